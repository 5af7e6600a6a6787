"""Damaged inputs through both readers and the native read loop: truncations, flipped bytes and
inserted garbage in every input form (SAM / BAM, plain / BGZF / gzip).  A reader may reject such an
input (htslib does: truncated file, bad magic, corrupt record), but it must do so with an error the
caller sees -- never a crash, a hang or a read outside its buffers.  The seeds are fixed; under
scripts/sanitize_host.sh (ASan / UBSan builds of the host code) the same cases check memory safety.
"""
import gzip
import random
import zlib

import pytest

from find_circ2_amd import cli
from find_circ2_amd.ingest import NativeIngest
from find_circ2_amd.samio import AlignmentFile
from oracle_engine import oracle_evaluator_factory
from samgen import bgzf_compress, sam_to_bam
from test_ingest import _mixed_sam


@pytest.fixture(scope="module")
def forms(tmp_path_factory):
    d = tmp_path_factory.mktemp("fuzz")
    sam = str(d / "mixed.sam")
    fa = _mixed_sam(sam, 160, seed=815)
    text = open(sam, "rb").read()
    data = {"sam": text, "sam_bgzf": bgzf_compress(text), "sam_gzip": gzip.compress(text)}
    for form, comp in (("bam_bgzf", "bgzf"), ("bam_gzip", "gzip"), ("bam_raw", "none")):
        p = str(d / (form + ".tmp"))
        sam_to_bam(text.decode("latin-1"), p, compress=comp)
        data[form] = open(p, "rb").read()
    return d, fa, data


def _damage(rng, data: bytes) -> bytes:
    kind = rng.randrange(4)
    if kind == 0:                                   # cut anywhere, the header included
        return data[:rng.randrange(len(data))]
    b = bytearray(data)
    if kind == 1:                                   # flip bytes past the first block's header
        for _ in range(rng.randint(1, 8)):
            i = rng.randrange(min(18, len(b) - 1), len(b))
            b[i] ^= 1 << rng.randrange(8)
        return bytes(b)
    if kind == 2:                                   # garbage spliced in
        i = rng.randrange(len(b))
        return bytes(b[:i]) + bytes(rng.randrange(256) for _ in range(rng.randint(1, 64))) + bytes(b[i:])
    return bytes(rng.randrange(256) for _ in range(rng.randint(0, 300)))   # noise


def _native_all(path):
    ing = NativeIngest(path, True)
    try:
        n = 0
        for _ in range(100000):
            frags = ing.next_chunk(15, False, False, 64)
            n += len(frags)
            if ing.eof and not frags:
                break
        return n
    finally:
        ing.close()


def _python_all(path):
    af = AlignmentFile(path, "rb")
    try:
        return sum(1 for _ in af)
    finally:
        af.close()


@pytest.mark.parametrize("form", ["sam", "sam_bgzf", "sam_gzip", "bam_bgzf", "bam_gzip", "bam_raw"])
def test_damaged_inputs_fail_cleanly_in_both_readers(forms, tmp_path, form):
    d, _, data = forms
    rng = random.Random(zlib.crc32(form.encode()))
    outcomes = {"ok": 0, "error": 0}
    for k in range(12):
        p = str(tmp_path / ("case%d" % k))
        with open(p, "wb") as fh:
            fh.write(_damage(rng, data[form]))
        for reader in (_native_all, _python_all):
            try:
                reader(p)
                outcomes["ok"] += 1
            except (OSError, ValueError, RuntimeError) as ex:     # the native reader: Fc2Error (RuntimeError)
                assert str(ex) or type(ex).__name__
                outcomes["error"] += 1
    assert outcomes["error"] > 0                 # the damage is seen, not read past


@pytest.mark.parametrize("form", ["sam", "bam_bgzf"])
def test_damaged_inputs_through_the_native_read_loop(forms, tmp_path, form):
    """The CLI's default loop (C++ read loop, oracle evaluator): a damaged input exits 1 or completes;
    its process survives either way."""
    d, fa, data = forms
    rng = random.Random(4711 + len(form))
    for k in range(8):
        p = str(tmp_path / ("in%d" % k))
        with open(p, "wb") as fh:
            fh.write(_damage(rng, data[form]))
        try:
            rc = cli.main(["-G", fa, "-o", str(tmp_path / ("o%d" % k)), "-q", p],
                          evaluator_factory=oracle_evaluator_factory)
        except (IOError, OSError, ValueError, RuntimeError, EOFError, KeyError, IndexError):
            rc = 1
        assert rc in (0, 1)


def _raw_bam(records):
    """Uncompressed BAM: one reference 'chr1' (1000 bp), then the given record bodies."""
    import struct
    text = b"@SQ\tSN:chr1\tLN:1000\n"
    out = b"BAM\x01" + struct.pack("<i", len(text)) + text + struct.pack("<i", 1)
    out += struct.pack("<i", 5) + b"chr1\x00" + struct.pack("<i", 1000)
    for body in records:
        out += struct.pack("<i", len(body)) + body
    return out


def _record(name=b"r1\x00", seq_len=4, tags=b"", l_seq=None, l_name=None):
    import struct
    cigar = struct.pack("<I", (seq_len << 4) | 0)                  # seq_len M
    body = struct.pack("<iiBBHHHiiii", 0, 10, len(name) if l_name is None else l_name, 60, 0, 1, 0,
                       seq_len if l_seq is None else l_seq, -1, -1, 0)
    return body + name + cigar + b"\x12" * ((seq_len + 1) // 2) + b"\x1e" * seq_len + tags


BAD_RECORDS = {
    "int_tag_cut_short": _record(tags=b"ASi\x05\x00"),
    "array_count_past_record": _record(tags=b"XBBi\x00\xca\x9a\x3b\x01\x00\x00\x00"),
    "string_without_nul": _record(tags=b"XZZabc"),
    "unknown_tag_type": _record(tags=b"ASq\x05\x00\x00\x00"),
    "seq_past_block": _record(l_seq=400),
    "name_without_nul": _record(name=b"r1x"),
    "tag_header_cut": _record(tags=b"AS"),
}


@pytest.mark.parametrize("case", sorted(BAD_RECORDS))
def test_corrupt_bam_records_are_errors(tmp_path, case):
    """Records htslib rejects (bam_read1's layout checks, corrupted aux data): both readers raise,
    neither reads past the record (the aux parser of round 3 did, found by the fuzz above)."""
    good = tmp_path / "good.bam"
    good.write_bytes(_raw_bam([_record(tags=b"ASC\x04"), _record(name=b"r2\x00", tags=b"ASi\x04\x00\x00\x00")]))
    assert _python_all(str(good)) == 2
    _native_all(str(good))
    p = tmp_path / "bad.bam"
    p.write_bytes(_raw_bam([_record(tags=b"ASC\x04"), BAD_RECORDS[case]]))
    with pytest.raises(RuntimeError, match="invalid BAM record|corrupted aux data"):
        _native_all(str(p))
    with pytest.raises(ValueError):
        _python_all(str(p))


@pytest.mark.parametrize("block", [None, "900"])
@pytest.mark.parametrize("form", ["bam_bgzf", "bam_gzip", "bam_raw", "sam"])
def test_parse_ahead_equals_sequential_reader_on_damage(forms, tmp_path, monkeypatch, form, block):
    """The native loop's parse-ahead threads (BAM: records cut into blocks from the decompressed
    stream; SAM: newline-aligned blocks; fragments grouped on the parse threads from each block's
    first closing record on) against the sequential reader the loop uses with -B: the same exit
    status on every damaged input and, when a run completes, the same files.  The reader must stop
    exactly where the sequential one reports the damage.  block: the parse block size in bytes
    (FC2_PARSE_BLOCK; default 4 MiB), small enough here for fragments to straddle blocks."""
    import gzip as gz
    import os
    if block:
        monkeypatch.setenv("FC2_PARSE_BLOCK", block)
    d, fa, data = forms
    rng = random.Random(2027 + len(form))
    n_err = 0
    for k in range(10):
        p = str(tmp_path / ("in%d" % k))
        with open(p, "wb") as fh:
            fh.write(data[form] if k == 0 else _damage(rng, data[form]))
        rcs, outs = [], []
        for tag, extra in (("ahead", []), ("seq", ["-B"])):
            o = str(tmp_path / ("o%d_%s" % (k, tag)))
            try:
                rc = cli.main(["-G", fa, "-o", o, "-q"] + extra + [p], evaluator_factory=oracle_evaluator_factory)
            except (IOError, OSError, ValueError, RuntimeError, EOFError, KeyError, IndexError):
                rc = 1
            rcs.append(rc)
            outs.append(o)
        assert rcs[0] == rcs[1], (k, rcs)
        n_err += rcs[0] != 0
        if rcs[0] == 0:
            for f in ("circ_splice_sites.bed", "lin_splice_sites.bed", "multi_events.tsv"):
                assert open(os.path.join(outs[0], f)).read() == open(os.path.join(outs[1], f)).read(), (k, f)
            with gz.open(os.path.join(outs[0], "spliced_reads.fastq.gz"), "rt") as a, \
                    gz.open(os.path.join(outs[1], "spliced_reads.fastq.gz"), "rt") as b:
                assert a.read() == b.read(), k
    assert n_err > 0


@pytest.fixture(scope="module")
def long_bam(tmp_path_factory):
    """The rich SAM with 80-kb unspliced reads spliced in (records longer than the inflated
    batches' 64-KiB headroom), as raw BAM bytes."""
    from test_native_caller import _rich_sam
    d = tmp_path_factory.mktemp("bgzf_split")
    sam = str(d / "rich.sam")
    fa = _rich_sam(sam, 600, seed=5150)
    lines = open(sam).read().splitlines()
    rng = random.Random(99)
    out, k = [], 0
    for l in lines:
        out.append(l)
        if not l.startswith("@") and rng.random() < 0.01:
            L = 80_000
            seq = "".join(rng.choice("ACGT") for _ in range(L))
            out.append("long%d\t0\tchr1\t%d\t60\t%dM\t*\t0\t0\t%s\t%s\tAS:i:%d" % (k, 1001, L, seq, "I" * L, L))
            k += 1
    text = "\n".join(out) + "\n"
    p = str(d / "raw.bam")
    sam_to_bam(text, p, compress="none")
    return d, fa, open(p, "rb").read()


@pytest.mark.parametrize("bgzf_block,batch,parse_block", [(3000, 2, None), (9000, 5, "20000"), (65280, 1, None),
                                                       (65280, 8, "100000"), (20000, 16, "7000")])
def test_bgzf_inplace_splitter_equals_copying_and_sequential(long_bam, tmp_path, monkeypatch, bgzf_block, batch,
                                                             parse_block):
    """The BGZF splitter that cuts parse blocks in place in the inflated batches (bgzf_split_loop:
    a record cut by a batch's end moved into the next batch's headroom, or joined by copy when it
    is longer than the headroom) against the sequential reader (-B): tiny BGZF blocks and batches of 1-16 blocks put batch boundaries inside
    records of every size; parse blocks smaller and larger than a BGZF block put the cuts inside the
    record lists the inflating threads made (RecLists: jumps to a list's cut or exit, a block inside an
    80-kb record with no list, the lists' guessed starts inside such records); the files are identical,
    on the whole input and on truncations."""
    import os
    d, fa, raw = long_bam
    monkeypatch.setenv("FC2_BGZF_BATCH", str(batch))
    monkeypatch.setenv("FC2_PARSE_INFLIGHT", "3")       # parse batches reused soon after they are read
    if parse_block:
        monkeypatch.setenv("FC2_PARSE_BLOCK", parse_block)
    data = bgzf_compress(raw, block=bgzf_block, level=1)
    rng = random.Random(bgzf_block)
    cuts = [len(data)] + [rng.randrange(len(data) // 3, len(data)) for _ in range(3)]
    for k, n in enumerate(cuts):
        p = str(tmp_path / ("in%d.bam" % k))
        with open(p, "wb") as fh:
            fh.write(data[:n])
        res = []
        for tag, extra in (("inplace", []), ("seq", ["-B"])):
            o = str(tmp_path / ("o%d_%s" % (k, tag)))
            try:
                rc = cli.main(["-G", fa, "-o", o, "-q"] + extra + [p], evaluator_factory=oracle_evaluator_factory)
            except (IOError, OSError, ValueError, RuntimeError, EOFError, KeyError, IndexError):
                rc = 1
            files = {}
            for f in ("circ_splice_sites.bed", "lin_splice_sites.bed", "multi_events.tsv"):
                fp = os.path.join(o, f)
                files[f] = open(fp).read() if os.path.exists(fp) else None
            fq = os.path.join(o, "spliced_reads.fastq.gz")
            files["reads"] = gzip.open(fq, "rt").read() if rc == 0 else None
            res.append((rc, files))
        assert res[0] == res[1], (k, n, [r[0] for r in res])
        if k == 0:
            assert res[0][0] == 0 and res[0][1]["circ_splice_sites.bed"].count("\n") > 20


_CLI_SCRIPT = """
import sys
sys.path[:0] = [%r]
from oracle_engine import oracle_evaluator_factory
from find_circ2_amd import cli
try:
    rc = cli.main(sys.argv[1:], evaluator_factory=oracle_evaluator_factory)
except Exception as e:
    print("RAISED", type(e).__name__, e, file=sys.stderr)
    rc = 1
sys.exit(rc)
"""


def test_libdeflate_and_zlib_give_the_same_run(long_bam, tmp_path):
    """BGZF blocks inflated and CRC-checked by libdeflate (default) or by zlib (FC2_LIBDEFLATE=0,
    the fallback without the library), spliced_reads.fastq.gz compressed by either: the same exit
    status and the same text on the whole input and on damaged copies (a flipped byte inside a
    block is caught by the CRC or the inflater in both)."""
    import os
    import subprocess
    import sys
    d, fa, raw = long_bam
    data = bgzf_compress(raw, block=20000, level=1)
    rng = random.Random(7)
    inputs = [data]
    for _ in range(3):
        b = bytearray(data)
        i = rng.randrange(100, len(b))
        b[i] ^= 1 << rng.randrange(8)
        inputs.append(bytes(b))
    script = _CLI_SCRIPT % os.path.dirname(os.path.abspath(__file__))
    for k, blob in enumerate(inputs):
        p = str(tmp_path / ("in%d.bam" % k))
        with open(p, "wb") as fh:
            fh.write(blob)
        res = []
        for lib in ("1", "0"):
            o = str(tmp_path / ("o%d_%s" % (k, lib)))
            env = dict(os.environ, FC2_LIBDEFLATE=lib, FC2_BGZF_BATCH="3")
            r = subprocess.run([sys.executable, "-c", script, "-G", fa, "-o", o, "-q", p], env=env,
                               capture_output=True, text=True, timeout=300)
            files = {}
            for f in ("circ_splice_sites.bed", "lin_splice_sites.bed", "multi_events.tsv"):
                fp = os.path.join(o, f)
                files[f] = open(fp).read() if os.path.exists(fp) else None
            fq = os.path.join(o, "spliced_reads.fastq.gz")
            files["reads"] = gzip.open(fq, "rt").read() if os.path.exists(fq) and r.returncode == 0 else None
            res.append((r.returncode, files))
        assert res[0] == res[1], (k, res[0][0], res[1][0])
        if k == 0:
            assert res[0][0] == 0 and res[0][1]["reads"].count("\n") > 100


def test_bgzf_splitter_jumps_through_record_lists(tmp_path):
    """A bwa-mem-shaped BAM of 60,000 reads in standard ~64-KiB BGZF blocks (scripts/gen_reads +
    fc2_sam_to_bam): the splitter finds nearly every parse block's cut through the record lists the
    inflating threads made (FC2_CALLER_TIMING's "bgzf split" line: jumps, and records read one at a
    time only where a list does not reach -- the first batch, a block's first record, a batch's
    end), with small parse blocks so the cuts land inside the lists too; the files equal the
    sequential reader's (-B)."""
    import os
    import re
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    gen = os.path.join(root, "scripts", "gen_reads")
    if not os.path.exists(gen):
        subprocess.check_call(["gcc", "-O2", "-o", gen, gen + ".c"])
    sq = tmp_path / "sq.tsv"
    sq.write_text("chrA\t300000\nchrB\t450000\nchrC\t250000\n")
    fa, sam, bam = str(tmp_path / "g.fa"), str(tmp_path / "r.sam"), str(tmp_path / "r.bam")
    subprocess.check_call([gen, str(sq), "60000", "11", fa, sam])
    from find_circ2_amd.ingest import sam_to_bam as native_sam_to_bam
    native_sam_to_bam(sam, bam)
    n_records = sum(1 for l in open(sam) if l[0] != "@")
    script = _CLI_SCRIPT % os.path.dirname(os.path.abspath(__file__))
    files = []
    for tag, extra, env_extra in (("lists", [], {"FC2_CALLER_TIMING": "1", "FC2_PARSE_BLOCK": "200000",
                                                 "FC2_BGZF_BATCH": "24"}),
                                  ("seq", ["-B"], {})):
        o = str(tmp_path / tag)
        env = dict(os.environ, **env_extra)
        r = subprocess.run([sys.executable, "-c", script, "-G", fa, "-o", o, "-q"] + extra + [bam], env=env,
                           capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stderr[-2000:]
        if tag == "lists":
            m = re.search(r"bgzf split: (\d+) records read one at a time, (\d+) jumps", r.stderr)
            assert m, r.stderr[-2000:]
            steps, jumps = int(m.group(1)), int(m.group(2))
            assert jumps > 100 and steps < n_records // 10, (steps, jumps, n_records)
        got = {}
        for f in ("circ_splice_sites.bed", "lin_splice_sites.bed", "multi_events.tsv"):
            got[f] = open(os.path.join(o, f)).read()
        got["reads"] = gzip.open(os.path.join(o, "spliced_reads.fastq.gz"), "rt").read()
        files.append(got)
    assert files[0] == files[1]
    assert files[0]["lin_splice_sites.bed"].count("\n") > 1000


@pytest.mark.parametrize("batch", ["2", "3", "8"])
def test_bgzf_oversized_members_through_the_splitter(long_bam, tmp_path, monkeypatch, batch):
    """Gzip members that inflate to far more than BGZF's 64 KiB (htslib reads them) in batches of 2-8
    blocks, through the in-place splitter and its record lists: the files equal the sequential
    reader's (-B), on the whole input and on truncations."""
    import os
    import subprocess
    import sys
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from test_input_format import _bgzf_blocks
    d, fa, raw = long_bam
    n = len(raw)
    import zlib

    def fits(a, b):                                  # a BGZF block holds at most 64 KiB compressed
        co = zlib.compressobj(6, zlib.DEFLATED, -15)
        return len(co.compress(raw[a:b]) + co.flush()) + 26 <= 65536

    edges = [0, 1, 7, 7, 5000, 70000, 70000]
    while edges[-1] < n:                             # then members of ~120-kB of input where they fit
        a, b = edges[-1], min(n, edges[-1] + 120000)
        while not fits(a, b):
            b = a + (b - a) // 2
        edges.append(b)
    data = _bgzf_blocks(raw, edges[1:-1])
    rng = random.Random(int(batch))
    script = _CLI_SCRIPT % os.path.dirname(os.path.abspath(__file__))
    for k, size in enumerate([len(data)] + [rng.randrange(len(data) // 3, len(data)) for _ in range(2)]):
        p = str(tmp_path / ("in%d.bam" % k))
        with open(p, "wb") as fh:
            fh.write(data[:size])
        res = []
        for tag, extra, env_extra in (("inplace", [], {}), ("seq", ["-B"], {})):
            o = str(tmp_path / ("o%d_%s" % (k, tag)))
            env = dict(os.environ, FC2_BGZF_BATCH=batch, FC2_INGEST_THREADS="3", **env_extra)
            r = subprocess.run([sys.executable, "-c", script, "-G", fa, "-o", o, "-q"] + extra + [p], env=env,
                               capture_output=True, text=True, timeout=300)
            files = {}
            for f in ("circ_splice_sites.bed", "lin_splice_sites.bed", "multi_events.tsv"):
                fp = os.path.join(o, f)
                files[f] = open(fp).read() if os.path.exists(fp) else None
            fq = os.path.join(o, "spliced_reads.fastq.gz")
            files["reads"] = gzip.open(fq, "rt").read() if os.path.exists(fq) and r.returncode == 0 else None
            res.append((r.returncode, files))
        assert res[0] == res[1], (k, size, [x[0] for x in res])
        if k == 0:
            assert res[0][0] == 0 and res[0][1]["circ_splice_sites.bed"].count("\n") > 20
