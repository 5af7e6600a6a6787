"""The alignment input's format comes from its bytes, never from its name or from stdin.

The reference opens ``pysam.Samfile(args[0], 'r' if args[0].endswith('sam') else 'rb')`` or
``pysam.Samfile('-', 'r')`` for stdin (find_circ.py:461-469); htslib's hts_open, under pysam,
detects the byte source (plain, BGZF, other gzip) and the format (BAM magic or SAM text) for
every read mode, so ``samtools view -b ... | find_circ.py`` reads BAM from stdin.  Both readers
here (the native ingest, include/fc2_ingest.h, and samio.AlignmentFile under --python-ingest)
must do the same: every form below writes files identical to the plain SAM file given by path.
"""
import gzip
import os
import subprocess
import sys

import pytest

from conftest import GOLDEN, ROOT, TESTS
from find_circ2_amd import cli
from find_circ2_amd.ingest import NativeIngest
from find_circ2_amd.samio import AlignmentFile
from oracle_engine import oracle_evaluator_factory
from samgen import bgzf_compress, sam_to_bam
from test_ingest import _mixed_sam, same

FORMS = {   # name -> (format, compression)
    "sam": ("sam", "plain"), "sam_bgzf": ("sam", "bgzf"), "sam_gzip": ("sam", "gzip"),
    "bam_bgzf": ("bam", "bgzf"), "bam_gzip": ("bam", "gzip"), "bam_raw": ("bam", "plain"),
}


@pytest.fixture(scope="module")
def inputs(tmp_path_factory):
    d = tmp_path_factory.mktemp("fmt")
    sam = str(d / "mixed.sam")
    fa = _mixed_sam(sam, 700, seed=4711)
    text = open(sam, "rb").read()
    data = {"sam": text, "sam_bgzf": bgzf_compress(text), "sam_gzip": gzip.compress(text)}
    for form, comp in (("bam_bgzf", "bgzf"), ("bam_gzip", "gzip"), ("bam_raw", "none")):
        p = str(d / (form + ".tmp"))
        sam_to_bam(text.decode("latin-1"), p, compress=comp)
        data[form] = open(p, "rb").read()
    base = {}
    for loop, ing in (("native", []), ("py", ["--python-ingest"])):
        out = str(d / ("base_" + loop))
        assert cli.main(["-G", fa, "-o", out, "-n", "fmt", "-q"] + ing + [sam],
                        evaluator_factory=oracle_evaluator_factory) == 0
        base[loop] = out
    same(base["native"], base["py"])
    return d, fa, data, base


def _write(d, name, data):
    p = str(d / name)
    with open(p, "wb") as fh:
        fh.write(data)
    return p


@pytest.mark.parametrize("form", sorted(FORMS))
def test_readers_detect_format_from_bytes(inputs, form):
    d, _, data, _ = inputs
    for name in ("x.sam", "x.bam", "x.txt"):
        p = _write(d, form + "_" + name, data[form])
        ing = NativeIngest(p, not name.endswith("sam"))
        try:
            assert ing.format() == FORMS[form]
            assert len(ing.references) == 3
        finally:
            ing.close()
        af = AlignmentFile(p, "r" if name.endswith("sam") else "rb")
        try:
            assert (af.format, af.compression) == FORMS[form]
            assert len(af.references) == 3 and sum(1 for _ in af) > 700
        finally:
            af.close()


@pytest.mark.parametrize("form", sorted(FORMS))
@pytest.mark.parametrize("name", ["x.sam", "x.bam"])
def test_cli_by_path_any_name(inputs, tmp_path, form, name):
    """A BAM named x.sam, SAM named x.bam, bgzip'ed / gzip'ed SAM: the same files as the SAM run."""
    d, fa, data, base = inputs
    p = _write(tmp_path, name, data[form])
    for loop, ing in (("native", []), ("py", ["--python-ingest"])):
        out = str(tmp_path / loop)
        assert cli.main(["-G", fa, "-o", out, "-n", "fmt", "-q"] + ing + [p],
                        evaluator_factory=oracle_evaluator_factory) == 0
        same(base[loop], out)


def _pipe(args, stdin_bytes, timeout=120):
    """The CLI as its own process, its stdin a pipe fed with stdin_bytes (``aligner | find_circ``)."""
    env = dict(os.environ, PYTHONPATH=os.pathsep.join([ROOT, TESTS]))
    return subprocess.run([sys.executable, os.path.join(TESTS, "cli_oracle_main.py")] + args, input=stdin_bytes,
                          stdout=subprocess.PIPE, stderr=subprocess.PIPE, env=env, timeout=timeout)


@pytest.mark.parametrize("form", ["bam_bgzf", "bam_gzip", "bam_raw", "sam", "sam_gzip"])
def test_cli_stdin_pipe(inputs, tmp_path, form):
    """``samtools view -b ... | find_circ -G g.fa -o out``: north_star's stdin-BAM CLI."""
    d, fa, data, base = inputs
    loops = (("native", []), ("py", ["--python-ingest"])) if form in ("bam_bgzf", "sam") else (("native", []),)
    for loop, ing in loops:
        out = str(tmp_path / loop)
        r = _pipe(["-G", fa, "-o", out, "-n", "fmt", "-q"] + ing, data[form])
        assert r.returncode == 0, r.stderr.decode()[-2000:]
        same(base[loop], out)


def test_cli_stdin_bam_writes_same_anchor_bam(inputs, tmp_path):
    """-B with BAM on stdin copies the same records as with the BAM file by path."""
    d, fa, data, base = inputs
    p = _write(tmp_path, "in.bam", data["bam_bgzf"])
    o1, o2 = str(tmp_path / "path"), str(tmp_path / "pipe")
    assert cli.main(["-G", fa, "-o", o1, "-n", "fmt", "-q", "-B", p], evaluator_factory=oracle_evaluator_factory) == 0
    r = _pipe(["-G", fa, "-o", o2, "-n", "fmt", "-q", "-B"], data["bam_bgzf"])
    assert r.returncode == 0, r.stderr.decode()[-2000:]
    same(o1, o2)
    b1 = gzip.open(os.path.join(o1, "spliced_alignments.bam")).read()
    b2 = gzip.open(os.path.join(o2, "spliced_alignments.bam")).read()
    assert b1 == b2 and len(b1) > 1000


@pytest.mark.parametrize("form", ["bam_bgzf", "bam_gzip", "sam_bgzf", "sam_gzip"])
def test_truncated_compressed_input_fails(inputs, tmp_path, form):
    """A compressed stream cut short is an error (htslib: truncated file), not a silent end."""
    d, fa, data, _ = inputs
    p = _write(tmp_path, "cut", data[form][:len(data[form]) * 3 // 5])
    for ing in ([], ["--python-ingest"]):
        out = str(tmp_path / ("o%d" % len(ing)))
        try:
            rc = cli.main(["-G", fa, "-o", out, "-q"] + ing + [p], evaluator_factory=oracle_evaluator_factory)
        except Exception:
            rc = 1
        assert rc == 1, (form, ing)


def test_cram_is_refused(tmp_path):
    p = _write(tmp_path, "x.cram", b"CRAM\x03\x00" + b"\x00" * 64)
    with pytest.raises(Exception, match="CRAM"):
        NativeIngest(p, True)
    with pytest.raises(ValueError, match="CRAM"):
        AlignmentFile(p, "rb")


def test_golden_known_answers_through_stdin_bam(tmp_path):
    """The reference's own known answers (test_reads.fa truth, find_circ.py --test) with BAM on stdin."""
    from bwa_emul import read_fasta
    from samgen import sam_text
    from test_cli import _reads, bed_rows
    fa = os.path.join(GOLDEN, "test_ref.fa")
    sam = sam_text(read_fasta(fa), _reads(os.path.join(GOLDEN, "test_reads.fa")))
    p = str(tmp_path / "in.bam")
    sam_to_bam(sam, p)
    out = str(tmp_path / "o")
    r = _pipe(["-G", fa, "-o", out, "-n", "test", "-q", "--test"], open(p, "rb").read())
    assert r.returncode == 0, r.stderr.decode()[-2000:]
    circ = bed_rows(os.path.join(out, "circ_splice_sites.bed"))
    assert {("testbed_plus", 240, 320, "+"), ("testbed_plus", 80, 640, "+")} <= set(circ)


def test_native_sam_to_bam_reads_back_as_the_sam(inputs, tmp_path):
    """fc2_sam_to_bam (the bench's BAM maker) against the Python test encoder: the CLI on either BAM
    writes the SAM run's files."""
    from find_circ2_amd.ingest import sam_to_bam as native_sam_to_bam
    d, fa, data, base = inputs
    sam = _write(tmp_path, "in.sam", data["sam_gzip"])
    bam = str(tmp_path / "n.bam")
    native_sam_to_bam(sam, bam)
    ing = NativeIngest(bam, True)
    assert ing.format() == ("bam", "bgzf")
    ing.close()
    r = _pipe(["-G", fa, "-o", str(tmp_path / "o"), "-n", "fmt", "-q"], open(bam, "rb").read())
    assert r.returncode == 0, r.stderr.decode()[-2000:]
    same(base["native"], str(tmp_path / "o"))
    with pytest.raises(Exception, match="BAM already"):
        native_sam_to_bam(bam, str(tmp_path / "again.bam"))


def _bgzf_blocks(data: bytes, cuts):
    """BGZF with block boundaries at `cuts` (and an empty block at each cut listed twice)."""
    import struct
    import zlib
    out = bytearray()
    edges = [0] + list(cuts) + [len(data)]
    for a, b in zip(edges, edges[1:]):
        chunk = data[a:b]
        co = zlib.compressobj(6, zlib.DEFLATED, -15)
        cdata = co.compress(chunk) + co.flush()
        bsize = 18 + len(cdata) + 8
        out += b"\x1f\x8b\x08\x04\x00\x00\x00\x00\x00\xff\x06\x00BC\x02\x00" + struct.pack("<H", bsize - 1)
        out += cdata + struct.pack("<II", zlib.crc32(chunk) & 0xFFFFFFFF, len(chunk))
    return bytes(out)


def test_edge_forms_read_like_the_plain_sam(inputs, tmp_path):
    """BGZF with empty blocks and record-splitting block edges, no EOF marker; concatenated gzip
    members of SAM; the same bytes on a stdin pipe: the SAM run's files, both loops."""
    d, fa, data, base = inputs
    sam = data["sam"]
    bam = gzip.decompress(data["bam_gzip"])
    forms = {
        "bam_odd_blocks": _bgzf_blocks(bam, [1, 7, 7, 5000, 65000, 65000, len(bam) - 3]),
        "sam_odd_blocks": _bgzf_blocks(sam, [10, 10, len(sam) // 2]),
        "sam_gzip_members": gzip.compress(sam[:len(sam) // 3]) + gzip.compress(sam[len(sam) // 3:]),
    }
    for name, blob in forms.items():
        p = _write(tmp_path, name, blob)
        for loop, ing in (("native", []), ("py", ["--python-ingest"])):
            out = str(tmp_path / (name + loop))
            assert cli.main(["-G", fa, "-o", out, "-n", "fmt", "-q"] + ing + [p],
                            evaluator_factory=oracle_evaluator_factory) == 0, (name, loop)
            same(base[loop], out)
    r = _pipe(["-G", fa, "-o", str(tmp_path / "pipe_odd"), "-n", "fmt", "-q"], forms["bam_odd_blocks"])
    assert r.returncode == 0, r.stderr.decode()[-2000:]
    same(base["native"], str(tmp_path / "pipe_odd"))


@pytest.mark.parametrize("form", ["empty", "sam_header_only", "bam_header_only", "bgzf_eof_only"])
def test_inputs_without_records(tmp_path, form):
    """No alignment records at all.  With a header that declares the references both loops finish
    with empty tables (no UnboundLocalError, which the reference raises only for exactly one record,
    find_circ.py:1486).  Without one -- an empty stream, an empty BGZF file -- pysam.Samfile's header
    check (check_sq) raises ValueError when the reference opens the input (find_circ.py:461-469):
    both loops exit with status 1 and that error, and write no table rows."""
    fa = os.path.join(GOLDEN, "test_ref.fa")
    hdr = "@SQ\tSN:testbed_plus\tLN:720\n@SQ\tSN:testbed_minus\tLN:720\n"
    if form == "empty":
        blob = b""
    elif form == "sam_header_only":
        blob = hdr.encode()
    elif form == "bam_header_only":
        p = str(tmp_path / "h.bam")
        sam_to_bam(hdr, p)
        blob = open(p, "rb").read()
    else:
        blob = bytes.fromhex("1f8b08040000000000ff0600424302001b0003000000000000000000")
    outs = []
    for loop, ing in (("native", []), ("py", ["--python-ingest"])):
        out = str(tmp_path / loop)
        r = _pipe(["-G", fa, "-o", out, "-q"] + ing, blob)
        outs.append(out)
        rows = [l for l in open(os.path.join(out, "circ_splice_sites.bed")) if not l.startswith("#")]
        assert rows == []
        if form in ("empty", "bgzf_eof_only"):
            assert r.returncode == 1, (form, loop)
            assert "ValueError: file has no sequences defined (mode='r')" in r.stderr.decode(), r.stderr.decode()
            continue
        assert r.returncode == 0, (form, loop, r.stderr.decode()[-2000:])
    if form not in ("empty", "bgzf_eof_only"):
        same(outs[0], outs[1])


@pytest.mark.parametrize("body", ["", "sam_no_sq", "sam_text"])
def test_bam_named_inputs(tmp_path, body):
    """A path not ending in 'sam' is opened with mode 'rb' by the reference (find_circ.py:463-466).
    An empty x.bam (what a crashed aligner leaves behind) or one holding SAM text without @SQ fails
    pysam's header check with ValueError; SAM text with a header is read as SAM (htslib detects the
    format from the bytes), with a warning in run.log.  All three read loops agree."""
    fa = os.path.join(GOLDEN, "test_ref.fa")
    rec = "r1\t0\ttestbed_plus\t10\t60\t20M\t*\t0\t0\t%s\t*\tAS:i:20\n" % ("A" * 20)
    text = {"": "", "sam_no_sq": rec + rec.replace("r1", "r2"),
            "sam_text": "@SQ\tSN:testbed_plus\tLN:720\n" + rec + rec.replace("r1", "r2")}[body]
    p = str(tmp_path / "aln.bam")
    open(p, "w").write(text)
    for loop, mode in (("native", []), ("pyc", ["--python-caller"]), ("py", ["--python-ingest"])):
        out = str(tmp_path / loop)
        rc = cli.main(["-G", fa, "-o", out, "-q"] + mode + [p], evaluator_factory=oracle_evaluator_factory)
        log = open(os.path.join(out, "run.log")).read()
        if body == "sam_text":
            assert rc == 0, (loop, log[-1000:])
            assert "holds SAM text: read as SAM" in log
        else:
            assert rc == 1, loop
            assert "ValueError: file has no sequences defined (mode='rb')" in log, log[-1000:]
