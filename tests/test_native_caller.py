"""Native caller (include/fc2_caller.h) == the Python caller, file for file.

The default CLI runs the whole read loop in C++ (grouping, process_mate,
record_hits, the junction tables, the writers) and hands only the breakpoint
search to the batch evaluator.  ``--python-caller`` keeps the loop in Python
(find_circ2_amd.caller, the line-by-line restatement of find_circ.py:1450-1527
and :976-1447) on the same native ingest, and ``--python-ingest`` in Python
end to end.  With the CPU oracle as the breakpoint search behind both hooks,
every output file and every counter in run.log must agree across the three,
for SAM and BAM input, every option that changes the host logic, known
junction files, and the inputs on which the reference raises.
"""
import os

import numpy as np
import pytest

from conftest import GOLDEN, ROOT
from find_circ2_amd import cli
from oracle_engine import oracle_evaluator_factory
from bwa_emul import read_fasta
from samgen import sam_text, sam_to_bam
from test_cli import _reads, run_cli
from test_ingest import _mixed_sam, counters, same


def _three(tmp_path, fa, inp, extra, tag=""):
    outs, rcs = [], []
    for t, mode in (("py", ["--python-ingest"]), ("pyc", ["--python-caller"]), ("nat", [])):
        out = str(tmp_path / (tag + t))
        rcs.append(cli.main(["-G", fa, "-o", out, "-n", "mix", "-q"] + list(extra) + mode + [inp],
                            evaluator_factory=oracle_evaluator_factory))
        outs.append(out)
    return rcs, outs


@pytest.fixture(scope="module")
def mixed(tmp_path_factory):
    d = tmp_path_factory.mktemp("mixed")
    sam = str(d / "mixed.sam")
    fa = _mixed_sam(sam, 2000, seed=4242)
    bam = str(d / "mixed.bam")
    sam_to_bam(open(sam).read(), bam)
    return fa, sam, bam


OPTION_SETS = [[], ["--test"], ["--all-hits", "--non-canonical"], ["--all-hits", "--strand-pref", "-d", "0"],
               ["-d", "0"], ["--half-unique", "--report-nobridges"], ["--no-linear"], ["--no-multi"], ["--noop"],
               ["--min-uniq-qual", "0", "-a", "12", "-m", "0"], ["--min-uniq-qual", "9", "-m", "4", "-d", "3"],
               ["--short-threshold", "1000", "--huge-threshold", "2000"], ["--chunk-size", "13"],
               ["--stdout", "multi"]]


@pytest.mark.parametrize("extra", OPTION_SETS, ids=[" ".join(e) or "default" for e in OPTION_SETS])
def test_native_caller_equals_python_mixed(tmp_path, mixed, extra, capsys):
    fa, sam, bam = mixed
    rcs, outs = _three(tmp_path, fa, sam, extra)
    assert rcs == [0, 0, 0]
    if "--stdout" in extra:
        cap = capsys.readouterr().out
        third = len(cap) // 3
        assert cap[:third] == cap[third:2 * third] == cap[2 * third:]
    same(outs[0], outs[1])
    same(outs[0], outs[2])
    if not extra:
        c = counters(outs[2])
        assert c["circ_spliced"] > 5 and c["lin_spliced"] + c["lin_no_bp"] > 200


def test_native_caller_bam_equals_sam(tmp_path, mixed):
    fa, sam, bam = mixed
    rc1 = cli.main(["-G", fa, "-o", str(tmp_path / "s"), "-q", sam], evaluator_factory=oracle_evaluator_factory)
    rc2 = cli.main(["-G", fa, "-o", str(tmp_path / "b"), "-q", bam], evaluator_factory=oracle_evaluator_factory)
    assert rc1 == rc2 == 0
    same(str(tmp_path / "s"), str(tmp_path / "b"))


@pytest.mark.parametrize("fa,rf", [("test_ref.fa", "test_reads.fa"), ("CDR1as_locus.fa", "cdr1as_reads.fa")])
@pytest.mark.parametrize("extra", [["--test"], ["--test", "--all-hits", "--non-canonical"]])
def test_native_caller_equals_python_golden(tmp_path, fa, rf, extra):
    fa = os.path.join(GOLDEN, fa)
    rd = _reads(os.path.join(GOLDEN, rf))
    _, o1 = run_cli(tmp_path, fa, rd, extra=extra + ["--python-caller"], tag="py")
    _, o2 = run_cli(tmp_path, fa, rd, extra=extra, tag="native")
    same(o1, o2)


def _known_bed(path, rows, extra_rows):
    with open(path, "w") as f:
        f.write("#chrom\tstart\tend\tname\tscore\tstrand\n")
        for r in rows + extra_rows:
            f.write("\t".join(str(x) for x in r) + "\n")


def test_native_caller_known_sites(tmp_path, mixed):
    """--known-circ/--known-lin: known names replace novel ones, the table keeps file order
    and a repeated coordinate keeps its first position; unobserved known sites stay unreported."""
    fa, sam, _ = mixed
    rcs, outs = _three(tmp_path, fa, sam, [], tag="pre")
    circ = [l.split("\t") for l in open(os.path.join(outs[0], "circ_splice_sites.bed")) if l[0] != "#"]
    lin = [l.split("\t") for l in open(os.path.join(outs[0], "lin_splice_sites.bed")) if l[0] != "#"]
    assert len(circ) > 4 and len(lin) > 4
    rng = np.random.default_rng(3)
    pick = lambda rows: [rows[i] for i in sorted(rng.choice(len(rows), len(rows) // 2, replace=False))]  # noqa
    kc = [(r[0], r[1], r[2], "KC%d" % i, 0, r[5]) for i, r in enumerate(pick(circ))]
    kl = [(r[0], r[1], r[2], "KL%d" % i, 0, r[5]) for i, r in enumerate(pick(lin))]
    c0 = circ[0][0]
    _known_bed(str(tmp_path / "kc.bed"), kc, [(c0, 5, 900, "never_seen", 0, "+"), kc[0][:3] + ("dup", 0, kc[0][5])])
    _known_bed(str(tmp_path / "kl.bed"), kl, [(c0, 7, 77, "never_seen_lin", 0, "-")])
    extra = ["--known-circ", str(tmp_path / "kc.bed"), "--known-lin", str(tmp_path / "kl.bed")]
    rcs, outs = _three(tmp_path, fa, sam, extra)
    assert rcs == [0, 0, 0]
    same(outs[0], outs[1])
    same(outs[0], outs[2])
    txt = open(os.path.join(outs[2], "circ_splice_sites.bed")).read()
    assert "never_seen" not in txt and txt.count("\tKC") > 1
    log = open(os.path.join(outs[2], "run.log")).read()
    assert "loaded %d known splice sites" % (len(kc) + 2) in log


def test_native_caller_missing_chromosome_fails_like_python(tmp_path, mixed):
    """A SAM reference absent from the FASTA: KeyError(chrom) in get_data (find_circ.py:193)."""
    fa, sam, _ = mixed
    txt = open(sam).read().replace("SN:chr2\t", "SN:chrX\t").replace("\tchr2\t", "\tchrX\t")
    bad = str(tmp_path / "bad.sam")
    open(bad, "w").write(txt)
    rcs, outs = _three(tmp_path, fa, bad, [])
    assert rcs == [1, 1, 1]
    for o in outs[1:]:
        assert "KeyError: 'chrX'" in open(os.path.join(o, "run.log")).read()


def test_native_caller_stranded_fails_like_reference(tmp_path):
    fa = os.path.join(GOLDEN, "test_ref.fa")
    rd = _reads(os.path.join(GOLDEN, "test_reads.fa"))
    rc1, _ = run_cli(tmp_path, fa, rd, extra=["--stranded", "--python-caller"], tag="py")
    rc2, o2 = run_cli(tmp_path, fa, rd, extra=["--stranded"], tag="nat")
    assert rc1 == rc2 == 1
    assert "AttributeError" in open(os.path.join(o2, "run.log")).read()


def test_native_caller_single_record_fails_like_reference(tmp_path):
    fa = os.path.join(GOLDEN, "test_ref.fa")
    sam = tmp_path / "one.sam"
    sam.write_text("@SQ\tSN:testbed_plus\tLN:720\nr\t0\ttestbed_plus\t10\t60\t20M\t*\t0\t0\t%s\t*\tAS:i:20\n"
                   % ("A" * 20))
    rcs, outs = _three(tmp_path, fa, str(sam), [])
    assert rcs == [1, 1, 1]
    assert "UnboundLocalError" in open(os.path.join(outs[2], "run.log")).read()


def _rich_sam(path, n_frag, seed, secondary_same_chrom=False):
    """bwa-mem-like SAM with GT/AG (or CT/AC) planted at every junction: 2- and 3-segment linear
    and circular reads, paired mates (unspliced inside/outside the circle, on another chromosome,
    linearly spliced), supplementary/secondary records, uniqueness from AS/XS, N and mismatches."""
    rng = np.random.default_rng(seed)
    names = ["chr1", "chr2", "chr3"]
    size = 90_000
    g = {c: bytearray(np.frombuffer(b"ACGT", np.uint8)[rng.integers(0, 4, size)].tobytes()) for c in names}

    def plant(c, istart, iend, minus):
        g[c][istart:istart + 2] = b"CT" if minus else b"GT"
        g[c][iend - 2:iend] = b"AC" if minus else b"AG"

    frags = []                          # list of mates; a mate = list of (chrom, gpos, qlen)
    for i in range(n_frag):
        c = names[int(rng.integers(3))]
        minus = rng.random() < 0.4

        def unspliced(L=100, lo=1000, hi=size - 1000, chrom=c):
            p = int(rng.integers(lo, max(lo + 1, hi - L)))
            return [(chrom, min(max(p, 0), size - L - 1), L)]

        def lin(nseg, L=100):
            cuts = sorted(rng.choice(np.arange(12, L - 12), nseg - 1, replace=False))
            lens = np.diff([0] + list(cuts) + [L])
            p = int(rng.integers(2000, size - 20000))
            segs = []
            for k, ln in enumerate(lens):
                segs.append((c, p, int(ln)))
                if k < nseg - 1:
                    nxt = p + int(ln) + int(rng.integers(60, 3000))
                    plant(c, p + int(ln), nxt, minus)
                    p = nxt
            return segs

        def circ(nseg, L=100):
            kA = int(rng.integers(12, L - 12))
            span = int(rng.integers(150, 6000))
            E = int(rng.integers(span + 500, size - 2000))
            S = E - span
            plant(c, E, S, minus)
            if nseg == 2:
                return [(c, E - kA, kA), (c, S, L - kA)]
            k1 = int(rng.integers(12, L - kA - 12 + 1)) if L - kA - 24 > 0 else (L - kA) // 2
            mid = S + k1 + int(rng.integers(40, max(41, span - k1 - kA - 40)))
            mid = min(mid, E - kA - 20)
            plant(c, S + k1, mid, minus)
            return [(c, E - kA, kA), (c, S, k1), (c, mid, L - kA - k1)]

        kind = rng.random()
        if kind < 0.15:
            frags.append([unspliced()])
        elif kind < 0.3:
            frags.append([lin(2)])
        elif kind < 0.4:
            frags.append([lin(3)])
        elif kind < 0.55:
            frags.append([circ(2)])
        elif kind < 0.6:
            frags.append([circ(3)])
        else:
            m1 = circ(2) if rng.random() < 0.75 else lin(2)
            lo = min(s[1] for s in m1)
            hi = max(s[1] + s[2] for s in m1)
            r = rng.random()
            if r < 0.35:
                m2 = unspliced(lo=lo, hi=hi + 100)                           # inside the circle
            elif r < 0.6:
                m2 = unspliced(lo=hi + 200, hi=hi + 5000)                    # outside
            elif r < 0.7:
                m2 = unspliced(chrom=names[(names.index(c) + 1) % 3])        # another chromosome
            elif r < 0.9:
                m2 = lin(2)
            else:
                m2 = circ(2)
            frags.append([m1, m2])

    ok = lambda segs: all(ln > 0 and 0 <= p and p + ln <= size for _, p, ln in segs)  # noqa: E731
    frags = [[m if ok(m) else [(m[0][0], 5000, 100)] for m in mates] for mates in frags]
    lines = ["@HD\tVN:1.5"] + ["@SQ\tSN:%s\tLN:%d" % (c, size) for c in names]
    for i, mates in enumerate(frags):
        qn = "f%05d" % i
        if rng.random() < 0.03:
            lines.append("%s\t4\t*\t0\t0\t*\t*\t0\t0\t%s\t*" % (qn, "A" * 100))
            continue
        for mi, segs in enumerate(mates):
            mf = 0 if len(mates) == 1 else (0x41 if mi == 0 else 0x81)
            if mf and rng.random() < 0.7:
                mf |= 0x2
            rev = 16 if rng.random() < 0.3 else 0
            read = bytearray(b"".join(bytes(g[c][p:p + ln]) for c, p, ln in segs))
            for _ in range(int(rng.integers(0, 3))):                        # mismatches
                k = int(rng.integers(len(read)))
                read[k] = b"ACGT"[(b"ACGT".index(read[k]) + 1) % 4] if read[k] in b"ACGT" else read[k]
            if rng.random() < 0.05:
                read[int(rng.integers(len(read)))] = ord("N")
            seq = read.decode()
            qual = "*" if rng.random() < 0.1 else "".join(chr(33 + int(q)) for q in rng.integers(2, 40, len(seq)))
            prim = int(rng.integers(len(segs)))
            q0 = 0
            recs = []
            for k, (c, p, ln) in enumerate(segs):
                before, after = q0, len(seq) - q0 - ln
                clip = "S" if k == prim else "H"
                cig = ("%d%s" % (before, clip) if before else "") + "%dM" % ln + ("%d%s" % (after, clip) if after else "")
                s_ = seq if k == prim else seq[q0:q0 + ln]
                qq = qual if (k == prim or qual == "*") else qual[q0:q0 + ln]
                asv = ln - int(rng.integers(0, 3))
                tags = "AS:i:%d" % asv
                if rng.random() < 0.6:
                    tags += "\tXS:i:%d" % int(rng.integers(0, asv + 2))
                fl = mf | rev | (0 if k == prim else 2048)
                recs.append((k != prim, "%s\t%d\t%s\t%d\t%d\t%s\t*\t0\t0\t%s\t%s\t%s" %
                             (qn, fl, c, p + 1, int(rng.integers(0, 61)), cig, s_, qq, tags)))
                q0 += ln
            recs.sort(key=lambda t: t[0])
            lines += [t[1] for t in recs]
            if rng.random() < 0.05:
                c, p, ln = segs[0]
                if not secondary_same_chrom:
                    c = names[(names.index(c) + 1) % 3]
                lines.append("%s\t%d\t%s\t%d\t0\t%dM\t*\t0\t0\t*\t*\tAS:i:%d" % (qn, mf | 256, c, p + 501, ln, ln - 3))
    with open(path, "w") as f:
        f.write("\n".join(lines) + "\n")
    fa = path + ".fa"
    with open(fa, "w") as f:
        for c in names:
            f.write(">%s\n" % c)
            s = g[c].decode()
            for k in range(0, size, 70):
                f.write(s[k:k + 70] + "\n")
    return fa


RICH_SETS = [[], ["--all-hits", "--non-canonical", "--strand-pref"], ["--half-unique", "--report-nobridges"],
             ["-d", "0", "--min-uniq-qual", "0"], ["--no-linear"], ["--chunk-size", "5", "--all-hits"]]


@pytest.mark.parametrize("extra", RICH_SETS, ids=[" ".join(e) or "default" for e in RICH_SETS])
def test_native_caller_equals_python_rich(tmp_path, extra):
    sam = str(tmp_path / "rich.sam")
    fa = _rich_sam(sam, 2500, seed=97)
    rcs, outs = _three(tmp_path, fa, sam, extra)
    assert rcs == [0, 0, 0]
    same(outs[0], outs[1])
    same(outs[0], outs[2])
    if not extra:
        c = counters(outs[2])
        assert c["circ_spliced"] > 300 and c["lin_spliced"] > 300
        multi = open(os.path.join(outs[2], "multi_events.tsv")).read().splitlines()
        assert len(multi) > 50


def test_native_caller_secondary_without_seq_fails_like_python(tmp_path):
    """A SEQ-less secondary hit next to the primary joins proper_segs; len(None) raises
    (find_circ.py:1101, pysam query of SEQ "*") in all three read loops."""
    sam = str(tmp_path / "sec.sam")
    fa = _rich_sam(sam, 800, seed=5, secondary_same_chrom=True)
    rcs, outs = _three(tmp_path, fa, sam, [])
    assert rcs == [1, 1, 1]
    assert "TypeError: object of type 'NoneType' has no len()" in open(os.path.join(outs[2], "run.log")).read()


@pytest.mark.parametrize("threads", ["1", "3"])
def test_bam_plain_gzip_and_bgzf_agree(tmp_path, mixed, threads, monkeypatch):
    """BGZF blocks are inflated in parallel batches (FC2_INGEST_THREADS); a BAM written as one
    plain gzip member takes the streaming path.  Both give the SAM run's files."""
    fa, sam, bam = mixed
    plain = str(tmp_path / "plain.bam")
    sam_to_bam(open(sam).read(), plain, bgzf=False)
    monkeypatch.setenv("FC2_INGEST_THREADS", threads)
    outs = []
    for tag, inp in (("sam", sam), ("bgzf", bam), ("plain", plain)):
        out = str(tmp_path / tag)
        assert cli.main(["-G", fa, "-o", out, "-q", "--all-hits", inp], evaluator_factory=oracle_evaluator_factory) == 0
        outs.append(out)
    same(outs[0], outs[1])
    same(outs[0], outs[2])


def test_corrupt_bgzf_block_fails(tmp_path, mixed):
    fa, sam, bam = mixed
    data = bytearray(open(bam, "rb").read())
    data[len(data) // 2] ^= 0xFF                   # inside some block's deflate data
    bad = str(tmp_path / "bad.bam")
    open(bad, "wb").write(bytes(data))
    out = str(tmp_path / "o")
    # small input: the first batch of blocks holds the BAM header too, so opening fails (an uncaught
    # exception where pysam opens the input, find_circ.py:461-469: traceback, exit status 1)
    assert cli.main(["-G", fa, "-o", out, "-q", bad], evaluator_factory=oracle_evaluator_factory) == 1
    assert "corrupt BGZF block" in open(os.path.join(out, "run.log")).read()


def test_native_caller_reads_stdin(tmp_path, mixed):
    """No input argument: SAM text from stdin (find_circ.py:461-469), as from `bwa mem | find_circ`."""
    import subprocess
    import sys
    fa, sam, _ = mixed
    here = os.path.dirname(os.path.abspath(__file__))
    out1, out2 = str(tmp_path / "file"), str(tmp_path / "stdin")
    assert cli.main(["-G", fa, "-o", out1, "-q", sam], evaluator_factory=oracle_evaluator_factory) == 0
    code = ("import sys; sys.path[:0] = [%r, %r]\n"
            "from oracle_engine import oracle_evaluator_factory\n"
            "from find_circ2_amd import cli\n"
            "sys.exit(cli.main(['-G', %r, '-o', %r, '-q'], evaluator_factory=oracle_evaluator_factory))"
            % (here, os.path.dirname(here), fa, out2))
    with open(sam, "rb") as fh:
        r = subprocess.run([sys.executable, "-c", code], stdin=fh, capture_output=True, timeout=300)
    assert r.returncode == 0, r.stderr.decode()[-2000:]
    same(out1, out2)
    assert "reading from stdin" in open(os.path.join(out2, "run.log")).read()


@pytest.mark.parametrize("body", ["", "u1\t4\t*\t0\t0\t*\t*\t0\t0\tACGT\t####\nu2\t4\t*\t0\t0\t*\t*\t0\t0\tACGT\t####\n",
                                  "\n\n"], ids=["header_only", "only_unmapped", "blank_lines"])
def test_native_caller_degenerate_inputs(tmp_path, body):
    """Header-only input (the reference's generator ends at the first next(), find_circ.py:1458),
    unmapped-only input (the first record still opens a mate, :1462-1463) and blank lines."""
    fa = os.path.join(GOLDEN, "test_ref.fa")
    sam = str(tmp_path / "d.sam")
    open(sam, "w").write("@SQ\tSN:testbed_plus\tLN:720\n" + body)
    rcs, outs = _three(tmp_path, fa, sam, [])
    assert rcs[0] == rcs[1] == rcs[2] == 0
    same(outs[0], outs[1])
    same(outs[0], outs[2])
    rows = [l for l in open(os.path.join(outs[2], "circ_splice_sites.bed")) if not l.startswith("#")]
    assert rows == []


@pytest.mark.parametrize("n_filler", [0, 9, 62, 70])
def test_native_caller_many_sam_tags(tmp_path, n_filler):
    """The SAM parser collects a line's tabs in one pass (64 at most, then it falls back to a
    per-tag scan): AS / XS found after many filler tags, first occurrence winning, the same files
    as the Python ingest."""
    sam0 = str(tmp_path / "base.sam")
    fa = _rich_sam(sam0, 300, seed=4242)
    out_lines = []
    for line in open(sam0).read().splitlines():
        if line.startswith("@"):
            out_lines.append(line)
            continue
        f = line.split("\t")
        filler = ["Z%d:i:%d" % (k % 10, k) for k in range(n_filler)]
        # a second, later AS: uniqness() reads the first (get_tag, find_circ.py:814), Hit.add the
        # last (dict(tags), :556-557) -- the anchor-quality columns show which one was used
        first_as = [int(t[5:]) for t in f[11:] if t.startswith("AS:i:")][:1]
        dup = ["AS:i:%d" % (first_as[0] + 5)] if first_as else []
        out_lines.append("\t".join(f[:11] + filler + f[11:] + dup))
    sam = str(tmp_path / "t.sam")
    open(sam, "w").write("\n".join(out_lines) + "\n")
    o1, o2 = str(tmp_path / "py"), str(tmp_path / "native")
    rc1 = cli.main(["-G", fa, "-o", o1, "-q", "--python-caller", sam], evaluator_factory=oracle_evaluator_factory)
    rc2 = cli.main(["-G", fa, "-o", o2, "-q", sam], evaluator_factory=oracle_evaluator_factory)
    assert rc1 == rc2 == 0
    same(o1, o2)
    assert sum(1 for l in open(os.path.join(o2, "circ_splice_sites.bed")) if l[0] != "#") > 20
    bam = str(tmp_path / "t.bam")                  # the BAM aux parser: same rule
    sam_to_bam(open(sam).read(), bam)
    o3 = str(tmp_path / "native_bam")
    assert cli.main(["-G", fa, "-o", o3, "-q", bam], evaluator_factory=oracle_evaluator_factory) == 0
    same(o1, o3)


def test_native_reads_gz_members(tmp_path, monkeypatch):
    """spliced_reads.fastq.gz compressed by the native loop (fc2_caller_set_reads_gz) in small
    pieces -- many gzip members, written in order on worker threads -- reads back as the text the
    Python loop writes."""
    import gzip
    import zlib
    from find_circ2_amd import gzout
    sam = str(tmp_path / "rich.sam")
    fa = _rich_sam(sam, 800, seed=77)
    o1, o2 = str(tmp_path / "py"), str(tmp_path / "native")
    assert cli.main(["-G", fa, "-o", o1, "-q", "--python-caller", sam], evaluator_factory=oracle_evaluator_factory) == 0
    orig = gzout.ParallelGzipWriter.__init__

    def small_pieces(self, path, level=6, threads=0, piece=4 << 20, encoding="latin-1"):
        orig(self, path, level=level, threads=3, piece=4096, encoding=encoding)
    monkeypatch.setattr(gzout.ParallelGzipWriter, "__init__", small_pieces)
    assert cli.main(["-G", fa, "-o", o2, "-q", sam], evaluator_factory=oracle_evaluator_factory) == 0
    same(o1, o2)
    raw = open(os.path.join(o2, "spliced_reads.fastq.gz"), "rb").read()
    members, text = 0, b""
    while raw:                                      # walk the members one by one
        d = zlib.decompressobj(16 + zlib.MAX_WBITS)
        text += d.decompress(raw)
        raw = d.unused_data
        members += 1
    assert members > 20
    with gzip.open(os.path.join(o1, "spliced_reads.fastq.gz"), "rb") as f:
        assert text == f.read()


def _large_sam(tmp_path, n_frag, seed, crlf_every=7, blank_every=997):
    sam0 = str(tmp_path / "base.sam")
    fa = _rich_sam(sam0, n_frag, seed=seed)
    lines = open(sam0).read().splitlines()
    hdr = [l for l in lines if l.startswith("@")]
    body = []
    for k, l in enumerate(l for l in lines if not l.startswith("@")):
        body.append(l + ("\r" if k % crlf_every == 3 else ""))
        if k % blank_every == 5:
            body.append("")
    return fa, hdr, body


@pytest.mark.parametrize("case", ["ok", "no_final_newline", "bad_line_late"])
def test_native_caller_multi_block_sam(tmp_path, case):
    """A SAM of several 4 MiB blocks (the native ingest's splitter cuts the input at newlines, two
    parser threads parse blocks, the loop takes them in order), with CRLF and blank lines: the same
    files as the Python loop; a malformed line in a late block fails both the same way."""
    fa, hdr, body = _large_sam(tmp_path, 20000, seed=2718)
    if case == "bad_line_late":
        body.insert(int(len(body) * 0.85), "broken\tline")
    text = "\n".join(hdr + body) + ("" if case == "no_final_newline" else "\n")
    assert len(text) > (9 << 20)
    sam = str(tmp_path / "big.sam")
    open(sam, "w").write(text)
    o1, o2 = str(tmp_path / "py"), str(tmp_path / "native")
    rc1 = cli.main(["-G", fa, "-o", o1, "-q", "--python-caller", sam], evaluator_factory=oracle_evaluator_factory)
    rc2 = cli.main(["-G", fa, "-o", o2, "-q", sam], evaluator_factory=oracle_evaluator_factory)
    assert rc1 == rc2 == (1 if case == "bad_line_late" else 0)
    if rc1 == 0:
        same(o1, o2)
    else:
        import gzip
        for f in ("multi_events.tsv",):
            assert open(os.path.join(o1, f)).read() == open(os.path.join(o2, f)).read()
        with gzip.open(os.path.join(o1, "spliced_reads.fastq.gz"), "rt") as a, \
                gzip.open(os.path.join(o2, "spliced_reads.fastq.gz"), "rt") as b:
            ta, tb = a.read(), b.read()
        assert ta == tb and len(ta) > 1000


def test_native_reads_gz_unwritable_path(tmp_path):
    """fc2_caller_set_reads_gz on a path that cannot be created fails at open (FC2_E_IO), before
    any input is read."""
    from find_circ2_amd import _native as N
    from find_circ2_amd.native_caller import NativeCaller
    from oracle_engine import oracle_batch_engine
    from find_circ2_amd.hotpath import Options as HPOptions
    sam = str(tmp_path / "rich.sam")
    fa = _rich_sam(sam, 20, seed=5)
    options, _ = cli.build_parser().parse_args(["-G", fa, "-o", str(tmp_path / "o"), sam])
    hp = HPOptions(asize=options.asize, margin=options.margin, maxdist=options.maxdist)
    _, names, fasta, dummy = oracle_batch_engine(options, hp)
    nc = NativeCaller(sam, False, options, names, fasta, genome_dummy=dummy,
                      reads_gz=(str(tmp_path / "no_such_dir" / "r.fastq.gz"), 2, 2, 0))
    try:
        with pytest.raises(N.Fc2Error):
            nc.open()
    finally:
        nc.close()


def _retag(lines, rng, rewrite):
    """The SAM lines with each record's tag fields (after the 11 mandatory ones) passed through
    rewrite(tags, rng) -> tags."""
    out = []
    for l in lines:
        if l.startswith("@"):
            out.append(l)
            continue
        f = l.split("\t")
        out.append("\t".join(f[:11] + rewrite(f[11:], rng)))
    return out


def _float_tags(tags, rng):
    """AS / XS of one record as floats in the ways an aligner may write them: an integral float, a
    value float32 cannot hold exactly (pysam hands back the float32), an extra float XS, an integer
    AS with a float XS, and a later float AS that only dict(tags) sees (find_circ.py:556-559)."""
    r = rng.random()
    asv = [t for t in tags if t.startswith("AS:i:")]
    if not asv:
        return tags
    a = int(asv[0][5:])
    if r < 0.2:
        return [("AS:f:%d.0" % a) if t.startswith("AS:i:") else t for t in tags]
    if r < 0.4:
        return [("AS:f:%.1f" % (a - 0.9)) if t.startswith("AS:i:") else t for t in tags]
    if r < 0.55:
        return [t for t in tags if not t.startswith("XS:")] + ["XS:f:%.2f" % (a - 2.5 + rng.random())]
    if r < 0.65:
        return tags + ["AS:f:%.3f" % (rng.random() * 3)]
    if r < 0.75:
        return [("XS:f:%.1f" % (float(t[5:]) + 0.5)) if t.startswith("XS:i:") else t for t in tags]
    return tags


@pytest.mark.parametrize("extra", [[], ["--half-unique", "--min-uniq-qual", "1"], ["--all-hits", "--non-canonical"]],
                         ids=["default", "half-unique", "all-hits"])
def test_native_caller_float_as_xs(tmp_path, extra):
    """Float AS / XS tags (type 'f'): JunctionSpan.uniq (:809-831), Hit.add's qA / qB, the uniqueness
    of bridges and best_qual_left/right (:556-566, :593, :704-713) follow Python's mixed int / float
    arithmetic and Python 2's str(float) in all three read loops, from SAM and from BAM."""
    sam0 = str(tmp_path / "base.sam")
    fa = _rich_sam(sam0, 800, seed=5150)
    rng = np.random.default_rng(77)
    sam = str(tmp_path / "float.sam")
    open(sam, "w").write("\n".join(_retag(open(sam0).read().splitlines(), rng, _float_tags)) + "\n")
    bam = str(tmp_path / "float.bam")
    sam_to_bam(open(sam).read(), bam)
    rcs, outs = _three(tmp_path, fa, sam, extra)
    assert rcs == [0, 0, 0]
    same(outs[0], outs[1])
    same(outs[0], outs[2])
    rows = open(os.path.join(outs[2], "circ_splice_sites.bed")).read().splitlines()[1:]
    quals = [c for r in rows for c in r.split("\t")[10:12]]
    assert any("." in q for q in quals) and any(q.endswith(".0") for q in quals), quals[:20]
    o_bam = str(tmp_path / "nat_bam")
    assert cli.main(["-G", fa, "-o", o_bam, "-n", "mix", "-q"] + extra + [bam], evaluator_factory=oracle_evaluator_factory) == 0
    same(outs[0], o_bam)


def test_float32_rounding_of_sam_tags(tmp_path):
    """A SAM 'f' value is kept as the float32 htslib stores (pysam returns it widened): AS:f:30.1
    prints as Python 2's str() of float32(30.1) = 30.1000003815 in best_qual_left."""
    fa = os.path.join(GOLDEN, "test_ref.fa")
    rd = _reads(os.path.join(GOLDEN, "test_reads.fa"))
    _, o0 = run_cli(tmp_path, fa, rd, extra=[], tag="base")
    base = open(os.path.join(o0, "circ_splice_sites.bed")).read().splitlines()
    assert len(base) > 1
    lines = sam_text(read_fasta(fa), rd).splitlines()        # the SAM run_cli feeds the CLI
    sam = str(tmp_path / "f.sam")
    open(sam, "w").write("\n".join(_retag(lines, None, lambda t, _: [("AS:f:30.1" if x.startswith("AS:") else x)
                                                                      for x in t])) + "\n")
    outs = []
    for tag, mode in (("py", ["--python-ingest"]), ("nat", [])):
        o = str(tmp_path / tag)
        assert cli.main(["-G", fa, "-o", o, "-q"] + mode + [sam], evaluator_factory=oracle_evaluator_factory) == 0
        outs.append(o)
    same(*outs)
    rows = open(os.path.join(outs[1], "circ_splice_sites.bed")).read().splitlines()[1:]
    assert rows and all(r.split("\t")[10] == "30.1000003815" for r in rows), rows


@pytest.mark.parametrize("case", ["str_as_with_xs", "str_last_as_in_hit", "str_as_no_xs", "array_xs"])
def test_native_caller_non_numeric_as_xs(tmp_path, case):
    """A str (A / Z / H) or array (B) AS / XS: Python raises TypeError where it subtracts one
    (uniqness, :816-817; Hit.add, :558-559) and orders a non-number above every int (min() at :831
    and `uniq >= min_uniq_qual` at :1299, :1351) -- the three read loops agree on the outcome."""
    sam0 = str(tmp_path / "base.sam")
    fa = _rich_sam(sam0, 300, seed=5151)
    rng = np.random.default_rng(3)

    def rewrite(tags, rng):
        if case == "str_as_with_xs":       # AS:Z - XS -> TypeError in JunctionSpan.__init__
            return [("AS:Z:x%s" % t[5:]) if t.startswith("AS:i:") and any(u.startswith("XS:") for u in tags)
                    and rng.random() < 0.02 else t for t in tags]
        if case == "str_last_as_in_hit":   # a later AS:Z: only dict(tags) in Hit.add sees it
            return tags + ["AS:Z:late"] if rng.random() < 0.02 else tags
        if case == "str_as_no_xs":         # AS:A without XS: uniq is a str, which passes uniqueness
            return [("AS:A:q" if t.startswith("AS:i:") else t) for t in tags if not t.startswith("XS:")] \
                if rng.random() < 0.3 else tags
        return [("XS:B:i,1,2" if t.startswith("XS:i:") else t) for t in tags] if rng.random() < 0.02 else tags

    sam = str(tmp_path / "t.sam")
    open(sam, "w").write("\n".join(_retag(open(sam0).read().splitlines(), rng, rewrite)) + "\n")
    rcs, outs = _three(tmp_path, fa, sam, [])
    assert rcs[0] == rcs[1] == rcs[2], rcs
    if case == "str_as_no_xs":
        assert rcs[2] in (0, 1)
    else:
        assert rcs[2] == 1
    if rcs[2] == 0:
        same(outs[0], outs[1])
        same(outs[0], outs[2])
    else:
        logs = [open(os.path.join(o, "run.log")).read() for o in outs]
        assert all("TypeError: unsupported operand type(s) for -" in g for g in logs), logs[2][-500:]
        assert logs[1].splitlines()[-1].split("\t")[-1] == logs[2].splitlines()[-1].split("\t")[-1]


@pytest.mark.parametrize("width", [4, 2])
@pytest.mark.parametrize("extra", [[], ["--all-hits"], ["--strand-pref", "-d", "0"], ["--chunk-size", "7"]])
def test_native_caller_compact_results_equal_raw(tmp_path, extra, width):
    """fc2_caller_submit_compact (results in a compact transfer form, expanded per chunk) records exactly
    what fc2_caller_submit records from the 8-byte words."""
    from oracle_engine import compact_factory
    sam = str(tmp_path / "rich.sam")
    fa = _rich_sam(sam, 500, seed=3141)
    o1, o2 = str(tmp_path / "raw"), str(tmp_path / "compact")
    assert cli.main(["-G", fa, "-o", o1, "-q"] + extra + [sam], evaluator_factory=oracle_evaluator_factory) == 0
    assert cli.main(["-G", fa, "-o", o2, "-q"] + extra + [sam], evaluator_factory=compact_factory(width)) == 0
    same(o1, o2)
    assert sum(1 for l in open(os.path.join(o2, "circ_splice_sites.bed")) if l[0] != "#") > 10


def test_native_caller_close_before_parse_threads_run(tmp_path):
    """Closing right after the first pull on a tiny SAM input: the parse-ahead threads may only
    start running once close has begun (which resets the handle's pointer to them before joining);
    they must not reach the object through that pointer.  Repeated so the window is hit (the bug
    crashed about 1 run in 200 under load)."""
    import ctypes
    from find_circ2_amd import _native as N
    from find_circ2_amd.caller import CallerOptions
    from find_circ2_amd.native_caller import NativeCaller
    fa = os.path.join(GOLDEN, "test_ref.fa")
    for k, body in enumerate(["\n\n", "", "u1\t4\t*\t0\t0\t*\t*\t0\t0\tACGT\t####\n"]):
        sam = str(tmp_path / ("d%d.sam" % k))
        open(sam, "w").write("@SQ\tSN:testbed_plus\tLN:720\n" + body)
        for _ in range(400):
            nc = NativeCaller(sam, False, CallerOptions(), ["testbed_plus"], write_reads=False,
                              write_multi=False, genome_dummy=True)
            nc.open()
            batch, eof = N.CallerBatch(), ctypes.c_int(0)
            rc = N.lib().fc2_caller_next(nc.h, ctypes.byref(batch), ctypes.byref(eof))
            assert rc == (N.FC2_OK if k < 2 else rc)   # one record: the reference's UnboundLocalError
            nc.close()


def test_submit_compact_checks_word_count(tmp_path):
    """fc2_caller_submit_compact takes the words' count and refuses one that is not the queued
    chunk's pair count (it would read past the words otherwise)."""
    import ctypes

    import numpy as np

    from find_circ2_amd import _native as N
    from find_circ2_amd.caller import CallerOptions
    from find_circ2_amd.native_caller import NativeCaller
    sam = str(tmp_path / "rich.sam")
    fa = _rich_sam(sam, 50, seed=7)
    from bwa_emul import read_fasta
    nc = NativeCaller(sam, False, CallerOptions(), list(read_fasta(fa)), write_reads=False, write_multi=False,
                      genome_dummy=True)
    nc.open()
    try:
        batch, eof = N.CallerBatch(), ctypes.c_int(0)
        while True:
            N.check(N.lib().fc2_caller_next(nc.h, ctypes.byref(batch), ctypes.byref(eof)))
            if batch.n or eof.value:
                break
        n = int(batch.n)
        assert n > 1
        words = np.zeros(n, np.uint32)
        L = N.lib()
        rc = L.fc2_caller_submit_compact(nc.h, words.ctypes.data, 4, n - 1, None, 0, None, 0, n)
        assert rc == N.FC2_E_PARAM and b"words for a batch of" in L.fc2_last_error()
        assert L.fc2_caller_submit_compact(nc.h, words.ctypes.data, 4, n, None, 0, None, 0, n) == N.FC2_OK
    finally:
        nc.close()


def test_rows_release_the_read_side(tmp_path):
    """fc2_caller_rows, once the input is read and every chunk recorded, hands the read side (the
    input, its parse blocks, the chunk buffers) to a thread that frees it: fc2_caller_ingest is NULL
    after, fc2_caller_next keeps reporting the end, and the counters and the second table's rows are
    those of a run without the release (the Python loop's)."""
    import ctypes
    from find_circ2_amd import _native as N
    from find_circ2_amd.native_caller import NativeCaller
    from oracle_engine import oracle_batch_engine
    from find_circ2_amd.hotpath import Options as HPOptions
    sam = str(tmp_path / "rich.sam")
    fa = _rich_sam(sam, 300, seed=17)
    options, _ = cli.build_parser().parse_args(["-G", fa, "-o", str(tmp_path / "o"), sam])
    hp = HPOptions(asize=options.asize, margin=options.margin, maxdist=options.maxdist)
    ev, names, fasta, dummy = oracle_batch_engine(options, hp)
    nc = NativeCaller(sam, False, options, names, fasta, genome_dummy=dummy, write_reads=False)
    L = N.lib()
    try:
        nc.open()
        nc.run(ev, {}, threads=True)
        before = nc.counters()
        assert L.fc2_caller_ingest(nc.h)
        circ = nc.rows_bytes(0)
        assert not L.fc2_caller_ingest(nc.h)
        lin = nc.rows_bytes(1)
        assert nc.counters() == before
        b, eof = N.CallerBatch(), ctypes.c_int(0)
        assert L.fc2_caller_next(nc.h, ctypes.byref(b), ctypes.byref(eof)) == N.FC2_OK
        assert eof.value == 1 and b.n == 0 and b.n_long == 0
        assert circ.count(b"\n") > 5 and lin.count(b"\n") > 5
    finally:
        nc.close()
    # the same tables from the Python loop
    o1, o2 = str(tmp_path / "py"), str(tmp_path / "nat")
    from oracle_engine import oracle_evaluator_factory
    assert cli.main(["-G", fa, "-o", o1, "-q", "--python-caller", sam], evaluator_factory=oracle_evaluator_factory) == 0
    assert cli.main(["-G", fa, "-o", o2, "-q", sam], evaluator_factory=oracle_evaluator_factory) == 0
    for f in ("circ_splice_sites.bed", "lin_splice_sites.bed"):
        rows = lambda o: [l for l in open(os.path.join(o, f), "rb") if not l.startswith(b"#")]   # noqa: E731
        assert sorted(rows(o1)) == sorted(rows(o2))
    nat = [l for l in open(os.path.join(o2, "circ_splice_sites.bed"), "rb") if not l.startswith(b"#")]
    assert sorted(circ.splitlines(True)) == sorted(nat)


def test_native_caller_many_reads_per_junction(tmp_path):
    """Junctions supported by hundreds of reads (scripts/gen_reads with a junction-site pool: 20 sites,
    20k reads, repeated read sequences among a junction's reads): the per-junction read-name and
    uniq-read sets (fc2_caller.cpp StrSet, past 16 members an open-addressing table) give n_frags and
    n_uniq -- the files equal the Python loop's."""
    import subprocess
    gen = os.path.join(ROOT, "scripts", "gen_reads")
    if not os.path.exists(gen):
        subprocess.check_call(["gcc", "-O2", "-o", gen, gen + ".c"])
    sq = tmp_path / "sq.tsv"
    sq.write_text("chrA\t300000\nchrB\t450000\nchrC\t250000\n")
    fa, sam = str(tmp_path / "g.fa"), str(tmp_path / "r.sam")
    subprocess.check_call([gen, str(sq), "20000", "7", fa, sam, "20"])
    o1, o2 = str(tmp_path / "py"), str(tmp_path / "nat")
    assert cli.main(["-G", fa, "-o", o1, "-q", "--python-caller", sam], evaluator_factory=oracle_evaluator_factory) == 0
    assert cli.main(["-G", fa, "-o", o2, "-q", sam], evaluator_factory=oracle_evaluator_factory) == 0
    same(o1, o2)
    rows = [l.split("\t") for l in open(os.path.join(o2, "circ_splice_sites.bed")) if l[0] != "#"]
    assert rows and max(int(r[4]) for r in rows) > 100          # n_frags: hundreds of reads per junction
    assert any(int(r[8]) < int(r[4]) for r in rows)             # n_uniq < n_frags: repeated read sequences
