"""CLI (find_circ.py-compatible) on CPU with the oracle evaluator: known answers,
formats, --test mode, BAM input, option edge cases.  The GPU evaluator is
compared file-for-file with these runs in tests/test_cli_gpu.py."""
import gzip
import os

import pytest

from bwa_emul import read_fasta
from conftest import GOLDEN
from find_circ2_amd import cli
from find_circ2_amd.caller import py2_str
from find_circ2_amd.samio import AlignmentFile
from oracle_engine import oracle_evaluator_factory
from samgen import sam_text, sam_to_bam


def _reads(path):
    names = [l[1:].strip() for l in open(path) if l.startswith('>')]
    seqs = read_fasta(path)
    return [(n, seqs[n.split()[0]]) for n in names]


def run_cli(tmp_path, fa, reads, extra=(), bam=False, evaluator=oracle_evaluator_factory, tag="out", genome_arg=None):
    """Align `reads` to `fa` (tests/bwa_emul.py) and run the CLI on them; `genome_arg` is what -G
    gets (default: fa itself)."""
    genome = read_fasta(fa)
    sam = sam_text(genome, reads)
    inp = str(tmp_path / ("in.bam" if bam else "in.sam"))
    if bam:
        sam_to_bam(sam, inp)
    else:
        open(inp, "w").write(sam)
    out = str(tmp_path / tag)
    rc = cli.main(["-G", genome_arg or fa, "-o", out, "-n", "test", "-q"] + list(extra) + [inp],
                  evaluator_factory=evaluator)
    return rc, out


def bed_rows(path):
    rows = [l.rstrip("\n").split("\t") for l in open(path) if not l.startswith("#")]
    return {(r[0], int(r[1]), int(r[2]), r[5]): r for r in rows}


def test_py2_str():
    assert py2_str(1.0) == "1.0" and py2_str(0.5) == "0.5" and py2_str(1 / 3.) == "0.333333333333"
    assert py2_str(2.0 / 3) == "0.666666666667" and py2_str(1e16) == "1e+16" and py2_str(3) == "3"
    assert py2_str(False) == "False" and py2_str(123456789012.0) == "123456789012.0"


def test_cli_test_reads_known_answers(tmp_path):
    fa = os.path.join(GOLDEN, "test_ref.fa")
    rc, out = run_cli(tmp_path, fa, _reads(os.path.join(GOLDEN, "test_reads.fa")), extra=["--test"])
    assert rc == 0
    circ = bed_rows(os.path.join(out, "circ_splice_sites.bed"))
    lin = bed_rows(os.path.join(out, "lin_splice_sites.bed"))
    assert {("testbed_plus", 240, 320, "+"), ("testbed_plus", 80, 640, "+"),
            ("testbed_minus", 240, 320, "-")} == set(circ)
    assert {("testbed_plus", 160, 240, "+"), ("testbed_plus", 320, 400, "+"), ("testbed_plus", 480, 560, "+"),
            ("testbed_minus", 160, 240, "-"), ("testbed_minus", 320, 400, "-")} <= set(lin)
    header = open(os.path.join(out, "circ_splice_sites.bed")).readline()
    assert header.startswith("#chrom\tstart\tend\tname\tn_frags") and header.count("\t") == 21
    # the 3-segment circular read supports its junction twice in one fragment: a closure
    r = circ[("testbed_plus", 240, 320, "+")]
    assert r[3] == "test_circ_000001" and r[17] == "GTAG" and r[14] == "0" and r[16] == "1"
    assert "SUPPORT_CLOSURE" in r[20].split(",")
    assert r[6] == "1.0" and r[7] == "2"          # weight 1/(3-1) twice; spanned twice
    tests = [l.rstrip("\n").split("\t") for l in open(os.path.join(out, "test_results.tsv"))]
    by = {t[0].split("___")[0]: t for t in tests}
    assert by["test_ref_plus_lin_triple_exons1-3"][1] == "LIN_OK"
    assert by["test_ref_plus_circ_triple_exon2"][2] == "CIRC_OK"
    m = by["test_ref_plus_circ_mixed_exon3,4,1"]
    assert m[1] == "LIN_OK" and m[2] == "CIRC_OK"
    with gzip.open(os.path.join(out, "spliced_reads.fastq.gz"), "rt") as fh:
        fq = fh.read().splitlines()
    assert len(fq) % 4 == 0 and fq[0].startswith("@test_ref_plus_lin_triple_exons1-3")


def test_cli_cdr1as_matches_reference_bed(tmp_path):
    fa = os.path.join(GOLDEN, "CDR1as_locus.fa")
    rc, out = run_cli(tmp_path, fa, _reads(os.path.join(GOLDEN, "cdr1as_reads.fa")))
    assert rc == 0
    circ = bed_rows(os.path.join(out, "circ_splice_sites.bed"))
    ref = [l.rstrip("\n").split("\t") for l in open(os.path.join(GOLDEN, "cdr1as_reference.bed"))
           if not l.startswith("#")]
    # cmp_bed.py's notion of parity: identical (chrom, start, end, strand) sets (cmp_bed.py:6-26, 59-60)
    assert set(circ) == {(r[0], int(r[1]), int(r[2]), r[5]) for r in ref}
    row = circ[("CDR1as_locus", 728, 2213, "+")]
    # same-meaning columns of the v1 reference row: n_reads 3, edits 0, anchor_overlap 0, breakpoints 1, GTAG
    assert (row[4], row[14], row[15], row[16], row[17]) == ("3", "0", "0", "1", "GTAG")


def test_cli_bam_input_equals_sam(tmp_path):
    fa = os.path.join(GOLDEN, "test_ref.fa")
    reads = _reads(os.path.join(GOLDEN, "test_reads.fa"))
    _, o1 = run_cli(tmp_path, fa, reads, tag="sam")
    _, o2 = run_cli(tmp_path, fa, reads, bam=True, tag="bam")
    for f in ("circ_splice_sites.bed", "lin_splice_sites.bed", "multi_events.tsv"):
        assert open(os.path.join(o1, f)).read() == open(os.path.join(o2, f)).read(), f


def test_samio_fields(tmp_path):
    line = ("r1\t2048\tchr22\t50648608\t19\t52H24M\t*\t0\t0\tAGGTGACGCGGCGCACGGCGCGGA\t*\tNM:i:0\tAS:i:24\t"
            "XS:i:18\tSA:Z:chr22,50647092,+,56M20S,60,0;")
    p = tmp_path / "x.sam"
    p.write_text("@SQ\tSN:chr21\tLN:100\n@SQ\tSN:chr22\tLN:51304566\n" + line + "\n")
    recs = list(AlignmentFile(str(p)))
    r = recs[0]
    assert r.tid == 1 and r.pos == 50648607 and r.aend == 50648607 + 24 and r.is_supplementary
    assert r.query == r.seq and r.qual is None and r.get_tag("AS") - r.get_tag("XS") == 6
    assert r.cigar == [(5, 52), (0, 24)]


@pytest.mark.parametrize("extra", [["--non-canonical"], ["--all-hits"], ["--strand-pref"], ["-d", "0"],
                                   ["--no-linear"], ["--half-unique", "--report-nobridges"], ["--no-multi"]])
def test_cli_options_run(tmp_path, extra):
    fa = os.path.join(GOLDEN, "test_ref.fa")
    rc, out = run_cli(tmp_path, fa, _reads(os.path.join(GOLDEN, "test_reads.fa")), extra=extra)
    assert rc == 0
    circ = bed_rows(os.path.join(out, "circ_splice_sites.bed"))
    assert ("testbed_plus", 240, 320, "+") in circ
    if extra == ["-d", "0"]:
        assert circ[("testbed_plus", 240, 320, "+")][14] == "False"   # simple_match's bool (find_circ.py:865-871)
    if extra == ["--no-linear"]:
        lin = bed_rows(os.path.join(out, "lin_splice_sites.bed"))
        assert ("testbed_plus", 160, 240, "+") not in lin


def test_cli_stranded_fails_like_reference(tmp_path):
    fa = os.path.join(GOLDEN, "test_ref.fa")
    rc, out = run_cli(tmp_path, fa, _reads(os.path.join(GOLDEN, "test_reads.fa")), extra=["--stranded"])
    assert rc == 1     # AttributeError in Hit.add (find_circ.py:532-533) -> sys.exit(1)


def test_cmp_bed_semantics(tmp_path, capsys):
    from find_circ2_amd import cmp_bed
    fa = os.path.join(GOLDEN, "CDR1as_locus.fa")
    rc, out = run_cli(tmp_path, fa, _reads(os.path.join(GOLDEN, "cdr1as_reads.fa")))
    mine = os.path.join(out, "circ_splice_sites.bed")
    ref = os.path.join(GOLDEN, "cdr1as_reference.bed")
    assert cmp_bed.main([ref, mine]) == 0
    cap = capsys.readouterr()
    assert "files contain identical splice sites!" in cap.err and "overlap\t1" in cap.err
    other = tmp_path / "other.bed"
    other.write_text("#h\nCDR1as_locus\t728\t2214\tx\t1\t+\n")
    assert not cmp_bed.compare(ref, str(other))
    cap = capsys.readouterr()
    assert cap.out.startswith("MISSING\tCDR1as_locus\t728\t2213") and "input2_not_in_input1\t1" in cap.err


@pytest.mark.parametrize("mode", [[], ["--python-caller"], ["--python-ingest"]])
def test_non_ascii_bytes_written_back_unchanged(tmp_path, mode):
    """a qname byte >= 0x80 (here 0xE9) comes back as that single byte in
    spliced_reads.fastq.gz and as the same byte in the BED read lists (no UTF-8 re-encoding),
    in all three read loops."""
    import gzip
    fa = os.path.join(GOLDEN, "CDR1as_locus.fa")
    reads = [("r\xe9ad%d_%s" % (i, n), s) for i, (n, s) in enumerate(_reads(os.path.join(GOLDEN, "cdr1as_reads.fa")))]
    genome = read_fasta(fa)
    sam = str(tmp_path / "in.sam")
    with open(sam, "wb") as f:
        f.write(sam_text(genome, reads).encode("latin-1"))
    out = str(tmp_path / "o")
    assert cli.main(["-G", fa, "-o", out, "-q"] + mode + [sam], evaluator_factory=oracle_evaluator_factory) == 0
    raw = gzip.open(os.path.join(out, "spliced_reads.fastq.gz"), "rb").read()
    assert b"r\xe9ad" in raw and b"r\xc3\xa9ad" not in raw
    bed = open(os.path.join(out, "circ_splice_sites.bed"), "rb").read()
    assert b"\xc3\xa9" not in bed


def test_default_cli_fails_loudly_without_a_gpu(tmp_path):
    """The shipped search has no CPU fallback: with no HIP device the default CLI (native read loop,
    ctxpipe) exits 1 with the device error -- also for an input in which no span is searched."""
    from find_circ2_amd.ctxpipe import device_count
    try:
        if device_count() > 0:
            pytest.skip("a GPU is present")
    except Exception:
        pass                                    # no HIP runtime at all: the same failure is expected
    import shutil
    fa = str(tmp_path / "test_ref.fa")               # (the default CLI writes the .byo_index next to it)
    shutil.copy(os.path.join(GOLDEN, "test_ref.fa"), fa)
    for reads in (_reads(os.path.join(GOLDEN, "test_reads.fa")), []):
        rc, out = run_cli(tmp_path, fa, reads, evaluator=None, tag="default%d" % len(reads))
        assert rc == 1
        assert "fc2_ctx_create" in open(os.path.join(out, "run.log")).read()
