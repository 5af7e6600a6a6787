"""The native read loop on many workers -- fc2_caller_next's process_mate over fragment ranges and
fc2_caller_submit's phases A-D -- against the Python loop (find_circ2_amd.caller, a line-by-line
restatement of find_circ.py:1276-1439): every output file and counter identical whatever the number of workers and of fragment ranges -- junction
names by first appearance (:684-686), float weight sums in input order (:544, :563, :579) -- and,
on a run that fails part-way, the same partial outputs (spliced reads and multi_events rows of
the fragments before the failing one, its test row when written before the failure)."""
import gzip
import os

import pytest

from find_circ2_amd import cli
from oracle_engine import oracle_evaluator_factory, pipelined_factory
from test_ingest import same
from test_native_caller import _rich_sam

MODES = [dict(FC2_CALLER_THREADS="1", FC2_NEXT_THREADS="1"),
         dict(FC2_CALLER_THREADS="3", FC2_NEXT_THREADS="2", FC2_CALLER_MIN_RANGE="1"),
         dict(FC2_CALLER_THREADS="8", FC2_NEXT_THREADS="7", FC2_CALLER_MIN_RANGE="5"), dict(FC2_CALLER_THREADS="16"),
         # fragments grouped on the parse threads across many small parse blocks (a fragment cut
         # by a block boundary, regions of one fragment, none), on one parse thread
         dict(FC2_PARSE_BLOCK="700", FC2_NEXT_THREADS="2", FC2_CALLER_MIN_RANGE="1", FC2_PARSE_INFLIGHT="2"),
         dict(FC2_PARSE_BLOCK="4000", FC2_PARSE_THREADS="5", FC2_CALLER_THREADS="3"),
         dict(FC2_PARSE_THREADS="1", FC2_PARSE_BLOCK="1500"),
         # chunks cut short by the pinned-batch cap (one 400-byte block per chunk; some chunks empty)
         dict(FC2_PARSE_BLOCK="400", FC2_PIN_MAX="1", FC2_PARSE_INFLIGHT="3")]


@pytest.fixture(scope="module")
def rich(tmp_path_factory):
    d = tmp_path_factory.mktemp("rich")
    sam = str(d / "rich.sam")
    fa = _rich_sam(sam, 900, seed=4242)
    return fa, sam


@pytest.fixture(scope="module")
def hit_names(tmp_path_factory, rich):
    """Fragments with a recorded junction, in input order (their reads are written)."""
    fa, sam = rich
    o = str(tmp_path_factory.mktemp("clean") / "py")
    assert cli.main(["-G", fa, "-o", o, "-q", "--python-caller", sam], evaluator_factory=oracle_evaluator_factory) == 0
    names = {l[1:].split(" ")[0] for l in _gz(os.path.join(o, "spliced_reads.fastq.gz")).splitlines()
             if l.startswith("@")}
    order = [l.split("\t")[0] for l in open(sam) if not l.startswith("@")]
    return [q for k, q in enumerate(order) if q in names and q not in order[:k]]


@pytest.mark.parametrize("mode", range(len(MODES)))
@pytest.mark.parametrize("extra", [[], ["--all-hits", "--non-canonical"], ["--test", "--chunk-size", "61"],
                                   ["--half-unique", "--report-nobridges", "--strand-pref"]])
def test_parallel_recording_equals_python_loop(tmp_path, monkeypatch, rich, mode, extra):
    fa, sam = rich
    o1 = str(tmp_path / "py")
    assert cli.main(["-G", fa, "-o", o1, "-q", "--python-caller"] + extra + [sam],
                    evaluator_factory=oracle_evaluator_factory) == 0
    for k, v in MODES[mode].items():
        monkeypatch.setenv(k, v)
    o2 = str(tmp_path / "native")
    assert cli.main(["-G", fa, "-o", o2, "-q"] + extra + [sam], evaluator_factory=pipelined_factory(3)) == 0
    same(o1, o2)
    assert sum(1 for l in open(os.path.join(o2, "circ_splice_sites.bed")) if l[0] != "#") > 20


def _gz(path):
    with gzip.open(path, "rt") as f:
        return f.read()


@pytest.mark.parametrize("mode", range(len(MODES)))
@pytest.mark.parametrize("bad", ["seq", "unspliced_none", "no_as", "b_no_cigar"])
def test_parallel_recording_fails_where_python_loop_fails(tmp_path, monkeypatch, rich, hit_names, mode, bad):
    """A read sequence with a byte outside the IUPAC table (rev_comp's KeyError in Hit.add,
    find_circ.py:573-582), or -- with --test -- a test name that parse_truth cannot read, in a
    fragment in the middle of the input: both loops exit 1, with the same partial outputs."""
    fa, sam = rich
    lines = open(sam).read().splitlines()
    target = hit_names[len(hit_names) // 2]
    out = []
    for l in lines:
        f = l.split("\t")
        if not l.startswith("@") and f[0] == target:
            if bad == "seq" and f[9] != "*":
                f[9] = f[9][:40] + "." + f[9][41:]
            elif bad == "unspliced_none":
                f[0] = target + "___O:chr1:x:+"          # int('x') in parse_truth (:1148-1200)
            elif bad == "no_as":                         # uniqness: KeyError in process_mate (:809-819)
                f = f[:11] + [t for t in f[11:] if not t.startswith("AS:")]
            elif bad == "b_no_cigar" and int(f[1]) & 2048:   # B.aend None: int(None) packing the pair
                f[5] = "*"
                if f[9] == "*":
                    f[9], f[10] = "A" * 60, "I" * 60
        out.append("\t".join(f))
    p = str(tmp_path / "bad.sam")
    open(p, "w").write("\n".join(out) + "\n")
    extra = ["--test"] if bad == "unspliced_none" else []
    o1 = str(tmp_path / "py")
    rc1 = cli.main(["-G", fa, "-o", o1, "-q", "--python-caller"] + extra + [p], evaluator_factory=oracle_evaluator_factory)
    for k, v in MODES[mode].items():
        monkeypatch.setenv(k, v)
    o2 = str(tmp_path / "native")
    rc2 = cli.main(["-G", fa, "-o", o2, "-q"] + extra + [p], evaluator_factory=pipelined_factory(3))
    assert rc1 == rc2 == 1
    if bad == "b_no_cigar":
        err = [l for l in open(os.path.join(o2, "run.log")) if "Error" in l]
        assert err and "NoneType" in err[-1], err
    for f in ("multi_events.tsv", "test_results.tsv"):
        p1, p2 = os.path.join(o1, f), os.path.join(o2, f)
        assert os.path.exists(p1) == os.path.exists(p2)
        if os.path.exists(p1):
            assert open(p1).read() == open(p2).read(), f
    r1, r2 = _gz(os.path.join(o1, "spliced_reads.fastq.gz")), _gz(os.path.join(o2, "spliced_reads.fastq.gz"))
    assert r1 == r2 and r1.count("\n@") > 10


def _edge_sam(src, dst, seed, first):
    """The rich SAM with grouping edge cases spliced in: unmapped records with fresh qnames and with
    the qname of the record before them, a fragment's records repeated later (its qname seen again
    after others), and a first record that is unmapped -- with the first mapped qname ("same") or
    another ("other")."""
    import random
    rng = random.Random(seed)
    lines = open(src).read().splitlines()
    head = [l for l in lines if l.startswith("@")]
    body = [l for l in lines if not l.startswith("@")]
    out = []
    for k, l in enumerate(body):
        f = l.split("\t")
        r = rng.random()
        if r < 0.03:
            out.append("\t".join(["unm%d" % k, "4", "*", "0", "0", "*", "*", "0", "0", "ACGTACGTAC", "IIIIIIIIII"]))
        elif r < 0.06:
            out.append("\t".join([f[0], str(4 | (int(f[1]) & 0x40)), "*", "0", "0", "*", "*", "0", "0", "ACGT", "IIII"]))
        out.append(l)
        if r > 0.985 and k > 10:                         # an earlier fragment's records again
            q = body[k - 7].split("\t")[0]
            out.extend(x for x in body[max(0, k - 12):k] if x.split("\t")[0] == q)
    q0 = out[0].split("\t")[0] if first == "same" else "lead"
    out.insert(0, "\t".join([q0, "4", "*", "0", "0", "*", "*", "0", "0", "ACGTAC", "IIIIII"]))
    open(dst, "w").write("\n".join(head + out) + "\n")


@pytest.mark.parametrize("first", ["same", "other"])
@pytest.mark.parametrize("mode", [dict(FC2_PARSE_BLOCK="300", FC2_PARSE_INFLIGHT="2"),
                                  dict(FC2_PARSE_BLOCK="1100", FC2_NEXT_THREADS="3", FC2_CALLER_MIN_RANGE="1"),
                                  dict(FC2_PARSE_THREADS="1", FC2_PARSE_BLOCK="500")])
@pytest.mark.parametrize("bam", [False, True])
def test_grouping_edge_cases_equal_python_ingest(tmp_path, monkeypatch, rich, first, mode, bam):
    """Fragments grouped on the parse threads (group_batch) at tiny parse blocks against the pure
    Python reader and loop (--python-ingest: samio + caller, find_circ.py:1450-1486): every file
    and every run.log counter identical, with unmapped records inside and between fragments, a
    qname seen again after others, and an unmapped first record."""
    from samgen import sam_to_bam
    from test_ingest import same as same_files
    fa, sam = rich
    p = str(tmp_path / "edge.sam")
    _edge_sam(sam, p, seed=len(first) + len(mode), first=first)
    if bam:
        sam_to_bam(open(p).read(), str(tmp_path / "edge.bam"))
        p = str(tmp_path / "edge.bam")
    o1 = str(tmp_path / "py")
    rc1 = cli.main(["-G", fa, "-o", o1, "-q", "--python-ingest"] + [p], evaluator_factory=oracle_evaluator_factory)
    for k, v in mode.items():
        monkeypatch.setenv(k, v)
    o2 = str(tmp_path / "native")
    rc2 = cli.main(["-G", fa, "-o", o2, "-q", p], evaluator_factory=pipelined_factory(3))
    assert rc1 == rc2 == 0
    same_files(o1, o2)
