"""The native read loop reading ahead (NativeCaller.run with a pipelined evaluator, chunks queued
by fc2_caller_next, include/fc2_caller.h): every output file and counter must equal the
one-chunk-at-a-time loop's, for option sets that change the host logic, small chunks (many
chunks in flight), and the inputs on which the reference raises -- there the read-ahead loop
must record the fragments before the failure exactly like the sequential one (an error of
fc2_caller_next is raised after the queued chunks are submitted)."""
import os

import pytest

from conftest import GOLDEN
from find_circ2_amd import cli
from oracle_engine import oracle_evaluator_factory, pipelined_factory
from test_ingest import _mixed_sam, same
from test_native_caller import _rich_sam


def _pair(tmp_path, fa, inp, extra, depth=3):
    seq = str(tmp_path / "seq")
    ahead = str(tmp_path / "ahead")
    rc1 = cli.main(["-G", fa, "-o", seq, "-n", "s", "-q"] + extra + [inp], evaluator_factory=oracle_evaluator_factory)
    f = pipelined_factory(depth)
    rc2 = cli.main(["-G", fa, "-o", ahead, "-n", "s", "-q"] + extra + [inp], evaluator_factory=f)
    return rc1, rc2, seq, ahead, f


@pytest.fixture(params=[False, True], ids=["one_thread", "reader_thread"])
def threads(request, monkeypatch):
    """NativeCaller.run in its single-thread read-ahead form and in its two-thread form (a reader
    thread forming chunks with fc2_caller_next while this thread records them)."""
    from find_circ2_amd.native_caller import NativeCaller
    orig = NativeCaller.run

    def run(self, *a, **k):
        k["threads"] = request.param
        return orig(self, *a, **k)
    monkeypatch.setattr(NativeCaller, "run", run)
    return request.param


@pytest.mark.parametrize("extra", [[], ["--chunk-size", "7"], ["--chunk-size", "3", "--all-hits", "--non-canonical"],
                                   ["--test", "--chunk-size", "11"], ["--no-linear", "--chunk-size", "5"]])
def test_readahead_equals_sequential(tmp_path, extra, threads):
    sam = str(tmp_path / "rich.sam")
    fa = _rich_sam(sam, 1500, seed=41)
    rc1, rc2, a, b, f = _pair(tmp_path, fa, sam, extra)
    assert rc1 == rc2 == 0
    same(a, b)
    if "--chunk-size" in extra:
        if threads:
            assert 1 <= f.made[0].max_in_flight <= 3   # bounded by the evaluator's depth
        else:
            assert f.made[0].max_in_flight == 3        # the loop really held three chunks


def test_readahead_missing_chromosome(tmp_path, threads):
    sam = str(tmp_path / "m.sam")
    fa = _mixed_sam(sam, 1500, seed=77)
    txt = open(sam).read().replace("SN:chr2\t", "SN:chrX\t").replace("\tchr2\t", "\tchrX\t")
    open(sam, "w").write(txt)
    rc1, rc2, a, b, _ = _pair(tmp_path, fa, sam, ["--chunk-size", "9"])
    assert rc1 == rc2 == 1
    assert "KeyError: 'chrX'" in open(os.path.join(b, "run.log")).read()
    for fn in ("spliced_reads.fastq.gz", "multi_events.tsv"):
        pa, pb = os.path.join(a, fn), os.path.join(b, fn)
        import gzip
        rd = (lambda p: gzip.open(p, "rt").read()) if fn.endswith(".gz") else (lambda p: open(p).read())
        assert rd(pa) == rd(pb), fn                  # the same fragments recorded before the failure


def test_readahead_next_error_after_queued_chunks(tmp_path, threads):
    """A SEQ-less secondary record makes fc2_caller_next fail (TypeError, find_circ.py:1101):
    the chunks already queued are recorded first, as the sequential loop records them."""
    sam = str(tmp_path / "sec.sam")
    fa = _rich_sam(sam, 800, seed=5, secondary_same_chrom=True)
    rc1, rc2, a, b, _ = _pair(tmp_path, fa, sam, ["--chunk-size", "4"])
    assert rc1 == rc2 == 1
    assert "TypeError" in open(os.path.join(b, "run.log")).read()
    import gzip
    ra = gzip.open(os.path.join(a, "spliced_reads.fastq.gz"), "rt").read()
    rb = gzip.open(os.path.join(b, "spliced_reads.fastq.gz"), "rt").read()
    assert ra == rb
