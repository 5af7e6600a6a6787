"""Every pair of the bench batches against the oracle (full-size parity).

bench.py's headline batch (configs[2]: 50M synthetic 100 bp pairs, seed 1337, read order, on the
hg19-shaped synthetic genome) and its configs[4] share (25M pairs, read lengths 120..150 bp) are
generated exactly as bench.build_workload makes them, scanned by the product kernel, and every
one of the 8-byte result words is compared with the oracle's (oracle.scan_planes: the C
restatement of find_circ.py:854-974 fed from the batch's packed rows and the genome's 2-bit
planes, on 16 host threads).  Integer work: bit-exact, no tolerance.
"""
import argparse
import os
import sys
import time

import numpy as np
import pytest

import oracle

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from find_circ2_amd import _native as N, scan  # noqa: E402


def _check(args):
    import bench
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    dev = torch.device("cuda", 0)
    opt, g, b = bench.build_workload(args, 0, dev)
    return _check_batch(opt, g, b, dev)


def _check_batch(opt, g, b, dev):
    res = scan(opt, g, b).results[:b.n].cpu().numpy().view(np.uint64)
    torch.cuda.synchronize(dev)
    hp = b.pairs[:16 * b.n].cpu().numpy()
    words = b.read_words[:b.rw * b.stride].cpu().numpy()
    nwords = b.read_nwords[:b.nw * b.stride].cpu().numpy()
    units = g.units.cpu().numpy().view(np.uint64)
    nplane = g.nplane.cpu().numpy().view(np.uint64)
    p = oracle.params(opt.asize, opt.margin, opt.maxdist, opt.noncanonical, opt.strandpref, opt.allhits)
    t0 = time.time()
    exp, skipped = oracle.scan_planes(p, units, nplane, np.asarray(g.chrom_start, np.uint64),
                                      np.asarray(g.sizes, np.int64), hp, words, nwords, b.rw, b.nw, b.stride, b.n,
                                      n_threads=16)
    print("oracle: %d pairs in %.1f s" % (b.n, time.time() - t0))
    assert skipped == 0
    err = (exp >> np.uint64(48)) & np.uint64(0x6000)
    ok = err == 0
    mism = np.nonzero(res[ok] != exp[ok])[0]
    assert mism.size == 0, (mism.size, np.nonzero(ok)[0][mism[:5]], res[ok][mism[:5]], exp[ok][mism[:5]])
    assert np.array_equal((res[~ok] >> np.uint64(48)) & np.uint64(0x6000), err[~ok])
    hits = int(((res & np.uint64(0xFFFF)) != np.uint64(0xFFFF)).sum())
    assert hits > b.n // 3
    # the compact transfer forms (fc2_result_compact_launch -> fc2_result_expand) of every result word
    from find_circ2_amd import compact, expand
    dres = torch.from_numpy(res.view(np.int64)).to(dev)
    for width in (4, 2):
        c = compact(opt, dres, b.n, width=width)
        torch.cuda.synchronize(dev)
        n_esc = int(c.count.item())
        assert n_esc <= c.cap
        esc = c.esc.cpu().numpy().view(N.ESCAPE_DTYPE)[:n_esc]
        back = expand(opt, c.words[:b.n].cpu().numpy(), esc)
        assert np.array_equal(back.view(np.uint64), res)
        print("compact form, %d B: %d escapes of %d" % (width, n_esc, b.n))
    return b.n, hits


def test_configs2_bench_batch_every_pair():
    a = argparse.Namespace(workload="hg19", pairs=50_000_000, read_len=100, locus_ordered=False)
    n, hits = _check(a)
    assert n == 50_000_000


def test_configs4_share_every_pair():
    a = argparse.Namespace(workload="hg19", pairs=25_000_000, read_len=150, read_len_min=120, locus_ordered=False)
    n, hits = _check(a)
    assert n == 25_000_000


def test_stream_share_equals_slice_of_whole_stream():
    """bench.stream_share: pairs [lo, hi) of a seeded stream generated on their own (fc2_synth_cfg.first)
    are byte for byte the same rows as in the whole stream -- what lets each rank hold only its share."""
    import bench
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    dev = torch.device("cuda", 0)
    a = argparse.Namespace(workload="hg19", pairs=3_000_000, read_len=100, locus_ordered=False)
    opt, g, b = bench.build_workload(a, 0, dev)
    n, kw = bench.workload_cfg(a, 0)
    for lo, hi in ((0, 1000), (1_234_567, 2_000_000), (2_999_488, 3_000_000)):
        s = bench.stream_share(opt, g, kw, lo, hi)
        assert torch.equal(s.pairs[:16 * (hi - lo)], b.pairs[16 * lo:16 * hi])
        for j in range(b.rw):
            assert torch.equal(s.read_words[j * s.stride:j * s.stride + hi - lo],
                               b.read_words[j * b.stride + lo:j * b.stride + hi])
        for j in range(b.nw):
            assert torch.equal(s.read_nwords[j * s.stride:j * s.stride + hi - lo],
                               b.read_nwords[j * b.stride + lo:j * b.stride + hi])


def test_device_pipeline_both_result_forms():
    """bench.device_pipeline (pinned host SoA -> H2D -> scan -> D2H, 8 slices on two streams): the
    results that come back, as 2-B compact words expanded on the host or as raw 8-B words, equal the
    device-resident scan of the same batch for every pair."""
    import bench
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    dev = torch.device("cuda", 0)
    a = argparse.Namespace(workload="hg19", pairs=3_000_000, read_len=100, locus_ordered=False)
    opt, g, b = bench.build_workload(a, 0, dev)
    res = scan(opt, g, b).results[:b.n]
    b._bench_ref_results = res.cpu().clone()
    for width, d2h in ((2, 2), (8, 8)):
        r = bench.device_pipeline(opt, g, b, reps=1, width=width)
        assert r["results_equal_device_resident_scan"] is True, (width, r)
        assert abs(r["d2h_bytes_per_pair"] - d2h) < 0.1


def _read_bases(b, k):
    """Internal bases of pair k decoded from the batch's rows (lo plane bits [0, l), hi plane bits
    [l, 2l) of one bit stream; N rows): codes 0..3, 4 for N."""
    l = int(b._hp[k]["read_len"]) - 2 * b._e
    bits = np.concatenate([np.unpackbits(np.array([b._words[j * b.stride + k]], "<u8").view(np.uint8),
                                         bitorder="little") for j in range(b.rw)])
    nb = np.concatenate([np.unpackbits(np.array([b._nwords[j * b.stride + k]], "<u8").view(np.uint8),
                                       bitorder="little") for j in range(b.nw)])
    c = bits[:l].astype(np.int64) | (bits[l:2 * l].astype(np.int64) << 1)
    c[nb[:l] != 0] = 4
    return c


def test_three_segment_reads():
    """SURVEY.md 8(d) config 5's three-segment reads (fc2_synth_cfg.p_three_seg): the two pairs of a
    slot are (s1,s2) and (s2,s3) of one read wrapping a circle [start, end) -- the same chromosome and
    circle, s2's bases (mutations and N included) equal in both internal rows, the circle found by the
    scan for both -- every result equal to the oracle's, and shares that split a slot equal the
    whole stream's rows."""
    import bench
    from find_circ2_amd import PairBatch, SynthConfig
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    dev = torch.device("cuda", 0)
    a = argparse.Namespace(workload="hg19", pairs=1000, read_len=150, read_len_min=120, locus_ordered=False)
    opt, g, _ = bench.build_workload(a, 0, dev)
    kw = dict(seed=99, len_min=120, len_max=150, p_backsplice=1.0, p_planted=0.5, mut_rate=0.01, n_rate=0.002,
              span_min=150, span_max=20000, p_three_seg=1.0)
    n = 400_000
    b = PairBatch.synthetic(opt, g, n, SynthConfig(**kw), with_truth=True)
    hp = b.pairs[:16 * n].cpu().numpy().view(N.PAIR_DTYPE)
    truth = b.truth[:2 * n].cpu().numpy().reshape(n, 2)
    ok = (hp["flags"] & N.PAIR_SKIP) == 0
    assert ok.mean() > 0.99
    p0, p1 = hp[0::2], hp[1::2]
    both = ok[0::2] & ok[1::2]
    assert np.array_equal(truth[0::2][both], truth[1::2][both])
    assert np.array_equal(p0["chrom"][both], p1["chrom"][both])
    circ_all = p0["b_aend"] - p1["a_pos"]                     # (s1,s2) ends at end, (s2,s3) starts at start
    circ = circ_all[both]
    assert np.array_equal(circ, (truth[0::2, 1] - truth[0::2, 0])[both])
    assert (circ >= opt.asize).all() and (circ <= 150 - 2 * opt.asize).all()
    assert np.array_equal(p1["b_aend"][both] - p1["a_pos"][both], p1["read_len"][both].astype(np.int32) - circ)  # k3
    assert ((p0["flags"] & N.PAIR_BACKSPLICE) != 0).all() and ((p1["flags"] & N.PAIR_BACKSPLICE) != 0).all()
    # s2 in both rows: pair 0's internal base j is read position e + j, pair 1's is k1 + e + j
    b._hp, b._e = hp, opt.asize - opt.margin
    b._words = b.read_words[:b.rw * b.stride].cpu().numpy().view(np.uint64)
    b._nwords = b.read_nwords[:b.nw * b.stride].cpu().numpy().view(np.uint64)
    e = b._e
    for s in np.nonzero(both)[0][:300]:
        k1 = int(p0["read_len"][s]) - int(circ_all[s])
        i0, i1 = _read_bases(b, 2 * s), _read_bases(b, 2 * s + 1)
        lo, hi = k1 + e, min(e + len(i0), k1 + e + len(i1))   # read positions both rows hold
        assert hi > lo
        assert np.array_equal(i0[lo - e:hi - e], i1[lo - k1 - e:hi - k1 - e]), s
    # the oracle on every pair, and both pairs of a slot find the circle
    _check_batch(opt, g, b, dev)
    res = scan(opt, g, b).results[:n].cpu().numpy().view(N.RESULT_DTYPE)
    found = res["best_x"] >= 0
    assert (found[0::2] & found[1::2] & both).mean() > 0.4
    # shares that cut a slot in two are the whole stream's rows
    for lo, hi in ((1, 1001), (12_345, 20_000)):
        sb = PairBatch.synthetic(opt, g, hi - lo, SynthConfig(first=lo, **kw))
        assert torch.equal(sb.pairs[:16 * (hi - lo)], b.pairs[16 * lo:16 * hi])
        for j in range(b.rw):
            assert torch.equal(sb.read_words[j * sb.stride:j * sb.stride + hi - lo],
                               b.read_words[j * b.stride + lo:j * b.stride + hi])
