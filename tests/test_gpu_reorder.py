"""GPU: the device locality reorder (fc2_reorder_launch) in front of the scan.

The reorder only changes where each pair sits in the batch, so every pair's
result must be bit-identical to the scan of the input-order batch (which the
parity tests pin to the oracle), and the layout itself must be a stable sort of
the batch by genome bucket of the A window.
"""
import os

import numpy as np
import pytest

from conftest import GOLDEN
from synth_small import load_genome, make_spans

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from find_circ2_amd import Genome, Options, PairBatch, SynthConfig, decode_splices, reorder, scan, sq_table  # noqa
from find_circ2_amd import _native as N  # noqa: E402


def _dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return "cuda:0"


def _key(t):
    return [(s.start, s.end, s.strand, s.gtag, s.dist, s.ov, s.n_hits) for s in t] if isinstance(t, list) else repr(t)


def _check_layout(g, src: PairBatch, r: PairBatch):
    """slot is a permutation; buckets non-decreasing; slots increase inside a bucket;
    records and read rows are those of the input pair."""
    n = src.n
    slot = r.slot[:n].cpu().numpy().astype(np.int64)
    assert np.array_equal(np.sort(slot), np.arange(n))
    hp_in = src.fetch_host_pairs()
    hp_out = r.fetch_host_pairs()
    assert np.array_equal(hp_out.view(np.uint8).reshape(n, 16), hp_in[slot].view(np.uint8).reshape(n, 16))
    info = r.reorder_info
    cs = g.chrom_start.astype(np.int64) if len(g.chrom_start) else np.zeros(1, np.int64)
    ch = hp_out["chrom"].astype(np.int64)
    ok = ch < len(g.names)
    gb = np.where(ok, cs[np.minimum(ch, len(cs) - 1)] + np.maximum(hp_out["a_pos"].astype(np.int64), 0), 0)
    bk = np.minimum(gb >> int(info.shift), int(info.n_buckets) - 1)
    assert np.all(np.diff(bk) >= 0)
    same = np.diff(bk) == 0
    assert np.all(np.diff(slot)[same] > 0)
    w_in = src.read_words[:src.rw * src.stride].view(src.rw, src.stride)[:, :n].cpu().numpy()
    w_out = r.read_words[:r.rw * r.stride].view(r.rw, r.stride)[:, :n].cpu().numpy()
    assert np.array_equal(w_out, w_in[:, slot])
    rn = (hp_in["flags"][slot] & N.PAIR_READ_N) != 0
    if rn.any():
        n_in = src.read_nwords[:src.nw * src.stride].view(src.nw, src.stride)[:, :n].cpu().numpy()
        n_out = r.read_nwords[:r.nw * r.stride].view(r.nw, r.stride)[:, :n].cpu().numpy()
        assert np.array_equal(n_out[:, rn], n_in[:, slot[rn]])
    return slot


@pytest.mark.parametrize("o", [dict(), dict(allhits=True, noncanonical=True, strandpref=True), dict(maxdist=0)])
@pytest.mark.parametrize("fa", ["test_ref.fa", "CDR1as_locus.fa"])
def test_reorder_same_results(fa, o):
    opt = Options(**o)
    path = os.path.join(GOLDEN, fa)
    g = Genome.from_fasta(path, device=_dev())
    spans = make_spans(load_genome(path), 5000, seed=91, L=(40, 200), p_readN=0.1, p_edge=0.1)
    args = ([s.read_part for s in spans], [s.a_pos for s in spans], [s.b_aend for s in spans],
            [g.chrom_index(s.chrom) for s in spans],
            [(N.PAIR_BACKSPLICE if s.is_backsplice else 0) | (N.PAIR_PRIMARY_REV if s.primary_reverse else 0)
             for s in spans])
    b0 = PairBatch.pack(opt, g, *args)
    r = reorder(g, b0)
    torch.cuda.synchronize()
    _check_layout(g, b0, r)
    assert r.layout == N.BATCH_LOCUS_ORDERED
    r0 = decode_splices(opt, g, b0, scan(opt, g, b0), raise_errors=False)
    r1 = decode_splices(opt, g, r, scan(opt, g, r), raise_errors=False)
    assert [_key(t) for t in r0] == [_key(t) for t in r1]
    assert sum(1 for t in r0 if isinstance(t, list) and t) > 500
    if fa == "test_ref.fa":
        assert b0.m_bytepath > 0          # byte-path results land at the reordered positions


@pytest.mark.parametrize("n", [1, 63, 8191, 8193, 200_003])
def test_reorder_sizes_hg19(n):
    """Ragged sizes (chunk = 8192 pairs) on the hg19-shaped genome: raw results
    bit-identical to the input-order scan at the slot each pair came from."""
    dev = _dev()
    names, sizes = sq_table(os.path.join(GOLDEN, "test_norm.sam"))
    g = _hg19(dev, names, sizes)
    opt = Options()
    b = PairBatch.synthetic(opt, g, n, SynthConfig(seed=5 + n, span_max=20000))
    r = reorder(g, b)
    torch.cuda.synchronize()
    slot = _check_layout(g, b, r)
    if n > 1000:
        assert r.reorder_info.n_buckets > 500
    res0 = scan(opt, g, b).results[:n].cpu().numpy()
    res1 = scan(opt, g, r).results[:n].cpu().numpy()
    assert np.array_equal(res1, res0[slot])


_HG = {}


def _hg19(dev, names, sizes):
    if "g" not in _HG:
        _HG["g"] = Genome.synthetic(names, sizes, seed=4711, device=dev)
    return _HG["g"]


def test_reorder_full_size_reuse():
    """50M pairs (the bench batch), buffers reused across calls: checksum of the
    raw results equals the input-order scan's; every result written."""
    dev = _dev()
    names, sizes = sq_table(os.path.join(GOLDEN, "test_norm.sam"))
    g = _hg19(dev, names, sizes)
    opt = Options()
    n = 50_000_000
    b = PairBatch.synthetic(opt, g, n, SynthConfig(seed=1337, span_max=20000))
    out0 = scan(opt, g, b)
    r = reorder(g, b)
    r2 = reorder(g, b, into=r)
    assert r2 is r
    out1 = scan(opt, g, r)
    torch.cuda.synchronize()
    slot = r.slot[:n].long()
    a = out0.results[:n]
    c = torch.empty_like(a)
    c[slot] = out1.results[:n]
    assert torch.equal(a, c)
    info = (a >> 48) & 0xFFFF
    assert bool(((info & N.RES_DONE) != 0).all())
    del out0, out1, r, b, a, c
    torch.cuda.empty_cache()


def test_reorder_dummy_genome():
    dev = _dev()
    g = Genome.dummy_genome(device=dev)
    opt = Options()
    spans = make_spans({"chrX": "ACGT" * 500}, 300, seed=3)
    b = PairBatch.pack(opt, g, [s.read_part for s in spans], [s.a_pos for s in spans], [s.b_aend for s in spans],
                       [0] * len(spans), [N.PAIR_BACKSPLICE] * len(spans))
    r = reorder(g, b)
    torch.cuda.synchronize()
    slot = r.slot[:b.n].cpu().numpy()
    assert np.array_equal(slot, np.arange(b.n))      # one bucket: stable = identity
    r0 = decode_splices(opt, g, b, scan(opt, g, b), raise_errors=False)
    r1 = decode_splices(opt, g, r, scan(opt, g, r), raise_errors=False)
    assert [_key(t) for t in r0] == [_key(t) for t in r1]
