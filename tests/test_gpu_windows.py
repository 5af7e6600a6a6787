"""GPU: window-carrying batches (fc2_batch_view.win_words) give the same results as the gather.

North_star's form: each pair's Af / Bf travel with the batch, packed on the host
from the mmap'd FASTA (fc2_pack_windows) or gathered on the device from the
resident genome (fc2_gather_windows_launch), and the scan reads no genome at all
-- here it is handed a genome view that holds ONLY the chromosome sizes.  Both
forms must match the oracle and the gathering scan bit for bit (results and
--all-hits tie masks), on every option set; at the bench's full size (50M pairs)
the device-gathered rows must reproduce the gathering scan exactly.
"""
import ctypes
import os

import numpy as np
import pytest

from conftest import GOLDEN
from gpu_helpers import assert_same, gpu_arrays, oracle_arrays
from synth_small import load_genome, make_spans

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from find_circ2_amd import Genome, Options, PairBatch, SynthConfig, scan, sq_table  # noqa: E402
from find_circ2_amd import _native as N  # noqa: E402
from find_circ2_amd.hotpath import ScanOutput  # noqa: E402
from test_gpu_parity import OPTS, oracle_spans  # noqa: E402


def _sizes_only_view(g):
    """A genome view without any sequence: the window-carrying scan may read chromosome sizes only."""
    return N.GenomeView(None, None, None, None, g.d_chrom_size.data_ptr(), 0, len(g.names), 0, None, None, 0, 0,
                        None, 0, 0)


def _scan_carried(opt, g, b):
    p = opt.params()
    res = torch.empty(b.stride, dtype=torch.int64, device=b.device)
    tm = torch.zeros(b.tw * b.stride, dtype=torch.int64, device=b.device) if opt.allhits else None
    out = ScanOutput(res, tm, b.tw, b.stride)
    gv, bv = _sizes_only_view(g), b.view()
    s = torch.cuda.current_stream(b.device).cuda_stream
    N.check(N.lib().fc2_bp_scan_launch(ctypes.byref(p), ctypes.byref(gv), ctypes.byref(bv), res.data_ptr(),
                                       tm.data_ptr() if tm is not None else None, b.tw, s))
    if b.m_bytepath:
        v = b.bytes_view()
        N.check(N.lib().fc2_bp_scan_bytes_launch(ctypes.byref(p), ctypes.byref(v), res.data_ptr(),
                                                 tm.data_ptr() if tm is not None else None, b.tw, b.stride, s))
    torch.cuda.synchronize()
    return out


def _pack(opt, g, spans):
    flags = [(N.PAIR_BACKSPLICE if s.is_backsplice else 0) | (N.PAIR_PRIMARY_REV if s.primary_reverse else 0)
             for s in spans]
    return PairBatch.pack(opt, g, [s.read_part for s in spans], [s.a_pos for s in spans], [s.b_aend for s in spans],
                          [g.chrom_index_or_missing(s.chrom) for s in spans], flags)


@pytest.mark.parametrize("fa", ["CDR1as_locus.fa", "test_ref.fa"])
@pytest.mark.parametrize("oi", range(len(OPTS)))
def test_carried_windows_vs_gather_and_oracle(fa, oi):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    o = OPTS[oi]
    opt = Options(**o)
    path = os.path.join(GOLDEN, fa)
    g = Genome.from_fasta(path, device="cuda:0")
    e = opt.asize - opt.margin
    spans = make_spans(load_genome(path), 3000, seed=77 + oi, asize=opt.asize, L=(2 * e, 2 * e + 126),
                       p_readN=0.1, p_edge=0.2)
    ref_b = _pack(opt, g, spans)
    ref = scan(opt, g, ref_b)
    torch.cuda.synchronize()
    r = oracle_spans(opt, path, spans, g.names)
    for how in ("fasta", "device"):
        b = _pack(opt, g, spans)
        if how == "fasta":
            b.carry_windows_from_fasta(g)
        else:
            b.carry_windows_from_device(g)
        out = _scan_carried(opt, g, b)
        assert torch.equal(out.results[:b.n], ref.results[:b.n]), how
        if opt.allhits:
            assert torch.equal(out.tiemask, ref.tiemask), how
        ga = gpu_arrays(opt, b.fetch_host_pairs(), out.host(b.n))
        assert ga["done"].all()
        hits = assert_same(ga, oracle_arrays(r), label=f"carried {how} {fa} {o}")
        assert hits > 100
        if how == "fasta":
            flagged = int(((b.host_pairs["flags"] & N.PAIR_WIN_N) != 0).sum())
            assert flagged > 10                      # windows over chromosome ends carry N rows


def test_carried_windows_full_size_bench_batch():
    """BASELINE configs[2]: 50M pairs on the hg19-shaped genome; device-gathered rows, sizes-only genome."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    names, sizes = sq_table(os.path.join(GOLDEN, "test_norm.sam"))
    g = Genome.synthetic(names, sizes, seed=4711, device="cuda:0")
    opt = Options()
    n = 50_000_000
    b = PairBatch.synthetic(opt, g, n, SynthConfig(seed=1337, span_min=150, span_max=20000, p_backsplice=1.0,
                                                   mut_rate=0.005, n_rate=0.0005))
    ref = scan(opt, g, b).results[:n].clone()
    torch.cuda.synchronize()
    b.carry_windows_from_device(g)
    out = _scan_carried(opt, g, b)
    neq = int((out.results[:n] != ref).sum())
    assert neq == 0, "%d of %d pairs differ" % (neq, n)
    hit = (ref & 0xFFFF) != 0xFFFF
    assert float(hit.float().mean()) > 0.4
