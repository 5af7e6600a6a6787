"""GPU: every form of the scan kernel agrees bit for bit at the bench's full size.

bp_scan32 has an LDS-staged form with cooperative window loads (read-order
batches over a large genome) and a plain form (locus-ordered batches, small
genomes); bp_scan is the 64-bit-word variant; the genome twin is optional.  They
share no window-loading code path, so identical raw results on all 50M pairs of
the BASELINE configs[2] workload (read order and locus order) are a
size-independent parity property on top of the oracle comparisons of
test_gpu_parity.py, which run at sizes the oracle finishes in seconds.
"""
import os

import numpy as np
import pytest

from conftest import GOLDEN

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from find_circ2_amd import Genome, Options, PairBatch, SynthConfig, scan, sq_table  # noqa: E402
from find_circ2_amd import _native as N  # noqa: E402

# knob values per form: FC2_TUNE_KERNEL32 (2), STAGE (7), TWIN (6), PERSIST (10), WORDS (11), STAGE_BLOCK (13),
# TRI (14)
KNOBS = (2, 7, 6, 10, 11, 13, 14)
FORMS = {"scan32_staged_coop_words": (1, 1, 1, 0, 1, 256, 0), "scan32_staged_coop_words_512": (1, 1, 1, 0, 1, 512, 0),
         "scan32_staged_coop_words_1024": (1, 1, 1, 0, 1, 1024, 0),
         "scan32_staged_tri_words_512": (1, 1, 1, 0, 1, 512, 1),
         "scan32_staged_tri_words_256": (1, 1, 1, 0, 1, 256, 1),
         "scan32_staged_coop_units_twin": (1, 1, 1, 0, 0, 256, 0),
         "scan32_persistent_coop_words": (1, 1, 1, -1, 1, 256, 0),
         "scan32_persistent_coop_twin": (1, 1, 1, -1, 0, 256, 0),
         "scan32_persistent_3_per_cu": (1, 1, 1, 3, 0, 256, 0),
         "scan32_plain_words_no_twin": (1, 0, 0, 0, 1, 256, 0), "scan32_plain_words_twin": (1, 0, 1, 0, 1, 256, 0),
         "scan32_plain_units_no_twin": (1, 0, 0, 0, 0, 256, 0), "scan32_plain_units_twin": (1, 0, 1, 0, 0, 256, 0),
         "scan64": (0, 0, 0, 0, 1, 256, 0)}
DEFAULTS = {k: N.get_tuning(k) for k in KNOBS}


def _set(form):
    L = N.lib()
    for k, v in zip(KNOBS, FORMS[form]):
        N.check(L.fc2_set_tuning(k, v))


def _reset():
    L = N.lib()
    for k, v in DEFAULTS.items():
        L.fc2_set_tuning(k, v)


@pytest.fixture(scope="module")
def hg19():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    names, sizes = sq_table(os.path.join(GOLDEN, "test_norm.sam"))
    return Genome.synthetic(names, sizes, seed=4711, device="cuda:0")


@pytest.mark.parametrize("ordered", [False, True], ids=["read_order", "locus_order"])
def test_forms_agree_full_size(hg19, ordered):
    opt = Options()
    n = 50_000_000
    b = PairBatch.synthetic(opt, hg19, n, SynthConfig(seed=1337, span_max=20000, locus_ordered=ordered))
    ref = None
    try:
        for form in FORMS:
            _set(form)
            out = scan(opt, hg19, b)
            torch.cuda.synchronize()
            res = out.results[:n].clone()
            del out
            if ref is None:
                ref = res
                info = (ref >> 48) & 0xFFFF
                assert bool(((info & N.RES_DONE) != 0).all())
                hit = ((ref & 0xFFFF) != 0xFFFF)
                assert float(hit.float().mean()) > 0.4          # ~half of the pairs are planted junctions
            else:
                neq = int((res != ref).sum())
                assert neq == 0, "%s differs from %s on %d of %d pairs" % (form, next(iter(FORMS)), neq, n)
            del res
    finally:
        _reset()
        del b, ref
        torch.cuda.empty_cache()


def test_forms_agree_150bp(hg19):
    """BASELINE configs[4] shape: 120-150 bp reads (windows up to 126 bases, five word pairs): the
    three-lane form (default there), the two-lane form with the fifth-pair load and the plain form agree."""
    opt = Options()
    n = 25_000_000
    b = PairBatch.synthetic(opt, hg19, n, SynthConfig(seed=4242, len_min=120, len_max=150, span_max=20000))
    ref = None
    try:
        for form in ("scan32_staged_tri_words_512", "scan32_staged_coop_words_512", "scan32_staged_coop_words",
                     "scan32_plain_words_twin", "scan32_plain_units_twin", "scan64"):
            _set(form)
            out = scan(opt, hg19, b)
            torch.cuda.synchronize()
            res = out.results[:n].clone()
            del out
            if ref is None:
                ref = res
                assert float(((ref & 0xFFFF) != 0xFFFF).float().mean()) > 0.4
            else:
                neq = int((res != ref).sum())
                assert neq == 0, "%s differs on %d of %d pairs" % (form, neq, n)
    finally:
        _reset()
        torch.cuda.empty_cache()


def test_forms_agree_all_hits_ties(hg19):
    """--all-hits --non-canonical --strand-pref: results and tie masks of every form agree."""
    opt = Options(allhits=True, noncanonical=True, strandpref=True)
    n = 4_000_000
    b = PairBatch.synthetic(opt, hg19, n, SynthConfig(seed=99, span_max=20000, p_backsplice=0.5))
    ref = None
    try:
        for form in FORMS:
            _set(form)
            out = scan(opt, hg19, b)
            torch.cuda.synchronize()
            cur = (out.results[:n].clone(), out.tiemask.view(out.tw, out.stride)[:, :n].clone())
            if ref is None:
                ref = cur
                assert int((ref[1] != 0).any(dim=0).sum()) > n // 10
            else:
                assert torch.equal(cur[0], ref[0]), form
                assert torch.equal(cur[1], ref[1]), form
    finally:
        _reset()
        torch.cuda.empty_cache()
