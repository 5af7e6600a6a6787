"""GPU: every form of the scan kernel agrees bit for bit at the bench's full size.

bp_scan32 has an LDS-staged form with cooperative window loads (read-order batches over a large
genome; two- or three-lane loads of the word-pair table, or the 64-base unit planes) and a plain
form (locus-ordered batches, small genomes; word pairs or unit planes).  fc2_bp_scan_launch picks
one per batch; the per-call FC2_BATCH_FORM_* hints of fc2_batch_view.layout force each of them
(the shipped library has no process-global knobs; the measured-and-rejected forms live only in A/B
builds, libfc2_ab.so).  They share no window-loading code path, so identical raw results on all
50M pairs of the BASELINE configs[2] workload (read order and locus order) are a size-independent
parity property on top of the oracle comparisons of test_gpu_parity.py / test_gpu_fullsize.py.
"""
import os

import numpy as np
import pytest

from conftest import GOLDEN

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from find_circ2_amd import Genome, Options, PairBatch, SynthConfig, scan, sq_table  # noqa: E402
from find_circ2_amd import _native as N  # noqa: E402

FORMS = {"default": 0,
         "staged_words_twolane": N.BATCH_FORM_STAGED | N.BATCH_FORM_TWOLANE,
         "staged_words_tri": N.BATCH_FORM_STAGED | N.BATCH_FORM_TRI,
         "staged_words_five": N.BATCH_FORM_STAGED | N.BATCH_FORM_FIVE,
         "staged_units": N.BATCH_FORM_STAGED | N.BATCH_FORM_UNITS,
         "plain_words": N.BATCH_FORM_PLAIN,
         "plain_units": N.BATCH_FORM_PLAIN | N.BATCH_FORM_UNITS,
         "wave_per_pair": N.BATCH_FORM_WAVE}


def _scan_form(opt, g, b, form):
    keep = b.layout
    b.layout = keep | FORMS[form]
    try:
        return scan(opt, g, b)
    finally:
        b.layout = keep


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
            out = _scan_form(opt, hg19, b, form)
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
        for form in ("default", "staged_words_twolane", "staged_units", "plain_words", "plain_units", "wave_per_pair"):
            out = _scan_form(opt, hg19, b, form)
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
        torch.cuda.empty_cache()


def test_forms_agree_all_hits_ties(hg19):
    """--all-hits --non-canonical --strand-pref: results and tie masks of every form agree."""
    opt = Options(allhits=True, noncanonical=True, strandpref=True)
    n = 4_000_000
    b = PairBatch.synthetic(opt, hg19, n, SynthConfig(seed=99, span_max=20000, p_backsplice=0.5))
    ref = None
    try:
        for form in FORMS:
            out = _scan_form(opt, hg19, b, form)
            torch.cuda.synchronize()
            cur = (out.results[:n].clone(), out.tiemask.view(out.tw, out.stride)[:, :n].clone())
            if ref is None:
                ref = cur
                assert int((ref[1] != 0).any(dim=0).sum()) > n // 10
            else:
                assert torch.equal(cur[0], ref[0]), form
                assert torch.equal(cur[1], ref[1]), form
    finally:
        torch.cuda.empty_cache()
