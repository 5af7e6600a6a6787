"""The device packer of the compact result forms (fc2_result_compact_launch) where it must escape.
test_gpu_fullsize.py runs it on the 50M-pair bench batch, whose words all fit (0 escapes); here:
(a) the packer's words and escapes equal the numpy restatement of the rule (tests/test_compact_results.py)
word for word on synthetic result words of every shape, escapes included (errors, x > 125 / 254,
n_ties > 16 / 255, dist and ov past their fields); (b) real scan results with many escapes (long
reads, -d 6) expand back bit for bit; (c) an escape list longer than its slots is reported, and the
expansion refuses the truncated list instead of returning wrong words."""
import os

import numpy as np
import pytest

from conftest import GOLDEN
from synth_small import load_genome, make_spans
from test_compact_results import pack, sample_words

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from find_circ2_amd import CompactResults, Options, compact, expand  # noqa: E402
from find_circ2_amd import _native as N  # noqa: E402
from test_gpu_parity import genome, run_spans  # noqa: E402


def _dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda", 0)


def _device_form(opt, words8, width, cap=0):
    dev = _dev()
    d = torch.from_numpy(words8.astype(np.int64)).to(dev)
    c = compact(opt, d, len(words8), into=CompactResults(len(words8), dev, cap=cap, width=width))
    torch.cuda.synchronize(dev)
    k = int(c.count.item())
    esc = c.esc.cpu().numpy().view(N.ESCAPE_DTYPE)[:min(k, c.cap)]
    return c.words[:len(words8)].cpu().numpy(), np.sort(esc, order="index"), k, c.cap


@pytest.mark.parametrize("width", [2, 4])
def test_device_words_equal_the_restated_rule(width):
    w = sample_words(400_003, seed=17).astype(np.int64)
    got, esc, k, cap = _device_form(Options(), w, width, cap=len(w))
    exp, exp_esc = pack(w.view(np.uint64), width)
    assert np.array_equal(got.view(exp.dtype), exp)
    assert k == len(exp_esc) > 1000
    assert np.array_equal(esc["index"], exp_esc["index"])
    assert np.array_equal(esc["result"].view(np.int64), exp_esc["result"].view(np.int64))
    assert np.array_equal(expand(Options(), got, esc), w)


@pytest.mark.parametrize("width", [2, 4])
def test_scan_results_with_escapes_expand_back(width):
    path = os.path.join(GOLDEN, "CDR1as_locus.fa")
    opt = Options(maxdist=6, margin=0)
    spans = make_spans(load_genome(path), 6000, seed=606, asize=opt.asize, L=(60, 300), p_readN=0.05)
    b, out = run_spans(opt, genome(path), spans)
    res = out.results[:b.n].cpu().numpy()
    got, esc, k, cap = _device_form(opt, res, width)
    assert k <= cap
    if width == 2:
        assert k > 100                              # x > 125 and dist > 3 are common here
    assert np.array_equal(expand(opt, got, esc), res)


def test_escape_overflow_is_reported():
    w = sample_words(50_000, seed=23).astype(np.int64)
    got, esc, k, cap = _device_form(Options(), w, 2, cap=16)
    assert cap == 16 and k > cap
    with pytest.raises(Exception):
        expand(Options(), got, esc)
