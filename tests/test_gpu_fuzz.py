"""GPU parity fuzz: random option sets x random kernel forms against the CPU oracle.

Every case draws find_circ.py options (``-a/--asize``, ``-m/--margin``, ``-d/--maxdist``,
``--non-canonical``, ``--strand-pref``, ``--all-hits``; find_circ.py:393-404) and a kernel form
through the per-call FC2_BATCH_FORM_* hints (LDS-staged / plain / automatic, word pairs or unit
planes, two- or three-lane window loads, locus-ordered flag), then requires results bit-identical to
the oracle's literal restatement of find_breakpoints (find_circ.py:854-974), ties included.
Results never depend on the kernel form.
"""
import os

import numpy as np
import pytest

from conftest import GOLDEN
from gpu_helpers import assert_same, gpu_arrays, oracle_arrays
from synth_small import load_genome, make_spans

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from find_circ2_amd import Options, PairBatch, decode_splices  # noqa: E402
from find_circ2_amd import _native as N  # noqa: E402
from test_gpu_parity import genome, oracle_spans, run_spans  # noqa: E402

# per-call form hints (fc2_batch_view.layout, include/fc2_bp.h): one drawn from each group per case
HINTS = ((0, N.BATCH_FORM_STAGED, N.BATCH_FORM_PLAIN, N.BATCH_FORM_WAVE), (0, 0, N.BATCH_FORM_UNITS),
         (0, N.BATCH_FORM_TWOLANE, N.BATCH_FORM_TRI, N.BATCH_FORM_FIVE), (0, 0, N.BATCH_LOCUS_ORDERED))


@pytest.fixture
def form_hint(monkeypatch):
    """Every scan of the case runs with the drawn hints ORed into its batch view."""
    box = {"hint": 0}
    orig = PairBatch.view

    def view(self):
        v = orig(self)
        v.layout |= box["hint"]
        return v
    monkeypatch.setattr(PairBatch, "view", view)
    return box


# FC2_FUZZ_CASES widens the campaign (the suite runs 40; profiles/r03/gpu_fuzz_400.log ran 400)
@pytest.mark.parametrize("seed", range(int(os.environ.get("FC2_FUZZ_CASES", "40"))))
def test_random_options_and_kernel_forms(seed, form_hint):
    rng = np.random.default_rng(90210 + seed)
    asize = int(rng.integers(6, 26))
    margin = int(rng.integers(0, min(asize - 1, 7) + 1))
    opt = Options(asize=asize, margin=margin, maxdist=int(rng.choice([0, 1, 2, 3, 5, 8])),
                  noncanonical=bool(rng.random() < 0.3), strandpref=bool(rng.random() < 0.3),
                  allhits=bool(rng.random() < 0.3))
    knobs = 0
    for group in HINTS:
        knobs |= int(rng.choice(group))
    form_hint["hint"] = knobs
    fa = ["CDR1as_locus.fa", "test_ref.fa"][seed % 2]
    path = os.path.join(GOLDEN, fa)
    g = genome(path)
    e = asize - margin
    top = 2 * e + (126 if seed % 3 else 300)          # mostly word-pair-layout lengths, some long reads
    spans = make_spans(load_genome(path), 4000, seed=5150 + seed, asize=asize, L=(2 * e - 3, top),
                       p_readN=0.1, p_edge=0.1)
    b, out = run_spans(opt, g, spans)
    r = oracle_spans(opt, path, spans, g.names)
    ga = gpu_arrays(opt, b.host_pairs, out.host(b.n))
    label = "seed %d %s form hints 0x%x" % (seed, vars(opt), knobs)
    assert ga["done"].all(), label
    hits = assert_same(ga, oracle_arrays(r), label=label)
    assert hits > 20, label
    if opt.allhits:
        # decode_splices raises at the first pair the reference would raise on (KeyError /
        # get_data range); the tie lists are compared on a batch of the other pairs
        keep = np.nonzero(~(ga["err_key"] | ga["err_win"]))[0]
        b2, out2 = run_spans(opt, g, [spans[i] for i in keep])
        got = decode_splices(opt, g, b2, out2)
        for j, ties in enumerate(got):
            i = int(keep[j])
            exp = r.ties_of(i)
            assert [(t.start, t.end, t.strand, t.gtag, int(t.dist), t.ov, t.n_hits) for t in ties] == \
                [(int(x["start"]), int(x["end"]), x["strand"].decode(), x["gtag"].decode(), int(x["dist"]),
                  int(x["ov"]), int(x["n_hits"])) for x in exp], (label, i)
    if not opt.noncanonical and not opt.allhits and b.m_bytepath == 0:
        # the same scan writing the compact forms itself (fc2_bp_scan_compact_launch, same form hints):
        # the words and escapes expand back to the 8-byte results, which equal the oracle's (above)
        from find_circ2_amd import expand
        from find_circ2_amd.hotpath import scan_compact
        res = out.results[:b.n].cpu().numpy()
        for width in (2, 4):
            dev = torch.device("cuda", 0)
            words = torch.empty(width * b.n, dtype=torch.uint8, device=dev)
            esc = torch.zeros(16 * b.n, dtype=torch.uint8, device=dev)
            ctr = torch.zeros(1, dtype=torch.int32, device=dev)
            scan_compact(opt, g, b, words.data_ptr(), width, esc.data_ptr(), b.n, ctr.data_ptr())
            torch.cuda.synchronize(dev)
            k = int(ctr.item())
            w = words.cpu().numpy().view(np.uint16 if width == 2 else np.uint32)
            e = esc.cpu().numpy().view(N.ESCAPE_DTYPE)[:k]
            assert np.array_equal(expand(opt, w, e), res), (label, width)
