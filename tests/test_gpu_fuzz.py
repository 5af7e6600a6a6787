"""GPU parity fuzz: random option sets x random kernel forms against the CPU oracle.

Every case draws find_circ.py options (``-a/--asize``, ``-m/--margin``, ``-d/--maxdist``,
``--non-canonical``, ``--strand-pref``, ``--all-hits``; find_circ.py:393-404) and a kernel form
through the FC2_TUNE_* knobs (64- or 32-bit words, LDS staging on/off, 256/512/1024-pair blocks,
three-lane window loads never/always/auto, persistent grid), then requires results bit-identical to
the oracle's literal restatement of find_breakpoints (find_circ.py:854-974), ties included.
Results never depend on the kernel form; the knobs are restored afterwards.
"""
import os

import numpy as np
import pytest

from conftest import GOLDEN
from gpu_helpers import assert_same, gpu_arrays, oracle_arrays
from synth_small import load_genome, make_spans

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from find_circ2_amd import Options, decode_splices  # noqa: E402
from find_circ2_amd import _native as N  # noqa: E402
from test_gpu_parity import genome, oracle_spans, run_spans  # noqa: E402

# FC2_TUNE_* (include/fc2_bp.h): knob -> value drawn per case
KNOBS = {2: (0, 1), 7: (0, 1), 13: (256, 512, 1024), 14: (0, 1, 2), 10: (0, 0, -1)}


@pytest.fixture
def restore_knobs():
    before = {k: N.get_tuning(k) for k in KNOBS}
    yield
    for k, v in before.items():
        N.lib().fc2_set_tuning(k, v)


@pytest.mark.parametrize("seed", range(40))
def test_random_options_and_kernel_forms(seed, restore_knobs):
    rng = np.random.default_rng(90210 + seed)
    asize = int(rng.integers(6, 26))
    margin = int(rng.integers(0, min(asize - 1, 7) + 1))
    opt = Options(asize=asize, margin=margin, maxdist=int(rng.choice([0, 1, 2, 3, 5, 8])),
                  noncanonical=bool(rng.random() < 0.3), strandpref=bool(rng.random() < 0.3),
                  allhits=bool(rng.random() < 0.3))
    knobs = {k: int(rng.choice(v)) for k, v in KNOBS.items()}
    for k, v in knobs.items():
        N.lib().fc2_set_tuning(k, v)
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
    label = "seed %d %s knobs %s" % (seed, vars(opt), knobs)
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
