"""GPU parity on genome shapes the golden FASTAs do not have.

* many contigs (1500 > the 512 a scan block stages in LDS): the staged kernel
  reads the chromosome table from L2 instead;
* N-heavy sequence (runs of 1..5000 N plus isolated N, ~30 % of bases): windows
  that touch N take the N-plane path — in round trip 3 via the super-coarse map
  (staged kernel) or one round trip later via the coarse map (plain kernel);
  chromosome ends give partial windows.
Every case runs through both kernel forms and with the genome twin on and off,
and must be bit-identical to the CPU oracle.
"""
import numpy as np
import pytest

import oracle
from gpu_helpers import assert_same, gpu_arrays, oracle_arrays
from synth_small import load_genome, make_spans

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from find_circ2_amd import Genome, Options, PairBatch, scan  # noqa: E402
from find_circ2_amd import _native as N  # noqa: E402


def _write_fasta(path, seqs, width=60):
    with open(path, "w") as f:
        for name, s in seqs.items():
            f.write(">%s\n" % name)
            for k in range(0, len(s), width):
                f.write(s[k:k + width] + "\n")


def _many_contigs(path, n=1500, seed=5):
    rng = np.random.default_rng(seed)
    seqs = {}
    for c in range(n):
        L = int(rng.integers(200, 4000))
        s = np.frombuffer(b"ACGTacgt", np.uint8)[rng.integers(0, 8, L)].tobytes().decode()
        seqs["scaffold_%d" % c] = s
    _write_fasta(path, seqs)


def _n_heavy(path, seed=6):
    rng = np.random.default_rng(seed)
    seqs = {}
    for c in range(6):
        L = int(rng.integers(150_000, 260_000))
        s = np.frombuffer(b"ACGT", np.uint8)[rng.integers(0, 4, L)].copy()
        covered = 0
        while covered < 0.3 * L:            # N runs of 1..5000
            a = int(rng.integers(0, L))
            b = min(L, a + int(rng.integers(1, 5001)))
            s[a:b] = ord('N')
            covered += b - a
        iso = rng.integers(0, L, L // 500)  # isolated N
        s[iso] = ord('N')
        seqs["chr%d" % (c + 1)] = s.tobytes().decode()
    _write_fasta(path, seqs, width=50)


def _run(opt, g, spans, stage, twin, words=1):
    """Scan through one kernel form, chosen per call by fc2_batch_view.layout hints: stage -> the
    LDS-staged or the plain form, words=0 -> the 64-base unit planes, twin=0 -> the batch flagged
    locus-ordered (no shifted twin, XCD-contiguous blocks; results never depend on the flag)."""
    flags = [(N.PAIR_BACKSPLICE if s.is_backsplice else 0) | (N.PAIR_PRIMARY_REV if s.primary_reverse else 0)
             for s in spans]
    b = PairBatch.pack(opt, g, [s.read_part for s in spans], [s.a_pos for s in spans],
                       [s.b_aend for s in spans], [g.chrom_index_or_missing(s.chrom) for s in spans], flags)
    b.layout |= (N.BATCH_FORM_STAGED if stage else N.BATCH_FORM_PLAIN) | (0 if words else N.BATCH_FORM_UNITS) | \
        (0 if twin else N.BATCH_LOCUS_ORDERED)
    out = scan(opt, g, b)
    torch.cuda.synchronize()
    return b, out


def _oracle(opt, path, spans):
    of = oracle.OracleFasta(path)
    p = oracle.params(opt.asize, opt.margin, opt.maxdist, opt.noncanonical, opt.strandpref, opt.allhits)
    return oracle.scan_fasta(p, of, [s.read_part for s in spans], [of.names.index(s.chrom) for s in spans],
                             [s.a_pos for s in spans], [s.b_aend for s in spans], [s.is_backsplice for s in spans],
                             [s.primary_reverse for s in spans], use_fast=False, all_ties=True)


@pytest.fixture(scope="module")
def genomes(tmp_path_factory):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    d = tmp_path_factory.mktemp("genomes")
    out = {}
    for name, fn in (("many_contigs", _many_contigs), ("n_heavy", _n_heavy)):
        p = str(d / (name + ".fa"))
        fn(p)
        out[name] = (p, Genome.from_fasta(p, device="cuda:0"), load_genome(p))
    return out


@pytest.mark.parametrize("kind", ["many_contigs", "n_heavy"])
@pytest.mark.parametrize("stage,twin,words", [(1, 1, 1), (1, 1, 0), (1, 0, 0), (0, 1, 1), (0, 0, 1)])
@pytest.mark.parametrize("o", [dict(), dict(allhits=True, noncanonical=True)])
def test_genome_shapes_vs_oracle(genomes, kind, stage, twin, words, o):
    path, g, seqs = genomes[kind]
    opt = Options(**o)
    if kind == "many_contigs":
        assert len(g.names) > 512
    spans = make_spans(seqs, 4000, seed=17, L=(40, 150), p_readN=0.1, p_edge=0.1)
    b, out = _run(opt, g, spans, stage, twin, words)
    r = _oracle(opt, path, spans)
    ga = gpu_arrays(opt, b.host_pairs, out.host(b.n))
    assert ga["done"].all()
    hits = assert_same(ga, oracle_arrays(r), label="%s stage=%d twin=%d words=%d %s" % (kind, stage, twin, words, o))
    assert hits > 300
    if kind == "n_heavy":
        # the case under test: windows that overlap N runs (exact, from the FASTA text)
        e = opt.asize - opt.margin
        touched = 0
        for s in spans[:2000]:
            l = len(s.read_part) - 2 * e
            sq = seqs[s.chrom]
            wa = sq[max(0, s.a_pos + e):max(0, s.a_pos + e + l + 2)]
            wb = sq[max(0, s.b_aend - e - l - 2):max(0, s.b_aend - e)]
            touched += ('N' in wa.upper()) or ('N' in wb.upper())
        assert touched > 200
