"""GPU parity: the HIP path (through the C ABI) against the CPU oracle.

Every test here is ``@pytest.mark.gpu`` and runs on a real MI355X.  Results
must be bit-identical to the oracle (integer/byte work): breakpoint x, strand,
coordinates, edit distance, anchor overlap, tie count, splice signal, and the
reference's error conditions.
"""
import os

import numpy as np
import pytest

import oracle
from conftest import GOLDEN
from gpu_helpers import assert_same, gpu_arrays, oracle_arrays
from synth_small import load_genome, make_odd_spans, make_spans, truncated_fasta

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from find_circ2_amd import Genome, Options, PairBatch, SynthConfig, decode_splices, scan  # noqa: E402
from find_circ2_amd import _native as N  # noqa: E402
from oracle.bp_oracle import Options as ROptions, RefIndexedFasta, Span, find_breakpoints  # noqa: E402


@pytest.fixture(params=[N.BATCH_FORM_STAGED, N.BATCH_FORM_PLAIN, N.BATCH_FORM_WAVE], ids=["stage", "nostage", "wave"],
                autouse=True)
def scan_variant(request, monkeypatch):
    """Every parity case runs through both bp_scan32 forms: LDS-staged (chromosome table +
    super-coarse N map) and unstaged (coarse map from L2), and through the one-wavefront-per-pair
    form of BASELINE's north_star (bp_wave_kernel; batches it cannot take -- no word-pair table,
    l + 2 > 128 -- run the default form), forced per call by the FC2_BATCH_FORM_* hint in the batch
    view; the default picks per batch."""
    orig = PairBatch.view

    def view(self):
        v = orig(self)
        v.layout |= request.param
        return v
    monkeypatch.setattr(PairBatch, "view", view)
    yield request.param


def _dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return "cuda:0"


_GENOMES = {}


def genome(path):
    if path not in _GENOMES:
        _GENOMES[path] = Genome.from_fasta(path, device=_dev())
    return _GENOMES[path]


def run_spans(opt: Options, g: Genome, spans):
    flags = [(N.PAIR_BACKSPLICE if s.is_backsplice else 0) | (N.PAIR_PRIMARY_REV if s.primary_reverse else 0)
             for s in spans]
    b = PairBatch.pack(opt, g, [s.read_part for s in spans], [s.a_pos for s in spans], [s.b_aend for s in spans],
                       [g.chrom_index_or_missing(s.chrom) for s in spans], flags)
    out = scan(opt, g, b)
    torch.cuda.synchronize()
    return b, out


def oracle_spans(opt: Options, path, spans, names):
    of = oracle.OracleFasta(path)
    p = oracle.params(opt.asize, opt.margin, opt.maxdist, opt.noncanonical, opt.strandpref, opt.allhits)
    return oracle.scan_fasta(p, of, [s.read_part for s in spans], [of.names.index(s.chrom) for s in spans],
                             [s.a_pos for s in spans], [s.b_aend for s in spans], [s.is_backsplice for s in spans],
                             [s.primary_reverse for s in spans], use_fast=False, all_ties=True)


OPTS = [
    dict(),
    dict(maxdist=0),
    dict(maxdist=4, margin=0),
    dict(noncanonical=True),
    dict(strandpref=True),
    dict(allhits=True),
    dict(allhits=True, noncanonical=True),
    dict(asize=20, margin=5, maxdist=3),
    dict(asize=10, margin=1, maxdist=1, strandpref=True, noncanonical=True, allhits=True),
]


@pytest.mark.parametrize("fa", ["CDR1as_locus.fa", "test_ref.fa"])
@pytest.mark.parametrize("oi", range(len(OPTS)))
def test_spans_vs_oracle(fa, oi):
    o = OPTS[oi]
    opt = Options(**o)
    path = os.path.join(GOLDEN, fa)
    g = genome(path)
    spans = make_spans(load_genome(path), 3000, seed=4711 + oi, asize=opt.asize, L=(40, 300), p_readN=0.1)
    b, out = run_spans(opt, g, spans)
    r = oracle_spans(opt, path, spans, g.names)
    ga = gpu_arrays(opt, b.host_pairs, out.host(b.n))
    assert ga["done"].all()
    hits = assert_same(ga, oracle_arrays(r), label=f"{fa} {o}")
    assert hits > 100
    if opt.allhits:
        got = decode_splices(opt, g, b, out)
        for i, ties in enumerate(got):
            exp = r.ties_of(i)
            assert [(t.start, t.end, t.strand, t.gtag, int(t.dist), t.ov, t.n_hits) for t in ties] == \
                [(int(e["start"]), int(e["end"]), e["strand"].decode(), e["gtag"].decode(), int(e["dist"]),
                  int(e["ov"]), int(e["n_hits"])) for e in exp], i


@pytest.mark.parametrize("fa", ["CDR1as_locus.fa", "test_ref.fa"])
@pytest.mark.parametrize("oi", range(len(OPTS)))
def test_word_layout_vs_oracle(fa, oi):
    """Batches with l + 2 <= 128 read their windows from the word-pair layout (both kernel forms via
    the autouse stage fixture: cooperative and plain loads, the fifth pair for W > 97, the shifted
    copy, windows hanging over chromosome ends), every option set."""
    o = OPTS[oi]
    opt = Options(**o)
    path = os.path.join(GOLDEN, fa)
    g = genome(path)
    e = opt.asize - opt.margin
    spans = make_spans(load_genome(path), 3000, seed=911 + oi, asize=opt.asize, L=(2 * e, 2 * e + 126),
                       p_readN=0.1, p_edge=0.2)
    b, out = run_spans(opt, g, spans)
    assert b.max_l + 2 <= 128
    r = oracle_spans(opt, path, spans, g.names)
    ga = gpu_arrays(opt, b.host_pairs, out.host(b.n))
    assert ga["done"].all()
    hits = assert_same(ga, oracle_arrays(r), label=f"word layout {fa} {o}")
    assert hits > 100


ODD_OPTS = [
    dict(asize=2, margin=2, maxdist=0),          # eff_a = 0: read[0:0] == '' (find_circ.py:895)
    dict(asize=2, margin=2, maxdist=2),
    dict(asize=10, margin=12, maxdist=0),        # eff_a < 0: read[-2:2]
    dict(asize=10, margin=12, maxdist=3),
    dict(asize=3, margin=3, maxdist=1, noncanonical=True, allhits=True),
    dict(),                                       # one-base internal parts against over-long windows
    dict(asize=6, margin=2, maxdist=40, noncanonical=True),
]


@pytest.mark.parametrize("dummy", [False, True], ids=["fasta", "dummy"])
@pytest.mark.parametrize("oi", range(len(ODD_OPTS)))
def test_degenerate_spans_vs_oracle(oi, dummy):
    """asize <= margin (every pair takes the byte-exact kernel), read parts of 0..4 bases and of
    2e +- 3 bases, windows past either chromosome end, on the FASTA and on GenomeAccessor's dummy
    genome (find_circ.py:338-345): pair by pair against the oracle, incl. numpy's broadcast of a
    one-byte operand and its shape failure (:861-863)."""
    o = ODD_OPTS[oi]
    opt = Options(**o)
    path = os.path.join(GOLDEN, "CDR1as_locus.fa")
    g = Genome.dummy_genome(device=_dev()) if dummy else genome(path)
    spans = make_odd_spans(load_genome(path), 2000, seed=31 + oi, asize=opt.asize, margin=opt.margin)
    flags = [(N.PAIR_BACKSPLICE if s.is_backsplice else 0) | (N.PAIR_PRIMARY_REV if s.primary_reverse else 0)
             for s in spans]
    b = PairBatch.pack(opt, g, [s.read_part for s in spans], [s.a_pos for s in spans], [s.b_aend for s in spans],
                       [0 if dummy else g.chrom_index_or_missing(s.chrom) for s in spans], flags)
    if opt.eff_a <= 0:
        assert b.m_bytepath == len(spans)
    out = scan(opt, g, b)
    torch.cuda.synchronize()
    of = oracle.OracleFasta.dummy_genome() if dummy else oracle.OracleFasta(path)
    r = oracle.scan_fasta(oracle.params(**o), of, [s.read_part for s in spans],
                          [0 if dummy else of.names.index(s.chrom) for s in spans], [s.a_pos for s in spans],
                          [s.b_aend for s in spans], [s.is_backsplice for s in spans],
                          [s.primary_reverse for s in spans], use_fast=False, all_ties=True)
    ga = gpu_arrays(opt, b.host_pairs, out.host(b.n))
    assert ga["done"].all()
    assert_same(ga, oracle_arrays(r), label=f"odd spans {o} dummy={dummy}")
    if opt.allhits:
        got = decode_splices(opt, g, b, out, raise_errors=False)
        for i, ties in enumerate(got):
            if r.n_ties[i] < 0:
                continue
            exp = r.ties_of(i)
            assert [(t.start, t.end, t.strand, t.gtag, int(t.dist), t.ov, t.n_hits) for t in ties] == \
                [(int(e["start"]), int(e["end"]), e["strand"].decode(), e["gtag"].decode(), int(e["dist"]),
                  int(e["ov"]), int(e["n_hits"])) for e in exp], i


@pytest.mark.parametrize("o", [dict(), dict(allhits=True, noncanonical=True, strandpref=True)])
def test_locus_ordered_layout_same_results(o):
    """PairBatch.pack(locus_order=True) lays the batch out in genome order; decoded
    results (all ties) must be those of the input-order layout, pair by pair."""
    opt = Options(**o)
    path = os.path.join(GOLDEN, "test_ref.fa")
    g = genome(path)
    spans = make_spans(load_genome(path), 4000, seed=27, L=(40, 200), p_readN=0.05)
    args = ([s.read_part for s in spans], [s.a_pos for s in spans], [s.b_aend for s in spans],
            [g.chrom_index(s.chrom) for s in spans],
            [(N.PAIR_BACKSPLICE if s.is_backsplice else 0) | (N.PAIR_PRIMARY_REV if s.primary_reverse else 0)
             for s in spans])
    b0 = PairBatch.pack(opt, g, *args)
    b1 = PairBatch.pack(opt, g, *args, locus_order=True)
    assert b1.perm is not None and not np.array_equal(b1.perm, np.arange(len(spans)))
    r0 = decode_splices(opt, g, b0, scan(opt, g, b0), raise_errors=False)
    r1 = decode_splices(opt, g, b1, scan(opt, g, b1), raise_errors=False)
    key = lambda t: [(s.start, s.end, s.strand, s.gtag, s.dist, s.ov, s.n_hits) for s in t] \
        if isinstance(t, list) else repr(t)
    assert [key(t) for t in r0] == [key(t) for t in r1]
    assert sum(1 for t in r0 if isinstance(t, list) and t) > 500


def test_known_answers_through_gpu():
    from bwa_emul import emulate_pairs, read_fasta, truth_from_name
    from find_circ2_amd import BreakpointEngine, JunctionSpan
    for fa, rf in [("test_ref.fa", "test_reads.fa"), ("CDR1as_locus.fa", "cdr1as_reads.fa")]:
        path = os.path.join(GOLDEN, fa)
        g = genome(path)
        gen = read_fasta(path)
        names = [l[1:].strip() for l in open(os.path.join(GOLDEN, rf)) if l.startswith('>')]
        seqs = read_fasta(os.path.join(GOLDEN, rf))
        spans = [(n, p) for n in names for p in emulate_pairs(n, seqs[n.split()[0]], gen)]
        opt = Options()
        b, out = run_spans(opt, g, [p for _, p in spans])
        got = decode_splices(opt, g, b, out)
        calls = {}
        for (n, p), ties in zip(spans, got):
            d = calls.setdefault(n, (set(), set()))
            for t in ties[:1]:
                (d[1] if p.is_backsplice else d[0]).add(t.coord)
        for n, (lin, circ) in calls.items():
            t = truth_from_name(n)
            if t:
                assert (lin, circ) == t, n
        if fa == "CDR1as_locus.fa":
            circ = [t[0] for (n, p), t in zip(spans, got) if t and p.is_backsplice]
            assert {c.coord for c in circ} == {("CDR1as_locus", 728, 2213, "+")} and len(circ) == 3
            assert all(c.gtag == "GTAG" and c.dist == 0 and c.ov == 0 and c.n_hits == 1 for c in circ)


WEIRD = (b">c1 desc\nACGTNacgtnRYKMacgtACGTACGTAGGTAAGTCCAG\nGTAGAGTCAGGTCAGTCAGGTAG\n"
         b">c2\nAAAAACCCCCGGAGGTTTTT\r\nGGTAAGTCAGTCAGGTCAGT\r\nNNNNNACGTAGGTAGGTCAG\r\nAC\r\n"
         b">c3\nACGTACGTACGGTAAGTCAG\nACG\nTACGTACAGGTCAGTCAGG\nAGGTCAGTCAGTCAGTCAGTTTAG\n")


def test_byte_path_exotic_and_irregular(tmp_path):
    """IUPAC bytes, CRLF lines and an irregular chromosome go through the byte-exact kernel."""
    path = str(tmp_path / "weird.fa")
    open(path, "wb").write(b"".join(WEIRD.replace(b">c", b">r%dc" % k) for k in range(3)))
    g = Genome.from_fasta(path, device=_dev())
    gen = load_genome(path)
    for o in (dict(asize=6, margin=1, maxdist=3), dict(asize=6, margin=1, maxdist=3, noncanonical=True),
              dict(asize=6, margin=2, maxdist=2, allhits=True, noncanonical=True)):
        opt = Options(**o)
        spans = make_spans(gen, 2000, seed=99, asize=opt.asize, L=(12, 60), p_edge=0.3, p_readN=0.2)
        b, out = run_spans(opt, g, spans)
        assert b.m_bytepath > 0
        r = oracle_spans(opt, path, spans, g.names)
        ga = gpu_arrays(opt, b.host_pairs, out.host(b.n))
        assert ga["done"].all()
        assert_same(ga, oracle_arrays(r), label=str(o))
        if o.get("noncanonical"):
            assert (r.n_ties == -oracle.ORC_ERR_KEY).any(), "expected some reference KeyErrors"


def test_byte_path_truncated_fasta(tmp_path):
    """Windows of every length mix: A cut short at the truncated end against B padded long
    before the chromosome's start, and the other way round.  The string form of find_circ.py:907-908
    then reads B up to byte 2l+2, which the byte kernel's B slot holds.  Pair by pair vs the oracle,
    which reads the same .byo_index."""
    path, gen = truncated_fasta(tmp_path)
    g = Genome.from_fasta(path, device=_dev())
    rng = np.random.default_rng(12)
    from synth_small import SmallSpan
    n_mixed = 0
    for o in (dict(asize=6, margin=1, maxdist=60), dict(asize=6, margin=1, maxdist=60, noncanonical=True, allhits=True),
              dict(asize=8, margin=2, maxdist=0), dict(asize=6, margin=1, maxdist=3)):
        opt = Options(**o)
        e = opt.eff_a
        spans = []
        for _ in range(3000):
            c = "u2" if rng.random() < 0.8 else "u1"
            size = len(gen[c])
            L = int(rng.integers(2 * e, 2 * e + 40))
            l = L - 2 * e
            a_pos = int(rng.integers(size - 30, size + 70)) - e         # A around the real / claimed end
            b_aend = int(rng.integers(-l - 10, 30)) + e                  # B around the start
            if rng.random() < 0.3:
                a_pos, b_aend = int(rng.integers(-l - 10, 20)) - e, int(rng.integers(size - 20, size + 70)) + e
            src = gen[c][max(0, size - L):] + gen[c][:L]
            read = src[:L].encode() if rng.random() < 0.5 else bytes(rng.choice(np.frombuffer(b"ACGTN", np.uint8), L))
            bs = rng.random() < 0.5
            spans.append(SmallSpan(c, 0, a_pos, a_pos + L // 2, (a_pos - 5) if bs else (a_pos + L), b_aend, read,
                                   bool(rng.random() < 0.5)))
            la = len(oracle.OracleFasta(path).get_upper(0 if c == "u1" else 1, a_pos + e, a_pos + e + l + 2)) \
                if len(spans) <= 60 else l + 2
            n_mixed += la < l + 2
        b, out = run_spans(opt, g, spans)
        assert b.m_bytepath > 0
        r = oracle_spans(opt, path, spans, g.names)
        ga = gpu_arrays(opt, b.host_pairs, out.host(b.n))
        assert ga["done"].all()
        assert_same(ga, oracle_arrays(r), label="truncated %s" % o)
    assert n_mixed > 0


def test_edge_lengths_and_long_reads():
    """l < 0, l == 0, l just below/above the 2/4/8-word kernels, and l > 510 (byte path)."""
    path = os.path.join(GOLDEN, "CDR1as_locus.fa")
    g = genome(path)
    gen = load_genome(path)
    opt = Options()
    spans = []
    for L in (20, 25, 26, 27, 28, 100, 127, 128, 129, 130, 150, 254, 255, 256, 257, 258, 300, 520, 522, 523, 524,
              700, 1000):
        spans += make_spans(gen, 20, seed=L, L=(L, L), asize=15, p_short=0.0)
    b, out = run_spans(opt, g, spans)
    assert b.m_bytepath > 0
    r = oracle_spans(opt, path, spans, g.names)
    ga = gpu_arrays(opt, b.host_pairs, out.host(b.n))
    assert_same(ga, oracle_arrays(r), label="edge lengths")


def test_dummy_genome_all_n():
    """GenomeAccessor dummy mode (find_circ.py:340-345): windows are all N."""
    g = Genome.dummy_genome(device=_dev())
    path = os.path.join(GOLDEN, "CDR1as_locus.fa")
    spans = make_spans(load_genome(path), 300, seed=3, p_readN=0.0)
    # reads of mostly N so that non-canonical hits exist
    for k, s in enumerate(spans[:100]):
        s.read_part = b"A" * 13 + b"N" * (len(s.read_part) - 26) + b"T" * 13
    for o in (dict(), dict(noncanonical=True, maxdist=5)):
        opt = Options(**o)
        b, out = run_spans(opt, g, spans)
        res = out.host(b.n)
        ga = gpu_arrays(opt, b.host_pairs, res)
        # oracle with an all-N FASTA-free genome = windows of N
        wins, off = [], []
        pos = 0
        for s in spans:
            l = max(0, len(s.read_part) - 2 * opt.eff_a)
            off.append(pos)
            wins.append(b"N" * (2 * (l + 2)))
            pos += 2 * (l + 2)
        p = oracle.params(**o)
        r = oracle.scan_windows(p, [s.read_part for s in spans], np.frombuffer(b"".join(wins) + b"\0", np.uint8),
                                np.array(off), [s.a_pos for s in spans], [s.b_aend for s in spans],
                                [s.is_backsplice for s in spans], [s.primary_reverse for s in spans])
        hits = assert_same(ga, oracle_arrays(r), label="dummy " + str(o))
        if o.get("noncanonical"):
            assert hits >= 100


def test_skip_flag_and_empty_batch():
    path = os.path.join(GOLDEN, "CDR1as_locus.fa")
    g = genome(path)
    spans = make_spans(load_genome(path), 50, seed=8)
    opt = Options()
    flags = [N.PAIR_SKIP | (N.PAIR_BACKSPLICE if s.is_backsplice else 0) for s in spans]
    b = PairBatch.pack(opt, g, [s.read_part for s in spans], [s.a_pos for s in spans], [s.b_aend for s in spans],
                       [0] * len(spans), flags)
    res = scan(opt, g, b).host(b.n)
    assert (res["best_x"] == -1).all() and ((res["info"] & N.RES_DONE) != 0).all()
    b0 = PairBatch.pack(opt, g, [], [], [], [], [])
    out0 = scan(opt, g, b0)
    torch.cuda.synchronize()
    assert decode_splices(opt, g, b0, out0) == []


def _synth_vs_fasta_oracle(opt, path, n, cfg, check_naive=20000):
    g = genome(path)
    b = PairBatch.synthetic(opt, g, n, cfg)
    out = scan(opt, g, b)
    torch.cuda.synchronize()
    hp = b.fetch_host_pairs()
    res = out.host(n)
    ga = gpu_arrays(opt, hp, res)
    assert ga["done"].all()
    from planes import decode_reads_vec
    words = b.read_words.cpu().numpy().view(np.uint64)
    nwords = b.read_nwords.cpu().numpy().view(np.uint64)
    e = opt.eff_a
    ls = hp["read_len"].astype(np.int64) - 2 * e
    has_n = (hp["flags"] & N.PAIR_READ_N) != 0
    mat, ls = decode_reads_vec(words, nwords, b.stride, n, ls, has_n)
    L = hp["read_len"].astype(np.int64)
    # read_part = anchors (unused by the search) + internal part
    parts = np.full((n, int(L.max())), ord('A'), np.uint8)
    for j in range(mat.shape[1]):
        sel = j < ls
        parts[sel, e + j] = mat[sel, j]
    buf = np.ascontiguousarray(parts).ravel()
    off = (np.arange(n, dtype=np.int64) * parts.shape[1])
    of = oracle.OracleFasta(path)
    p = oracle.params(opt.asize, opt.margin, opt.maxdist, opt.noncanonical, opt.strandpref, opt.allhits)
    chrom = np.array([of.names.index(g.names[c]) for c in hp["chrom"]], np.int32)
    bs = (hp["flags"] & N.PAIR_BACKSPLICE) != 0
    rev = (hp["flags"] & N.PAIR_PRIMARY_REV) != 0
    skip = (hp["flags"] & N.PAIR_SKIP) != 0
    r = oracle.scan_fasta(p, of, (buf, off, L.astype(np.int32)), chrom, hp["a_pos"], hp["b_aend"], bs, rev,
                          use_fast=True)
    hits = assert_same(ga, oracle_arrays(r), mask=~skip, label="synthetic fast-oracle")
    k = min(check_naive, n)
    rn = oracle.scan_fasta(p, of, (buf, off[:k], L[:k].astype(np.int32)), chrom[:k], hp["a_pos"][:k],
                           hp["b_aend"][:k], bs[:k], rev[:k], use_fast=False)
    orr = oracle_arrays(rn)
    sub = {kk: np.asarray(v)[:k] for kk, v in ga.items()}
    assert_same(sub, orr, mask=~skip[:k], label="synthetic naive-oracle")
    return hits, b, res


def test_config2_1M_cdr1as_bit_exact():
    """BASELINE config 2: 1M synthetic 100 bp anchor pairs on CDR1as_locus.fa, bit-exact vs CPU."""
    opt = Options()
    cfg = SynthConfig(seed=1337, len_min=100, len_max=100, p_backsplice=1.0, mut_rate=0.005, n_rate=0.0005,
                      span_min=150, span_max=2500)
    hits, b, res = _synth_vs_fasta_oracle(opt, os.path.join(GOLDEN, "CDR1as_locus.fa"), 1_000_000, cfg)
    assert hits > 200_000


def test_config5_shape_variable_length_150bp():
    """Config-5 shaped reads: L in [120, 150], 30 % linear pairs, all options on one seed."""
    for o in (dict(), dict(noncanonical=True), dict(strandpref=True, maxdist=3)):
        opt = Options(**o)
        cfg = SynthConfig(seed=815, len_min=120, len_max=150, p_backsplice=0.7, mut_rate=0.01, n_rate=0.001)
        _synth_vs_fasta_oracle(opt, os.path.join(GOLDEN, "CDR1as_locus.fa"), 200_000, cfg, check_naive=5000)


def test_hg19_shaped_sampled_parity_and_shard_invariance():
    """Config-3 shaped: hg19 @SQ table (test_norm.sam), synthetic genome with N runs.

    Sampled pairs are checked against the oracle on windows decoded from the
    device genome; the whole batch is checked for shard invariance (splitting it
    in two and scanning the halves gives the same results) and determinism.
    """
    from find_circ2_amd import sq_table
    from planes import decode_reads_vec, window
    dev = _dev()
    names, sizes = sq_table(os.path.join(GOLDEN, "test_norm.sam"))
    assert len(names) == 93 and sum(sizes) == 3_137_161_264
    g = Genome.synthetic(names, sizes, seed=4711, device=dev)
    opt = Options()
    n = 4_000_000
    cfg = SynthConfig(seed=110112, len_min=100, len_max=100, p_backsplice=1.0)
    b = PairBatch.synthetic(opt, g, n, cfg)
    out1 = scan(opt, g, b)
    out2 = scan(opt, g, b)
    torch.cuda.synchronize()
    r1 = out1.results[:n].clone()
    assert torch.equal(r1, out2.results[:n])
    # shard invariance: scan each half as its own batch view
    half = n // 2
    for lo, hi in ((0, half), (half, n)):
        sub = PairBatch()
        sub.__dict__.update(b.__dict__)
        sub.n = hi - lo
        sub.pairs = b.pairs[16 * lo:]
        sub.read_words = b.read_words[lo:]
        sub.read_nwords = b.read_nwords[lo:]
        o = scan(opt, g, sub)
        torch.cuda.synchronize()
        assert torch.equal(o.results[:hi - lo], r1[lo:hi])
    hp = b.fetch_host_pairs()
    res = out1.host(n)
    ga = gpu_arrays(opt, hp, res)
    assert ga["done"].all()
    frac = ga["n_ties"].astype(bool).mean()
    assert 0.3 < frac < 0.95, frac
    # sampled oracle parity
    rng = np.random.default_rng(5)
    idx = np.sort(rng.choice(n, 50_000, replace=False))
    units, nplane = g.host_planes()
    # sampled rows, still column-major (stride = number of samples)
    m = len(idx)
    words = b.read_words.cpu().numpy().view(np.uint64).reshape(b.rw, b.stride)[:, idx].ravel()
    nwords = b.read_nwords.cpu().numpy().view(np.uint64).reshape(b.nw, b.stride)[:, idx].ravel()
    shp = hp[idx]
    e = opt.eff_a
    ls = shp["read_len"].astype(np.int64) - 2 * e
    has_n = (shp["flags"] & N.PAIR_READ_N) != 0
    mat, ls = decode_reads_vec(words, nwords, m, m, ls, has_n)
    reads, wins, woff = [], [], []
    pos = 0
    for k in range(m):
        l = int(ls[k])
        c = int(shp["chrom"][k])
        cs, sz = int(g.chrom_start[c]), int(g.sizes[c])
        a0 = int(shp["a_pos"][k]) + e
        b1 = int(shp["b_aend"][k]) - e
        A = window(units, nplane, cs, sz, a0, a0 + l + 2)
        B = window(units, nplane, cs, sz, b1 - l - 2, b1)
        reads.append(b"A" * e + mat[k, :l].tobytes() + b"A" * e)
        woff.append(pos)
        wins.append(A + B)
        pos += len(A) + len(B)
    p = oracle.params()
    r = oracle.scan_windows(p, reads, np.frombuffer(b"".join(wins) + b"\0", np.uint8), np.array(woff),
                            shp["a_pos"], shp["b_aend"], (shp["flags"] & 1) != 0, (shp["flags"] & 2) != 0,
                            use_fast=True)
    sub = {kk: np.asarray(v)[idx] for kk, v in ga.items()}
    skip = (shp["flags"] & N.PAIR_SKIP) != 0
    hits = assert_same(sub, oracle_arrays(r), mask=~skip, label="hg19 sampled")
    assert hits > 10_000
