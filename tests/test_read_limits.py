"""Read parts longer than FC2_MAX_READ_LEN = 32767 bases.  A batch pair's fc2_result.best_x is
16-bit, so fc2_pack_pairs refuses them (FC2_E_RANGE) instead of wrapping; the reference's x-loop has
no limit (find_circ.py:873, :904-906), so the read loop hands them out as fc2_long_pair records whose
search runs on the long path (32-bit results, fc2_bp_scan_long_launch): the whole CLI with 33-40 kb
reads writes the Python loop's files, and on the GPU the long path equals the oracle tie for tie."""
import ctypes
import gzip
import os

import numpy as np
import pytest

import oracle
from find_circ2_amd import _native as N


def _fasta(tmp_path, seq, name="big"):
    path = str(tmp_path / "g.fa")
    with open(path, "w") as f:
        f.write(">%s\n" % name)
        for i in range(0, len(seq), 60):
            f.write(seq[i:i + 60] + "\n")
    return path


def _long_pair(seq, L, x_frac=0.95):
    """A linear junction read of length L: G[d-k:d] + G[a:a+L-k], donor GT at d, acceptor AG at a-2."""
    k = int(L * x_frac)
    d = 1000 + k
    a = d + 5000
    read = seq[d - k:d] + seq[a:a + L - k]
    return read, d - k, a + L - k, k


def _genome_seq(L):
    rng = np.random.default_rng(3)
    g = list(rng.choice(list("ACGT"), 2 * L + 20000))
    return g


def _long_read_genome(L):
    """Four chromosomes of 3L + 20 kb: one per long read, one for the 100-bp reads."""
    rng = np.random.default_rng(11)
    return {c: bytearray(rng.choice(np.frombuffer(b"ACGT", np.uint8), 3 * L + 20000).tobytes())
            for c in ("g1", "g2", "g3", "g4")}


def _long_reads(g, L):
    """bwa-mem-shaped reads as (name, seq, segments): a linear 2-segment read of L bases, a backsplice
    read of L - 2000, a 3-segment circle of L - 3000, each on its own chromosome, and 100-bp reads next
    to them; a segment = (chrom, query start, query end, genome position).  GT..AG are planted first,
    then the reads are cut from the genome."""
    k = int(L * 0.7)
    d, a = 1000 + k, 1000 + k + 5000
    Lc, kA = L - 2000, 300
    start, end = 2000, 2000 + Lc + 8000
    L3 = L - 3000
    s0, e0 = 3000, 3000 + L3 + 5000
    k1 = L3 // 2
    mid = s0 + k1 + 2000
    plants = [("g1", d, a), ("g2", end, start), ("g3", e0, s0), ("g3", s0 + k1, mid)]
    rng = np.random.default_rng(4)
    shorts = []
    for i in range(20):
        p0 = 1000 + 4000 * i
        q0 = p0 + int(rng.integers(200, 1500))
        plants.append(("g4", p0 + 50, q0))
        shorts.append((p0, q0))
    for c, donor, acceptor in plants:          # GT at the donor, AG before the acceptor
        g[c][donor:donor + 2] = b"GT"
        g[c][acceptor - 2:acceptor] = b"AG"
    G = {c: bytes(sq) for c, sq in g.items()}
    reads = [("lin_long", G["g1"][d - k:d] + G["g1"][a:a + L - k], [("g1", 0, k, d - k), ("g1", k, L, a)]),
             ("circ_long", G["g2"][end - kA:end] + G["g2"][start:start + Lc - kA],
              [("g2", 0, kA, end - kA), ("g2", kA, Lc, start)]),
             ("circ3_long", G["g3"][e0 - 200:e0] + G["g3"][s0:s0 + k1] + G["g3"][mid:mid + L3 - 200 - k1],
              [("g3", 0, 200, e0 - 200), ("g3", 200, 200 + k1, s0), ("g3", 200 + k1, L3, mid)])]
    for i, (p0, q0) in enumerate(shorts):
        reads.append(("short%d" % i, G["g4"][p0:p0 + 50] + G["g4"][q0:q0 + 50], [("g4", 0, 50, p0), ("g4", 50, 100, q0)]))
    return reads


def _sam_of(g, reads):
    """SAM text in bwa mem's shape (tests/samgen.py): the longest segment is the primary record (full
    SEQ, soft clips), the others supplementary (hard clips, their part of SEQ); AS = segment length."""
    lines = ["@HD\tVN:1.5"] + ["@SQ\tSN:%s\tLN:%d" % (c, len(sq)) for c, sq in g.items()]
    for name, seq, segs in reads:
        seq = bytes(seq).decode()
        L = len(seq)
        prim = max(range(len(segs)), key=lambda k: segs[k][2] - segs[k][1])
        for k in [prim] + [k for k in range(len(segs)) if k != prim]:
            c, qs, qe, gp = segs[k]
            clip = "S" if k == prim else "H"
            cig = ("%d%s" % (qs, clip) if qs else "") + "%dM" % (qe - qs) + ("%d%s" % (L - qe, clip) if L - qe else "")
            lines.append("\t".join([name, str(0 if k == prim else 2048), c, str(gp + 1), "60", cig, "*", "0", "0",
                                    seq if k == prim else seq[qs:qe], ("I" * L) if k == prim else "*",
                                    "AS:i:%d" % (qe - qs)]))
    return "\n".join(lines) + "\n"


@pytest.mark.parametrize("extra", [[], ["--all-hits", "--non-canonical", "-d", "3"], ["--chunk-size", "1"],
                                   ["--strand-pref", "--half-unique"]],
                         ids=["default", "all-hits", "chunk1", "strand-pref"])
def test_long_reads_native_equals_python(tmp_path, extra):
    """A 36 kb read (and 34 / 33 kb ones): the native read loop hands them out as long pairs (its
    evaluator's long path, here the oracle) and writes the files of the Python loop, for SAM and BAM;
    every long junction is called (at the coordinates planted, find_circ.py:929-945)."""
    from find_circ2_amd import cli
    from oracle_engine import oracle_evaluator_factory, pipelined_factory
    from samgen import sam_to_bam
    from test_ingest import same
    L = 36000
    g = _long_read_genome(L)
    reads = _long_reads(g, L)
    fa = str(tmp_path / "g.fa")
    with open(fa, "w") as f:
        for c, sq in g.items():
            f.write(">%s\n" % c)
            t = sq.decode()
            for i in range(0, len(t), 60):
                f.write(t[i:i + 60] + "\n")
    sam = str(tmp_path / "in.sam")
    open(sam, "w").write(_sam_of(g, reads))
    bam = str(tmp_path / "in.bam")
    sam_to_bam(open(sam).read(), bam)
    outs = []
    for tag, mode, inp, fac in (("py", ["--python-caller"], sam, oracle_evaluator_factory),
                                ("nat", [], sam, oracle_evaluator_factory),
                                ("nat_bam", [], bam, pipelined_factory(3))):
        o = str(tmp_path / tag)
        assert cli.main(["-G", fa, "-o", o, "-n", "lr", "-q"] + extra + [inp], evaluator_factory=fac) == 0, tag
        outs.append(o)
    same(outs[0], outs[1])
    same(outs[0], outs[2])
    circ = open(os.path.join(outs[1], "circ_splice_sites.bed")).read()
    lin = open(os.path.join(outs[1], "lin_splice_sites.bed")).read()
    rd = gzip.open(os.path.join(outs[1], "spliced_reads.fastq.gz"), "rt").read()
    for name in ("circ_long", "circ3_long"):          # reads of circ junctions (write_read, :1442-1447)
        assert "@" + name in rd, name
    assert "g2\t2000\t%d\t" % (2000 + (L - 2000) + 8000) in circ, circ[:3000]         # circ_long's junction
    assert "g3\t3000\t%d\t" % (3000 + (L - 3000) + 5000) in circ, circ[:3000]         # circ3_long's
    assert "g1\t%d\t%d\t" % (1000 + int(L * 0.7), 1000 + int(L * 0.7) + 5000) in lin, lin[:3000]   # lin_long's intron


def test_pack_refuses_reads_longer_than_limit(tmp_path):
    assert N.MAX_READ_LEN == 32767
    g = _genome_seq(40000)
    path = _fasta(tmp_path, "".join(g))
    h = ctypes.c_void_p()
    N.check(N.lib().fc2_fasta_open(path.encode(), 0, ctypes.byref(h)))
    try:
        nu, ncw = ctypes.c_uint64(), ctypes.c_uint64()
        cs = np.zeros(1, np.uint64)
        N.check(N.lib().fc2_fasta_layout(h, ctypes.byref(nu), ctypes.byref(ncw), cs.ctypes.data))
        units = np.zeros(2 * nu.value, np.uint64)
        nplane = np.zeros(nu.value, np.uint64)
        ncoarse = np.zeros(max(1, ncw.value), np.uint32)
        exo = ctypes.c_uint64()
        N.check(N.lib().fc2_fasta_pack(h, units.ctypes.data, nplane.ctypes.data, ncoarse.ctypes.data,
                                       ctypes.byref(exo), 0))
        p = N.Params(15, 2, 2, 0, 0, 0, 0)
        for L, ok in ((32767, True), (32768, False), (40000, False)):
            buf = np.frombuffer(("A" * L).encode() + b"\0" * 16, np.uint8)
            off = np.zeros(1, np.uint64)
            hp = np.zeros(1, N.PAIR_DTYPE)
            hp["a_pos"], hp["b_aend"], hp["read_len"] = 100, 30000, L
            rw, nw, tw = ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_uint32()
            N.check(N.lib().fc2_batch_geometry(ctypes.byref(p), L, ctypes.byref(rw), ctypes.byref(nw), ctypes.byref(tw)))
            words = np.zeros(rw.value, np.uint64)
            nwords = np.zeros(nw.value, np.uint64)
            nbp = ctypes.c_uint64()
            rc = N.lib().fc2_pack_pairs(ctypes.byref(p), h, 1, buf.ctypes.data, off.ctypes.data, hp.ctypes.data,
                                        words.ctypes.data, rw.value, nwords.ctypes.data, nw.value, 1,
                                        ctypes.byref(nbp), 1)
            if ok:
                assert rc == N.FC2_OK and nbp.value == 1          # l > 510: byte path
            else:
                assert rc == N.FC2_E_RANGE
                assert b"32767" in N.lib().fc2_last_error()
    finally:
        N.lib().fc2_fasta_close(h)


@pytest.mark.gpu
def test_longest_reads_vs_oracle(tmp_path):
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from find_circ2_amd import Genome, Options, PairBatch, decode_splices, scan
    L = 32767
    g = _genome_seq(L + 8000)
    reads, a_pos, b_aend = [], [], []
    for frac in (0.95, 0.5, 0.999):
        k = int(L * frac)
        d, a = 1000 + k, 1000 + k + 5000
        g[d:d + 2] = list("GT")
        g[a - 2:a] = list("AG")
    seq = "".join(g)
    for frac in (0.95, 0.5, 0.999):
        r, ap, be, k = _long_pair(seq, L, frac)
        reads.append(r.encode())
        a_pos.append(ap)
        b_aend.append(be)
    path = _fasta(tmp_path, seq)
    opt = Options()
    gen = Genome.from_fasta(path, device="cuda:0")
    b = PairBatch.pack(opt, gen, reads, a_pos, b_aend, [0] * 3, [0] * 3)
    assert b.m_bytepath == 3
    got = decode_splices(opt, gen, b, scan(opt, gen, b))
    of = oracle.OracleFasta(path)
    r = oracle.scan_fasta(oracle.params(), of, reads, [0] * 3, a_pos, b_aend, [False] * 3, [False] * 3,
                          use_fast=True)
    for i in range(3):
        assert r.n_ties[i] >= 1
        f = r.first[i]
        assert got[i] and (got[i][0].start, got[i][0].end, got[i][0].n_hits) == \
            (int(f["start"]), int(f["end"]), int(r.n_ties[i])), i
    assert int(r.first[0]["x"]) > 30000 and int(r.first[2]["x"]) > 32000


@pytest.mark.gpu
@pytest.mark.parametrize("o", [dict(), dict(allhits=True, noncanonical=True, maxdist=4), dict(maxdist=0),
                               dict(strandpref=True, allhits=True)], ids=["default", "allhits-nc", "d0", "sp"])
def test_long_path_vs_oracle(tmp_path, o):
    """fc2_bp_scan_long_launch on 33-60 kb read parts (breakpoints near either end, reads of random
    bases with no hit, a pair on a missing chromosome, one whose windows leave the chromosome):
    first tie, tie count and every --all-hits tie equal the oracle's."""
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from find_circ2_amd import Genome, Options
    from find_circ2_amd.hotpath import decode_long_splices, scan_long
    opt = Options(**o)
    L0 = 60000
    g = _genome_seq(L0 + 8000)
    fr = (0.95, 0.5, 0.001, 0.999, 0.3)
    lens = (60000, 40000, 33000, 32768, 45000)
    for frac, L in zip(fr, lens):
        k = max(20, int(L * frac))
        d, a = 1000 + k, 1000 + k + 5000
        g[d:d + 2] = list("GT")
        g[a - 2:a] = list("AG")
    seq = "".join(g)
    reads, a_pos, b_aend, chrom, flags = [], [], [], [], []
    for frac, L in zip(fr, lens):
        r, ap, be, k = _long_pair(seq, L, max(20, int(L * frac)) / L)
        reads.append(r.encode())
        a_pos.append(ap)
        b_aend.append(be)
        chrom.append(0)
        flags.append(N.PAIR_PRIMARY_REV if frac < 0.4 else 0)
    rng = np.random.default_rng(9)
    reads.append(bytes(rng.choice(np.frombuffer(b"ACGT", np.uint8), 35000).tobytes()))   # no hit
    a_pos.append(2000), b_aend.append(50000), chrom.append(0), flags.append(0)
    reads.append(reads[0][:34000])                                                         # windows past the end
    a_pos.append(len(seq) - 10000), b_aend.append(len(seq) + 20000), chrom.append(0), flags.append(0)
    path = _fasta(tmp_path, seq)
    gen = Genome.from_fasta(path, device="cuda:0")
    buf = b"".join(reads) + b"\0" * 16
    lp = np.zeros(len(reads), N.LONG_PAIR_DTYPE)
    ln = np.array([len(r) for r in reads], np.uint64)
    lp["read_off"][1:] = np.cumsum(ln[:-1])
    lp["read_len"], lp["a_pos"], lp["b_aend"], lp["chrom"], lp["flags"] = ln, a_pos, b_aend, chrom, flags
    res, ties, toff = scan_long(opt, gen, np.frombuffer(buf, np.uint8), lp)
    assert ((res["info"] & N.RES_DONE) != 0).all()
    of = oracle.OracleFasta(path)
    r = oracle.scan_fasta(oracle.params(opt.asize, opt.margin, opt.maxdist, opt.noncanonical, opt.strandpref,
                                        opt.allhits), of, reads, chrom, a_pos, b_aend, [False] * len(reads),
                          [bool(f & N.PAIR_PRIMARY_REV) for f in flags], use_fast=True, all_ties=True)
    got = decode_long_splices(opt, gen, lp, res, ties, toff)
    n_hit = 0
    for i in range(len(reads)):
        nt = int(r.n_ties[i])
        if nt <= 0:
            assert got[i] == [] or isinstance(got[i], BaseException), (i, nt, got[i])
            assert int(res["best_x"][i]) == -1
            continue
        n_hit += 1
        assert int(res["best_x"][i]) == int(r.first[i]["x"]) and int(res["n_ties"][i]) == nt, i
        exp = r.ties_of(i)
        assert [(t.start, t.end, t.strand, t.gtag, int(t.dist), t.ov, t.n_hits) for t in got[i]] == \
            [(int(e["start"]), int(e["end"]), e["strand"].decode(), e["gtag"].decode(), int(e["dist"]), int(e["ov"]),
              int(e["n_hits"])) for e in (exp if opt.allhits else exp[:1])], i
    assert n_hit >= 5 if opt.maxdist else n_hit >= 4
    assert int(r.first[0]["x"]) > 55000


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [21, 22])
def test_long_path_fuzz_vs_oracle(tmp_path, seed):
    """The long path over random 32768-36000-base read parts whose windows are drawn independently
    from three buckets each -- past the chromosome's end, before its start, inside (get_data's 'N'
    padding, find_circ.py:194-211) -- on a genome with tandem repeats (many ties) and N runs, reads
    cut around a random junction or random bases with N, both strands, --all-hits with -d 2 and
    --non-canonical: every pair's first tie, tie count and tie list equal the oracle's."""
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from find_circ2_amd import Genome, Options
    from find_circ2_amd.hotpath import decode_long_splices, scan_long
    rng = np.random.default_rng(seed)
    G = 90000
    g = bytearray(rng.choice(np.frombuffer(b"ACGT", np.uint8), G).tobytes())
    for _ in range(12):                                   # tandem repeats: runs of equal-scoring x
        p = int(rng.integers(0, G - 3000))
        unit = bytes(rng.choice(np.frombuffer(b"ACGT", np.uint8), int(rng.integers(1, 4))).tobytes())
        g[p:p + 2000] = (unit * 2000)[:2000]
    for _ in range(4):                                    # N runs
        p, n = int(rng.integers(0, G - 500)), int(rng.integers(1, 400))
        g[p:p + n] = b"N" * n
    for _ in range(40):                                   # GT / AG signals
        p = int(rng.integers(2, G - 2))
        g[p:p + 2] = b"GT" if rng.random() < 0.5 else b"AG"
    opt = Options(allhits=True, noncanonical=bool(seed % 2), maxdist=2)
    spec, a_pos, b_aend, flags = [], [], [], []
    for i in range(24):
        L = int(rng.integers(32768, 36001))
        kA = int(rng.integers(20, L - 20))
        v, w = rng.random(), rng.random()
        if v < 0.25:
            ap = G + int(rng.integers(-L, 2 * L))
        elif v < 0.5:
            ap = int(rng.integers(-2 * L, 100))
        else:
            ap = int(rng.integers(0, G - L))
        if w < 0.25:
            be = G + int(rng.integers(-L, 2 * L))
        elif w < 0.5:
            be = int(rng.integers(-L, L))
        else:
            be = int(rng.integers(L, G))
        cut = 0 <= ap and ap + kA <= G - 2 and be - (L - kA) >= 2 and be <= G and rng.random() < 0.8
        if cut and rng.random() < 0.7:                     # a donor / acceptor signal at the junction
            g[ap + kA:ap + kA + 2] = b"GT"
            g[be - (L - kA) - 2:be - (L - kA)] = b"AG"
        spec.append((cut, L, kA, ap, be))
        a_pos.append(ap)
        b_aend.append(be)
        flags.append(N.PAIR_PRIMARY_REV if rng.random() < 0.5 else 0)
    seq = g.decode()
    reads = [(seq[ap:ap + kA] + seq[be - (L - kA):be] if cut else
              "".join("ACGTN"[int(c)] for c in rng.integers(0, 5, L))).encode() for cut, L, kA, ap, be in spec]
    path = _fasta(tmp_path, seq)
    gen = Genome.from_fasta(path, device="cuda:0")
    buf = b"".join(reads) + b"\0" * 16
    lp = np.zeros(len(reads), N.LONG_PAIR_DTYPE)
    ln = np.array([len(r) for r in reads], np.uint64)
    lp["read_off"][1:] = np.cumsum(ln[:-1])
    lp["read_len"], lp["a_pos"], lp["b_aend"], lp["flags"] = ln, a_pos, b_aend, flags
    res, ties, toff = scan_long(opt, gen, np.frombuffer(buf, np.uint8), lp)
    assert ((res["info"] & N.RES_DONE) != 0).all()
    of = oracle.OracleFasta(path)
    r = oracle.scan_fasta(oracle.params(opt.asize, opt.margin, opt.maxdist, opt.noncanonical, opt.strandpref,
                                        opt.allhits), of, reads, [0] * len(reads), a_pos, b_aend,
                          [False] * len(reads), [bool(f & N.PAIR_PRIMARY_REV) for f in flags],
                          use_fast=True, all_ties=True)
    got = decode_long_splices(opt, gen, lp, res, ties, toff)
    n_hit = n_multi = 0
    for i in range(len(reads)):
        nt = int(r.n_ties[i])
        if nt <= 0:
            assert got[i] == [] or isinstance(got[i], BaseException), (i, nt, got[i])
            assert int(res["best_x"][i]) == -1, i
            continue
        n_hit += 1
        n_multi += nt > 1
        assert int(res["best_x"][i]) == int(r.first[i]["x"]) and int(res["n_ties"][i]) == nt, i
        assert [(t.start, t.end, t.strand, t.gtag, int(t.dist), t.ov, t.n_hits) for t in got[i]] == \
            [(int(e["start"]), int(e["end"]), e["strand"].decode(), e["gtag"].decode(), int(e["dist"]), int(e["ov"]),
              int(e["n_hits"])) for e in r.ties_of(i)], i
    assert n_hit >= 3, n_hit
