"""asize <= margin, one-base internal parts and over-long windows (CPU side).

With eff_a = asize - margin <= 0 the reference's internal part read[eff_a:-eff_a]
(find_circ.py:895) is empty (eff_a == 0) or a short slice from the read's end, and
l = L - 2*eff_a exceeds the read: with -d 0 simple_match's string `!=` never holds
(:865-871), otherwise numpy compares byte arrays of different lengths (:861-863),
which fails -- except where one operand has one byte and is broadcast.  These tests
pin the literal Python restatement (oracle/bp_oracle.py, numpy itself does the
comparison) against the C oracle, and the product's host packer routing such pairs
to the byte-exact path.
"""
import ctypes
import os

import numpy as np
import pytest

import oracle
from conftest import GOLDEN
from oracle.bp_oracle import (DummyGenome, Options, RefIndexedFasta, ReferenceKeyError, ReferenceShapeError, Span,
                              find_breakpoints)
from synth_small import load_genome, make_odd_spans

from find_circ2_amd import _native as N

OPTS = [
    dict(asize=2, margin=2, maxdist=0),
    dict(asize=2, margin=2, maxdist=2),
    dict(asize=10, margin=12, maxdist=0),
    dict(asize=10, margin=12, maxdist=3),
    dict(asize=3, margin=3, maxdist=1, noncanonical=True, allhits=True),
    dict(asize=15, margin=2, maxdist=2),                       # one-base internal parts, long windows
    dict(asize=6, margin=2, maxdist=40, noncanonical=True),    # broadcast counts up to the window length
]


def _literal(spans, genome, opt):
    out = []
    for s in spans:
        sp = Span(s.chrom, s.a_pos, s.a_aend, s.b_pos, s.b_aend, s.read_part, s.primary_reverse)
        try:
            out.append(find_breakpoints(sp, genome, opt))
        except ReferenceKeyError:
            out.append("key")
        except ReferenceShapeError:
            out.append("shape")
    return out


def _check(spans, lit, r):
    kinds = {"key": 0, "shape": 0, "hit": 0, "none": 0}
    for i, h in enumerate(lit):
        if h == "key":
            assert r.n_ties[i] == -oracle.ORC_ERR_KEY, i
        elif h == "shape":
            assert r.n_ties[i] == -oracle.ORC_ERR_SHAPE, (i, r.n_ties[i])
        else:
            assert r.n_ties[i] == len(h), (i, r.n_ties[i], len(h), spans[i])
            got = [(int(t['x']), int(t['start']), int(t['end']), t['strand'].decode(), t['gtag'].decode(),
                    int(t['dist']), int(t['ov']), int(t['score']), int(t['n_hits'])) for t in r.ties_of(i)]
            exp = [(x.x, x.start, x.end, x.strand, x.gtag, int(x.dist), x.ov, x.score, x.n_hits) for x in h]
            assert got == exp, (i, got, exp)
        kinds[h if isinstance(h, str) else ("hit" if h else "none")] += 1
    return kinds


@pytest.mark.parametrize("fa", ["CDR1as_locus.fa", "test_ref.fa"])
@pytest.mark.parametrize("oi", range(len(OPTS)))
def test_literal_vs_c_oracle(fa, oi):
    o = OPTS[oi]
    opt = Options(**o)
    path = os.path.join(GOLDEN, fa)
    spans = make_odd_spans(load_genome(path), 1500, seed=77 + oi, asize=opt.asize, margin=opt.margin)
    lit = _literal(spans, RefIndexedFasta(path), opt)
    of = oracle.OracleFasta(path)
    r = oracle.scan_fasta(oracle.params(**o), of, [s.read_part for s in spans], [s.chrom_idx for s in spans],
                          [s.a_pos for s in spans], [s.b_aend for s in spans], [s.is_backsplice for s in spans],
                          [s.primary_reverse for s in spans], use_fast=False, all_ties=True)
    kinds = _check(spans, lit, r)
    print(fa, o, kinds)
    if opt.maxdist > 0:
        assert kinds["shape"] > 0
    if opt.asize - opt.margin > 0:
        assert kinds["hit"] > 0, kinds


@pytest.mark.parametrize("oi", range(len(OPTS)))
def test_literal_vs_c_oracle_dummy_genome(oi):
    """GenomeAccessor's dummy mode (find_circ.py:338-345, 370-371): all-N windows of exactly
    end - start bytes, any chromosome."""
    o = OPTS[oi]
    opt = Options(**o)
    path = os.path.join(GOLDEN, "CDR1as_locus.fa")
    spans = make_odd_spans(load_genome(path), 800, seed=5 + oi, asize=opt.asize, margin=opt.margin)
    lit = _literal(spans, DummyGenome(), opt)
    r = oracle.scan_fasta(oracle.params(**o), oracle.OracleFasta.dummy_genome(), [s.read_part for s in spans],
                          [0] * len(spans), [s.a_pos for s in spans], [s.b_aend for s in spans],
                          [s.is_backsplice for s in spans], [s.primary_reverse for s in spans], use_fast=False,
                          all_ties=True)
    _check(spans, lit, r)


def test_numpy_broadcast_is_the_reference_rule():
    """The rule oracle/bp_oracle.py._mismatches delegates to numpy: a one-byte operand is
    broadcast, other unequal lengths fail (numpy 1.x: scalar True, .sum() raises)."""
    from oracle.bp_oracle import _mismatches
    assert _mismatches(b"A", b"AAC") == 1
    assert _mismatches(b"ACGT", b"T") == 3
    assert _mismatches(b"", b"G") == 0
    assert _mismatches(b"", b"") == 0
    with pytest.raises(ReferenceShapeError):
        _mismatches(b"", b"AC")
    with pytest.raises(ReferenceShapeError):
        _mismatches(b"AC", b"ACG")


@pytest.mark.parametrize("asize,margin", [(2, 2), (10, 12), (3, 5)])
def test_pack_routes_every_pair_to_byte_path(asize, margin):
    """eff_a <= 0: fc2_pack_pairs flags every evaluated pair FC2_PAIR_BYTEPATH and
    fc2_bytepath_fill stores read[e:-e] with Python's slice rules (find_circ.py:895)."""
    L = N.lib()
    p = N.Params(asize, margin, 2, 0, 0, 0, 0)
    path = os.path.join(GOLDEN, "CDR1as_locus.fa")
    h = ctypes.c_void_p()
    N.check(L.fc2_fasta_open(path.encode(), 0, ctypes.byref(h)))
    try:
        nu, ncw = ctypes.c_uint64(), ctypes.c_uint64()
        cs = np.zeros(4, np.uint64)
        N.check(L.fc2_fasta_layout(h, ctypes.byref(nu), ctypes.byref(ncw), cs.ctypes.data))
        units = np.empty(2 * nu.value, np.uint64)
        npl = np.empty(nu.value, np.uint64)
        nco = np.zeros(max(1, ncw.value), np.uint32)
        n_exo = ctypes.c_uint64()
        N.check(L.fc2_fasta_pack(h, units.ctypes.data, npl.ctypes.data, nco.ctypes.data, ctypes.byref(n_exo), 1))
        reads = [b"", b"A", b"acg", b"ACGTACGTAC", b"TTGCAAGGCTTAAACC" * 3]
        buf = np.frombuffer(b"".join(reads) + b"\0" * 16, np.uint8).copy()
        off = np.zeros(len(reads), np.uint64)
        off[1:] = np.cumsum([len(r) for r in reads])[:-1]
        pairs = np.zeros(len(reads), N.PAIR_DTYPE)
        pairs["read_len"] = [len(r) for r in reads]
        pairs["a_pos"] = [100, 200, 300, 400, 500]
        pairs["b_aend"] = [900, 800, 700, 600, 1500]
        pairs["flags"] = N.PAIR_BACKSPLICE
        rw, nw, tw = ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_uint32()
        N.check(L.fc2_batch_geometry(ctypes.byref(p), 48, ctypes.byref(rw), ctypes.byref(nw), ctypes.byref(tw)))
        words = np.zeros(rw.value * len(reads), np.uint64)
        nwords = np.zeros(nw.value * len(reads), np.uint64)
        nbp = ctypes.c_uint64()
        N.check(L.fc2_pack_pairs(ctypes.byref(p), h, len(reads), buf.ctypes.data, off.ctypes.data, pairs.ctypes.data,
                                 words.ctypes.data, rw.value, nwords.ctypes.data, nw.value, len(reads),
                                 ctypes.byref(nbp), 1))
        assert nbp.value == len(reads)
        assert ((pairs["flags"] & N.PAIR_BYTEPATH) != 0).all()
        m, nbytes = ctypes.c_uint64(), ctypes.c_uint64()
        N.check(L.fc2_bytepath_size(ctypes.byref(p), len(reads), pairs.ctypes.data, ctypes.byref(m), ctypes.byref(nbytes)))
        idx = np.zeros(m.value, np.uint64)
        bp = np.zeros(m.value, N.PAIR_DTYPE)
        offs = np.zeros(m.value, np.uint64)
        arena = np.zeros(nbytes.value + 16, np.uint8)
        N.check(L.fc2_bytepath_fill(ctypes.byref(p), h, len(reads), buf.ctypes.data, off.ctypes.data, pairs.ctypes.data,
                                    idx.ctypes.data, bp.ctypes.data, offs.ctypes.data, arena.ctypes.data))
        e = asize - margin
        ref = RefIndexedFasta(path)
        for k, r in enumerate(reads):
            o = int(offs[k])
            lenI, lenA, lenB = arena[o:o + 12].view(np.int32)
            internal = r[e:-e].upper()                                  # Python's own slice
            assert bytes(arena[o + 16:o + 16 + lenI]) == internal, (k, r)
            l = len(r) - 2 * e
            flank = l + 2
            a = ref.get_data("CDR1as_locus", 100 * (k + 1) + e, 100 * (k + 1) + e + flank).upper()
            assert lenA == len(a)
            assert bytes(arena[o + 16 + lenI:o + 16 + lenI + min(lenA, l + 3)]) == a[:l + 3]
    finally:
        L.fc2_fasta_close(h)


@pytest.mark.parametrize("opts", [["-a", "2", "-m", "2", "-d", "0"], ["-a", "10", "-m", "12", "-d", "0"],
                                  ["-a", "2", "-m", "2", "-d", "2"]])
def test_cli_asize_le_margin(tmp_path, opts):
    """The whole CLI (oracle search): -d 0 completes with no junction ('' != spliced, :865-871);
    -d > 0 exits 1 at the first evaluated span (numpy shape failure, :861-863, caught at
    :1578-1583); the native read loop and the Python one agree."""
    from oracle_engine import oracle_evaluator_factory, pipelined_factory
    from test_cli import _reads, bed_rows, run_cli
    fa = os.path.join(GOLDEN, "test_ref.fa")
    rd = _reads(os.path.join(GOLDEN, "test_reads.fa"))
    rc1, o1 = run_cli(tmp_path, fa, rd, extra=opts + ["--python-caller"], evaluator=oracle_evaluator_factory, tag="py")
    rc2, o2 = run_cli(tmp_path, fa, rd, extra=opts, evaluator=pipelined_factory(2), tag="native")
    assert rc1 == rc2 == (0 if opts[-1] == "0" else 1)
    if rc1 == 0:
        for o in (o1, o2):
            assert bed_rows(os.path.join(o, "circ_splice_sites.bed")) == {}
            assert bed_rows(os.path.join(o, "lin_splice_sites.bed")) == {}
        for f in ("circ_splice_sites.bed", "lin_splice_sites.bed", "multi_events.tsv"):
            assert open(os.path.join(o1, f)).read() == open(os.path.join(o2, f)).read()
