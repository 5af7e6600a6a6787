"""The full-size parity checker (oracle.scan_planes, orc_scan_planes in oracle/bp_oracle.c) against
the FASTA-fed oracle (orc_scan_fasta) -- CPU only.

scan_planes reads a batch exactly as the GPU gets it: pairs packed by the host packer
(fc2_pack_pairs) and the 2-bit genome planes (fc2_fasta_pack), decoded back to bytes by the
oracle's own reading of include/fc2_bp.h.  Its 8-byte result words must encode the FASTA-fed
oracle's first tie for every pair (non-byte-path pairs; byte-path pairs are reported as skipped).
This pins the checker the -m gpu full-size tests use at 50M pairs.
"""
import ctypes
import os

import numpy as np
import pytest

import oracle
from conftest import GOLDEN
from synth_small import load_genome, make_spans

from find_circ2_amd import _native as N

_RC = {ord('A'): 'T', ord('C'): 'G', ord('G'): 'C', ord('T'): 'A', ord('N'): 'N'}
_C3 = {"A": 0, "C": 1, "G": 2, "T": 3, "N": 4}


def host_genome(path):
    h = ctypes.c_void_p()
    N.check(N.lib().fc2_fasta_open(path.encode(), 0, ctypes.byref(h)))
    nc = N.lib().fc2_fasta_n_chrom(h)
    nu, ncw = ctypes.c_uint64(), ctypes.c_uint64()
    cs = np.zeros(nc, np.uint64)
    N.check(N.lib().fc2_fasta_layout(h, ctypes.byref(nu), ctypes.byref(ncw), cs.ctypes.data))
    units = np.zeros(2 * nu.value, np.uint64)
    nplane = np.zeros(nu.value, np.uint64)
    ncoarse = np.zeros(max(1, ncw.value), np.uint32)
    exo = ctypes.c_uint64()
    N.check(N.lib().fc2_fasta_pack(h, units.ctypes.data, nplane.ctypes.data, ncoarse.ctypes.data,
                                   ctypes.byref(exo), 0))
    sizes = np.zeros(nc, np.int64)
    names = []
    for i in range(nc):
        nm, sz, o, ld, sk, rg = ctypes.c_char_p(), ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64(), \
            ctypes.c_int64(), ctypes.c_int()
        N.check(N.lib().fc2_fasta_chrom(h, i, ctypes.byref(nm), ctypes.byref(sz), ctypes.byref(o), ctypes.byref(ld),
                                        ctypes.byref(sk), ctypes.byref(rg)))
        names.append(nm.value.decode())
        sizes[i] = sz.value
    return h, names, units, nplane, cs, sizes


def expected_words(r: "oracle.OracleResult", n: int) -> np.ndarray:
    out = np.zeros(n, np.uint64)
    for i in range(n):
        t = int(r.n_ties[i])
        if t < 0:
            err = 0x2000 if t == -oracle.ORC_ERR_KEY else 0x4000
            out[i] = 0xFFFF | ((0x8000 | err) << 48)
            continue
        if t == 0:
            out[i] = 0xFFFF | (0x8000 << 48)
            continue
        f = r.first[i]
        minus = f["strand"] == b"-"
        g = f["gtag"].decode()
        raw = "".join(_RC[ord(c)] for c in reversed(g)) if minus else g
        g12 = sum(_C3[c] << (3 * k) for k, c in enumerate(raw))
        info = 0x8000 | (1 if minus else 0) | ((g12 << 1) & 0x1FFE)
        out[i] = (int(f["x"]) & 0xFFFF) | (min(int(f["dist"]), 255) << 16) | ((int(f["ov"]) & 0xFF) << 24) | \
            (min(t, 0xFFFF) << 32) | (info << 48)
    return out


@pytest.mark.parametrize("fa", ["CDR1as_locus.fa", "test_ref.fa"])
@pytest.mark.parametrize("o", [dict(), dict(maxdist=0), dict(noncanonical=True, strandpref=True),
                               dict(asize=20, margin=5, maxdist=3), dict(asize=10, margin=0, maxdist=4)])
def test_scan_planes_equals_fasta_oracle(fa, o):
    path = os.path.join(GOLDEN, fa)
    h, names, units, nplane, cs, sizes = host_genome(path)
    try:
        p = oracle.params(**o)
        fp = N.Params(p.asize, p.margin, p.maxdist, p.noncanonical, p.strandpref, 0, 0)
        spans = make_spans(load_genome(path), 3000, seed=77, asize=p.asize, L=(20, 300), p_readN=0.1, p_edge=0.2)
        n = len(spans)
        reads = [s.read_part for s in spans]
        lens = np.array([len(r) for r in reads], np.int64)
        off = np.zeros(n, np.uint64)
        off[1:] = np.cumsum(lens[:-1])
        buf = np.frombuffer(b"".join(reads) + b"\0" * 16, np.uint8)
        hp = np.zeros(n, N.PAIR_DTYPE)
        hp["a_pos"] = [s.a_pos for s in spans]
        hp["b_aend"] = [s.b_aend for s in spans]
        hp["chrom"] = [names.index(s.chrom) for s in spans]
        hp["read_len"] = lens
        hp["flags"] = [(N.PAIR_BACKSPLICE if s.is_backsplice else 0) | (N.PAIR_PRIMARY_REV if s.primary_reverse else 0)
                       for s in spans]
        hp["flags"][::97] |= N.PAIR_SKIP
        rw, nw, tw = ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_uint32()
        N.check(N.lib().fc2_batch_geometry(ctypes.byref(fp), int(lens.max()), ctypes.byref(rw), ctypes.byref(nw),
                                           ctypes.byref(tw)))
        words = np.zeros(rw.value * n, np.uint64)
        nwords = np.zeros(nw.value * n, np.uint64)
        nbp = ctypes.c_uint64()
        N.check(N.lib().fc2_pack_pairs(ctypes.byref(fp), h, n, buf.ctypes.data, off.ctypes.data, hp.ctypes.data,
                                       words.ctypes.data, rw.value, nwords.ctypes.data, nw.value, n,
                                       ctypes.byref(nbp), 1))
        got, skipped = oracle.scan_planes(p, units, nplane, cs, sizes, hp, words, nwords, rw.value, nw.value, n, n,
                                          n_threads=4)
        bp = (hp["flags"] & N.PAIR_BYTEPATH) != 0
        assert skipped == int(bp.sum())
        of = oracle.OracleFasta(path)
        r = oracle.scan_fasta(p, of, reads, [of.names.index(s.chrom) for s in spans], hp["a_pos"], hp["b_aend"],
                              (hp["flags"] & 1) != 0, (hp["flags"] & 2) != 0, use_fast=False)
        exp = expected_words(r, n)
        skip = (hp["flags"] & N.PAIR_SKIP) != 0
        exp[skip] = 0xFFFF | (0x8000 << 48)
        check = ~bp
        bad = np.nonzero(got[check] != exp[check])[0]
        assert bad.size == 0, (fa, o, np.nonzero(check)[0][bad[:5]], got[check][bad[:5]], exp[check][bad[:5]])
        assert (((got[check] & np.uint64(0xFFFF)) != np.uint64(0xFFFF)).sum()) > 100
    finally:
        N.lib().fc2_fasta_close(h)
