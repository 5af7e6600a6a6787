"""CPU: the window-carrying batch form's host packer (fc2_pack_windows) against the oracle.

North_star's design streams each pair's two genome windows from the mmap'd
FASTA with the batch (win_2bit in the SoA).  fc2_pack_windows
reads Af = G[A.pos+e : A.pos+e+l+2] and Bf = G[B.aend-e-l-2 : B.aend-e]
(find_circ.py:900-902) with get_data's semantics (find_circ.py:189-215, N
padding outside the chromosome) and encodes them as bit planes; here every
row is decoded back and compared with the oracle's get_data(...).upper().
"""
import ctypes
import os

import numpy as np
import pytest

from conftest import GOLDEN
from find_circ2_amd import _native as N
from oracle.bp_oracle import RefIndexedFasta
from synth_small import load_genome, make_spans
from test_abi import _open, _pack, _pack_pairs

CODE = b"ACGT"


def _decode_row(ww, wn, stride, i, pw, W, flagged):
    w32 = []
    for j in range(2 * pw):
        v = int(ww[j * stride + i])
        w32 += [v & 0xFFFFFFFF, v >> 32]
    n32 = []
    for j in range(pw):
        v = int(wn[j * stride + i]) if flagged else 0
        n32 += [v & 0xFFFFFFFF, v >> 32]
    out = []
    for x in range(2):
        s = bytearray()
        for pos in range(32 * pw):
            k, b = divmod(pos, 32)
            lo = (w32[(2 * x) * pw + k] >> b) & 1
            hi = (w32[(2 * x + 1) * pw + k] >> b) & 1
            nn = (n32[x * pw + k] >> b) & 1
            if pos >= W:
                assert lo == hi == nn == 0, (i, x, pos)
                continue
            s.append(ord("N") if nn else CODE[lo | (hi << 1)])
        out.append(bytes(s))
    return out


@pytest.mark.parametrize("fa", ["CDR1as_locus.fa", "test_ref.fa"])
@pytest.mark.parametrize("asize,margin", [(15, 2), (10, 1), (20, 5)])
def test_pack_windows_match_get_data(fa, asize, margin):
    L = N.lib()
    path = os.path.join(GOLDEN, fa)
    rc, h = _open(path)
    assert rc == 0
    _pack(h)
    genome = load_genome(path)
    names = list(genome)
    e = asize - margin
    spans = make_spans(genome, 1500, seed=23 + asize, asize=asize, L=(2 * e, 2 * e + 126), p_edge=0.3)
    p = N.Params(asize, margin, 2, 0, 0, 0, 0)
    rc, hp, words, nwords, stride, nbp, _, _ = _pack_pairs(L, p, h, spans, [names.index(s.chrom) for s in spans])
    assert rc == 0, L.fc2_last_error()
    pw, ww_, wnw = ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_uint32()
    maxlen = max(len(s.read_part) for s in spans)
    assert L.fc2_window_geometry(ctypes.byref(p), maxlen, ctypes.byref(pw), ctypes.byref(ww_), ctypes.byref(wnw)) == 0
    pw = pw.value
    assert (ww_.value, wnw.value) == (2 * pw, pw) and 1 <= pw <= 4
    ww = np.full(2 * pw * stride, 0xDEAD, np.uint64)       # stale contents must be overwritten
    wn = np.full(pw * stride, 0xBEEF, np.uint64)
    hp["flags"] |= N.PAIR_WIN_N                             # and stale flags cleared
    assert L.fc2_pack_windows(ctypes.byref(p), h, len(spans), hp.ctypes.data, ww.ctypes.data, wn.ctypes.data, pw,
                              stride, 3) == 0, L.fc2_last_error()
    ref = RefIndexedFasta(path)
    checked = flagged = 0
    for i, s in enumerate(spans):
        l = len(s.read_part) - 2 * e
        W = l + 2
        f = int(hp["flags"][i])
        if (f & (N.PAIR_SKIP | N.PAIR_BYTEPATH)) or l < 0:      # not evaluated: all-zero rows
            assert not any(int(ww[j * stride + i]) for j in range(2 * pw)), i
            assert not any(int(wn[j * stride + i]) for j in range(pw)), i
            assert not f & N.PAIR_WIN_N
            continue
        got = _decode_row(ww, wn, stride, i, pw, W, bool(f & N.PAIR_WIN_N))
        Af = ref.get_data(s.chrom, s.a_pos + e, s.a_pos + e + W).upper()
        Bf = ref.get_data(s.chrom, s.b_aend - e - W, s.b_aend - e).upper()
        assert (got[0], got[1]) == (Af, Bf), (i, s.chrom, s.a_pos, s.b_aend, W)
        assert bool(f & N.PAIR_WIN_N) == (b"N" in Af or b"N" in Bf), i
        checked += 1
        flagged += bool(f & N.PAIR_WIN_N)
    assert checked > 1000 and flagged > 20           # windows hanging over chromosome ends read as N
    L.fc2_fasta_close(h)


def test_window_geometry_limits():
    L = N.lib()
    p = N.Params(15, 2, 2, 0, 0, 0, 0)
    pw, ww, wnw = ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_uint32()
    assert L.fc2_window_geometry(ctypes.byref(p), 100, ctypes.byref(pw), ctypes.byref(ww), ctypes.byref(wnw)) == 0
    assert (pw.value, ww.value, wnw.value) == (3, 6, 3)           # W = 76
    assert L.fc2_window_geometry(ctypes.byref(p), 152, ctypes.byref(pw), ctypes.byref(ww), ctypes.byref(wnw)) == 0
    assert pw.value == 4                                            # W = 128
    assert L.fc2_window_geometry(ctypes.byref(p), 153, ctypes.byref(pw), ctypes.byref(ww),
                                 ctypes.byref(wnw)) == N.FC2_E_RANGE
