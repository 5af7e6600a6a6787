"""CPU oracle package -- TEST INFRASTRUCTURE ONLY (see bp_oracle.py / bp_oracle.c).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this package.  The product package ``find_circ2_amd`` never does.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from typing import List, Optional

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = os.path.join(_HERE, "liboracle.so")


class OrcParams(ctypes.Structure):
    _fields_ = [("asize", ctypes.c_int32), ("margin", ctypes.c_int32), ("maxdist", ctypes.c_int32),
                ("noncanonical", ctypes.c_uint8), ("strandpref", ctypes.c_uint8),
                ("allhits", ctypes.c_uint8), ("_pad", ctypes.c_uint8)]


class OrcHit(ctypes.Structure):
    _fields_ = [("x", ctypes.c_int32), ("start", ctypes.c_int32), ("end", ctypes.c_int32),
                ("dist", ctypes.c_int32), ("ov", ctypes.c_int32), ("score", ctypes.c_int32),
                ("n_hits", ctypes.c_int32), ("strand", ctypes.c_char), ("gtag", ctypes.c_char * 5)]


ORC_HIT_DTYPE = np.dtype([("x", "<i4"), ("start", "<i4"), ("end", "<i4"), ("dist", "<i4"),
                          ("ov", "<i4"), ("score", "<i4"), ("n_hits", "<i4"), ("strand", "S1"),
                          ("gtag", "S5")], align=True)
assert ORC_HIT_DTYPE.itemsize == ctypes.sizeof(OrcHit), (ORC_HIT_DTYPE.itemsize, ctypes.sizeof(OrcHit))

ORC_ERR_KEY = 1
ORC_ERR_SHAPE = 2
ORC_ERR_CHROM = 3


def build(force: bool = False) -> str:
    src = os.path.join(_HERE, "bp_oracle.c")
    if force or not os.path.exists(_LIB) or os.path.getmtime(_LIB) < os.path.getmtime(src):
        subprocess.check_call(["make", "-s", "-C", _HERE, "liboracle.so"])
    return _LIB


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB):
            build()
        L = ctypes.CDLL(_LIB)
        vp = ctypes.c_void_p
        L.orc_fasta_index.restype = vp
        L.orc_fasta_index.argtypes = [vp, ctypes.c_int64]
        L.orc_fasta_free.argtypes = [vp]
        L.orc_fasta_dummy.restype = vp
        L.orc_fasta_dummy.argtypes = []
        L.orc_fasta_n_chrom.argtypes = [vp]
        L.orc_fasta_chrom_name.restype = ctypes.c_char_p
        L.orc_fasta_chrom_name.argtypes = [vp, ctypes.c_int]
        L.orc_fasta_chrom_size.restype = ctypes.c_int64
        L.orc_fasta_chrom_size.argtypes = [vp, ctypes.c_int]
        L.orc_fasta_find.argtypes = [vp, ctypes.c_char_p]
        L.orc_get_upper.restype = ctypes.c_int64
        L.orc_get_upper.argtypes = [vp, ctypes.c_int, ctypes.c_int64, ctypes.c_int64, vp, ctypes.c_int64]
        L.orc_scan_fasta.restype = ctypes.c_int64
        L.orc_scan_fasta.argtypes = [ctypes.POINTER(OrcParams), vp, ctypes.c_int64,
                                     vp, vp, vp, vp, vp, vp, vp, vp, ctypes.c_int,
                                     vp, vp, vp, ctypes.c_int64, vp, ctypes.c_int]
        L.orc_scan_windows.restype = ctypes.c_int64
        L.orc_scan_windows.argtypes = [ctypes.POINTER(OrcParams), ctypes.c_int64,
                                       vp, vp, vp, vp, vp, vp, vp, vp, vp, ctypes.c_int,
                                       vp, vp, vp, ctypes.c_int64, vp]
        _lib = L
    return _lib


def params(asize=15, margin=2, maxdist=2, noncanonical=False, strandpref=False, allhits=False) -> OrcParams:
    return OrcParams(asize, margin, maxdist, int(bool(noncanonical)), int(bool(strandpref)), int(bool(allhits)), 0)


class OracleFasta:
    """A FASTA indexed with the reference's semantics (find_circ.py:120-155)."""

    dummy = False

    def __init__(self, path: str = None, data: bytes = None):
        if data is None:
            with open(path, "rb") as f:
                data = f.read()
        self._buf = np.frombuffer(data, dtype=np.uint8).copy()
        self.h = lib().orc_fasta_index(self._buf.ctypes.data, len(self._buf))
        if path is not None and os.access(path + ".byo_index", os.R_OK):
            self._load_index(path + ".byo_index")     # find_circ.py:110-112
        n = lib().orc_fasta_n_chrom(self.h)
        self.names = [lib().orc_fasta_chrom_name(self.h, i).decode() for i in range(n)]
        self.sizes = [lib().orc_fasta_chrom_size(self.h, i) for i in range(n)]

    def _load_index(self, ipath: str):
        """load_index (find_circ.py:182-187): one line per chromosome, the skip characters as a
        Python-2 repr (string_escape)."""
        import codecs
        rows = []
        with open(ipath, "rb") as f:
            for line in f:
                chrom, ofs, ldata, skip, skipchar, size = line.rstrip().split(b"\t")
                rows.append((chrom, int(ofs), int(ldata), int(skip), codecs.escape_decode(skipchar[1:-1])[0],
                             int(size)))
        # the chromosomes keep the positions index() gave them (callers index them in FASTA order, the
        # reference looks them up by name); names only the index file holds come after them
        L = lib()
        first = [L.orc_fasta_chrom_name(self.h, i) for i in range(L.orc_fasta_n_chrom(self.h))]
        rank = {nm: k for k, nm in enumerate(first)}
        rows.sort(key=lambda r: rank.get(r[0], len(first)))
        n = len(rows)
        if not hasattr(L, "_set_chroms_sig"):
            vp, i64p = ctypes.c_void_p, ctypes.POINTER(ctypes.c_int64)
            L.orc_fasta_set_chroms.argtypes = [vp, ctypes.c_int, ctypes.POINTER(ctypes.c_char_p), i64p, i64p, i64p,
                                               ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(ctypes.c_int32), i64p]
            L._set_chroms_sig = True
        col = lambda k: (ctypes.c_int64 * max(n, 1))(*[r[k] for r in rows])       # noqa: E731
        names = (ctypes.c_char_p * max(n, 1))(*[r[0] for r in rows])
        skipc = (ctypes.c_char_p * max(n, 1))(*[r[4] for r in rows])
        skipl = (ctypes.c_int32 * max(n, 1))(*[len(r[4]) for r in rows])
        L.orc_fasta_set_chroms(self.h, n, names, col(1), col(2), col(3), skipc, skipl, col(5))

    @classmethod
    def dummy_genome(cls) -> "OracleFasta":
        """GenomeAccessor's dummy mode (find_circ.py:338-345, 370-371): all-N windows for every
        chromosome, used when indexed_fasta() raises IOError (e.g. -G <directory>)."""
        g = cls.__new__(cls)
        g._buf = None
        g.h = lib().orc_fasta_dummy()
        g.names, g.sizes, g.dummy = [], [], True
        return g

    @classmethod
    def open_or_dummy(cls, path: str) -> "OracleFasta":
        """GenomeAccessor.__init__ (find_circ.py:338-345): IOError -> dummy mode.  Python 3's
        IOError is OSError; the reference's file() raises it for a missing file, a directory or
        missing permissions."""
        try:
            return cls(path)
        except OSError:
            return cls.dummy_genome()

    def __del__(self):
        try:
            lib().orc_fasta_free(self.h)
        except Exception:
            pass

    def get_upper(self, chrom: int, start: int, end: int) -> bytes:
        cap = max(0, end - start) + 64
        out = np.zeros(cap, dtype=np.uint8)
        k = lib().orc_get_upper(self.h, chrom, start, end, out.ctypes.data, cap)
        if k > cap:   # outside get_data's defined range the slice can wrap (Python slice semantics)
            out = np.zeros(k, dtype=np.uint8)
            k = lib().orc_get_upper(self.h, chrom, start, end, out.ctypes.data, k)
        return bytes(out[:k])


def _ptr(a):
    return a.ctypes.data if a is not None else None


class OracleResult:
    def __init__(self, n_ties, first, all_ties, all_off):
        self.n_ties = n_ties          # int32 [n]: 0 no hit, >0 ties, <0 -error
        self.first = first            # ORC_HIT_DTYPE [n]
        self.all_ties = all_ties      # ORC_HIT_DTYPE [total] or None
        self.all_off = all_off        # int64 [n] or None

    def ties_of(self, i) -> List:
        if self.all_ties is None or self.n_ties[i] <= 0:
            return [self.first[i]] if self.n_ties[i] > 0 else []
        o = self.all_off[i]
        return list(self.all_ties[o:o + self.n_ties[i]])


def _pack_reads(reads):
    if isinstance(reads, tuple):
        return reads
    lens = np.array([len(r) for r in reads], dtype=np.int32)
    off = np.zeros(len(reads), dtype=np.int64)
    if len(reads):
        off[1:] = np.cumsum(lens[:-1])
    buf = np.frombuffer(b"".join(reads) + b"\0" * 8, dtype=np.uint8).copy()
    return buf, off, lens


def scan_fasta(p: OrcParams, fasta: OracleFasta, reads, chrom_idx, a_pos, b_aend, is_bs, primary_rev,
               use_fast=False, all_ties=False) -> OracleResult:
    buf, off, lens = _pack_reads(reads)
    n = len(lens)
    chrom_idx = np.ascontiguousarray(chrom_idx, dtype=np.int32)
    a_pos = np.ascontiguousarray(a_pos, dtype=np.int32)
    b_aend = np.ascontiguousarray(b_aend, dtype=np.int32)
    is_bs = np.ascontiguousarray(is_bs, dtype=np.uint8)
    primary_rev = np.ascontiguousarray(primary_rev, dtype=np.uint8)
    n_ties = np.zeros(n, dtype=np.int32)
    first = np.zeros(n, dtype=ORC_HIT_DTYPE)
    at = ao = None
    cap = 0
    if all_ties:
        cap = int(2 * (lens.astype(np.int64) + 2 + 2 * max(0, p.margin - p.asize)).sum()) + 16
        at = np.zeros(cap, dtype=ORC_HIT_DTYPE)
        ao = np.zeros(n, dtype=np.int64)
    lib().orc_scan_fasta(ctypes.byref(p), fasta.h, n, _ptr(buf), _ptr(off), _ptr(lens), _ptr(chrom_idx),
                         _ptr(a_pos), _ptr(b_aend), _ptr(is_bs), _ptr(primary_rev), int(use_fast),
                         _ptr(n_ties), _ptr(first), _ptr(at), cap, _ptr(ao), 1)
    return OracleResult(n_ties, first, at, ao)


def scan_windows(p: OrcParams, reads, wins: np.ndarray, win_off: np.ndarray, a_pos, b_aend, is_bs,
                 primary_rev, use_fast=False, all_ties=False) -> OracleResult:
    buf, off, lens = _pack_reads(reads)
    n = len(lens)
    a_pos = np.ascontiguousarray(a_pos, dtype=np.int32)
    b_aend = np.ascontiguousarray(b_aend, dtype=np.int32)
    is_bs = np.ascontiguousarray(is_bs, dtype=np.uint8)
    primary_rev = np.ascontiguousarray(primary_rev, dtype=np.uint8)
    wins = np.ascontiguousarray(wins, dtype=np.uint8)
    win_off = np.ascontiguousarray(win_off, dtype=np.int64)
    n_ties = np.zeros(n, dtype=np.int32)
    first = np.zeros(n, dtype=ORC_HIT_DTYPE)
    at = ao = None
    cap = 0
    if all_ties:
        cap = int(2 * (lens.astype(np.int64) + 2 + 2 * max(0, p.margin - p.asize)).sum()) + 16
        at = np.zeros(cap, dtype=ORC_HIT_DTYPE)
        ao = np.zeros(n, dtype=np.int64)
    lib().orc_scan_windows(ctypes.byref(p), n, _ptr(buf), _ptr(off), _ptr(lens), _ptr(wins), _ptr(win_off),
                           _ptr(a_pos), _ptr(b_aend), _ptr(is_bs), _ptr(primary_rev), int(use_fast),
                           _ptr(n_ties), _ptr(first), _ptr(at), cap, _ptr(ao))
    return OracleResult(n_ties, first, at, ao)


def scan_planes(p: OrcParams, units: np.ndarray, nplane: np.ndarray, chrom_start: np.ndarray,
                chrom_size: np.ndarray, pairs: np.ndarray, read_words: np.ndarray, read_nwords: np.ndarray,
                rw: int, nw: int, stride: int, n: int, n_threads: int = 16):
    """First tie of every pair of a batch in the device layouts of include/fc2_bp.h (packed rows +
    2-bit genome planes), encoded as the kernel's 8-byte fc2_result words (uint64 [n]); see
    orc_scan_planes.  Returns (words, number of pairs that could not be checked)."""
    L = lib()
    if not hasattr(L, "_planes_sig"):
        vp = ctypes.c_void_p
        L.orc_scan_planes.restype = ctypes.c_int64
        L.orc_scan_planes.argtypes = [ctypes.POINTER(OrcParams), vp, vp, vp, vp, ctypes.c_int, vp, vp, vp,
                                      ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_int64, vp,
                                      ctypes.c_int]
        L._planes_sig = True
    arrs = [np.ascontiguousarray(a) for a in (units, nplane, chrom_start, chrom_size, pairs, read_words, read_nwords)]
    assert arrs[0].dtype.itemsize * arrs[0].size >= 16 and arrs[4].nbytes >= 16 * n
    assert arrs[5].nbytes >= 8 * rw * stride and arrs[6].nbytes >= 8 * nw * stride
    out = np.zeros(n, np.uint64)
    skipped = L.orc_scan_planes(ctypes.byref(p), *[a.ctypes.data for a in arrs[:4]], len(chrom_size),
                                *[a.ctypes.data for a in arrs[4:]], rw, nw, stride, n, out.ctypes.data,
                                int(n_threads))
    return out, int(skipped)
