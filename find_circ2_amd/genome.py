"""Device-resident genome for the breakpoint search.

Replaces the reference's per-pair window fetch chain
``Track.get -> GenomeAccessor.get_data -> indexed_fasta.get_data``
(find_circ.py:310-312, 362-368, 189-215) with a genome packed once into HBM:

* ``units``   [2 * n_units] u64 -- bit-sliced 2-bit codes, 64 bases per unit
                                    (low plane word, high plane word)
* ``nplane``  [n_units]     u64 -- 1 where the uppercased base is 'N'
* ``ncoarse`` [...]         u32 -- 1 bit per 1024 bases that contain an N

hg19 (3.1 Gbp) takes 0.78 GB of code planes + 0.39 GB of N plane: a fraction
of one MI355X's 288 GB, so every rank keeps its own copy.

The host side keeps the mmap'd FASTA with the reference's index semantics
(``.byo_index`` compatible) for the rare pairs evaluated byte-exactly.
"""
from __future__ import annotations

import ctypes
from typing import List, Optional, Sequence

from ._lazy import LazyModule

np = LazyModule("numpy", globals(), "np")

from . import _native as N


def _torch():
    import torch
    return torch


def _require_gpu(device) -> None:
    torch = _torch()
    if not torch.cuda.is_available():
        raise RuntimeError("find_circ2_amd needs a HIP device (MI355X); no CPU fallback exists")


class Genome:
    """A genome resident in device memory (see module docstring)."""

    def __init__(self):
        self.device = None
        self.names: List[str] = []
        self.sizes: np.ndarray = np.zeros(0, np.int64)
        self.chrom_start: np.ndarray = np.zeros(0, np.uint64)
        self.n_units = 0
        self.units = self.nplane = self.ncoarse = None      # torch device tensors
        self.units_twin = None                              # units shifted by half a line (fc2_twin_launch)
        self.nsuper = None                                  # LDS-sized N map (fc2_nsuper_launch)
        self.nsuper_shift = self.nsuper_words = 0
        self.wt = None                                      # word-pair layout + shifted copy (fc2_wtab_launch)
        self.wt_bytes = self.wt_twin_off = 0
        self.d_chrom_start = self.d_chrom_size = None
        self.dummy = False
        self.fasta = None                                   # ctypes handle (host FASTA) or None
        self.n_exotic = 0
        self.regular: List[int] = []
        self._index = {}

    # ------------------------------------------------------------------ build
    @classmethod
    def from_fasta(cls, path: str, device="cuda", write_index: bool = False, n_threads: int = 0) -> "Genome":
        """Index (reference semantics, find_circ.py:110-155) + pack + upload a FASTA."""
        _require_gpu(device)
        torch = _torch()
        g = cls()
        g.device = torch.device(device)
        h = ctypes.c_void_p()
        N.check(N.lib().fc2_fasta_open(path.encode(), int(write_index), ctypes.byref(h)))
        g.fasta = h
        g._read_chroms()
        n_units = ctypes.c_uint64()
        n_cw = ctypes.c_uint64()
        cs = np.zeros(max(1, len(g.names)), np.uint64)
        N.check(N.lib().fc2_fasta_layout(h, ctypes.byref(n_units), ctypes.byref(n_cw), cs.ctypes.data))
        g.n_units = int(n_units.value)
        units = np.empty(2 * g.n_units, np.uint64)
        nplane = np.empty(g.n_units, np.uint64)
        ncoarse = np.zeros(max(1, int(n_cw.value)), np.uint32)
        n_exo = ctypes.c_uint64()
        N.check(N.lib().fc2_fasta_pack(h, units.ctypes.data, nplane.ctypes.data, ncoarse.ctypes.data,
                                       ctypes.byref(n_exo), int(n_threads)))
        g.n_exotic = int(n_exo.value)
        g._read_chroms()          # regularity is known after packing
        g.chrom_start = cs[:len(g.names)].copy()
        g._upload(units, nplane, ncoarse)
        return g

    @classmethod
    def synthetic(cls, names: Sequence[str], sizes: Sequence[int], seed: int = 1337, device="cuda",
                  n_fraction: float = 0.07) -> "Genome":
        """Seeded random genome with hg19-like N runs, generated on the device."""
        _require_gpu(device)
        torch = _torch()
        g = cls()
        g.device = torch.device(device)
        g.names = list(names)
        g._index = {n: i for i, n in enumerate(g.names)}
        g.sizes = np.asarray(sizes, np.int64)
        padded = (g.sizes + 63) // 64 * 64
        g.chrom_start = np.zeros(len(g.sizes), np.uint64)
        if len(g.sizes) > 1:
            g.chrom_start[1:] = np.cumsum(padded[:-1]).astype(np.uint64)
        g.n_units = int(max(1, padded.sum() // 64))
        g.regular = [1] * len(g.names)
        lo, hi = synthetic_n_intervals(g.sizes, g.chrom_start, seed, n_fraction)
        units = torch.empty(2 * g.n_units, dtype=torch.int64, device=g.device)
        nplane = torch.empty(g.n_units, dtype=torch.int64, device=g.device)
        ncoarse = torch.zeros(max(1, (((g.n_units + 15) >> 4) + 31) >> 5), dtype=torch.int32, device=g.device)
        d_lo = torch.from_numpy(lo).to(g.device)
        d_hi = torch.from_numpy(hi).to(g.device)
        stream = torch.cuda.current_stream(g.device).cuda_stream
        N.check(N.lib().fc2_synth_genome_launch(int(seed), units.data_ptr(), nplane.data_ptr(), ncoarse.data_ptr(),
                                                g.n_units, d_lo.data_ptr() if len(lo) else None,
                                                d_hi.data_ptr() if len(hi) else None, len(lo), stream))
        g.units, g.nplane, g.ncoarse = units, nplane, ncoarse
        g._upload_tables()
        torch.cuda.synchronize(g.device)
        return g

    @classmethod
    def dummy_genome(cls, device="cuda") -> "Genome":
        """GenomeAccessor dummy mode (find_circ.py:340-345): every window is all 'N'."""
        _require_gpu(device)
        torch = _torch()
        g = cls()
        g.device = torch.device(device)
        g.dummy = True
        return g

    def replicate(self, device) -> "Genome":
        """The same genome resident on another device (one copy per GPU): device
        tables copied device to device, the host FASTA handle shared (this object keeps owning it;
        the replica must not outlive it)."""
        torch = _torch()
        g = Genome()
        g.device = torch.device(device)
        for k in ("names", "sizes", "chrom_start", "n_units", "nsuper_shift", "nsuper_words", "wt_bytes",
                  "wt_twin_off", "dummy", "n_exotic", "regular", "_index"):
            setattr(g, k, getattr(self, k))
        for k in ("units", "nplane", "ncoarse", "units_twin", "nsuper", "wt", "d_chrom_start", "d_chrom_size"):
            t = getattr(self, k)
            setattr(g, k, None if t is None else t.to(g.device, copy=True))
        g.fasta = self.fasta
        g._owner = self                  # keeps the FASTA handle alive; close() leaves it to the owner
        torch.cuda.synchronize(g.device)
        return g

    def _read_chroms(self):
        L = N.lib()
        n = L.fc2_fasta_n_chrom(self.fasta)
        names, sizes, reg = [], [], []
        for i in range(n):
            nm = ctypes.c_char_p()
            sz = ctypes.c_int64()
            r = ctypes.c_int()
            N.check(L.fc2_fasta_chrom(self.fasta, i, ctypes.byref(nm), ctypes.byref(sz), None, None, None,
                                      ctypes.byref(r)))
            names.append(nm.value.decode("latin-1"))
            sizes.append(sz.value)
            reg.append(r.value)
        self.names, self.sizes, self.regular = names, np.asarray(sizes, np.int64), reg
        self._index = {nm: i for i, nm in enumerate(names)}

    def _upload(self, units, nplane, ncoarse):
        torch = _torch()
        self.units = torch.from_numpy(units.view(np.int64)).to(self.device)
        self.nplane = torch.from_numpy(nplane.view(np.int64)).to(self.device)
        self.ncoarse = torch.from_numpy(ncoarse.view(np.int32)).to(self.device)
        self._upload_tables()

    def _upload_tables(self):
        torch = _torch()
        cs = self.chrom_start.astype(np.int64) if len(self.chrom_start) else np.zeros(1, np.int64)
        sz = self.sizes.astype(np.int64) if len(self.sizes) else np.zeros(1, np.int64)
        self.d_chrom_start = torch.from_numpy(cs.copy()).to(self.device)
        self.d_chrom_size = torch.from_numpy(sz.copy()).to(self.device)
        if self.n_units:
            self.units_twin = torch.empty(2 * (self.n_units + 8), dtype=torch.int64, device=self.device)
            N.check(N.lib().fc2_twin_launch(self.units.data_ptr(), self.n_units, self.units_twin.data_ptr(),
                                            torch.cuda.current_stream(self.device).cuda_stream))
            sh, nw = ctypes.c_uint32(), ctypes.c_uint32()
            N.check(N.lib().fc2_nsuper_geometry(self.n_units, ctypes.byref(sh), ctypes.byref(nw)))
            self.nsuper_shift, self.nsuper_words = sh.value, nw.value
            self.nsuper = torch.empty((nw.value + 3) // 4 * 4, dtype=torch.int32, device=self.device)
            N.check(N.lib().fc2_nsuper_launch(self.ncoarse.data_ptr(), self.n_units, self.nsuper.data_ptr(),
                                              torch.cuda.current_stream(self.device).cuda_stream))
            nb, to = ctypes.c_uint64(), ctypes.c_uint64()
            if N.lib().fc2_wtab_geometry(self.n_units, ctypes.byref(nb), ctypes.byref(to)) == 0:
                self.wt_bytes, self.wt_twin_off = nb.value, to.value
                self.wt = torch.empty(nb.value // 4, dtype=torch.int32, device=self.device)
                N.check(N.lib().fc2_wtab_launch(self.units.data_ptr(), self.n_units, self.wt.data_ptr(),
                                                torch.cuda.current_stream(self.device).cuda_stream))

    # ------------------------------------------------------------------ access
    def view(self) -> N.GenomeView:
        if self.dummy:
            return N.GenomeView(None, None, None, None, None, 0, 0xFFFFFFFF, 1, None, None, 0, 0)
        return N.GenomeView(self.units.data_ptr(), self.nplane.data_ptr(), self.ncoarse.data_ptr(),
                            self.d_chrom_start.data_ptr(), self.d_chrom_size.data_ptr(), self.n_units,
                            len(self.names), 0, self.units_twin.data_ptr() if self.units_twin is not None else None,
                            self.nsuper.data_ptr() if self.nsuper is not None else None, self.nsuper_shift,
                            self.nsuper_words, self.wt.data_ptr() if self.wt is not None else None,
                            self.wt_bytes, self.wt_twin_off)

    def chrom_index(self, name: str) -> int:
        """Chromosome -> table index; KeyError like indexed_fasta.get_data (find_circ.py:193)."""
        if self.dummy:
            return 0
        return self._index[name]

    def chrom_index_or_missing(self, name: str) -> int:
        if self.dummy:
            return 0
        return self._index.get(name, 0xFFFFFFFF)

    def get_upper(self, chrom: int, start: int, end: int) -> bytes:
        """Host ``get_data(chrom, start, end, '+').upper()`` with the reference's semantics."""
        if self.fasta is None:
            if self.dummy:
                return b"N" * max(0, end - start)
            raise RuntimeError("synthetic genome has no host FASTA")
        cap = max(0, end - start) + 64
        buf = np.zeros(cap, np.uint8)
        ln = ctypes.c_int64()
        N.check(N.lib().fc2_fasta_get_upper(self.fasta, chrom, start, end, buf.ctypes.data, cap, ctypes.byref(ln)))
        if ln.value > cap:   # outside get_data's defined range the mmap slice can wrap
            buf = np.zeros(ln.value, np.uint8)
            N.check(N.lib().fc2_fasta_get_upper(self.fasta, chrom, start, end, buf.ctypes.data, ln.value,
                                                ctypes.byref(ln)))
        return bytes(buf[:ln.value])

    def host_planes(self):
        """Device planes copied back to host numpy (tests / oracle decoding)."""
        return (self.units.cpu().numpy().view(np.uint64), self.nplane.cpu().numpy().view(np.uint64))

    def close(self):
        if getattr(self, "_owner", None) is not None:      # a replica: the owner closes the FASTA
            self.fasta = None
            return
        if self.fasta is not None:
            N.lib().fc2_fasta_close(self.fasta)
            self.fasta = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def synthetic_n_intervals(sizes: np.ndarray, chrom_start: np.ndarray, seed: int, n_fraction: float = 0.07):
    """hg19-like 'N' runs (global half-open intervals, sorted, non-overlapping).

    Per chromosome: telomeric runs at both ends, one centromere-like run, a few
    random gaps, and the 64-alignment padding after each chromosome -- about
    ``n_fraction`` of all bases (hg19 is ~7 % N).
    """
    rng = np.random.default_rng(seed ^ 0x5EED)
    iv = []
    for size, cs in zip(sizes.tolist(), chrom_start.tolist()):
        cs = int(cs)
        if size >= 200_000:
            tel = 10_000
            iv.append((cs, cs + tel))
            iv.append((cs + size - tel, cs + size))
            cen = int(size * max(0.0, n_fraction - 2 * tel / size) * 0.7)
            if cen > 0:
                c0 = int(rng.integers(size // 3, size // 2))
                iv.append((cs + c0, cs + c0 + cen))
            gaps = int(size * max(0.0, n_fraction - 2 * tel / size) * 0.3)
            k = 4
            for _ in range(k):
                g0 = int(rng.integers(tel, size - tel))
                iv.append((cs + g0, cs + g0 + max(1, gaps // k)))
        elif size >= 5_000 and rng.random() < 0.5:
            g0 = int(rng.integers(0, size - 100))
            iv.append((cs + g0, cs + g0 + int(rng.integers(1, 100))))
        padded = (size + 63) // 64 * 64
        if padded > size:
            iv.append((cs + size, cs + padded))
    if not iv:
        return np.zeros(0, np.int64), np.zeros(0, np.int64)
    iv.sort()
    merged = [list(iv[0])]
    for a, b in iv[1:]:
        if a <= merged[-1][1]:
            merged[-1][1] = max(merged[-1][1], b)
        else:
            merged.append([a, b])
    arr = np.asarray(merged, np.int64)
    return arr[:, 0].copy(), arr[:, 1].copy()


def sq_table(sam_path: str):
    """Chromosome names and lengths from a SAM header's @SQ lines."""
    names, sizes = [], []
    with open(sam_path) as f:
        for line in f:
            if not line.startswith("@"):
                break
            if line.startswith("@SQ"):
                d = dict(kv.split(":", 1) for kv in line.rstrip("\n").split("\t")[1:] if ":" in kv)
                names.append(d["SN"])
                sizes.append(int(d["LN"]))
    return names, sizes
