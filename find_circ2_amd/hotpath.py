"""The hot path: ``JunctionSpan.find_breakpoints`` for batches of anchor pairs on MI355X.

Reference interface (find_circ.py 1.99, Python 2):

* ``Splice``                         find_circ.py:766-806
* ``JunctionSpan.__init__``          find_circ.py:821-844
* ``JunctionSpan.find_breakpoints``  find_circ.py:854-974 (called from
  ``record_hits`` at :1303 / :1355, one pair at a time)

Here the same function is evaluated for a whole ``PairBatch`` by one HIP
launch (``fc2_bp_scan_launch``; rare pairs with exotic bytes / irregular FASTA
layout / very long reads by ``fc2_bp_scan_bytes_launch``), and the per-pair
results decode to exactly the ``Splice`` lists the reference returns.
``JunctionSpan.find_breakpoints()`` is kept as a drop-in (one-pair batch) so
code written against the reference keeps working; real callers batch.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass, field
from typing import Iterable, List, Optional, Sequence, Tuple

from ._lazy import LazyModule

np = LazyModule("numpy", globals(), "np")

from . import _native as N
from .genome import Genome, _require_gpu, _torch

_CODE = "ACGTN"
_COMP = {"A": "T", "C": "G", "G": "C", "T": "A", "N": "N"}


def rev_comp4(s: str) -> str:
    return "".join(_COMP[c] for c in reversed(s))


# ---------------------------------------------------------------------------
# options (find_circ.py:393-404)
# ---------------------------------------------------------------------------
@dataclass
class Options:
    asize: int = 15            # -a/--anchor
    margin: int = 2            # -m/--margin
    maxdist: int = 2           # -d/--max-mismatch
    noncanonical: bool = False # --non-canonical
    strandpref: bool = False   # --strand-pref
    allhits: bool = False      # --all-hits

    def params(self) -> N.Params:
        return N.Params(int(self.asize), int(self.margin), int(self.maxdist), int(bool(self.noncanonical)),
                        int(bool(self.strandpref)), int(bool(self.allhits)), 0)

    @property
    def eff_a(self) -> int:   # find_circ.py:882
        return self.asize - self.margin


@dataclass
class SynthConfig:
    """Synthetic anchor-pair workload."""
    seed: int = 1337
    len_min: int = 100
    len_max: int = 100
    p_planted: float = 0.5
    p_minus_site: float = 0.2
    p_backsplice: float = 1.0
    mut_rate: float = 0.005
    n_rate: float = 0.0005
    p_clip: float = 0.2
    span_min: int = 150
    span_max: int = 5000
    locus_ordered: bool = False
    p_three_seg: float = 0.0  # slots whose two pairs come from one three-segment read (config 5: 0.1)
    first: int = 0          # generate pairs [first, first + n) of the seeded stream

    def cfg(self) -> N.SynthCfg:
        return N.SynthCfg(int(self.seed), int(self.len_min), int(self.len_max), float(self.p_planted),
                          float(self.p_minus_site), float(self.p_backsplice), float(self.mut_rate),
                          float(self.n_rate), float(self.p_clip), int(self.span_min), int(self.span_max),
                          int(bool(self.locus_ordered)), float(self.p_three_seg), int(self.first))


# ---------------------------------------------------------------------------
# batches
# ---------------------------------------------------------------------------
def sparse_nrows(host_pairs: np.ndarray, nwords: np.ndarray, nw: int, stride: int):
    """The read N rows of the pairs that carry them (FC2_PAIR_READ_N): (pair index [k] int64,
    rows [nw, k] int64).  Every other pair's N row is zero, and the scan reads a pair's N row only
    when its READ_N flag is set, so this is all the N information a batch has to move."""
    idx = np.nonzero((host_pairs["flags"] & N.PAIR_READ_N) != 0)[0].astype(np.int64)
    rows = nwords.view(np.int64).reshape(nw, stride)[:, idx]
    return idx, np.ascontiguousarray(rows)


def scatter_nrows(dst, idx, rows, nw: int, stride: int) -> None:
    """Device side of sparse_nrows: dst (torch int64 [nw*stride]) row j, column idx[t] = rows[j, t]."""
    if idx.numel():
        dst.view(nw, stride)[:, idx] = rows


def upload_nrows(host_pairs: np.ndarray, nwords: np.ndarray, nw: int, stride: int, dev):
    """Device N rows of a packed batch: zeros plus the flagged pairs' rows scattered in.  At 100 bp
    the dense rows are 16 of the 56 B a pair moves over PCIe; the sparse form moves 8 + 8*nw B per
    pair with an 'N' (a few percent of reads) instead."""
    torch = _torch()
    out = torch.zeros(nw * stride, dtype=torch.int64, device=dev)
    idx, rows = sparse_nrows(host_pairs, nwords, nw, stride)
    scatter_nrows(out, torch.from_numpy(idx).to(dev), torch.from_numpy(rows).to(dev), nw, stride)
    return out


def narrow_tail(words: np.ndarray, rw: int, stride: int) -> bool:
    """True when the last read row holds only 32-bit values (at 100 bp the rows carry 2l = 148
    bits: row 2 uses 20), so it can cross PCIe as uint32 and be widened on the device."""
    return rw > 1 and not np.any(words.view(np.uint64).reshape(rw, stride)[rw - 1] >> np.uint64(32))


def widen_tail(dst, tail32) -> None:
    """Device side of narrow_tail: dst (torch int64 [m]) = zero-extended tail32 (torch int32 [m])."""
    dst.copy_(tail32.to(dst.dtype) & 0xFFFFFFFF)


def upload_read_rows(words: np.ndarray, rw: int, stride: int, dev):
    """Device read rows of a packed batch: rows 0..rw-2 as they are, the last row as uint32 when
    narrow_tail allows (24 -> 20 B per pair at 100 bp), widened on the device."""
    torch = _torch()
    w = words.view(np.int64).reshape(rw, stride)
    if not narrow_tail(words, rw, stride):
        return torch.from_numpy(w.ravel()).to(dev)
    out = torch.empty(rw * stride, dtype=torch.int64, device=dev)
    out[:(rw - 1) * stride].copy_(torch.from_numpy(w[:rw - 1].ravel()))
    tail = np.ascontiguousarray(w[rw - 1]).view(np.int32)[0::2]          # low halves (little-endian)
    widen_tail(out[(rw - 1) * stride:], torch.from_numpy(np.ascontiguousarray(tail)).to(dev))
    return out


class PairBatch:
    """A batch of anchor pairs resident in device memory (layout: include/fc2_bp.h)."""

    def __init__(self):
        self.n = 0
        self.stride = 0
        self.rw = self.nw = self.tw = 1
        self.max_l = 0
        self.device = None
        self.pairs = None          # torch uint8 [n*16]
        self.read_words = None     # torch int64 [rw*stride]
        self.read_nwords = None    # torch int64 [nw*stride]
        self.host_pairs: Optional[np.ndarray] = None   # PAIR_DTYPE [n]
        self.truth = None          # synthetic only: torch int32 [2n]
        self.m_bytepath = 0
        self.bp_index = self.bp_pairs = self.bp_arena = self.bp_off = None
        self.options: Optional[Options] = None
        self.perm: Optional[np.ndarray] = None   # packed slot k holds input pair perm[k] (locus order)
        self.layout = 0            # FC2_BATCH_* hints for the scan
        self.slot = None           # reorder() output: torch int32 [n], device twin of perm
        self.reorder_info = None
        self.workspace = None
        self.win_words = self.win_nwords = None   # window-carrying form (fc2_batch_view.win_words)
        self.pw = 0

    # -------------------------------------------------------------- from reads
    @classmethod
    def pack(cls, options: Options, genome: Genome, reads, a_pos, b_aend, chrom, flags,
             device=None, n_threads: int = 0, locus_order: bool = False) -> "PairBatch":
        """Pack anchor pairs (``read_part`` bytes + JunctionSpan fields) and upload them.

        ``reads``: list of ``bytes`` (``JunctionSpan.read_part``, find_circ.py:844) or a
        ``(buffer uint8, offsets uint64, lengths)`` triple.  ``flags``: PAIR_* bits
        (BACKSPLICE, PRIMARY_REV, SKIP).  ``locus_order``: lay the batch out in genome
        order of the A window (the windows of a wave then share L2 lines); results are
        returned in input order all the same.
        """
        torch = _torch()
        dev = torch.device(device) if device is not None else genome.device
        p = options.params()
        if isinstance(reads, tuple):
            buf, off, lens = reads
            buf = np.ascontiguousarray(buf, np.uint8)
            off = np.ascontiguousarray(off, np.uint64)
            lens = np.ascontiguousarray(lens, np.int64)
        else:
            reads = [r.encode("latin-1") if isinstance(r, str) else r for r in reads]
            lens = np.fromiter((len(r) for r in reads), np.int64, len(reads))
            off = np.zeros(len(reads), np.uint64)
            if len(reads):
                off[1:] = np.cumsum(lens[:-1]).astype(np.uint64)
            buf = np.frombuffer(b"".join(reads) + b"\0" * 16, np.uint8)
        n = len(lens)
        if n and lens.max() > N.MAX_READ_LEN:
            raise ValueError("read_part longer than %d bases (fc2_result.best_x is 16-bit)" % N.MAX_READ_LEN)
        hp = np.zeros(n, N.PAIR_DTYPE)
        hp["a_pos"] = np.asarray(a_pos, np.int64)
        hp["b_aend"] = np.asarray(b_aend, np.int64)
        hp["chrom"] = np.asarray(chrom, np.int64).astype(np.uint32)
        hp["read_len"] = lens
        hp["flags"] = np.asarray(flags, np.uint8)
        perm = None
        if locus_order and n > 1 and not genome.dummy and len(genome.chrom_start):
            cs = genome.chrom_start.astype(np.int64)
            c = np.minimum(hp["chrom"].astype(np.int64), len(cs) - 1)
            perm = np.argsort(cs[c] + hp["a_pos"].astype(np.int64), kind="stable")
            hp = hp[perm]
            off = off[perm]
            lens = lens[perm]
        max_len = int(lens.max()) if n else 0
        rw, nw, tw = ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_uint32()
        N.check(N.lib().fc2_batch_geometry(ctypes.byref(p), max_len, ctypes.byref(rw), ctypes.byref(nw),
                                           ctypes.byref(tw)))
        b = cls()
        b.options = options
        b.n, b.stride = n, max(n, 1)
        b.rw, b.nw, b.tw = rw.value, nw.value, tw.value
        words = np.zeros(b.rw * b.stride, np.uint64)
        nwords = np.zeros(b.nw * b.stride, np.uint64)
        nbp = ctypes.c_uint64()
        N.check(N.lib().fc2_pack_pairs(ctypes.byref(p), genome.fasta if not genome.dummy else None, n,
                                       buf.ctypes.data, off.ctypes.data, hp.ctypes.data, words.ctypes.data, b.rw,
                                       nwords.ctypes.data, b.nw, b.stride, ctypes.byref(nbp), int(n_threads)))
        fast = (hp["flags"] & (N.PAIR_BYTEPATH | N.PAIR_SKIP)) == 0
        ls = hp["read_len"].astype(np.int64) - 2 * options.eff_a
        b.max_l = int(max(0, ls[fast].max())) if fast.any() else 0
        b.host_pairs = hp
        b.perm = perm
        b.layout = N.BATCH_LOCUS_ORDERED if perm is not None else 0
        b.device = dev
        b.pairs = torch.from_numpy(hp.view(np.uint8)).to(dev)
        b.read_words = upload_read_rows(words, b.rw, b.stride, dev)
        b.read_nwords = upload_nrows(hp, nwords, b.nw, b.stride, dev)
        b.m_bytepath = int(nbp.value)
        if b.m_bytepath and genome.fasta is None and not genome.dummy:
            raise RuntimeError("%d pairs need byte-exact windows, which come from a FASTA-backed genome"
                               % b.m_bytepath)
        if b.m_bytepath:
            b._pack_bytepath(p, genome, buf, off)
        return b

    def _pack_bytepath(self, p, genome, buf, off):
        torch = _torch()
        m, nbytes = ctypes.c_uint64(), ctypes.c_uint64()
        hp = self.host_pairs
        N.check(N.lib().fc2_bytepath_size(ctypes.byref(p), self.n, hp.ctypes.data, ctypes.byref(m),
                                          ctypes.byref(nbytes)))
        m = int(m.value)
        idx = np.zeros(m, np.uint64)
        bpairs = np.zeros(m, N.PAIR_DTYPE)
        offs = np.zeros(m, np.uint64)
        arena = np.zeros(max(16, int(nbytes.value)), np.uint8)
        N.check(N.lib().fc2_bytepath_fill(ctypes.byref(p), genome.fasta if not genome.dummy else None, self.n,
                                          buf.ctypes.data, off.ctypes.data, hp.ctypes.data, idx.ctypes.data,
                                          bpairs.ctypes.data, offs.ctypes.data, arena.ctypes.data))
        dev = self.device
        self.bp_index = torch.from_numpy(idx.view(np.int64)).to(dev)
        self.bp_pairs = torch.from_numpy(bpairs.view(np.uint8)).to(dev)
        self.bp_off = torch.from_numpy(offs.view(np.int64)).to(dev)
        self.bp_arena = torch.from_numpy(arena).to(dev)

    # -------------------------------------------------------------- synthetic
    @classmethod
    def synthetic(cls, options: Options, genome: Genome, n: int, cfg: SynthConfig = None,
                  with_truth: bool = False) -> "PairBatch":
        """Generate ``n`` pairs on the device from ``genome`` (see fc2_synth_pairs_launch)."""
        torch = _torch()
        cfg = cfg or SynthConfig()
        p = options.params()
        rw, nw, tw = ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_uint32()
        N.check(N.lib().fc2_batch_geometry(ctypes.byref(p), int(cfg.len_max), ctypes.byref(rw), ctypes.byref(nw),
                                           ctypes.byref(tw)))
        if cfg.len_max - 2 * options.eff_a > N.lib().fc2_max_fast_l():
            raise ValueError("synthetic reads longer than the register kernel supports")
        b = cls()
        b.options = options
        b.n, b.stride = n, max(n, 1)
        b.rw, b.nw, b.tw = rw.value, nw.value, tw.value
        b.max_l = max(0, cfg.len_max - 2 * options.eff_a)
        b.layout = N.BATCH_LOCUS_ORDERED if cfg.locus_ordered else 0
        dev = genome.device
        b.device = dev
        b.pairs = torch.empty(16 * b.stride, dtype=torch.uint8, device=dev)
        b.read_words = torch.empty(b.rw * b.stride, dtype=torch.int64, device=dev)
        b.read_nwords = torch.empty(b.nw * b.stride, dtype=torch.int64, device=dev)
        if with_truth:
            b.truth = torch.empty(2 * b.stride, dtype=torch.int32, device=dev)
        cum = np.zeros(len(genome.names) + 1, np.int64)
        cum[1:] = np.cumsum(genome.sizes)
        d_cum = torch.from_numpy(cum).to(dev)
        gv = genome.view()
        stream = torch.cuda.current_stream(dev).cuda_stream
        N.check(N.lib().fc2_synth_pairs_launch(ctypes.byref(p), ctypes.byref(cfg.cfg()), ctypes.byref(gv),
                                               d_cum.data_ptr(), n, b.pairs.data_ptr(), b.read_words.data_ptr(),
                                               b.rw, b.read_nwords.data_ptr(), b.nw, b.stride,
                                               b.truth.data_ptr() if with_truth else None, stream))
        torch.cuda.synchronize(dev)
        b.host_pairs = None   # fetched lazily
        return b

    def sub(self, lo: int, hi: int) -> "PairBatch":
        """Pairs [lo, hi) of this batch as a batch of their own, sharing its device memory (no copy):
        the SoA rows keep the parent's stride, so the view only moves each base pointer by lo.  This
        is how a rank scans its contiguous share of a pair stream (shard.my_batches)."""
        if not 0 <= lo <= hi <= self.n:
            raise ValueError("sub-batch [%d, %d) outside [0, %d)" % (lo, hi, self.n))
        if self.m_bytepath or self.perm is not None or self.slot is not None or self.win_words is not None:
            raise ValueError("sub-batches of byte-path, reordered or window-carrying batches are not supported")
        s = PairBatch()
        s.options, s.device = self.options, self.device
        s.n, s.stride = hi - lo, self.stride
        s.rw, s.nw, s.tw, s.max_l, s.layout = self.rw, self.nw, self.tw, self.max_l, self.layout
        s.pairs = self.pairs[16 * lo:16 * hi]
        s.read_words = self.read_words[lo:]
        s.read_nwords = self.read_nwords[lo:]
        if self.host_pairs is not None:
            s.host_pairs = self.host_pairs[lo:hi]
        return s

    def fetch_host_pairs(self) -> np.ndarray:
        if self.host_pairs is None:
            self.host_pairs = self.pairs[:16 * self.n].cpu().numpy().view(N.PAIR_DTYPE).copy()
        return self.host_pairs

    def fetch_perm(self) -> Optional[np.ndarray]:
        """perm (packed slot k holds input pair perm[k]) or None for input order."""
        if self.perm is None and self.slot is not None:
            self.perm = self.slot[:self.n].cpu().numpy().astype(np.int64)
        return self.perm

    def view(self) -> N.BatchView:
        carried = self.win_words is not None
        return N.BatchView(self.pairs.data_ptr(), self.read_words.data_ptr(), self.read_nwords.data_ptr(),
                           self.n, self.stride, self.rw, self.nw, self.max_l, self.layout,
                           self.win_words.data_ptr() if carried else None,
                           self.win_nwords.data_ptr() if carried else None,
                           2 * self.pw if carried else 0, self.pw if carried else 0)

    # -------------------------------------------------------------- window-carrying form
    def _alloc_windows(self):
        torch = _torch()
        p = self.options.params()
        pw, ww, wnw = ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_uint32()
        N.check(N.lib().fc2_window_geometry(ctypes.byref(p), self.max_l + 2 * self.options.eff_a, ctypes.byref(pw),
                                            ctypes.byref(ww), ctypes.byref(wnw)))
        self.pw = pw.value
        return torch, p

    def carry_windows_from_fasta(self, genome: Genome, n_threads: int = 0) -> "PairBatch":
        """North_star's form: Af / Bf of every pair read on the host from the mmap'd FASTA
        (fc2_pack_windows, get_data semantics find_circ.py:189-215) and uploaded with the
        batch; the scan then gathers nothing from the genome (only chromosome sizes)."""
        torch, p = self._alloc_windows()
        if genome.fasta is None:
            raise RuntimeError("host window packing needs a FASTA-backed genome")
        hp = self.fetch_host_pairs().copy()
        ww = np.zeros(2 * self.pw * self.stride, np.uint64)
        wn = np.zeros(self.pw * self.stride, np.uint64)
        N.check(N.lib().fc2_pack_windows(ctypes.byref(p), genome.fasta, self.n, hp.ctypes.data, ww.ctypes.data,
                                         wn.ctypes.data, self.pw, self.stride, int(n_threads)))
        self.host_pairs = hp
        self.pairs = torch.from_numpy(hp.view(np.uint8).copy()).to(self.device)
        self.win_words = torch.from_numpy(ww.view(np.int64)).to(self.device)
        self.win_nwords = torch.from_numpy(wn.view(np.int64)).to(self.device)
        return self

    def carry_windows_from_device(self, genome: Genome) -> "PairBatch":
        """The same rows gathered on the device from the resident genome
        (fc2_gather_windows_launch; synthetic workloads, which have no FASTA)."""
        torch, p = self._alloc_windows()
        self.win_words = torch.empty(2 * self.pw * self.stride, dtype=torch.int64, device=self.device)
        self.win_nwords = torch.empty(self.pw * self.stride, dtype=torch.int64, device=self.device)
        gv, bv = genome.view(), self.view()
        stream = torch.cuda.current_stream(self.device).cuda_stream
        N.check(N.lib().fc2_gather_windows_launch(ctypes.byref(p), ctypes.byref(gv), ctypes.byref(bv),
                                                  self.pairs.data_ptr(), self.win_words.data_ptr(),
                                                  self.win_nwords.data_ptr(), self.pw, stream))
        torch.cuda.synchronize(self.device)
        self.host_pairs = None
        return self

    def bytes_view(self) -> N.BytesView:
        return N.BytesView(self.bp_index.data_ptr(), self.bp_pairs.data_ptr(), self.bp_arena.data_ptr(),
                           self.bp_off.data_ptr(), self.m_bytepath)


# ---------------------------------------------------------------------------
# scan
# ---------------------------------------------------------------------------
class ScanOutput:
    def __init__(self, results, tiemask, tw, stride):
        self.results = results      # torch int64 [stride] (fc2_result)
        self.tiemask = tiemask      # torch int64 [tw*stride] or None
        self.tw = tw
        self.stride = stride

    def host(self, n: int) -> np.ndarray:
        return self.results[:n].cpu().numpy().view(N.RESULT_DTYPE).copy()


class CompactResults:
    """A compact transfer form of a run of results (include/fc2_bp.h "compact results"): device
    words [n] (int32 for width 4, int16 for width 2), escape slots [cap] (``N.ESCAPE_DTYPE`` as
    16 bytes each) and the escape count.  The count lives in the low 4 bytes of one more 16-byte slot
    after the escape slots, so ``esc_block`` (slots + count) crosses to the host in ONE copy: a
    separate 4-byte D2H copy per batch made the runtime serialise the copies with the next scan on
    some stream placements (profiles/r03/strong_small_copies.txt)."""

    def __init__(self, n: int, device, cap: int = 0, width: int = 4):
        torch = _torch()
        if width not in (2, 4):
            raise ValueError("width is 2 or 4")
        self.n, self.width = n, width
        self.cap = cap or max(1024, n // 256)
        self.words = torch.empty(max(n, 1), dtype=torch.int16 if width == 2 else torch.int32, device=device)
        self.esc_block = torch.zeros(2 * (self.cap + 1), dtype=torch.int64, device=device)
        self.esc = self.esc_block[:2 * self.cap]
        self.count = self.esc_block[2 * self.cap:2 * self.cap + 1].view(torch.int32)[:1]


def compact(options: Options, results, n: int, into: CompactResults = None, stream=None,
            width: int = 4) -> CompactResults:
    """Pack the first ``n`` 8-byte results of the device tensor ``results`` into a compact form
    (``fc2_result_compact_launch``, asynchronous on ``stream``); canonical mode only.  ``into``
    decides the width when given."""
    torch = _torch()
    c = into if into is not None else CompactResults(n, results.device, width=width)
    if c.n < n:
        raise ValueError("compact buffers hold %d results, %d given" % (c.n, n))
    s = stream if stream is not None else torch.cuda.current_stream(results.device).cuda_stream
    p = options.params()
    N.check(N.lib().fc2_result_compact_launch(ctypes.byref(p), results.data_ptr(), n, c.width, c.words.data_ptr(),
                                              c.esc.data_ptr(), c.cap, c.count.data_ptr(), s))
    return c


def host_device_pointer(host_ptr: int) -> int:
    """The device address of page-locked host memory (fc2_host_register'ed or pinned)."""
    d = ctypes.c_void_p()
    N.check(N.lib().fc2_host_device_pointer(host_ptr, ctypes.byref(d)))
    return d.value


def scan_compact(options: Options, genome: Genome, batch: "PairBatch", words: int, width: int, esc: int, cap: int,
                 esc_count: int, count_out: int = None, stream=None) -> None:
    """``find_breakpoints`` for every pair of ``batch`` with the results written by the scan itself in
    a compact form (``fc2_bp_scan_compact_launch``): ``words`` / ``esc`` are device addresses (device
    memory, or page-locked host memory through ``host_device_pointer``: the words then cross PCIe as
    the scan writes them), ``esc_count`` a device int32 that is zero before the launch and is moved to
    ``count_out`` (and zeroed) after it when that is given.  Canonical mode without --all-hits; a
    batch with byte-path pairs is refused (their results are 8-byte words from the byte kernel)."""
    torch = _torch()
    if batch.m_bytepath:
        raise ValueError("scan_compact: the batch has %d byte-path pairs" % batch.m_bytepath)
    s = stream if stream is not None else torch.cuda.current_stream(batch.device).cuda_stream
    p = options.params()
    gv = genome.view()
    bv = batch.view()
    co = N.CompactOut(width, cap, words, esc, esc_count, count_out)
    N.check(N.lib().fc2_bp_scan_compact_launch(ctypes.byref(p), ctypes.byref(gv), ctypes.byref(bv), ctypes.byref(co),
                                               s))


def expand(options: Options, words: np.ndarray, esc: np.ndarray, out: np.ndarray = None,
           n_threads: int = 0) -> np.ndarray:
    """Host: the 8-byte result words (int64) back from compact words (a 4-byte dtype: width 4, a
    2-byte dtype: width 2) and the escapes (``N.ESCAPE_DTYPE``), ``fc2_result_expand``."""
    words = np.ascontiguousarray(words)
    width = words.dtype.itemsize
    if width not in (2, 4):
        raise ValueError("compact words are 2 or 4 bytes, not %d" % width)
    esc = np.ascontiguousarray(esc, dtype=N.ESCAPE_DTYPE) if len(esc) else np.zeros(0, N.ESCAPE_DTYPE)
    n = len(words)
    if out is None:
        out = np.empty(n, np.int64)
    p = options.params()
    N.check(N.lib().fc2_result_expand(ctypes.byref(p), words.ctypes.data, width, n,
                                      esc.ctypes.data if len(esc) else None, len(esc), out.ctypes.data, int(n_threads)))
    return out


def scan(options: Options, genome: Genome, batch: PairBatch, out: ScanOutput = None, stream=None) -> ScanOutput:
    """Run find_breakpoints for every pair of ``batch`` (asynchronous on ``stream``)."""
    torch = _torch()
    dev = batch.device
    p = options.params()
    if out is None:
        res = torch.empty(batch.stride, dtype=torch.int64, device=dev)
        tm = torch.zeros(batch.tw * batch.stride, dtype=torch.int64, device=dev) if options.allhits else None
        out = ScanOutput(res, tm, batch.tw, batch.stride)
    s = stream if stream is not None else torch.cuda.current_stream(dev).cuda_stream
    gv = genome.view()
    bv = batch.view()
    tptr = out.tiemask.data_ptr() if out.tiemask is not None else None
    N.check(N.lib().fc2_bp_scan_launch(ctypes.byref(p), ctypes.byref(gv), ctypes.byref(bv), out.results.data_ptr(),
                                       tptr, out.tw, s))
    if batch.m_bytepath:
        v = batch.bytes_view()
        N.check(N.lib().fc2_bp_scan_bytes_launch(ctypes.byref(p), ctypes.byref(v), out.results.data_ptr(), tptr,
                                                 out.tw, batch.stride, s))
    return out


def reorder(genome: Genome, batch: PairBatch, into: PairBatch = None) -> PairBatch:
    """Device locality reorder (``fc2_reorder_launch``) of a batch in input order.

    Returns a batch holding the same pairs stably sorted by genome bucket of the
    A window, flagged locus-ordered, whose ``slot`` (device) / ``fetch_perm()``
    (host) map each position back to the input pair; ``decode_splices`` of a scan
    over it returns results in input order.  ``into``: a previous result for a
    batch of the same shape whose buffers are reused.  Runs on torch's current
    stream.
    """
    torch = _torch()
    if batch.slot is not None or batch.perm is not None:
        raise ValueError("batch is already locus-ordered")
    dev = batch.device
    gv = genome.view()
    r = into
    info = N.ReorderInfo()
    N.check(N.lib().fc2_reorder_plan(ctypes.byref(gv), batch.n, ctypes.byref(info)))
    if r is None or r.n != batch.n or r.rw != batch.rw or r.nw != batch.nw or \
            r.reorder_info.chunk != info.chunk or r.workspace.numel() < info.workspace_bytes:
        r = PairBatch()
        r.options = batch.options
        r.n, r.stride, r.rw, r.nw, r.tw, r.max_l = batch.n, batch.stride, batch.rw, batch.nw, batch.tw, batch.max_l
        r.device = dev
        r.pairs = torch.empty_like(batch.pairs)
        r.read_words = torch.empty_like(batch.read_words)
        r.read_nwords = torch.empty_like(batch.read_nwords)
        r.slot = torch.empty(max(batch.n, 1), dtype=torch.int32, device=dev)
        r.workspace = torch.empty(max(1, int(info.workspace_bytes)), dtype=torch.uint8, device=dev)
        r.reorder_info = info
        r.layout = N.BATCH_LOCUS_ORDERED
    r.host_pairs = None
    r.perm = None
    stream = torch.cuda.current_stream(dev).cuda_stream
    N.check(N.lib().fc2_reorder_launch(ctypes.byref(r.reorder_info), ctypes.byref(gv), ctypes.byref(batch.view()),
                                       r.pairs.data_ptr(), r.read_words.data_ptr(), r.read_nwords.data_ptr(),
                                       r.slot.data_ptr(), r.workspace.data_ptr(), stream))
    r.m_bytepath = batch.m_bytepath
    if batch.m_bytepath:             # byte-path results go to the pair's reordered position
        inv = torch.empty(batch.n, dtype=torch.int64, device=dev)
        inv[r.slot[:batch.n].long()] = torch.arange(batch.n, dtype=torch.int64, device=dev)
        r.bp_index = inv[batch.bp_index]
        r.bp_pairs, r.bp_arena, r.bp_off = batch.bp_pairs, batch.bp_arena, batch.bp_off
    return r


# ---------------------------------------------------------------------------
# decoding to the reference's Splice objects
# ---------------------------------------------------------------------------
class Splice:
    """Mirror of ``Splice`` (find_circ.py:766-806)."""

    __slots__ = ("junc_span", "chrom", "start", "end", "strand", "dist", "ov", "gtag", "n_hits", "_score")

    def __init__(self, junc_span, chrom, start, end, strand, dist, ov, gtag):
        self.junc_span = junc_span
        self.chrom = chrom
        self.start = start
        self.end = end
        self.strand = strand
        self.dist = dist
        self.ov = ov
        self.gtag = gtag
        self.n_hits = 1
        self._score = None

    @property
    def is_canonical(self):          # find_circ.py:778-780
        return self.gtag == 'GTAG'

    @property
    def is_backsplice(self):         # find_circ.py:782-785
        return self.junc_span.is_backsplice

    @property
    def score(self):                 # find_circ.py:791-799 (value computed with the options of the scan)
        return self._score

    @property
    def coord(self):                 # find_circ.py:801-806
        if self.start < self.end:
            return (self.chrom, self.start, self.end, self.strand)
        return (self.chrom, self.end, self.start, self.strand)

    def __repr__(self):
        return "Splice(%s:%d-%d:%s edits=%s ov=%d gtag=%s n_hits=%d)" % (
            self.chrom, self.start, self.end, self.strand, self.dist, self.ov, self.gtag, self.n_hits)


# What find_breakpoints raises for windows outside the range where indexed_fasta.get_data is defined
# (find_circ.py:194-211), when the spliced string and the internal read part differ in length: under
# the reference's Python 2 / numpy 1.x, ``fromstring(a) != fromstring(b)`` of unequal lengths returns
# the scalar True (a DeprecationWarning) and ``.sum()`` then fails (find_circ.py:861-863).  With -d 0
# (simple_match, :865-871) nothing is raised.  The numpy version is not pinned by the reference, so
# this parity is unpinned; the exception type and message follow numpy <= 1.16 (the last Python-2 one).
WINDOW_SHAPE_MESSAGE = "'bool' object has no attribute 'sum'"


class BreakpointError(AttributeError):
    """The reference's AttributeError for windows of unexpected length (see WINDOW_SHAPE_MESSAGE)."""


def first_tie_arrays(options: Options, host_pairs: np.ndarray, res: np.ndarray):
    """Vectorised decode of ties[0] for every pair -> dict of numpy arrays.

    start/end follow find_circ.py:929-945; ``gtag`` is the Splice's signal
    (rev_comp for '-' hits, find_circ.py:949/954).
    """
    e = options.eff_a
    L = host_pairs["read_len"].astype(np.int64)
    l = L - 2 * e
    x = res["best_x"].astype(np.int64)
    s0 = host_pairs["b_aend"].astype(np.int64) - e - l + x
    e0 = host_pairs["a_pos"].astype(np.int64) + e + x + 1
    start = np.minimum(s0, e0)
    end = np.maximum(s0, e0)
    bs = (host_pairs["flags"] & N.PAIR_BACKSPLICE) != 0
    end = np.where(bs, end - 1, end)
    start = np.where(bs, start, start - 1)
    info = res["info"].astype(np.int64)
    return dict(hit=x >= 0, x=x, start=start, end=end, minus=(info & N.RES_MINUS) != 0,
                dist=res["dist"].astype(np.int64), ov=res["ov"].astype(np.int64),
                n_ties=res["n_ties"].astype(np.int64), gtag12=(info & N.RES_GTAG_MASK) >> N.RES_GTAG_SHIFT,
                err_key=(info & N.RES_ERR_KEY) != 0, err_win=(info & N.RES_ERR_WIN) != 0,
                done=(info & N.RES_DONE) != 0)


def gtag_str(gtag12: int) -> str:
    return "".join(_CODE[(gtag12 >> (3 * k)) & 7] for k in range(4))


def raise_reference_errors(options: Options, host_pairs: np.ndarray, res: np.ndarray, evaluated=None):
    """Re-raise what the reference would raise for the first failing evaluated pair."""
    info = res["info"]
    bad = (info & (N.RES_ERR_KEY | N.RES_ERR_WIN)) != 0
    if evaluated is not None:
        bad &= evaluated
    if not bad.any():
        return
    i = int(np.nonzero(bad)[0][0])
    if info[i] & N.RES_ERR_KEY:
        raise KeyError("pair %d: splice signal with a byte outside ACGTN (reference KeyError in fast_4mer_RC, "
                       "find_circ.py:927)" % i)
    raise BreakpointError(WINDOW_SHAPE_MESSAGE)


def decode_splices(options: Options, genome: Genome, batch: PairBatch, out: ScanOutput,
                   spans: Sequence = None, raise_errors: bool = True) -> List[List[Splice]]:
    """Per pair, the list ``find_breakpoints`` returns (ties, find_circ.py:961-974).

    With ``raise_errors=False`` a pair the reference would fail on gets the
    exception instance instead of a list, so a caller that evaluated pairs
    speculatively can raise it exactly where the reference calls the method.
    """
    hp = batch.fetch_host_pairs()
    res = out.host(batch.n)
    slot = np.arange(batch.n)
    perm = batch.fetch_perm()
    if perm is not None:                 # locus-ordered layout: back to input order
        slot = np.empty_like(perm)
        slot[perm] = np.arange(batch.n)
        hp, res = hp[slot], res[slot]
    evaluated = (hp["flags"] & N.PAIR_SKIP) == 0
    if raise_errors:
        raise_reference_errors(options, hp, res, evaluated)
    a = first_tie_arrays(options, hp, res)
    e = options.eff_a
    tm = None
    if options.allhits:
        tm = out.tiemask[:batch.tw * batch.stride].cpu().numpy().view(np.uint64).reshape(batch.tw, batch.stride)
    return [_splices_of(options, genome, hp, a, evaluated, i, spans[i] if spans is not None else None,
                        lambda i=i: tm[:, int(slot[i])]) for i in range(batch.n)]


def _splices_of(options: Options, genome: Genome, hp, a, evaluated, i: int, span, tie_words):
    """Pair i's find_breakpoints result from its decoded first tie (``a``, first_tie_arrays) and,
    with --all-hits, its tie words (``tie_words()``: '+' half then '-' half): the tie list, or the
    exception the reference raises."""
    if evaluated[i] and (a["err_key"][i] or a["err_win"][i]):
        return (KeyError("splice signal with a byte outside ACGTN (find_circ.py:927)") if a["err_key"][i]
                else BreakpointError(WINDOW_SHAPE_MESSAGE))
    if not a["hit"][i] or not evaluated[i]:
        return []
    chrom = genome.names[hp["chrom"][i]] if not genome.dummy else (span.chrom if span is not None else "")
    g = gtag_str(int(a["gtag12"][i]))
    strand = '-' if a["minus"][i] else '+'
    sig = rev_comp4(g) if strand == '-' else g
    dist = int(a["dist"][i])
    dist_v = False if options.maxdist == 0 else dist     # simple_match returns a bool (find_circ.py:865-871)
    s = Splice(span, chrom, int(a["start"][i]), int(a["end"][i]), strand, dist_v, int(a["ov"][i]), sig)
    nt = int(a["n_ties"][i])
    s.n_hits = nt
    s._score = _score(options, sig, dist, s.ov, strand, hp["flags"][i])
    if options.allhits and nt > 1:
        return _expand_ties(options, genome, hp, i, tie_words(), s, span, chrom)
    return [s]


def scan_long(options: Options, genome: Genome, reads, long_pairs: np.ndarray, device=None):
    """find_breakpoints of anchor pairs whose read parts exceed MAX_READ_LEN (fc2_long_pair records,
    include/fc2_bp.h; the reference's x-loop has no length limit, find_circ.py:873, :904-906): the
    read parts and windows are laid out on the host (fc2_long_fill, windows from the mmap'd FASTA
    with get_data's semantics), the byte-exact long kernel runs on ``device`` (default: the genome's),
    and the call waits for it.  ``reads``: the buffer the records' read_off index (a uint8 array or an
    address).  Returns (results LONG_RESULT_DTYPE [n], tie words uint64 or None, tie_off [n+1])."""
    torch = _torch()
    dev = torch.device(device) if device is not None else genome.device
    lp = np.ascontiguousarray(long_pairs, N.LONG_PAIR_DTYPE)
    n = len(lp)
    p = options.params()
    nbytes = ctypes.c_uint64()
    tie_off = np.zeros(n + 1, np.uint64)
    N.check(N.lib().fc2_long_geometry(ctypes.byref(p), n, lp.ctypes.data, ctypes.byref(nbytes), tie_off.ctypes.data))
    res = np.zeros(n, N.LONG_RESULT_DTYPE)
    if n == 0:
        return res, (np.zeros(0, np.uint64) if options.allhits else None), tie_off
    off = np.zeros(n, np.uint64)
    arena = np.zeros(max(16, int(nbytes.value)), np.uint8)
    rptr = reads if isinstance(reads, int) else np.ascontiguousarray(reads, np.uint8).ctypes.data
    N.check(N.lib().fc2_long_fill(ctypes.byref(p), genome.fasta if not genome.dummy else None, n, rptr, lp.ctypes.data,
                                  off.ctypes.data, arena.ctypes.data))
    d_pairs = torch.from_numpy(lp.view(np.uint8)).to(dev)
    d_off = torch.from_numpy(off.view(np.int64)).to(dev)
    d_arena = torch.from_numpy(arena).to(dev)
    d_res = torch.empty(n * N.LONG_RESULT_DTYPE.itemsize, dtype=torch.uint8, device=dev)
    d_toff = d_ties = None
    if options.allhits:
        d_toff = torch.from_numpy(tie_off.view(np.int64)).to(dev)
        d_ties = torch.empty(max(1, int(tie_off[n])), dtype=torch.int64, device=dev)
    s = torch.cuda.current_stream(dev)
    N.check(N.lib().fc2_bp_scan_long_launch(ctypes.byref(p), n, d_pairs.data_ptr(), d_off.data_ptr(),
                                            d_arena.data_ptr(), d_toff.data_ptr() if d_toff is not None else None,
                                            d_res.data_ptr(), d_ties.data_ptr() if d_ties is not None else None,
                                            s.cuda_stream))
    res = d_res.cpu().numpy().view(N.LONG_RESULT_DTYPE).copy()
    ties = d_ties.cpu().numpy().view(np.uint64)[:int(tie_off[n])].copy() if d_ties is not None else None
    return res, ties, tie_off


def decode_long_splices(options: Options, genome: Genome, long_pairs: np.ndarray, res: np.ndarray, ties, tie_off,
                        spans: Sequence = None) -> List:
    """decode_splices for the results of scan_long (pairs' tie words at ties[tie_off[j]:tie_off[j+1]])."""
    a = first_tie_arrays(options, long_pairs, res)
    evaluated = (long_pairs["flags"] & N.PAIR_SKIP) == 0
    return [_splices_of(options, genome, long_pairs, a, evaluated, j, spans[j] if spans is not None else None,
                        lambda j=j: ties[int(tie_off[j]):int(tie_off[j + 1])]) for j in range(len(long_pairs))]


def _score(options, sig, dist, ov, strand, flags):
    sc = (sig == 'GTAG') * 20 - dist * 10 - ov
    if options.strandpref:
        prim = '-' if flags & N.PAIR_PRIMARY_REV else '+'
        sc += 100 * (strand == prim)
    return sc


def _expand_ties(options, genome, hp, i, tm, best: Splice, span, chrom):
    """All ties of pair i in (x asc, '+' before '-') order from the tie mask."""
    e = options.eff_a
    L = int(hp["read_len"][i])
    l = L - 2 * e
    half = tm.shape[0] // 2
    out = []
    for x in range(l + 1):
        k, b = x >> 6, x & 63
        for strand, row in (('+', k), ('-', half + k)):
            if not (int(tm[row]) >> b) & 1:
                continue
            s0 = int(hp["b_aend"][i]) - e - l + x
            e0 = int(hp["a_pos"][i]) + e + x + 1
            st, en = min(s0, e0), max(s0, e0)
            if hp["flags"][i] & N.PAIR_BACKSPLICE:
                en -= 1
            else:
                st -= 1
            ov = 0
            if options.margin:
                if x < options.margin:
                    ov = options.margin - x
                if l - x < options.margin:
                    ov = options.margin - (l - x)
            if options.noncanonical:
                g = _window_gtag(genome, hp, i, x, e, l)
                sig = g if strand == '+' else rev_comp4(g)
            else:
                sig = 'GTAG'
            canon = 20 * (sig == 'GTAG')
            sp = 0
            if options.strandpref:
                prim = '-' if hp["flags"][i] & N.PAIR_PRIMARY_REV else '+'
                sp = 100 * (strand == prim)
            dist = (canon - ov + sp - best.score) // 10
            s = Splice(span, chrom, st, en, strand, False if options.maxdist == 0 else dist, ov, sig)
            s.n_hits = best.n_hits
            s._score = best.score
            out.append(s)
    return out


def _window_gtag(genome: Genome, hp, i, x, e, l) -> str:
    # gt = A_flank[x:x+2], ag = B_flank[x:x+2] of the full windows (find_circ.py:901-902, 924-926)
    if genome.dummy:
        return "NNNN"
    c = int(hp["chrom"][i])
    a0 = int(hp["a_pos"][i]) + e
    b1 = int(hp["b_aend"][i]) - e
    A = genome.get_upper(c, a0, a0 + l + 2)
    B = genome.get_upper(c, b1 - l - 2, b1)
    return (A[x:x + 2] + B[x:x + 2]).decode("latin-1")


# ---------------------------------------------------------------------------
# drop-in mirror of the reference objects
# ---------------------------------------------------------------------------
def uniqness(align):
    """AS - XS (find_circ.py:809-819): an int, a float, or a str / array AS as it is."""
    u = align.get_tag('AS')
    if align.has_tag('XS'):
        u -= align.get_tag('XS')
    return u


def _is_number(v) -> bool:
    return isinstance(v, (int, float)) and not isinstance(v, bool)


def _py2_min(a, b):
    """min(a, b) with Python 2's ordering of mixed types: numbers by value (b only if strictly
    smaller, as the builtin), any number before a non-number (a str or array tag value)."""
    if _is_number(a) and _is_number(b):
        return b if b < a else a
    if _is_number(b):
        return b
    if _is_number(a):
        return a
    # two non-numbers: Python 2 compares values of one type by value (str lexicographically, arrays
    # element-wise) and values of different types by type name ('array' < 'str')
    if type(a) is type(b):
        return b if b < a else a
    return b if type(b).__name__ < type(a).__name__ else a


def uniq_ok(uniq, min_uniq_qual: int) -> bool:
    """``uniq >= options.min_uniq_qual`` (find_circ.py:1299, :1351) under Python 2: a non-number
    (str / array) orders above every int."""
    return uniq >= min_uniq_qual if _is_number(uniq) else True


class JunctionSpan:
    """Mirror of ``JunctionSpan`` (find_circ.py:821-852).

    ``align_A``/``align_B``/``primary`` are pysam-like records (``.pos``,
    ``.aend``, ``.seq``, ``.is_reverse``, ``get_tag``/``has_tag``); ``chrom`` is
    the reference name of ``align_A`` (``fast_chrom_lookup``, find_circ.py:471-477).
    """

    engine = None   # set by BreakpointEngine.install() (the reference uses globals)

    def __init__(self, align_A, align_B, primary, q_start, q_end, weight, chrom=None):
        self.primary = primary
        self.align_A = align_A
        self.align_B = align_B
        self.q_start = q_start
        self.q_end = q_end
        self.weight = weight
        self.uniq_A = uniqness(align_A)
        self.uniq_B = uniqness(align_B)
        self.uniq = _py2_min(self.uniq_A, self.uniq_B)
        self.strand = '-' if primary.is_reverse else '+'
        self.dist = align_B.pos - align_A.aend
        self.read_part = primary.seq[q_start:q_end]
        self.chrom = chrom

    min_uniq_qual = 2   # options.min_uniq_qual (find_circ.py:393), read by is_uniq like the reference

    def is_uniq_for(self, min_uniq_qual: int) -> bool:        # find_circ.py:846-848
        return uniq_ok(self.uniq, min_uniq_qual)

    @property
    def is_uniq(self) -> bool:                                # find_circ.py:846-848
        return uniq_ok(self.uniq, self.min_uniq_qual)

    @property
    def is_backsplice(self):                                  # find_circ.py:850-852
        return self.dist < 0

    def find_breakpoints(self):                               # find_circ.py:854
        """The reference method: the list of ties, or the exception the reference raises for this
        span (KeyError for a chromosome missing from the FASTA, :193, or a non-ACGTN splice
        signal, :927)."""
        if JunctionSpan.engine is None:
            raise RuntimeError("no BreakpointEngine installed (BreakpointEngine(...).install())")
        return splices_or_raise(JunctionSpan.engine.find_breakpoints_batch([self])[0])


def none_aend_error():
    """find_breakpoints of a span whose align_B.aend is None: B's window, ``B.aend - eff_a``
    (find_circ.py:902), after A's window has been fetched (a missing chromosome raises first)."""
    return TypeError("unsupported operand type(s) for -: 'NoneType' and 'int'")


def splices_or_raise(r):
    """A ``find_breakpoints_batch`` entry as the reference method returns it: raises the
    per-span exception, else returns the tie list."""
    if isinstance(r, BaseException):
        raise r
    return r


class BreakpointEngine:
    """Genome + options + device: evaluates lists of JunctionSpans in one launch."""

    def __init__(self, genome: Genome, options: Options):
        self.genome = genome
        self.options = options

    def install(self):
        JunctionSpan.engine = self
        return self

    def find_breakpoints_batch(self, spans: Sequence[JunctionSpan], locus_order: bool = False) -> List:
        """``find_breakpoints()`` of every span in ONE launch.  Entry i is span i's tie list, or
        -- where the reference method would raise -- the exception instance, so a caller that
        evaluates spans speculatively raises it only when ``record_hits`` reaches that span
        (``splices_or_raise``): KeyError(chrom) for a chromosome missing from the FASTA
        (indexed_fasta.get_data, find_circ.py:193; the pair is not scanned), KeyError for a
        non-ACGTN splice signal (:927), BreakpointError for windows outside get_data's range."""
        if not spans:
            return []
        reads = []
        for s in spans:
            r = s.read_part
            reads.append(r if isinstance(r, bytes) else r.encode("latin-1"))
        missing = 0xFFFFFFFF
        chrom = [self.genome.chrom_index_or_missing(s.chrom) for s in spans]
        flags = [(N.PAIR_BACKSPLICE if s.is_backsplice else 0) | (N.PAIR_PRIMARY_REV if s.strand == '-' else 0) |
                 (N.PAIR_SKIP if c == missing or s.align_B.aend is None else 0) for s, c in zip(spans, chrom)]
        # read parts over MAX_READ_LEN take the long path (fc2_long_pair); the rest one batch
        longs = [k for k, r in enumerate(reads) if len(r) > N.MAX_READ_LEN]
        short = [k for k, r in enumerate(reads) if len(r) <= N.MAX_READ_LEN] if longs else range(len(spans))
        res: List = [None] * len(spans)
        if len(short):
            sub = [spans[k] for k in short]
            b = PairBatch.pack(self.options, self.genome, [reads[k] for k in short], [s.align_A.pos for s in sub],
                               [s.align_B.aend or 0 for s in sub], [0 if chrom[k] == missing else chrom[k] for k in short],
                               [flags[k] for k in short], locus_order=locus_order)
            out = scan(self.options, self.genome, b)
            for k, r in zip(short, decode_splices(self.options, self.genome, b, out, sub, raise_errors=False)):
                res[k] = r
        if longs:
            buf = b"".join(reads[k] for k in longs) + b"\0" * 16
            lp = np.zeros(len(longs), N.LONG_PAIR_DTYPE)
            lens = np.array([len(reads[k]) for k in longs], np.uint64)
            lp["read_off"][1:] = np.cumsum(lens[:-1])
            lp["read_len"] = lens
            lp["chrom"] = [0 if chrom[k] == missing else chrom[k] for k in longs]
            lp["a_pos"] = [spans[k].align_A.pos for k in longs]
            lp["b_aend"] = [spans[k].align_B.aend or 0 for k in longs]
            lp["flags"] = [flags[k] for k in longs]
            lr, ties, toff = scan_long(self.options, self.genome, np.frombuffer(buf, np.uint8), lp)
            for k, r in zip(longs, decode_long_splices(self.options, self.genome, lp, lr, ties, toff,
                                                       [spans[k] for k in longs])):
                res[k] = r
        return [KeyError(s.chrom) if c == missing else none_aend_error() if s.align_B.aend is None else r
                for s, r, c in zip(spans, res, chrom)]
