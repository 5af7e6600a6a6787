"""Pipelined breakpoint search over a host pair stream: pinned staging, side streams, N GPUs.

This is the transfer path BASELINE.json's north_star names ("batches pysam anchor-pair records
into SoA arrays and streams ... via pinned hipMemcpyAsync on a side stream"), for the pairs the
read loop hands out (``fc2_caller_next``, include/fc2_caller.h) -- the spans ``record_hits`` will
evaluate (find_circ.py:1303, :1355).  Per chunk:

1. the host packer (``fc2_pack_pairs``, C++ threads) writes the 16-B records and the bit-sliced
   read rows straight into page-locked staging buffers (no intermediate numpy copies);
2. on the scanner's own HIP stream: async H2D of records + rows, ``fc2_bp_scan_launch``
   (+ the byte-exact launch for the rare byte-path pairs), async D2H of the 8-B results
   (and the --all-hits tie rows) into page-locked result buffers, an event;
3. ``result(ticket)`` waits for that event only.

Each scanner double-buffers (two slots), so while chunk k is in flight the host packs chunk k+1;
with several devices (``devices=[...]``) chunks are dealt round-robin and ``result`` is called in
submission order, so the caller sees results in input order -- junction names are given by first
appearance (find_circ.py:681-690) and weights accumulate in order (:544, :563, :579).  Pairs
stay in input order: the read-order scan is ~2e10 pairs/s, two orders of magnitude above what
the host packer feeds, so a host locality sort would only cost time.
"""
from __future__ import annotations

import ctypes
from typing import List, Optional, Sequence

import numpy as np

from . import _native as N
from .genome import Genome, _torch
from .hotpath import Options, PairBatch, ScanOutput, scan, scan_long


class _Slot:
    """Page-locked host staging + device buffers for one chunk on one device."""

    def __init__(self):
        self.cap = 0
        self.rw = self.nw = self.tw = 0
        self.event = None
        self.busy = False
        self.keep = None            # device objects of the chunk in flight (alive until its event)

    def ensure(self, torch, dev, n: int, rw: int, nw: int, tw: int, allhits: bool):
        if n <= self.cap and rw <= self.rw and nw <= self.nw and (not allhits or tw <= self.tw):
            return
        cap = max(n, 2 * self.cap, 4096)
        rw, nw, tw = max(rw, self.rw), max(nw, self.nw), max(tw, self.tw)
        pin = dict(pin_memory=True)
        self.h_pairs = torch.empty(16 * cap, dtype=torch.uint8, **pin)
        self.h_words = torch.empty(rw * cap, dtype=torch.int64, **pin)
        self.h_nwords = torch.empty(nw * cap, dtype=torch.int64, **pin)
        self.h_res = torch.empty(cap, dtype=torch.int64, **pin)
        self.d_pairs = torch.empty(16 * cap, dtype=torch.uint8, device=dev)
        self.d_words = torch.empty(rw * cap, dtype=torch.int64, device=dev)
        self.d_nwords = torch.empty(nw * cap, dtype=torch.int64, device=dev)
        self.d_res = torch.empty(cap, dtype=torch.int64, device=dev)
        self.h_tm = self.d_tm = None
        if allhits:
            self.h_tm = torch.empty(tw * cap, dtype=torch.int64, **pin)
            self.d_tm = torch.empty(tw * cap, dtype=torch.int64, device=dev)
        self.np_pairs = self.h_pairs.numpy().view(N.PAIR_DTYPE)
        self.np_words = self.h_words.numpy()
        self.np_nwords = self.h_nwords.numpy()
        self.np_res = self.h_res.numpy()
        self.np_tm = self.h_tm.numpy() if allhits else None
        self.cap, self.rw, self.nw, self.tw = cap, rw, nw, tw


class Ticket:
    __slots__ = ("scanner", "slot", "n", "tw", "gen", "res", "tm")

    def __init__(self, scanner, slot, n, tw, gen):
        self.scanner, self.slot, self.n, self.tw, self.gen = scanner, slot, n, tw, gen
        self.res = self.tm = None


class DeviceScanner:
    """One device: its genome copy, a side stream and two staging slots."""

    SLOTS = 2

    def __init__(self, genome: Genome, options: Options, n_threads: int = 0):
        torch = _torch()
        self.genome = genome
        self.options = options
        self.params = options.params()
        self.dev = genome.device
        self.stream = torch.cuda.Stream(self.dev)
        self.slots = [_Slot() for _ in range(self.SLOTS)]
        for s in self.slots:
            s.event = torch.cuda.Event()
        self.k = 0
        self.n_threads = int(n_threads)
        self._gen = [0] * self.SLOTS          # which ticket currently owns each slot
        self._pending = {}                    # slot -> ticket whose results are not taken yet

    def submit(self, reads_ptr: int, read_off: np.ndarray, pairs: np.ndarray) -> Ticket:
        """Pack (host, C++ threads, into page-locked staging), upload, scan and download one chunk;
        returns at once after queueing the device work.  reads_ptr/read_off/pairs: the chunk as
        fc2_caller_next hands it out (read_part bytes at reads_ptr + read_off[i], PAIR_DTYPE)."""
        torch = _torch()
        n = len(pairs)
        si = self.k % self.SLOTS
        self.k += 1
        slot = self.slots[si]
        if slot.busy:
            self._drain(si)
        self._gen[si] += 1
        t = Ticket(self, si, n, 0, self._gen[si])
        if n == 0:
            t.res = np.zeros(0, np.int64)
            return t
        opt = self.options
        e = opt.eff_a
        max_len = int(pairs["read_len"].max())
        rw, nw, tw = ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_uint32()
        N.check(N.lib().fc2_batch_geometry(ctypes.byref(self.params), max_len, ctypes.byref(rw), ctypes.byref(nw),
                                           ctypes.byref(tw)))
        rw, nw, tw = rw.value, nw.value, tw.value
        slot.ensure(torch, self.dev, n, rw, nw, tw, opt.allhits)
        hp = slot.np_pairs[:n]
        # 16-B records into page-locked staging (torch's CPU copy runs on its thread pool)
        slot.h_pairs[:16 * n].copy_(torch.from_numpy(np.ascontiguousarray(pairs).view(np.uint8).reshape(-1)))
        off = np.ascontiguousarray(read_off, np.uint64)
        nbp = ctypes.c_uint64()
        g = self.genome
        N.check(N.lib().fc2_pack_pairs(ctypes.byref(self.params), g.fasta if not g.dummy else None, n, reads_ptr,
                                       off.ctypes.data, hp.ctypes.data, slot.np_words.ctypes.data, rw,
                                       slot.np_nwords.ctypes.data, nw, n, ctypes.byref(nbp), self.n_threads))
        b = PairBatch()
        b.options, b.device = opt, self.dev
        b.n, b.stride, b.rw, b.nw, b.tw = n, n, rw, nw, tw
        b.max_l = max(0, min(max_len - 2 * e, N.lib().fc2_max_fast_l()))
        b.host_pairs = hp
        b.m_bytepath = int(nbp.value)
        s = self.stream
        with torch.cuda.stream(s):
            b.pairs = slot.d_pairs[:16 * n]
            b.read_words = slot.d_words[:rw * n]
            b.read_nwords = slot.d_nwords[:nw * n]
            b.pairs.copy_(slot.h_pairs[:16 * n], non_blocking=True)
            b.read_words.copy_(slot.h_words[:rw * n], non_blocking=True)
            b.read_nwords.copy_(slot.h_nwords[:nw * n], non_blocking=True)
            if b.m_bytepath:
                if g.fasta is None and not g.dummy:
                    raise RuntimeError("%d pairs need byte-exact windows, which come from a FASTA-backed genome"
                                       % b.m_bytepath)
                self._pack_bytepath(b, reads_ptr, off)
            tm = None
            if opt.allhits:
                tm = slot.d_tm[:tw * n]
                tm.zero_()
            out = ScanOutput(slot.d_res[:n], tm, tw, n)
            scan(opt, g, b, out=out, stream=s.cuda_stream)
            slot.h_res[:n].copy_(out.results, non_blocking=True)
            if tm is not None:
                slot.h_tm[:tw * n].copy_(tm, non_blocking=True)
            slot.event.record(s)
        slot.busy = True
        slot.keep = b
        t.tw = tw
        self._pending[si] = t
        return t

    def _pack_bytepath(self, b: PairBatch, reads_ptr: int, off: np.ndarray):
        """The rare byte-path pairs (exotic bytes, irregular FASTA layout, l > 510): their
        uppercased bytes and windows (fc2_bytepath_fill), uploaded on the scanner's stream."""
        torch = _torch()
        p = self.params
        g = self.genome
        m, nbytes = ctypes.c_uint64(), ctypes.c_uint64()
        hp = b.host_pairs
        N.check(N.lib().fc2_bytepath_size(ctypes.byref(p), b.n, hp.ctypes.data, ctypes.byref(m),
                                          ctypes.byref(nbytes)))
        m = int(m.value)
        idx = np.zeros(m, np.uint64)
        bpairs = np.zeros(m, N.PAIR_DTYPE)
        offs = np.zeros(m, np.uint64)
        arena = np.zeros(max(16, int(nbytes.value)), np.uint8)
        N.check(N.lib().fc2_bytepath_fill(ctypes.byref(p), g.fasta if not g.dummy else None, b.n, reads_ptr,
                                          off.ctypes.data, hp.ctypes.data, idx.ctypes.data, bpairs.ctypes.data,
                                          offs.ctypes.data, arena.ctypes.data))
        b.bp_index = torch.from_numpy(idx.view(np.int64)).to(self.dev)
        b.bp_pairs = torch.from_numpy(bpairs.view(np.uint8)).to(self.dev)
        b.bp_off = torch.from_numpy(offs.view(np.int64)).to(self.dev)
        b.bp_arena = torch.from_numpy(arena).to(self.dev)

    def _drain(self, si: int):
        """Wait for slot si's chunk; results not yet taken by result() are copied out to their
        ticket so the slot can be reused."""
        slot = self.slots[si]
        slot.event.synchronize()
        t = self._pending.pop(si, None)
        if t is not None:
            self._copy_out(t)
        slot.busy = False
        slot.keep = None

    def _copy_out(self, t: Ticket, copy: bool = True):
        slot = self.slots[t.slot]
        res = slot.np_res[:t.n]
        tm = slot.np_tm[:t.tw * t.n].reshape(t.tw, t.n).view(np.uint64) if self.options.allhits else None
        if copy:
            res = res.copy()
            tm = tm.copy() if tm is not None else None
        t.res, t.tm = res, tm

    def result(self, t: Ticket, copy: bool = True):
        """(results int64 [n] = raw fc2_result words, tie mask uint64 [tw, n] or None) of a chunk.
        ``copy=False`` returns views of the page-locked result buffers: valid until the next
        ``submit`` to this scanner (the native read loop hands them straight to fc2_caller_submit)."""
        if t.res is None:
            if self._gen[t.slot] != t.gen:
                raise RuntimeError("ticket's slot was reused before its results were taken")
            slot = self.slots[t.slot]
            slot.event.synchronize()
            self._pending.pop(t.slot, None)
            self._copy_out(t, copy)
            slot.busy = False
            slot.keep = None
        return t.res, t.tm


class ScanPipeline:
    """Chunks dealt round-robin over one DeviceScanner per device; results in submission order.

    ``genome`` lives on devices[0]; other devices get a replica (``Genome.replicate``), a device
    listed twice shares its genome (two scanners, two streams -- how a 1-GPU box rehearses
    ``--gpus 2``).  ``depth`` = chunks in flight the caller may hold (2 per scanner)."""

    def __init__(self, genome: Genome, options: Options, devices: Optional[Sequence] = None, n_threads: int = 0):
        torch = _torch()
        devs = [torch.device(d) for d in (devices or [genome.device])]
        genomes = {genome.device: genome}
        self.scanners: List[DeviceScanner] = []
        for d in devs:
            if d not in genomes:
                genomes[d] = genome.replicate(d)
            self.scanners.append(DeviceScanner(genomes[d], options, n_threads))
        self.options = options
        self.k = 0
        self.depth = DeviceScanner.SLOTS * len(self.scanners)

    def submit(self, reads_ptr: int, read_off: np.ndarray, pairs: np.ndarray) -> Ticket:
        sc = self.scanners[self.k % len(self.scanners)]
        self.k += 1
        return sc.submit(reads_ptr, read_off, pairs)

    def result(self, t: Ticket, copy: bool = True):
        return t.scanner.result(t, copy)

    def evaluate_long(self, reads_ptr: int, long_pairs: np.ndarray):
        """The chunk's pairs with read parts over MAX_READ_LEN (fc2_caller_batch.long_pairs), on the first
        scanner's device and synchronously -- they are rare (hotpath.scan_long): (results, tie words)."""
        sc = self.scanners[0]
        res, ties, _ = scan_long(self.options, sc.genome, int(reads_ptr), long_pairs)
        return res, ties

    def __call__(self, reads, read_off, pairs):
        """Synchronous form (evaluate(reads, read_off, pairs) of native_caller)."""
        reads = np.ascontiguousarray(reads, np.uint8)
        return self.result(self.submit(reads.ctypes.data, read_off, pairs))
