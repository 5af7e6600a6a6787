"""The read loop's breakpoint search over the torch-free C ABI (include/fc2_ctx.h).

``python -m find_circ2_amd.cli`` (the native read loop) hands every chunk of anchor pairs to this
evaluator: per device one ``fc2_ctx`` holding the resident genome (2-bit planes, N maps, word-pair
table, built on the host from the mmap'd FASTA and uploaded once), and sibling contexts
(``fc2_ctx_create_sibling``) that scan against the same tables with their own HIP stream and
page-locked staging.  A chunk goes to the next context round-robin: host packing (``fc2_pack_pairs``
on C++ threads, the byte path's windows from the FASTA), H2D, the scan and the D2H of the 8-byte
results are queued on that context's stream, and ``result`` waits for them only.  With two contexts
per device one chunk is on the GPU while the host packs the next; results come back in submission
order, so junctions are named by first appearance and weights summed in input order
(find_circ.py:681-690, :544, :563, :579).

This module imports neither PyTorch nor the torch-based Genome: the process pays for the HIP
runtime only, not for ``import torch`` (DESIGN.md §0a start-up).  ``pipeline.ScanPipeline`` is the
same evaluator on torch streams (the Python read loop's and bench.py's form).
"""
from __future__ import annotations

import ctypes
import threading
from typing import List, Optional, Sequence

from ._lazy import LazyModule

np = LazyModule("numpy", globals(), "np")

from . import _native as N


def device_count() -> int:
    n = ctypes.c_int(0)
    N.check(N.lib().fc2_device_count(ctypes.byref(n)))
    return int(n.value)


def device_index(device) -> int:
    """'cuda:k' / 'hip:k' / k -> k."""
    if isinstance(device, int):
        return device
    s = str(device)
    return int(s.split(":", 1)[1]) if ":" in s else 0


class FastaGenome:
    """The genome FASTA as the native read loop needs it: the fc2_fasta handle (mmap'd, .byo_index
    read or written as find_circ.py:110-115 does) and its chromosome names; ``fasta`` None for
    GenomeAccessor's dummy mode (find_circ.py:338-345)."""

    def __init__(self, path: Optional[str], write_index: bool = True):
        self.fasta = None
        self.names: List[str] = []
        self.dummy = path is None
        if path is None:
            return
        h = ctypes.c_void_p()
        rc = N.lib().fc2_fasta_open(path.encode(), int(write_index), ctypes.byref(h))
        N.check(rc)
        self.fasta = h
        for i in range(N.lib().fc2_fasta_n_chrom(h)):
            nm = ctypes.c_char_p()
            N.check(N.lib().fc2_fasta_chrom(h, i, ctypes.byref(nm), None, None, None, None, None))
            self.names.append(nm.value.decode("latin-1"))

    @classmethod
    def open_or_dummy(cls, path: str, on_dummy=None) -> "FastaGenome":
        """fc2_fasta_open, or the dummy genome where the reference's indexed_fasta() raises IOError."""
        try:
            return cls(path)
        except N.Fc2Error as ex:
            if ex.code != N.FC2_E_IO:
                raise
            if on_dummy is not None:
                on_dummy()
            return cls(None)

    @classmethod
    def adopt(cls, pre, on_dummy=None) -> "FastaGenome":
        """The FASTA the prestart opened (prestart.Prestart): open_or_dummy's outcome, raised or warned
        here as open_or_dummy does."""
        pre.fasta_ready.wait()
        if pre.fasta_error is not None:
            raise N.Fc2Error(*pre.fasta_error)
        g = cls(None)
        if pre.dummy:
            if on_dummy is not None:
                on_dummy()
            return g
        g.dummy = False
        g.fasta = ctypes.c_void_p(pre.fasta)
        for i in range(N.lib().fc2_fasta_n_chrom(g.fasta)):
            nm = ctypes.c_char_p()
            N.check(N.lib().fc2_fasta_chrom(g.fasta, i, ctypes.byref(nm), None, None, None, None, None))
            g.names.append(nm.value.decode("latin-1"))
        return g

    def close(self):
        if self.fasta is not None:
            N.lib().fc2_fasta_close(self.fasta)
            self.fasta = None


class _Ctx:
    def __init__(self, handle, device: int):
        self.h = handle
        self.device = device
        self.lock = threading.Lock()
        self.pending = None            # the ticket whose results the context still holds
        self.primary = False           # owns the device's genome tables (siblings read them)

    def check(self, rc: int):
        if rc != N.FC2_OK:
            msg = N.lib().fc2_ctx_last_error(self.h)
            raise N.Fc2Error(rc, msg.decode("utf-8", "replace") if msg else "")


class CtxTicket:
    __slots__ = ("ctx", "n", "res", "tm", "tw", "done", "deferred", "keep")

    def __init__(self, ctx, n, res, tm, tw=0):
        self.ctx, self.n, self.res, self.tm, self.tw, self.done = ctx, n, res, tm, tw, False
        self.deferred = None           # (reads_ptr, off_ptr, pairs_ptr) while the genome is being built
        self.keep = None               # submit(): the arrays those pointers point into


class CtxPipeline:
    """Chunks dealt round-robin over ``per_device`` contexts on each of ``devices`` (one genome copy
    per device, siblings share it); ``depth`` = chunks the caller may hold in flight."""

    def __init__(self, genome: FastaGenome, options, devices: Sequence = (0,), per_device: int = 2,
                 n_threads: int = 0, background: bool = False, prestart=None):
        """``background``: create the contexts and make the genome resident on a thread of their own,
        so the caller can open its input and read the first chunks meanwhile (the reference, too,
        touches the genome only when the first span is evaluated, find_circ.py:435-436); the first
        submit waits for it and raises its error.  ``prestart``: the contexts prestart.Prestart is
        building for these devices (the CLI; implies background)."""
        self.options = options
        self.params = options.params()
        self.n_threads = int(n_threads)
        self.ctxs: List[_Ctx] = []
        self.k = 0
        self.n_ctx = len(devices) * per_device      # per listing of a device: per_device contexts
        # chunks the caller may hold: tickets own their result buffers, so more than the contexts --
        # while the genome is being built the read loop reads this many chunks ahead; never more than
        # fc2_caller_next queues (FC2_CALLER_MAX_QUEUED, include/fc2_caller.h), or a run with many
        # --gpus entries would stop on 'too many chunks not submitted'
        self.depth = min(4 * self.n_ctx, N.CALLER_MAX_QUEUED)
        self._slock = threading.Lock()              # dispatch order (reader thread + recorder thread)
        self._wlock = threading.Lock()              # wait_ready's bookkeeping
        self._deferred: List[CtxTicket] = []
        self._ready = None
        self._error = None
        self.load_s = self.hip_init_s = None
        self.genome_load_s = 0.0                    # fc2_ctx_genome_load calls (pack + upload + tables)
        self.siblings_s = 0.0                       # fc2_ctx_create_sibling calls
        self.prepack_s = 0.0                        # fc2_fasta_prepack beside HIP init (prestart only)
        self.wait_s = 0.0
        if prestart is not None:
            self._ready = threading.Thread(target=self._adopt_guarded, args=(prestart,),
                                           name="fc2-genome-adopt", daemon=True)
            self._ready.start()
        elif background:
            self._ready = threading.Thread(target=self._build_guarded, args=(genome, devices, per_device),
                                           name="fc2-genome-load", daemon=True)
            self._ready.start()
        else:
            self._build(genome, devices, per_device)

    def _build_guarded(self, genome, devices, per_device):
        try:
            self._build(genome, devices, per_device)
        except BaseException as ex:     # noqa: BLE001 -- raised at the first submit
            self._error = ex

    def _adopt_guarded(self, pre):
        pre.thread.join()
        if pre.error is not None:
            self._error = N.Fc2Error(*pre.error)
            return
        if len(pre.ctxs) != self.n_ctx:
            self._error = RuntimeError("genome prestart built %d contexts for %d" % (len(pre.ctxs), self.n_ctx))
            return
        for h, dev, primary in pre.ctxs:
            c = _Ctx(ctypes.c_void_p(h), dev)
            c.primary = primary
            self.ctxs.append(c)
        self.hip_init_s, self.genome_load_s, self.siblings_s = pre.hip_init_s, pre.genome_load_s, pre.siblings_s
        self.prepack_s = pre.prepack_s
        self.load_s = pre.load_s

    def wait_ready(self):
        """The contexts and resident genome are built (raises what building them raised); the time
        spent waiting for them is added up in ``wait_s``."""
        ready = self._ready             # read once: another thread may clear it (evaluate_long runs on the
        if ready is not None:           # reader thread, result() on the recorder thread)
            import time
            t = time.time()
            ready.join()
            with self._wlock:
                if self._ready is ready:
                    self._ready = None
                self.wait_s += time.time() - t
        if self._error is not None:
            raise self._error

    def _build(self, genome, devices, per_device):
        import time
        t0 = time.time()
        L = N.lib()
        primary = {}
        try:
            for d in devices:
                dev = device_index(d)
                if dev not in primary:
                    h = ctypes.c_void_p()
                    N.check(L.fc2_ctx_create(dev, ctypes.byref(h)))
                    if self.hip_init_s is None:         # the first HIP call of the process
                        self.hip_init_s = time.time() - t0
                    c = _Ctx(h, dev)
                    c.primary = True
                    self.ctxs.append(c)
                    tg = time.time()
                    c.check(L.fc2_ctx_genome_load(h, genome.fasta, self.n_threads))
                    self.genome_load_s += time.time() - tg
                    primary[dev] = c
                    k0 = 1
                else:
                    k0 = 0                 # a device listed twice: more contexts on it (--gpus N > devices)
                for _ in range(k0, per_device):
                    ts = time.time()
                    h = ctypes.c_void_p()
                    N.check(L.fc2_ctx_create_sibling(primary[dev].h, ctypes.byref(h)))
                    self.ctxs.append(_Ctx(h, dev))
                    self.siblings_s += time.time() - ts
        except BaseException:
            self.close()
            raise
        assert len(self.ctxs) == self.n_ctx, (len(self.ctxs), self.n_ctx)
        self.load_s = time.time() - t0

    def close(self):
        """Siblings before the contexts whose genome they read."""
        if self._ready is not None and self._ready is not threading.current_thread():
            self._ready.join()          # (from _build's error path on that thread itself: nothing to wait for)
            self._ready = None
        L = N.lib()
        for primary_pass in (False, True):
            for c in self.ctxs:
                if c.h and c.primary == primary_pass:
                    L.fc2_ctx_destroy(c.h)
                    c.h = None
        self.ctxs = []

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @staticmethod
    def _sync(c: _Ctx):
        t = c.pending
        if t is not None:
            c.pending = None
            c.check(N.lib().fc2_ctx_sync(c.h))
            t.done = True

    def submit(self, reads_ptr: int, read_off: np.ndarray, pairs: np.ndarray) -> CtxTicket:
        """Pack, upload, scan and download one chunk on the next context; returns at once after the
        device work is queued.  reads_ptr / read_off / pairs: the chunk as fc2_caller_next hands it out
        (its memory stays valid while the chunk is queued).  While the genome is still being built the
        chunk is only noted, and dispatched in order once it is ready."""
        pairs = np.ascontiguousarray(pairs, N.PAIR_DTYPE)
        off = np.ascontiguousarray(read_off, np.uint64)
        n = len(pairs)
        tm, tw = None, 0
        if n and self.options.allhits:
            rw, nw, tw_ = ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_uint32()
            N.check(N.lib().fc2_batch_geometry(ctypes.byref(self.params), int(pairs["read_len"].max()),
                                               ctypes.byref(rw), ctypes.byref(nw), ctypes.byref(tw_)))
            tw = tw_.value
            tm = np.empty((tw, n), np.uint64)
        t = CtxTicket(None, n, np.empty(n, np.int64), tm, tw)
        if self._ready is not None and self._ready.is_alive():
            off, pairs = off.copy(), pairs.copy()      # noted for later: the caller may reuse its arrays
        t.keep = (off, pairs)
        self._queue(t, reads_ptr, off.ctypes.data, pairs.ctypes.data)
        return t

    def submit_ptr(self, reads_ptr: int, off_ptr: int, pairs_ptr: int, n: int) -> CtxTicket:
        """submit() of a chunk given as fc2_caller_batch's pointers (the native read loop): the results
        land in a ctypes buffer and nothing here needs numpy -- the default CLI never imports it.  The
        chunk's memory stays valid until its fc2_caller_submit, which follows result(), so a chunk
        noted while the genome is built is not copied.  --all-hits (the tie mask's geometry needs the
        longest read part) goes through submit()."""
        if n and self.options.allhits:
            pairs = np.ctypeslib.as_array(ctypes.cast(pairs_ptr, ctypes.POINTER(ctypes.c_uint8)),
                                          (16 * n,)).view(N.PAIR_DTYPE)
            off = np.ctypeslib.as_array(ctypes.cast(off_ptr, ctypes.POINTER(ctypes.c_uint64)), (n,))
            return self.submit(reads_ptr, off, pairs)
        t = CtxTicket(None, n, (ctypes.c_int64 * max(1, n))(), None, 0)
        self._queue(t, reads_ptr, off_ptr, pairs_ptr)
        return t

    def _queue(self, t: CtxTicket, reads_ptr, off_ptr, pairs_ptr):
        with self._slock:
            if self._ready is not None and self._ready.is_alive():
                t.deferred = (reads_ptr, off_ptr, pairs_ptr)
                self._deferred.append(t)
                return
            self.wait_ready()
            self._flush()
            self._dispatch(t, reads_ptr, off_ptr, pairs_ptr)

    def _flush(self):
        """Dispatch the chunks noted while the genome was being built (caller holds _slock)."""
        while self._deferred:
            t = self._deferred.pop(0)
            reads_ptr, off_ptr, pairs_ptr = t.deferred
            t.deferred = None
            self._dispatch(t, reads_ptr, off_ptr, pairs_ptr)

    @staticmethod
    def _addr(a):
        if a is None:
            return None
        return ctypes.addressof(a) if isinstance(a, ctypes.Array) else a.ctypes.data

    def _dispatch(self, t: CtxTicket, reads_ptr, off_ptr, pairs_ptr):
        c = self.ctxs[self.k % len(self.ctxs)]
        self.k += 1
        t.ctx = c
        with c.lock:
            self._sync(c)                  # the context's previous chunk: its results into its ticket
            if t.n == 0:
                t.done = True
                return
            c.check(N.lib().fc2_ctx_scan_async(c.h, ctypes.byref(self.params), t.n, reads_ptr, off_ptr, pairs_ptr,
                                               self._addr(t.res), self._addr(t.tm), t.tw, self.n_threads))
            c.pending = t

    def result(self, t: CtxTicket, copy: bool = True):
        """(results int64 [n] = raw fc2_result words, tie mask uint64 [tw, n] or None) of a chunk."""
        if t.ctx is None and not t.done:
            with self._slock:
                self.wait_ready()
                self._flush()
        if not t.done:
            with t.ctx.lock:
                if t.ctx.pending is t:
                    self._sync(t.ctx)
        return t.res, t.tm

    def evaluate_long(self, reads_ptr: int, long_pairs: np.ndarray):
        """The chunk's pairs with read parts over MAX_READ_LEN (fc2_caller_batch.long_pairs), on the first
        context, synchronously (fc2_ctx_scan_long): (results LONG_RESULT_DTYPE, tie words or None)."""
        self.wait_ready()
        lp = np.ascontiguousarray(long_pairs, N.LONG_PAIR_DTYPE)
        n = len(lp)
        res = np.zeros(n, N.LONG_RESULT_DTYPE)
        ties = None
        p = self.params
        if self.options.allhits:
            toff = np.zeros(n + 1, np.uint64)
            N.check(N.lib().fc2_long_geometry(ctypes.byref(p), n, lp.ctypes.data, None, toff.ctypes.data))
            ties = np.zeros(max(1, int(toff[n])), np.uint64)
        with self._slock:
            self._flush()
        c = self.ctxs[0]
        with c.lock:
            self._sync(c)
            c.check(N.lib().fc2_ctx_scan_long(c.h, ctypes.byref(p), n, reads_ptr, lp.ctypes.data, res.ctypes.data,
                                              ties.ctypes.data if ties is not None else None))
        if ties is not None:
            ties = ties[:int(toff[n])]
        return res, ties

    def __call__(self, reads, read_off, pairs):
        """Synchronous form (evaluate(reads, read_off, pairs) of native_caller)."""
        reads = np.ascontiguousarray(reads, np.uint8)
        return self.result(self.submit(reads.ctypes.data, read_off, pairs))
