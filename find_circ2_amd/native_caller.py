"""Driver of the native read loop (include/fc2_caller.h, fc2_caller.cpp).

The C++ side reads the alignments, forms the anchor pairs, and runs
``record_hits`` / the junction tables / the writers of find_circ.py 1.99 (the
same logic as :mod:`find_circ2_amd.caller`, which stays as the reference path
behind ``--python-caller``).  This module moves the pairs of each chunk to the
breakpoint search and the results back, writes the text the C++ side produced,
and turns its errors into the exceptions the reference raises.

``evaluate(reads, read_off, pairs) -> (results, tiemask)``: ``pairs`` is a
``PAIR_DTYPE`` array (chrom = genome index), ``results`` the raw ``fc2_result``
words (int64 [n]) in the same order, ``tiemask`` uint64 [tw, n] with
``--all-hits`` (else None).  :func:`gpu_batch_evaluator` is the MI355X one.
"""
from __future__ import annotations

import ctypes
import sys
import time
import queue
import threading
from collections import deque
from typing import Callable, Dict, NamedTuple, Optional

from ._lazy import LazyModule

np = LazyModule("numpy", globals(), "np")

from . import _native as N
from .hotpath import BreakpointError

_EXC = {"KeyError": KeyError, "TypeError": TypeError, "ValueError": ValueError, "AttributeError": AttributeError,
        "IndexError": IndexError, "IOError": OSError, "BreakpointError": BreakpointError,
        "UnboundLocalError": UnboundLocalError}


def _raise_native(rc: int):
    msg = N.lib().fc2_last_error()
    msg = msg.decode("utf-8", "replace") if msg else ""
    kind, _, rest = msg.partition(": ")
    exc = _EXC.get(kind)
    if exc is None:
        raise N.Fc2Error(rc, msg)
    if exc is KeyError and rest.startswith("'") and rest.endswith("'"):
        raise KeyError(rest[1:-1])
    raise exc(rest)


def _check(rc: int):
    if rc != N.FC2_OK:
        _raise_native(rc)


def gpu_batch_evaluator(genome, hp, devices=None, n_threads: int = 0):
    """The MI355X evaluator of the native read loop: a ScanPipeline (pinned staging, one side
    stream per device, chunks dealt round-robin over ``devices``, results in input order).  It
    has ``submit``/``result`` (NativeCaller.run reads ahead with them) and is callable as a plain
    synchronous ``evaluate(reads, read_off, pairs)``."""
    from .pipeline import ScanPipeline
    return ScanPipeline(genome, hp, devices=devices, n_threads=n_threads)



class CompactChunk(NamedTuple):
    """A chunk's results in a compact transfer form (include/fc2_bp.h "compact results"): words [n]
    (a 4- or 2-byte dtype: the width) and the escapes (N.ESCAPE_DTYPE, indices into the chunk)."""
    words: np.ndarray
    escapes: np.ndarray

class NativeCaller:
    """One pass over an alignment file (path or '-') with the native read loop."""

    def __init__(self, path: str, is_bam: bool, copts, genome_names, fasta_handle=None, write_reads=True,
                 write_multi=True, genome_dummy=False, known_circ: str = "", known_lin: str = "",
                 bam_out: str = "", reads_gz=None, inflate_device=None, inflate_after: int = 0):
        o = copts
        # the strings must outlive the handle's open call (fc2_caller_open copies them)
        self._keep = [o.name.encode(), known_circ.encode() if known_circ else None,
                      known_lin.encode() if known_lin else None]
        self.opts = N.CallerOpts(
            self._keep[0], self._keep[1], self._keep[2], int(o.min_uniq_qual), int(o.asize), int(o.margin),
            int(o.maxdist), int(o.short_threshold), int(o.huge_threshold), int(bool(o.noncanonical)),
            int(bool(o.allhits)), int(bool(o.stranded)), int(bool(o.strandpref)), int(bool(o.halfunique)),
            int(bool(o.report_nobridges)), int(bool(o.test)), int(bool(o.nolinear)), int(bool(o.multi_events)),
            int(bool(o.noop)), int(bool(write_reads)), int(bool(write_multi)), 0, int(o.chunksize))
        self.h = ctypes.c_void_p()
        self.genome_names = list(genome_names or [])
        self.genome_dummy = genome_dummy
        self.fasta_handle = fasta_handle
        self._path = path
        self._is_bam = is_bam
        self.bam_out = bam_out
        self.reads_gz = reads_gz     # (path, level, threads, piece): spliced_reads.fastq.gz written natively
        self.inflate_device = inflate_device   # a BGZF input's blocks inflated on this GPU (None: the CPU)
        self.inflate_after = inflate_after     # ... once this many bytes of the input were read
        self.opened = False
        self.format = None           # "sam" | "bam", detected from the bytes (open)
        self.loop_profile = {}       # seconds per stage of the last run (two-thread loop)

    def open(self):
        """Open the input, map its reference ids to genome indices, load the known sites.

        Returns (#known circ sites, #known linear sites)."""
        L = N.lib()
        _check(L.fc2_caller_open(self._path.encode(), 1 if self._is_bam else 0, ctypes.byref(self.opts),
                                 ctypes.byref(self.h)))
        self.opened = True
        ing = L.fc2_caller_ingest(self.h)
        self.format = "bam" if L.fc2_ingest_format(ing, None) == 1 else "sam"      # FC2_INGEST_BAM
        if self.bam_out:
            N.check(L.fc2_ingest_set_bam_out(ing, self.bam_out.encode()))
        if self.inflate_device is not None:
            N.check(L.fc2_ingest_set_gpu_inflate_from(ing, int(self.inflate_device), int(self.inflate_after)))
        if self.reads_gz:
            path, level, threads, piece = self.reads_gz
            N.check(L.fc2_caller_set_reads_gz(self.h, path.encode(), int(level), int(threads), int(piece)))
        n_ref = L.fc2_ingest_n_refs(ing)
        self.refs = [L.fc2_ingest_ref_name(ing, t).decode("latin-1") for t in range(n_ref)]
        index = {nm: k for k, nm in enumerate(self.genome_names)}
        if self.genome_dummy:             # every window is all 'N'; no chromosome is missing
            vals = [0] * max(1, n_ref)
        else:
            vals = [index.get(nm, -1) for nm in self.refs] or [-1]
        t2c = (ctypes.c_int32 * len(vals))(*vals)
        self._t2c = t2c
        nkc, nkl = ctypes.c_uint64(), ctypes.c_uint64()
        _check(L.fc2_caller_set_genome(self.h, ctypes.addressof(t2c), n_ref, self.fasta_handle, ctypes.byref(nkc),
                                       ctypes.byref(nkl)))
        return int(nkc.value), int(nkl.value)

    def close_bam_out(self):
        """Finish spliced_alignments.bam (EOF block); raises on a write error."""
        if self.bam_out:
            N.check(N.lib().fc2_ingest_close_bam_out(N.lib().fc2_caller_ingest(self.h)))

    def inflate_counts(self):
        """(BGZF blocks inflated on the GPU, on the CPU) since the GPU inflate was set (0, 0 without)."""
        g, c = ctypes.c_uint64(), ctypes.c_uint64()
        N.check(N.lib().fc2_caller_inflate_counts(self.h, ctypes.byref(g), ctypes.byref(c)))
        return int(g.value), int(c.value)

    def stats(self):
        nr, npairs = ctypes.c_uint64(), ctypes.c_uint64()
        N.check(N.lib().fc2_caller_stats(self.h, ctypes.byref(nr), ctypes.byref(npairs)))
        return int(nr.value), int(npairs.value)

    def finish_reads(self):
        """Compress and write the rest of spliced_reads.fastq.gz (when written natively)."""
        if self.opened and self.reads_gz:
            N.check(N.lib().fc2_caller_close_reads(self.h))

    def close(self):
        if self.opened:
            N.lib().fc2_caller_close(self.h)
            self.opened = False

    def _take(self, stream: int) -> str:
        t, n = ctypes.c_void_p(), ctypes.c_uint64()
        N.check(N.lib().fc2_caller_take(self.h, stream, ctypes.byref(t), ctypes.byref(n)))
        return ctypes.string_at(t.value, n.value).decode("latin-1") if n.value else ""

    def _write_outputs(self, outputs: Dict):
        for k, key in ((0, "reads"), (1, "multi"), (2, "test")):
            txt = self._take(k)
            if txt and outputs.get(key) is not None:
                outputs[key].write(txt)

    def run(self, evaluate, outputs: Dict, stderr=sys.stderr, throughput=False, chunksize=100000, threads=None):
        """Process the whole input; returns (seconds, n_reads, n_pairs, evaluate_seconds).

        By default (``threads`` None/True, no -B/--bam) the loop runs on two threads: a reader
        thread forms chunks (``fc2_caller_next``: ingest, process_mate, the pairs) and queues their
        search, while this thread records them in input order (``fc2_caller_submit``: record_hits,
        tables, writers) -- the two halves of the reference's per-fragment loop overlap, and the
        outputs are those of the sequential loop (``_run_sequential``, used with -B, where records
        are written while reading, or ``threads=False``).
        """
        if self.bam_out or threads is False:
            return self._run_sequential(evaluate, outputs, stderr, throughput, chunksize)
        return self._run_threaded(evaluate, outputs, stderr, throughput, chunksize)

    def _run_threaded(self, evaluate, outputs: Dict, stderr, throughput, chunksize):
        L = N.lib()
        t0 = time.time()
        pipelined = hasattr(evaluate, "submit") and hasattr(evaluate, "result")
        pointers = pipelined and hasattr(evaluate, "submit_ptr")
        depth = min(max(2, int(getattr(evaluate, "depth", 2))), N.CALLER_MAX_QUEUED)
        q: "queue.Queue" = queue.Queue()
        # at most `depth` chunks between being handed out and being recorded: a ScanPipeline slot is
        # only reused once its chunk's results were taken
        slots = threading.Semaphore(depth)
        stop = threading.Event()
        eval_s = [0.0, 0.0]                  # reader (pack/queue), recorder (waits for results)

        def reader():
            try:
                while True:
                    slots.acquire()
                    if stop.is_set():
                        return
                    batch = N.CallerBatch()
                    eof_c = ctypes.c_int(0)
                    tn = time.perf_counter()
                    rc = L.fc2_caller_next(self.h, ctypes.byref(batch), ctypes.byref(eof_c))
                    self.loop_profile["next_s"] += time.perf_counter() - tn
                    if rc != N.FC2_OK:
                        try:
                            _raise_native(rc)           # fc2_last_error is per thread: read it here
                        except Exception as ex:
                            q.put(("err", ex, 0, None))
                        return
                    n = int(batch.n)
                    te = time.perf_counter()
                    if not n:
                        item = None
                    elif pointers:          # (ctxpipe: the chunk's own memory, no numpy in the process)
                        item = evaluate.submit_ptr(batch.reads, batch.read_off, batch.pairs, n)
                    elif pipelined:
                        pairs = np.ctypeslib.as_array(ctypes.cast(batch.pairs, ctypes.POINTER(ctypes.c_uint8)),
                                                      (16 * n,)).view(N.PAIR_DTYPE)
                        off = np.ctypeslib.as_array(ctypes.cast(batch.read_off, ctypes.POINTER(ctypes.c_uint64)),
                                                    (n,))
                        item = evaluate.submit(batch.reads, off, pairs)
                    else:
                        item = evaluate(*self._host_batch(batch, n))
                    litem = self._eval_long(evaluate, batch)
                    eval_s[0] += time.perf_counter() - te
                    q.put(("chunk", item, n, litem))
                    if eof_c.value:
                        q.put(("eof", None, 0, None))
                        return
            except BaseException as ex:         # noqa: BLE001 -- handed to the recording thread
                q.put(("err", ex, 0, None))

        self.loop_profile = {"next_s": 0.0, "queue_wait_s": 0.0, "submit_s": 0.0, "write_s": 0.0}
        th = threading.Thread(target=reader, name="fc2-reader", daemon=True)
        th.start()
        t_last, last_reads = t0, 0
        try:
            while True:
                tq = time.perf_counter()
                kind, item, n, litem = q.get()
                self.loop_profile["queue_wait_s"] += time.perf_counter() - tq
                if kind == "err":
                    raise item
                if kind == "eof":
                    break
                res = tm = None
                if n:
                    te = time.perf_counter()
                    res, tm = evaluate.result(item, copy=False) if pipelined else item
                    eval_s[1] += time.perf_counter() - te
                ts = time.perf_counter()
                rc = self._submit_long(L, litem)
                if rc == N.FC2_OK:
                    rc = self._submit(L, res, tm, n)
                tw_ = time.perf_counter()
                self._write_outputs(outputs)
                self.loop_profile["submit_s"] += tw_ - ts
                self.loop_profile["write_s"] += time.perf_counter() - tw_
                slots.release()
                if rc != N.FC2_OK:
                    _raise_native(rc)
                if throughput:
                    nr, npairs = ctypes.c_uint64(), ctypes.c_uint64()
                    L.fc2_caller_stats(self.h, ctypes.byref(nr), ctypes.byref(npairs))
                    if nr.value // chunksize > last_reads // chunksize:
                        t1 = time.time()
                        stderr.write("\rprocessed {0:.1f}M (paired-end) reads in {1:.1f} minutes ({2:.2f}k "
                                     "reads/second)       \r".format(nr.value / 1e6, (t1 - t0) / 60.,
                                                                   (nr.value - last_reads) / max(t1 - t_last, 1e-9)
                                                                   / 1000.))
                        t_last, last_reads = t1, nr.value
        finally:
            stop.set()
            slots.release()                     # a reader blocked on the semaphore sees `stop`
            th.join()
        if throughput:
            stderr.write('\n')
        self.loop_profile.update(eval_pack_s=eval_s[0], eval_wait_s=eval_s[1])
        nr, npairs = ctypes.c_uint64(), ctypes.c_uint64()
        L.fc2_caller_stats(self.h, ctypes.byref(nr), ctypes.byref(npairs))
        return time.time() - t0, int(nr.value), int(npairs.value), eval_s[0] + eval_s[1]

    def _run_sequential(self, evaluate, outputs: Dict, stderr=sys.stderr, throughput=False, chunksize=100000):
        """One thread; reads ahead up to the evaluator's depth (none with -B/--bam).

        ``evaluate`` is either a plain ``evaluate(reads, read_off, pairs) -> (results, tiemask)``
        or a pipelined evaluator with ``submit(reads_ptr, read_off, pairs) -> ticket``,
        ``result(ticket)`` and ``depth`` (pipeline.ScanPipeline): then the loop reads up to
        ``depth`` chunks ahead (fc2_caller_next queues them) so the search of chunk k runs on the
        GPU while the host forms chunk k+1; results are still submitted in input order.  With
        -B/--bam (records written while reading) it does not read ahead: the reference stops
        writing at a failing fragment.  ``evaluate_seconds``: host time spent packing, queueing
        and waiting for the search."""
        L = N.lib()
        t0 = time.time()
        t_last, last_reads = t0, 0
        eval_s = 0.
        pipelined = hasattr(evaluate, "submit") and hasattr(evaluate, "result")
        depth = min(max(1, int(getattr(evaluate, "depth", 1))), N.CALLER_MAX_QUEUED) if pipelined and not self.bam_out else 1
        queue = deque()                      # (ticket or (results, tiemask), n) in input order
        eof = False
        deferred = None                      # an error of fc2_caller_next, raised after the queued chunks
        eof_c = ctypes.c_int(0)
        prof = self.loop_profile = {"next_s": 0.0, "submit_s": 0.0, "write_s": 0.0}
        while True:
            while not eof and deferred is None and len(queue) < depth:
                batch = N.CallerBatch()
                tn = time.perf_counter()
                rc = L.fc2_caller_next(self.h, ctypes.byref(batch), ctypes.byref(eof_c))
                prof["next_s"] += time.perf_counter() - tn
                if rc != N.FC2_OK:
                    try:
                        _raise_native(rc)
                    except Exception as ex:   # the reference reaches the queued fragments first
                        deferred = ex
                    break
                eof = bool(eof_c.value)
                n = int(batch.n)
                te = time.perf_counter()
                if not n:
                    item = (None, None)
                elif pipelined and hasattr(evaluate, "submit_ptr"):
                    item = evaluate.submit_ptr(batch.reads, batch.read_off, batch.pairs, n)
                elif pipelined:
                    pairs = np.ctypeslib.as_array(ctypes.cast(batch.pairs, ctypes.POINTER(ctypes.c_uint8)),
                                                  (16 * n,)).view(N.PAIR_DTYPE)
                    off = np.ctypeslib.as_array(ctypes.cast(batch.read_off, ctypes.POINTER(ctypes.c_uint64)), (n,))
                    item = evaluate.submit(batch.reads, off, pairs)
                else:
                    item = evaluate(*self._host_batch(batch, n))
                litem = self._eval_long(evaluate, batch)
                eval_s += time.perf_counter() - te
                queue.append((item, n, litem))
            if not queue:
                break
            item, n, litem = queue.popleft()
            res = tm = None
            if n:
                te = time.perf_counter()
                res, tm = evaluate.result(item, copy=False) if pipelined else item   # consumed by submit below
                eval_s += time.perf_counter() - te
            ts = time.perf_counter()
            rc = self._submit_long(L, litem)
            if rc == N.FC2_OK:
                rc = self._submit(L, res, tm, n)
            tw_ = time.perf_counter()
            self._write_outputs(outputs)        # what record_hits wrote before any failure
            prof["submit_s"] += tw_ - ts
            prof["write_s"] += time.perf_counter() - tw_
            if rc != N.FC2_OK:
                _raise_native(rc)
            if throughput:
                nr, npairs = ctypes.c_uint64(), ctypes.c_uint64()
                L.fc2_caller_stats(self.h, ctypes.byref(nr), ctypes.byref(npairs))
                if nr.value // chunksize > last_reads // chunksize:
                    t1 = time.time()
                    stderr.write("\rprocessed {0:.1f}M (paired-end) reads in {1:.1f} minutes ({2:.2f}k "
                                 "reads/second)       \r".format(nr.value / 1e6, (t1 - t0) / 60.,
                                                               (nr.value - last_reads) / max(t1 - t_last, 1e-9)
                                                               / 1000.))
                    t_last, last_reads = t1, nr.value
        if deferred is not None:
            raise deferred
        if throughput:
            stderr.write('\n')
        prof["eval_s"] = eval_s
        nr, npairs = ctypes.c_uint64(), ctypes.c_uint64()
        L.fc2_caller_stats(self.h, ctypes.byref(nr), ctypes.byref(npairs))
        return time.time() - t0, int(nr.value), int(npairs.value), eval_s

    @staticmethod
    def _eval_long(evaluate, batch):
        """The chunk's pairs with read parts over MAX_READ_LEN (fc2_caller_batch.long_pairs), evaluated
        at once by the evaluator's long path: (results LONG_RESULT_DTYPE, tie words or None), or None."""
        n_long = int(batch.n_long)
        if not n_long:
            return None
        ev = getattr(evaluate, "evaluate_long", None)
        if ev is None:
            raise RuntimeError("the evaluator has no long path for read parts over %d bases" % N.MAX_READ_LEN)
        lp = np.ctypeslib.as_array(ctypes.cast(batch.long_pairs, ctypes.POINTER(ctypes.c_uint8)),
                                   (N.LONG_PAIR_DTYPE.itemsize * n_long,)).view(N.LONG_PAIR_DTYPE).copy()
        return ev(batch.reads, lp)

    def _submit_long(self, L, litem):
        """fc2_caller_submit_long of a chunk's long-pair results (before its fc2_caller_submit)."""
        if litem is None:
            return N.FC2_OK
        res, ties = litem
        res = np.ascontiguousarray(res, N.LONG_RESULT_DTYPE)
        t_ptr, nt = None, 0
        if ties is not None:
            ties = np.ascontiguousarray(ties, np.uint64)
            t_ptr, nt = (ties.ctypes.data if len(ties) else None), len(ties)
        return L.fc2_caller_submit_long(self.h, res.ctypes.data, len(res), t_ptr, nt)

    def _submit(self, L, res, tm, n):
        """fc2_caller_submit of one chunk's results: raw 8-byte words, or a CompactChunk (a compact
        transfer form, fc2_caller_submit_compact); tm = the --all-hits tie mask [tw, n] or None."""
        tm_ptr, tw = None, 0
        if isinstance(res, ctypes.Array):           # ctxpipe.submit_ptr: words in a ctypes buffer
            return L.fc2_caller_submit(self.h, ctypes.addressof(res) if n else None, None, 0, n)
        if tm is not None:
            tm = np.ascontiguousarray(tm, dtype=np.uint64)
            tw = tm.shape[0]
            tm_ptr = tm.ctypes.data
        if isinstance(res, CompactChunk):
            words = np.ascontiguousarray(res.words)
            esc = np.ascontiguousarray(res.escapes, dtype=N.ESCAPE_DTYPE)
            return L.fc2_caller_submit_compact(self.h, words.ctypes.data if n else None, words.dtype.itemsize,
                                               len(words), esc.ctypes.data if len(esc) else None, len(esc), tm_ptr,
                                               tw, n)
        res_ptr = None
        if n:
            res = np.ascontiguousarray(res, dtype=np.int64)
            res_ptr = res.ctypes.data
        return L.fc2_caller_submit(self.h, res_ptr, tm_ptr, tw, n)

    @staticmethod
    def _host_batch(batch, n):
        """(reads, read_off, pairs) numpy copies of a handed-out chunk for a plain evaluator."""
        pairs = np.ctypeslib.as_array(ctypes.cast(batch.pairs, ctypes.POINTER(ctypes.c_uint8)),
                                      (16 * n,)).view(N.PAIR_DTYPE).copy()
        off = np.ctypeslib.as_array(ctypes.cast(batch.read_off, ctypes.POINTER(ctypes.c_uint64)), (n,)).copy()
        total = int((off + pairs["read_len"].astype(np.uint64)).max())
        reads = np.zeros(total + 16, np.uint8)          # zero tail: the packer reads whole words
        if total:
            reads[:total] = np.ctypeslib.as_array(ctypes.cast(batch.reads, ctypes.POINTER(ctypes.c_uint8)), (total,))
        return reads, off, pairs

    def counters(self) -> Dict[str, float]:
        L = N.lib()
        out = {}
        k = 0
        nm, v = ctypes.c_char_p(), ctypes.c_double()
        while L.fc2_caller_counter(self.h, k, ctypes.byref(nm), ctypes.byref(v)) == N.FC2_OK:
            out[nm.value.decode()] = float(v.value)
            k += 1
        return out

    def rows(self, kind: int) -> str:
        return self.rows_bytes(kind).decode("latin-1")

    def write_rows(self, kind: int, fh) -> int:
        """The BED rows written straight into the open file fh (flushed first; the rows go to its
        descriptor from the native workers, never through Python).  Falls back to rows_bytes for an
        object without a descriptor."""
        try:
            fd = fh.fileno()
        except (AttributeError, OSError, ValueError):
            fd = -1
        if fd < 0:
            data = self.rows_bytes(kind)
            buf = getattr(fh, "buffer", None)
            if buf is None:
                fh.write(data.decode("latin-1"))
            else:
                fh.flush()
                buf.write(data)
            return len(data)
        fh.flush()
        n = ctypes.c_uint64()
        N.check(N.lib().fc2_caller_write_rows(self.h, kind, fd, ctypes.byref(n)))
        return n.value

    def rows_bytes(self, kind: int) -> bytes:
        """The BED rows as the bytes written (the input's bytes: latin-1 both ways)."""
        t, n = ctypes.c_void_p(), ctypes.c_uint64()
        N.check(N.lib().fc2_caller_rows(self.h, kind, ctypes.byref(t), ctypes.byref(n)))
        return ctypes.string_at(t.value, n.value) if n.value else b""
