"""Test-only evaluator: the CPU oracle behind the caller's ``evaluate(spans)`` hook.

Lets the whole CLI (grouping, record_hits, aggregation, writers) run on CPU
with the oracle's breakpoint search, so that (a) the host logic is tested
without a GPU and (b) on a GPU box the outputs of the GPU evaluator can be
compared file-for-file with this one.
"""
import oracle
from find_circ2_amd.hotpath import WINDOW_SHAPE_MESSAGE, BreakpointError, Splice, none_aend_error


def oracle_evaluator_factory(options, hp):
    of = oracle.OracleFasta.open_or_dummy(options.genome)     # GenomeAccessor, find_circ.py:338-345
    if of.dummy:
        _dummy_warning(options.genome)
    p = oracle.params(hp.asize, hp.margin, hp.maxdist, hp.noncanonical, hp.strandpref, hp.allhits)

    def evaluate(spans):
        idx = [0 if of.dummy else of.names.index(s.chrom) if s.chrom in of.names else -1 for s in spans]
        none_b = [s.align_B.aend is None for s in spans]
        r = oracle.scan_fasta(p, of, [s.read_part.encode("latin-1") for s in spans],
                              [-1 if nb else i for i, nb in zip(idx, none_b)],
                              [s.align_A.pos for s in spans], [s.align_B.aend or 0 for s in spans],
                              [s.is_backsplice for s in spans], [s.strand == '-' for s in spans],
                              use_fast=False, all_ties=True)
        for i, s in enumerate(spans):
            nt = int(r.n_ties[i])
            if none_b[i]:                       # A's window first (a missing chromosome), then B.aend - eff_a
                s.result = KeyError(s.chrom) if idx[i] < 0 else none_aend_error()
            elif nt == -oracle.ORC_ERR_KEY:
                s.result = KeyError("gtag")
            elif nt == -oracle.ORC_ERR_CHROM:
                s.result = KeyError(s.chrom)
            elif nt < 0:
                s.result = BreakpointError(WINDOW_SHAPE_MESSAGE)
            else:
                out = []
                for t in r.ties_of(i):
                    sp = Splice(s, s.chrom, int(t["start"]), int(t["end"]), t["strand"].decode(),
                                False if hp.maxdist == 0 else int(t["dist"]), int(t["ov"]), t["gtag"].decode())
                    sp.n_hits = int(t["n_hits"])
                    sp._score = int(t["score"])
                    out.append(sp)
                s.result = out
    return evaluate


def oracle_batch_engine(options, hp):
    """The same oracle behind the native caller's batch hook (find_circ2_amd.native_caller).

    Returns (evaluate, genome names, fc2_fasta handle, dummy): ``evaluate`` turns the
    oracle's hits back into raw ``fc2_result`` words and the ``--all-hits`` tie mask,
    the form the HIP scan hands to fc2_caller_submit (include/fc2_bp.h).
    """
    import ctypes

    import numpy as np

    from find_circ2_amd import _native as N

    of = oracle.OracleFasta.open_or_dummy(options.genome)     # GenomeAccessor, find_circ.py:338-345
    p = oracle.params(hp.asize, hp.margin, hp.maxdist, hp.noncanonical, hp.strandpref, hp.allhits)
    h = ctypes.c_void_p()
    rc = N.lib().fc2_fasta_open(options.genome.encode(), 0, ctypes.byref(h))
    assert (rc == N.FC2_E_IO) == of.dummy, (rc, of.dummy)      # the product's test of the same condition
    if of.dummy:
        _dummy_warning(options.genome)
        h = None
    else:
        N.check(rc)
    names = []
    for i in range(N.lib().fc2_fasta_n_chrom(h) if h else 0):
        nm = ctypes.c_char_p()
        N.check(N.lib().fc2_fasta_chrom(h, i, ctypes.byref(nm), None, None, None, None, None))
        names.append(nm.value.decode())
    to_oracle = np.array([of.names.index(nm) for nm in names] or [0], np.int64)   # handle index -> oracle index
    if of.dummy:
        to_oracle = np.zeros(1, np.int64)
    code = {c: i for i, c in enumerate("ACGTN")}
    rc = str.maketrans("ACGTN", "TGCAN")
    hpp = hp.params()

    def evaluate(reads, read_off, pairs):
        n = len(pairs)
        lens = pairs["read_len"].astype(np.int64)
        rp = [bytes(reads[int(o):int(o) + int(l)]) for o, l in zip(read_off, lens)]
        skip = (pairs["flags"] & N.PAIR_SKIP) != 0
        idx = np.where(skip, -1, to_oracle[np.minimum(pairs["chrom"].astype(np.int64), len(to_oracle) - 1)])
        if of.dummy:
            idx = np.where(skip, -1, 0)
        r = oracle.scan_fasta(p, of, rp, idx, pairs["a_pos"], pairs["b_aend"],
                              (pairs["flags"] & N.PAIR_BACKSPLICE) != 0, (pairs["flags"] & N.PAIR_PRIMARY_REV) != 0,
                              use_fast=False, all_ties=True)
        res = np.zeros(n, N.RESULT_DTYPE)
        res["best_x"] = -1
        info = np.full(n, N.RES_DONE, np.int64)
        rw, nw, tw = ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_uint32()
        N.check(N.lib().fc2_batch_geometry(ctypes.byref(hpp), int(lens.max()) if n else 0, ctypes.byref(rw),
                                           ctypes.byref(nw), ctypes.byref(tw)))
        tm = np.zeros((tw.value, n), np.uint64) if hp.allhits else None
        half = tw.value // 2
        for i in range(n):
            nt = int(r.n_ties[i])
            if nt == -oracle.ORC_ERR_KEY:
                info[i] |= N.RES_ERR_KEY
            elif nt == -oracle.ORC_ERR_SHAPE:
                info[i] |= N.RES_ERR_WIN
            elif nt > 0:
                f = r.first[i]
                sig = f["gtag"].decode()
                minus = f["strand"] == b"-"
                raw = sig[::-1].translate(rc) if minus else sig     # the kernel keeps the genome-strand 4-mer
                assert len(raw) == 4, raw
                res["best_x"][i] = int(f["x"])
                res["dist"][i] = max(0, int(f["dist"]))
                res["ov"][i] = int(f["ov"])
                res["n_ties"][i] = nt
                g12 = sum(code[c] << (3 * k) for k, c in enumerate(raw))
                info[i] |= (N.RES_MINUS if minus else 0) | (g12 << N.RES_GTAG_SHIFT)
                if tm is not None:
                    for t in r.ties_of(i):
                        x = int(t["x"])
                        row = (half if t["strand"] == b"-" else 0) + (x >> 6)
                        tm[row, i] |= np.uint64(1) << np.uint64(x & 63)
        res["info"] = info.astype(np.uint16)
        return res.view(np.int64), tm

    def evaluate_long(reads_ptr, lp):
        """The long path (fc2_long_pair records, include/fc2_bp.h) from the same oracle: LONG_RESULT_DTYPE
        results and the tie words laid out by fc2_long_geometry."""
        n = len(lp)
        total = int((lp["read_off"] + lp["read_len"]).max())
        buf = np.ctypeslib.as_array(ctypes.cast(reads_ptr, ctypes.POINTER(ctypes.c_uint8)), (total,))
        rp = [bytes(buf[int(o):int(o) + int(l)]) for o, l in zip(lp["read_off"], lp["read_len"])]
        skip = (lp["flags"] & N.PAIR_SKIP) != 0
        idx = np.where(skip, -1, 0 if of.dummy else to_oracle[np.minimum(lp["chrom"].astype(np.int64),
                                                                         len(to_oracle) - 1)])
        r = oracle.scan_fasta(p, of, rp, idx, lp["a_pos"], lp["b_aend"], (lp["flags"] & N.PAIR_BACKSPLICE) != 0,
                              (lp["flags"] & N.PAIR_PRIMARY_REV) != 0, use_fast=True, all_ties=True)
        toff = np.zeros(n + 1, np.uint64)
        N.check(N.lib().fc2_long_geometry(ctypes.byref(hpp), n, lp.ctypes.data, None, toff.ctypes.data))
        ties = np.zeros(int(toff[n]), np.uint64) if hp.allhits else None
        res = np.zeros(n, N.LONG_RESULT_DTYPE)
        res["best_x"] = -1
        res["info"] = N.RES_DONE
        for i in range(n):
            nt = int(r.n_ties[i])
            if nt == -oracle.ORC_ERR_KEY:
                res["info"][i] |= N.RES_ERR_KEY
            elif nt == -oracle.ORC_ERR_SHAPE:
                res["info"][i] |= N.RES_ERR_WIN
            elif nt > 0:
                f = r.first[i]
                sig = f["gtag"].decode()
                minus = f["strand"] == b"-"
                raw = sig[::-1].translate(rc) if minus else sig
                res["best_x"][i] = int(f["x"])
                res["dist"][i] = max(0, int(f["dist"]))
                res["ov"][i] = int(f["ov"])
                res["n_ties"][i] = nt
                res["info"][i] |= (N.RES_MINUS if minus else 0) | \
                    (sum(code[c] << (3 * k) for k, c in enumerate(raw)) << N.RES_GTAG_SHIFT)
                if ties is not None:
                    half = int(toff[i + 1] - toff[i]) // 2
                    for t in r.ties_of(i):
                        x = int(t["x"])
                        ties[int(toff[i]) + (half if t["strand"] == b"-" else 0) + (x >> 6)] |= \
                            np.uint64(1) << np.uint64(x & 63)
        return res, ties

    evaluate.evaluate_long = evaluate_long
    return evaluate, names, h, of.dummy


def _dummy_warning(path):
    import logging
    logging.getLogger("GenomeAccessor").warning("Could not access '%s'. Switching to dummy mode (only Ns)" % path)


oracle_evaluator_factory.batch = oracle_batch_engine


class DeferredEvaluator:
    """The oracle batch engine behind the pipelined interface (submit / result / depth) of
    find_circ2_amd.pipeline.ScanPipeline: submit only copies the chunk the native caller handed
    out (so the caller reads ahead, fc2_caller_next queueing chunks), result evaluates it."""

    def __init__(self, evaluate, depth):
        self.evaluate = evaluate
        self.depth = depth
        self.max_in_flight = 0
        self._in_flight = 0

    def submit(self, reads_ptr, read_off, pairs):
        import ctypes

        import numpy as np
        pairs = np.array(pairs, copy=True)
        off = np.array(read_off, dtype=np.uint64, copy=True)
        total = int((off + pairs["read_len"].astype(np.uint64)).max()) if len(pairs) else 0
        reads = np.zeros(total + 16, np.uint8)
        if total:
            reads[:total] = np.ctypeslib.as_array(ctypes.cast(reads_ptr, ctypes.POINTER(ctypes.c_uint8)), (total,))
        self._in_flight += 1
        self.max_in_flight = max(self.max_in_flight, self._in_flight)
        return (reads, off, pairs)

    def result(self, ticket, copy=True):
        self._in_flight -= 1
        return self.evaluate(*ticket)

    def evaluate_long(self, reads_ptr, long_pairs):
        return self.evaluate.evaluate_long(reads_ptr, long_pairs)


def pipelined_factory(depth):
    """oracle_evaluator_factory whose native-caller batch hook reads `depth` chunks ahead."""
    made = []

    def factory(options, hp):
        return oracle_evaluator_factory(options, hp)

    def batch(options, hp):
        evaluate, names, h, dummy = oracle_batch_engine(options, hp)
        ev = DeferredEvaluator(evaluate, depth)
        made.append(ev)
        return ev, names, h, dummy

    factory.batch = batch
    factory.made = made
    return factory


def compact_factory(width=4):
    """oracle_evaluator_factory whose native-caller batch hook hands each chunk's results over in a
    compact transfer form (native_caller.CompactChunk -> fc2_caller_submit_compact), packed by the
    numpy restatement of fc2_result_compact_launch's rules (tests/test_compact_results.py); canonical
    mode only -- with --non-canonical the raw words go as before."""
    from find_circ2_amd.native_caller import CompactChunk
    from test_compact_results import pack

    def factory(options, hp):
        return oracle_evaluator_factory(options, hp)

    def batch(options, hp):
        evaluate, names, h, dummy = oracle_batch_engine(options, hp)

        def ev(reads, read_off, pairs):
            res, tm = evaluate(reads, read_off, pairs)
            if hp.noncanonical:
                return res, tm
            words, esc = pack(res.view(np.int64) if hasattr(res, "view") else res, width)
            return CompactChunk(words, esc), tm
        ev.evaluate_long = evaluate.evaluate_long
        return ev, names, h, dummy

    import numpy as np
    factory.batch = batch
    return factory
