"""find_circ.py 1.99-compatible command line with the MI355X breakpoint search.

    bwa mem -t<threads> [-p] -A2 -B10 -k 15 -T 1 $GENOME_INDEX reads.fastq.gz | \\
        python -m find_circ2_amd.cli -G genome.fa -n sample -o outdir
    python -m find_circ2_amd.cli [options] <bwa_mem_genome_alignments.bam|.sam>

Same options (find_circ.py:383-413), output directory layout and file formats
(circ_splice_sites.bed, lin_splice_sites.bed, spliced_reads.fastq.gz,
multi_events.tsv, test_results.tsv, run.log; find_circ.py:420-458).
Unsupported: ``-S/--system`` (needs the absent ``byo`` library).  ``-B/--bam``
writes spliced_alignments.bam through the native ingest (not with ``--python-ingest``).  ``--stranded`` fails
exactly like the reference (AttributeError in Hit.add, find_circ.py:532-533).
"""
from __future__ import annotations

import io
import logging
import os
import sys
import time
import traceback

from .cliopts import USAGE, apply_threads, build_parser  # noqa: F401  (cli.build_parser: the tests' entry)

__version__ = "1.99"


def gpu_evaluator(genome, hp_options):
    """evaluate(spans): one batched GPU scan (read parts over MAX_READ_LEN on the long path); per-span
    results or the reference's exception (BreakpointEngine.find_breakpoints_batch)."""
    from .hotpath import BreakpointEngine
    engine = BreakpointEngine(genome, hp_options)

    def evaluate(spans):
        for s, r in zip(spans, engine.find_breakpoints_batch(spans, locus_order=True)):
            s.result = r
    return evaluate


# set by `python -m find_circ2_amd.cli`: the process ends right after main() returns, so what only
# frees memory (the junction tables, the device contexts) is left to its exit
EXIT_AFTER_MAIN = False


def process_age() -> float:
    """Seconds since this process started (/proc/self/stat starttime, clock-tick resolution): what
    interpreter start-up and imports cost before main() runs."""
    try:
        with open("/proc/self/stat") as f:
            fields = f.read().rsplit(")", 1)[1].split()
        with open("/proc/uptime") as f:
            uptime = float(f.read().split()[0])
        return max(0.0, uptime - int(fields[19]) / os.sysconf("SC_CLK_TCK"))
    except (OSError, ValueError, IndexError):
        return float("nan")


def main(argv=None, evaluator_factory=None) -> int:
    startup = {"before_main_s": process_age()}
    parser = build_parser()
    options, args = parser.parse_args(argv)
    apply_threads(options)
    if options.version:
        print("find_circ.py version {0}\n\n(c) Marvin Jens 2012-2016.\nCheck http://www.circbase.org for more "
              "information.\n(MI355X breakpoint search: find_circ2_amd)".format(__version__))
        return 0
    if not os.path.isdir(options.output):
        os.makedirs(options.output)
    log_h = logging.FileHandler(os.path.join(options.output, "run.log"), mode="w")
    log_h.setFormatter(logging.Formatter('%(asctime)-20s\t%(levelname)s\t%(name)s\t%(message)s'))
    root = logging.getLogger()
    root.handlers = [log_h]
    root.setLevel(logging.INFO)
    logger = logging.getLogger('find_circ')
    logger.info("find_circ {0} invoked as '{1}'".format(__version__, " ".join(sys.argv)))
    if options.system:
        sys.stderr.write("-S/--system needs the byo library, which is not available\n")
        return 1
    if not options.genome:
        print("need to specify either model system database (-S) or genome FASTA file (-G).")
        return 1
    if options.bam and options.python_ingest:
        sys.stderr.write("-B/--bam needs the native ingest (drop --python-ingest)\n")
        return 1
    bam_path = os.path.join(options.output, "spliced_alignments.bam") if options.bam else ""

    from .caller import Caller, CallerOptions
    from .gzout import ParallelGzipWriter
    from .hotpath import Options as HPOptions
    from .samio import AlignmentFile

    # latin-1 both ways (readers decode input bytes as latin-1): the output bytes are the input bytes,
    # as the Python-2 reference writes them
    out = {"circs": open(os.path.join(options.output, "circ_splice_sites.bed"), "w", encoding="latin-1"),
           "lins": open(os.path.join(options.output, "lin_splice_sites.bed"), "w", encoding="latin-1"),
           "reads": ParallelGzipWriter(os.path.join(options.output, "spliced_reads.fastq.gz"),
                                       threads=min(8, options.threads) if options.threads > 0 else 0),
           "multi": open(os.path.join(options.output, "multi_events.tsv"), "w", encoding="latin-1"),
           "test": open(os.path.join(options.output, "test_results.tsv"), "w", encoding="latin-1")
           if options.test else None}
    if options.stdout:
        out[options.stdout].write('# redirected to stdout\n')
        out[options.stdout].close()
        logger.info('redirected {0} to stdout'.format(options.stdout))
        out[options.stdout] = sys.stdout

    hp = HPOptions(asize=options.asize, margin=options.margin, maxdist=options.maxdist,
                   noncanonical=options.noncanonical, strandpref=options.strandpref, allhits=options.allhits)
    genome = None
    dummy_warning = lambda: logging.getLogger("GenomeAccessor").warning(        # noqa: E731
        "Could not access '%s'. Switching to dummy mode (only Ns)" % options.genome)
    python_loop = options.python_ingest or options.python_caller
    if evaluator_factory is None and python_loop:
        from . import _native as N
        from .genome import Genome
        try:
            genome = Genome.from_fasta(options.genome, device=options.device, write_index=True)
        except N.Fc2Error as ex:       # GenomeAccessor dummy mode (find_circ.py:338-345): IOError only
            if ex.code != N.FC2_E_IO:
                raise
            dummy_warning()
            genome = Genome.dummy_genome(device=options.device)
        evaluate = gpu_evaluator(genome, hp)
    elif evaluator_factory is None:
        # the native read loop's search over the torch-free C ABI (ctxpipe): the genome is indexed
        # (.byo_index read or written, find_circ.py:110-115) and made resident on each device here
        from . import prestart
        from .ctxpipe import CtxPipeline, FastaGenome
        pre = prestart.take(options)
        if pre is not None:
            # `python -m`: the FASTA opened and the contexts being built since before the imports
            # (prestart.py) -- adopted here, their errors raised here as below
            genome = FastaGenome.adopt(pre, dummy_warning)
            startup["genome_index_s"] = pre.genome_index_s
            # (only the number of devices matters here: the prestart resolved them as _devices does)
            evaluate = CtxPipeline(genome, hp, devices=[options.device] * max(1, options.gpus), prestart=pre)
        else:
            t = time.time()
            genome = FastaGenome.open_or_dummy(options.genome, dummy_warning)
            startup["genome_index_s"] = time.time() - t
            # the device genome is built on a thread of its own while the input is opened and its first
            # chunks are read (the first search waits for it); its time is logged with the phases
            evaluate = CtxPipeline(genome, hp, devices=_devices(options), background=True)
        if options.gpus > 1:
            logger.info("--gpus %d: chunks dealt round-robin over %s; the search is a few percent of the read "
                        "loop, which is bound by the host's cores (DESIGN.md §6), so more GPUs add little here"
                        % (options.gpus, ",".join(_devices(options))))
    elif python_loop:
        evaluate = evaluator_factory(options, hp)

    path = args[0] if args else "-"
    # the reference's pysam mode ('r' for stdin and *sam names, else 'rb', find_circ.py:461-469) is only a
    # hint: as htslib does, both readers detect BAM / SAM and BGZF / gzip / plain from the bytes themselves
    is_bam = bool(args) and not args[0].endswith("sam")
    logger.info('reading from {0}'.format(args[0]) if args else 'reading from stdin')
    if not (options.python_ingest or options.python_caller):
        return _run_native_caller(options, path, is_bam, out, hp, logger, evaluator_factory, genome, bam_path,
                                  genome_eval=evaluate if evaluator_factory is None else None, startup=startup)
    try:
        if options.python_ingest:
            sam = AlignmentFile(path, "rb" if is_bam else "r")
            fmt = sam.format
            run = lambda: caller.run(sam)                          # noqa: E731
        else:
            from .ingest import NativeIngest
            sam = NativeIngest(path, is_bam)
            fmt = sam.format()[0]
            if bam_path:
                sam.set_bam_out(bam_path)
            run = lambda: caller.run_native(sam)                   # noqa: E731
    except Exception:
        return _open_failed(out)
    _warn_format(logger, path, is_bam, fmt)

    cache = {}

    def chrom_of(a):                  # fast_chrom_lookup (find_circ.py:471-477)
        t = a.tid
        if t not in cache:
            if t < 0:
                raise ValueError("reference id %d out of range" % t)
            cache[t] = sam.getrname(t)
        return cache[t]

    copts = CallerOptions(**{k: getattr(options, k) for k in (
        "name", "min_uniq_qual", "asize", "margin", "maxdist", "short_threshold", "huge_threshold", "noncanonical",
        "allhits", "stranded", "strandpref", "halfunique", "report_nobridges", "throughput", "chunksize", "noop",
        "test", "nolinear", "multi_events", "debug")})
    caller = Caller(copts, evaluate, chrom_of, out, options.known_circ, options.known_lin)
    try:
        if options.profile:
            import cProfile
            prof = cProfile.Profile()
            seconds = prof.runcall(run)
            prof.print_stats()
        else:
            seconds = run()
    except KeyboardInterrupt:
        logging.warning("KeyboardInterrupt by user while processing input")
        seconds = 0.0
    except Exception:
        logging.error("Unhandled exception raised while processing input")
        exc = traceback.format_exc()
        logging.error(exc)
        sys.stderr.write(exc)
        # sys.exit(1) in the reference (find_circ.py:1583) flushes what was written so far
        for fh in out.values():
            if fh is not None and fh is not sys.stdout:
                fh.close()
        return 1
    if bam_path:
        sam.close_bam_out()
    _finish(options, seconds, caller.n_reads, logger, caller.N, caller.n_spans_evaluated, caller.gpu_seconds)
    caller.circ_splices.store(out["circs"])
    caller.linear_splices.store(out["lins"])
    for k, fh in out.items():
        if fh is not None and fh is not sys.stdout:
            fh.close()
    return 0


def _open_failed(out) -> int:
    """The input could not be opened: the reference's pysam.Samfile raises at module level
    (find_circ.py:461-469), an uncaught exception -- traceback, exit status 1."""
    logging.error("Unhandled exception raised while opening the input")
    exc = traceback.format_exc()
    logging.error(exc)
    sys.stderr.write(exc)
    for fh in out.values():
        if fh is not None and fh is not sys.stdout:
            fh.close()
    return 1


def _warn_format(logger, path, is_bam, fmt):
    """A BAM-named input (the reference opens it with mode 'rb', find_circ.py:463-466) that holds SAM
    text is read as SAM, as htslib detects the format from the bytes; noted in run.log, since an
    older pysam would have refused it."""
    if is_bam and fmt == "sam":
        logger.warning("'{0}' is not named *sam but holds SAM text: read as SAM (format detected from the "
                       "bytes, as htslib does for pysam.Samfile(path, 'rb'))".format(path))


def _finish(options, seconds, n_reads, logger, counters, n_spans, eval_seconds):
    M = n_reads / 1e6
    krps = n_reads / seconds / 1000. if seconds > 0 else 0.0
    txt = "processed {0:.2f}M (paired or single end) reads in {1:.1f} minutes (overall {2:.2f}k reads/second on " \
          "average)".format(M, seconds / 60., krps)
    logger.info(txt)
    if not options.silent and not options.stdout:
        print("#", txt)
        print("# results stored in '{0}'".format(options.output))
    logger.info('run finished')
    for key in sorted(counters):
        logger.info('{0}={1}'.format(key, counters[key]))
    logger.info('breakpoint search: {0} spans, {1:.3f} s incl. pack/transfer/decode'.format(n_spans, eval_seconds))


def _devices(options):
    """--gpus N devices starting at --device (cuda:k, cuda:k+1, ...), wrapping round the devices
    present (a 1-GPU box runs N scanners on cuda:0); the HIP runtime's count, no torch import."""
    from .ctxpipe import device_count, device_index
    if options.gpus <= 1:
        return [options.device]
    ndev = max(1, device_count())
    first = device_index(options.device)
    return ["cuda:%d" % ((first + k) % ndev) for k in range(options.gpus)]


# BAM input read before its BGZF blocks move to the GPU (DESIGN.md §5 "The BAM input inflated on the
# GPU"): a smaller input never touches the device for it, where setting it up costs more than it saves
GPU_INFLATE_AFTER = 256 << 20


def _inflate_device(options):
    """The GPU that inflates a BAM input's BGZF blocks (the first of the run's devices) and after how
    many bytes of input: by default once GPU_INFLATE_AFTER bytes were read, at once with FC2_GPU_INFLATE
    1 or 2; FC2_GPU_INFLATE=0: (None, 0), the CPU inflates every block."""
    env = os.environ.get("FC2_GPU_INFLATE")
    if env == "0":
        return None, 0
    from .ctxpipe import device_index
    return device_index(options.device), (0 if env in ("1", "2") else GPU_INFLATE_AFTER)


def _run_native_caller(options, path, is_bam, out, hp, logger, evaluator_factory, genome, bam_path="",
                       genome_eval=None, startup=None) -> int:
    """The read loop in C++ (include/fc2_caller.h); only the breakpoint search is called from here."""
    from .caller import BED_HEADER, MULTI_HEADER
    from .gzout import ParallelGzipWriter
    from .native_caller import NativeCaller
    if evaluator_factory is None:
        evaluate = genome_eval
        names, fasta, dummy = genome.names, genome.fasta, genome.dummy
    else:
        engine = getattr(evaluator_factory, "batch", None)
        if engine is None:
            raise ValueError("evaluator_factory has no batch form for the native caller (use --python-caller)")
        evaluate, names, fasta, dummy = engine(options, hp)
    reads_gz = None
    if isinstance(out.get("reads"), ParallelGzipWriter):   # compressed by the read loop itself
        w = out["reads"]
        reads_gz = (w.hand_over(), w.level, w.threads, w.piece)
    nc = NativeCaller(path, is_bam, options, names, fasta, write_reads=out.get("reads") is not None,
                      write_multi=out.get("multi") is not None, genome_dummy=dummy,
                      known_circ=options.known_circ, known_lin=options.known_lin, bam_out=bam_path,
                      reads_gz=reads_gz,
                      **(dict(zip(("inflate_device", "inflate_after"), _inflate_device(options)))
                         if genome_eval is not None else {}))
    try:
        try:
            n_kc, n_kl = nc.open()
        except Exception:
            return _open_failed(out)
        _warn_format(logger, path, is_bam, nc.format)
        for n, p in ((n_kc, options.known_circ), (n_kl, options.known_lin)):
            if p:
                logger.info("loaded {0} known splice sites from '{1}'".format(n, p))
        if out.get("multi") is not None:
            out["multi"].write(MULTI_HEADER)
        try:
            if options.profile:
                import cProfile
                prof = cProfile.Profile()
                seconds, n_reads, n_pairs, eval_s = prof.runcall(nc.run, evaluate, out, sys.stderr,
                                                                 options.throughput, options.chunksize)
                prof.print_stats()
            else:
                seconds, n_reads, n_pairs, eval_s = nc.run(evaluate, out, sys.stderr, options.throughput,
                                                           options.chunksize)
            if genome_eval is not None:
                genome_eval.wait_ready()       # no GPU, no run: fails loudly even if no span was searched
        except KeyboardInterrupt:
            logging.warning("KeyboardInterrupt by user while processing input")
            (n_reads, n_pairs), seconds, eval_s = nc.stats(), 0.0, 0.0
        except Exception:
            logging.error("Unhandled exception raised while processing input")
            exc = traceback.format_exc()
            logging.error(exc)
            sys.stderr.write(exc)
            return 1
        nc.close_bam_out()
        _finish(options, seconds, n_reads, logger, nc.counters(), n_pairs, eval_s)
        if nc.loop_profile:
            logger.info("read loop stages: " + ", ".join("%s=%.3f" % kv for kv in sorted(nc.loop_profile.items())))
        t_rows = time.time()
        for kind, key in ((0, "circs"), (1, "lins")):
            out[key].write(BED_HEADER)
            nc.write_rows(kind, out[key])
        if startup is not None:
            # the process's phases: what runs before the first record and after the last
            # (device_genome_s overlaps the start of the read loop)
            startup.update(device_genome_s=getattr(evaluate, "load_s", None) or 0.0,
                           hip_init_s=getattr(evaluate, "hip_init_s", None) or 0.0,
                           prepack_s=getattr(evaluate, "prepack_s", 0.0),
                           genome_load_s=getattr(evaluate, "genome_load_s", 0.0),
                           siblings_s=getattr(evaluate, "siblings_s", 0.0), read_loop_s=seconds,
                           genome_wait_s=getattr(evaluate, "wait_s", 0.0), tables_s=time.time() - t_rows)
            startup.update(zip(("inflate_gpu_blocks", "inflate_cpu_blocks"), nc.inflate_counts()))
            logger.info("process phases: " + ", ".join("%s=%.3f" % kv for kv in startup.items()) +
                        ", process_age_s=%.3f, numpy_loaded=%d, torch_loaded=%d"
                        % (process_age(), "numpy" in sys.modules, "torch" in sys.modules))
    finally:
        t_close = time.time()
        try:
            nc.finish_reads()
        finally:
            t_fin = time.time()
            # (the junction tables: freed by the process's exit; closed with FC2_CALLER_TIMING, whose
            # per-stage CPU totals fc2_caller_close prints)
            if not EXIT_AFTER_MAIN or os.environ.get("FC2_CALLER_TIMING"):
                nc.close()
        t_files = time.time()
        for k, fh in out.items():
            if fh is not None and fh is not sys.stdout:
                fh.close()
        t_ctx = time.time()
        if genome_eval is not None and not EXIT_AFTER_MAIN:   # the contexts, then the FASTA
            genome_eval.close()
            genome.close()
        if startup is not None and "read_loop_s" in startup:
            import resource
            logger.info("process shutdown: reads_gz_finish_s=%.3f, caller_close_s=%.3f, files_close_s=%.3f, "
                        "device_release_s=%.3f, process_age_s=%.3f, max_rss_gb=%.2f"
                        % (t_fin - t_close, t_files - t_fin, t_ctx - t_files, time.time() - t_ctx, process_age(),
                           resource.getrusage(resource.RUSAGE_SELF).ru_maxrss / 1048576.))
    return 0


if __name__ == "__main__":
    EXIT_AFTER_MAIN = True
    try:
        rc = main()
    except Exception:                   # as the interpreter reports it (traceback, status 1), but without
        traceback.print_exc()           # a finalisation that the HIP runtime could meet mid-call on the
        rc = 1                          # genome thread
    # every output is closed and flushed by now: leave without the interpreter's and the HIP runtime's
    # teardown (freeing what the process's exit releases anyway)
    logging.shutdown()
    sys.stdout.flush()
    sys.stderr.flush()
    os._exit(rc)
