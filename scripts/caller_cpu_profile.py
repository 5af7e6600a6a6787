#!/usr/bin/env python
"""Host-side cost of the native read loop (dev tool, CPU only).

Runs the C++ read loop (fc2_caller_next / fc2_caller_submit) sequentially over a synthetic SAM on a
scaled hg19-shaped genome, with the CPU oracle behind the batch hook (tests/oracle_engine.py; its
time is excluded), and prints the seconds spent in next (ingest, process_mate, pairs) and submit
(record_hits, junction tables, writers) -- the two halves the CLI overlaps on two threads.

    python scripts/caller_cpu_profile.py [reads] [genome-scale] [--bam] [--all-hits --non-canonical ...]

--bam reads the input as a BGZF BAM.  Under scripts/prof/sampler.c the samples are tagged 1 in
fc2_caller_next, 2 in fc2_caller_submit, 3 during the search (the parse-ahead threads run on).
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "scripts"), os.path.join(ROOT, "tests")]

from cli_scale_check import make_genome, write_fasta, write_sam  # noqa: E402


def main():
    pos = [a for a in sys.argv[1:] if not a.startswith("-")]
    bam = "--bam" in sys.argv[1:]
    extra = [a for a in sys.argv[1:] if a.startswith("-") and a != "--bam"]
    reads = int(pos[0]) if pos else 200_000
    scale = float(pos[1]) if len(pos) > 1 else 0.01
    from find_circ2_amd import cli, sq_table
    from find_circ2_amd.native_caller import NativeCaller
    from oracle_engine import oracle_batch_engine
    d = "/tmp/fc2_cprof_%d_%g" % (reads, scale)
    fa, sam = os.path.join(d, "genome.fa"), os.path.join(d, "reads.sam")
    if not os.path.exists(sam):
        os.makedirs(d, exist_ok=True)
        rng = np.random.default_rng(2024)
        names, sizes = sq_table(os.path.join(ROOT, "tests", "golden", "test_norm.sam"))
        sizes = [max(1000, int(s * scale)) for s in sizes]
        seqs = make_genome(fa, names, sizes, rng)
        write_sam(sam, seqs, reads, rng)
        write_fasta(fa, seqs)
    if bam:
        from find_circ2_amd.ingest import sam_to_bam
        if not os.path.exists(sam + ".bam"):
            sam_to_bam(sam, sam + ".bam")
        sam = sam + ".bam"
    options, _ = cli.build_parser().parse_args(["-G", fa, "-o", os.path.join(d, "out"), "-n", "prof"] + extra + [sam])
    from find_circ2_amd.hotpath import Options as HPOptions
    hp = HPOptions(asize=options.asize, margin=options.margin, maxdist=options.maxdist,
                   noncanonical=options.noncanonical, strandpref=options.strandpref, allhits=options.allhits)
    evaluate, names, fasta, dummy = oracle_batch_engine(options, hp)
    nc = NativeCaller(sam, bam, options, names, fasta, write_reads=True, write_multi=True, genome_dummy=dummy)
    nc.open()

    class Sink:
        def write(self, s):
            pass
    sampler = None
    if os.environ.get("FC2_SAMPLE"):                 # scripts/prof/sampler.c: PC samples per side
        import ctypes
        sampler = ctypes.CDLL(os.environ.get("FC2_SAMPLER_LIB", "/tmp/libfc2_sampler.so"))
        sampler.sampler_start(int(os.environ.get("FC2_SAMPLE_USEC", "100")))
    t0 = time.time()
    if sampler is None:
        nc.run(evaluate, {"reads": Sink(), "multi": Sink(), "test": None}, sys.stderr, False, options.chunksize,
               threads=False)
    else:
        _sampled_loop(nc, evaluate, sampler)
    wall = time.time() - t0
    t1 = time.time()
    rows = len(nc.rows(0)) + len(nc.rows(1))
    prof = {k: round(v, 3) for k, v in nc.loop_profile.items()}
    prof.update(reads=reads, scale=scale, extra=extra, wall_s=round(wall, 2), rows_s=round(time.time() - t1, 3),
                rows_chars=rows, reads_per_s_next_plus_submit=round(reads / (prof["next_s"] + prof["submit_s"])))
    nc.close()
    if sampler is not None:
        prof["samples"] = sampler.sampler_stop(os.environ["FC2_SAMPLE"].encode())
    print(json.dumps(prof))


def _sampled_loop(nc, evaluate, sampler):
    """NativeCaller._run_sequential without read-ahead, tagging the samples: 1 next, 2 submit."""
    import ctypes
    from find_circ2_amd import _native as N
    L = N.lib()
    prof = nc.loop_profile = {"next_s": 0.0, "submit_s": 0.0, "write_s": 0.0, "eval_s": 0.0}
    eof = ctypes.c_int(0)
    while not eof.value:
        b = N.CallerBatch()
        t = time.perf_counter()
        sampler.sampler_phase(1)
        rc = L.fc2_caller_next(nc.h, ctypes.byref(b), ctypes.byref(eof))
        sampler.sampler_phase(0)
        prof["next_s"] += time.perf_counter() - t
        N.check(rc)
        n = int(b.n)
        t = time.perf_counter()
        sampler.sampler_phase(3)
        res, tm = evaluate(*nc._host_batch(b, n)) if n else (None, None)
        sampler.sampler_phase(0)
        prof["eval_s"] += time.perf_counter() - t
        res_ptr = tm_ptr = None
        tw = 0
        if n:
            res = np.ascontiguousarray(res, dtype=np.int64)
            res_ptr = res.ctypes.data
            if tm is not None:
                tm = np.ascontiguousarray(tm, dtype=np.uint64)
                tw, tm_ptr = tm.shape[0], tm.ctypes.data
        t = time.perf_counter()
        sampler.sampler_phase(2)
        rc = L.fc2_caller_submit(nc.h, res_ptr, tm_ptr, tw, n)
        sampler.sampler_phase(0)
        prof["submit_s"] += time.perf_counter() - t
        N.check(rc)
        t = time.perf_counter()
        for k in range(3):
            nc._take(k)
        prof["write_s"] += time.perf_counter() - t


if __name__ == "__main__":
    main()
