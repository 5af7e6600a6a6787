#!/usr/bin/env python
"""End-to-end CLI throughput (host-bound; reported separately from the kernel metric).

Writes a seeded synthetic genome FASTA and a bwa-mem-shaped SAM of single-end
reads (a mix of unspliced, linear-spliced and backspliced 100 bp reads with
known segment coordinates), then runs ``python -m find_circ2_amd.cli`` on it and
reports reads/s plus the time spent in the batched breakpoint search.

usage: python scripts/cli_throughput.py [--reads N] [--genome-mb M] [--frac-spliced F] [--out DIR]
                                       [--mode native|python-caller|python-ingest ...] [--null-eval]

``--mode`` picks the read loop (C++ caller by default; several modes run one after
the other on the same input).  ``--null-eval`` replaces the breakpoint search by
"no hit" results, which times the host loop alone (runs without a GPU).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def write_genome(path, n_chrom, size, rng):
    seqs = {}
    with open(path, "w") as f:
        for c in range(n_chrom):
            s = np.frombuffer(b"ACGT", np.uint8)[rng.integers(0, 4, size)].tobytes().decode()
            name = "chr%d" % (c + 1)
            seqs[name] = s
            f.write(">%s\n" % name)
            for k in range(0, size, 60):
                f.write(s[k:k + 60] + "\n")
    return seqs


def write_sam(path, seqs, n_reads, frac_spliced, L, rng):
    names = list(seqs)
    with open(path, "w") as f:
        f.write("@HD\tVN:1.5\n")
        for n in names:
            f.write("@SQ\tSN:%s\tLN:%d\n" % (n, len(seqs[n])))
        for i in range(n_reads):
            ci = int(rng.integers(len(names)))
            chrom, g = names[ci], seqs[names[ci]]
            G = len(g)
            q = "I" * L
            if rng.random() >= frac_spliced:
                p = int(rng.integers(0, G - L))
                f.write("u%d\t0\t%s\t%d\t60\t%dM\t*\t0\t0\t%s\t%s\tNM:i:0\tAS:i:%d\n" % (i, chrom, p + 1, L, g[p:p + L],
                                                                                     q, L))
                continue
            kA = int(rng.integers(20, L - 20))
            kB = L - kA
            span = int(rng.integers(200, 5000))
            if rng.random() < 0.5:          # backsplice: A = G[end-kA:end], B = G[start:start+kB]
                end = int(rng.integers(span + kA, G - 10))
                start = end - span
                read = g[end - kA:end] + g[start:start + kB]
                a_pos, b_pos = end - kA, start
            else:                           # linear: A = G[d-kA:d], B = G[a:a+kB]
                d = int(rng.integers(kA, G - span - kB - 10))
                a = d + span
                read = g[d - kA:d] + g[a:a + kB]
                a_pos, b_pos = d - kA, a
            if kA >= kB:
                f.write("s%d\t0\t%s\t%d\t60\t%dM%dS\t*\t0\t0\t%s\t%s\tNM:i:0\tAS:i:%d\n" % (i, chrom, a_pos + 1, kA, kB,
                                                                                        read, q, kA))
                f.write("s%d\t2048\t%s\t%d\t60\t%dH%dM\t*\t0\t0\t%s\t*\tNM:i:0\tAS:i:%d\n" % (i, chrom, b_pos + 1, kA,
                                                                                          kB, read[kA:], kB))
            else:
                f.write("s%d\t0\t%s\t%d\t60\t%dS%dM\t*\t0\t0\t%s\t%s\tNM:i:0\tAS:i:%d\n" % (i, chrom, b_pos + 1, kA, kB,
                                                                                        read, q, kB))
                f.write("s%d\t2048\t%s\t%d\t60\t%dM%dH\t*\t0\t0\t%s\t*\tNM:i:0\tAS:i:%d\n" % (i, chrom, a_pos + 1, kA,
                                                                                          kB, read[:kA], kA))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reads", type=int, default=200_000)
    ap.add_argument("--genome-mb", type=int, default=20)
    ap.add_argument("--frac-spliced", type=float, default=0.3)
    ap.add_argument("--out", default="/tmp/fc2_cli_tp")
    ap.add_argument("--mode", action="append", choices=["native", "python-caller", "python-ingest"])
    ap.add_argument("--null-eval", action="store_true")
    a = ap.parse_args()
    os.makedirs(a.out, exist_ok=True)
    rng = np.random.default_rng(27)
    fa = os.path.join(a.out, "genome.fa")
    sam = os.path.join(a.out, "reads.sam")
    t0 = time.time()
    seqs = write_genome(fa, 4, a.genome_mb * 250_000, rng)
    write_sam(sam, seqs, a.reads, a.frac_spliced, 100, rng)
    t_gen = time.time() - t0
    from find_circ2_amd import cli
    factory = null_factory if a.null_eval else None
    for mode in a.mode or ["native"]:
        flag = [] if mode == "native" else ["--" + mode]
        run = os.path.join(a.out, "run_" + mode)
        t0 = time.time()
        rc = cli.main(["-G", fa, "-o", run, "-n", "tp", "-q"] + flag + [sam], evaluator_factory=factory)
        wall = time.time() - t0
        log = open(os.path.join(run, "run.log")).read()
        bp = [l for l in log.splitlines() if "breakpoint search:" in l]
        circ = sum(1 for l in open(os.path.join(run, "circ_splice_sites.bed")) if not l.startswith("#"))
        print(json.dumps({"mode": mode, "null_eval": a.null_eval, "rc": rc, "reads": a.reads,
                          "frac_spliced": a.frac_spliced, "wall_s": round(wall, 2),
                          "reads_per_s": round(a.reads / wall, 1), "gen_s": round(t_gen, 1),
                          "breakpoint_search": bp[-1].split("\t")[-1] if bp else None, "circ_rows": circ}), flush=True)


def null_factory(options, hp):
    """Breakpoint search stub: every span "no hit" (host-loop timing only)."""
    def evaluate(spans):
        for s in spans:
            s.result = []
    return evaluate


def _null_batch(options, hp):
    from find_circ2_amd import _native as N
    names = [l[1:].split()[0] for l in open(options.genome) if l.startswith(">")]

    def evaluate(reads, read_off, pairs):
        res = np.zeros(len(pairs), N.RESULT_DTYPE)
        res["best_x"] = -1
        res["info"] = N.RES_DONE
        tw = 2 * ((int(pairs["read_len"].max()) + 64) // 64) if len(pairs) else 2
        tm = np.zeros((tw, len(pairs)), np.uint64) if hp.allhits else None
        return res.view(np.int64), tm
    return evaluate, names, None, False


null_factory.batch = _null_batch


if __name__ == "__main__":
    main()
