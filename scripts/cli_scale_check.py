#!/usr/bin/env python
"""End-to-end check at genome scale: the default CLI (C++ read loop + HIP scan) against the
Python read loop (--python-caller, same HIP scan) on an hg19-sized synthetic genome.

Writes an hg19-shaped FASTA (93 contigs of tests/golden/test_norm.sam, 50-nt lines, N runs)
with GT/AG (or CT/AC) planted at every simulated junction, and a bwa-mem-shaped SAM of
single-end 100-bp reads (unspliced, linear and backspliced; mismatches; AS/XS), then
runs both loops and requires byte-identical output files and identical run.log counters.
Prints one JSON line with both wall times.

usage: python scripts/cli_scale_check.py [--reads N] [--scale F] [--out DIR]
"""
import argparse
import gzip
import json
import os
import re
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def make_genome(path, names, sizes, rng, width=50):
    acgt = np.frombuffer(b"ACGT", np.uint8)
    seqs = {}
    for name, size in zip(names, sizes):
        s = acgt[rng.integers(0, 4, size, dtype=np.uint8)]
        for _ in range(max(1, size // 2_000_000)):
            a = int(rng.integers(0, size))
            s[a:a + int(rng.integers(1000, 140_000))] = ord("N")
        seqs[name] = s
    return seqs


def write_fasta(path, seqs, width=50):
    with open(path, "wb") as f:
        for name, s in seqs.items():
            f.write(b">" + name.encode() + b"\n")
            full = len(s) // width
            f.write(np.concatenate([s[:full * width].reshape(full, width),
                                    np.full((full, 1), 10, np.uint8)], axis=1).tobytes())
            if len(s) % width:
                f.write(s[full * width:].tobytes() + b"\n")


def write_sam(path, seqs, n, rng, L=100):
    names = [k for k in seqs if len(seqs[k]) > 200_000]
    w = np.array([len(seqs[k]) for k in names], np.float64)
    w /= w.sum()
    out = ["@HD\tVN:1.5"] + ["@SQ\tSN:%s\tLN:%d" % (k, len(v)) for k, v in seqs.items()]
    q = "I" * L

    def piece(g, a, b):
        return g[a:b].tobytes().decode()

    for i in range(n):
        c = names[int(rng.choice(len(names), p=w))]
        g = seqs[c]
        G = len(g)
        kind = rng.random()
        if kind < 0.6:
            p = int(rng.integers(0, G - L))
            out.append("u%d\t0\t%s\t%d\t60\t%dM\t*\t0\t0\t%s\t%s\tAS:i:%d\tXS:i:%d"
                       % (i, c, p + 1, L, piece(g, p, p + L), q, L, int(rng.integers(0, 40))))
            continue
        kA = int(rng.integers(20, L - 20))
        span = int(rng.integers(200, 20000))
        minus = rng.random() < 0.5
        if kind < 0.8:                                 # backsplice: A = G[E-kA:E], B = G[S:S+kB]
            E = int(rng.integers(span + kA + 10, G - 10))
            S = E - span
            g[E:E + 2] = np.frombuffer(b"CT" if minus else b"GT", np.uint8)
            g[S - 2:S] = np.frombuffer(b"AC" if minus else b"AG", np.uint8)
            a_pos, b_pos = E - kA, S
        else:                                          # linear: A = G[D-kA:D], B = G[D+span:...]
            D = int(rng.integers(kA + 10, G - span - L - 10))
            g[D:D + 2] = np.frombuffer(b"CT" if minus else b"GT", np.uint8)
            g[D + span - 2:D + span] = np.frombuffer(b"AC" if minus else b"AG", np.uint8)
            a_pos, b_pos = D - kA, D + span
        read = bytearray(g[a_pos:a_pos + kA].tobytes() + g[b_pos:b_pos + L - kA].tobytes())
        if rng.random() < 0.3:
            k = int(rng.integers(L))
            read[k] = ord("ACGT"[(("ACGT".find(chr(read[k])) + 1) % 4)]) if chr(read[k]) in "ACGT" else read[k]
        read = read.decode()
        xs = int(rng.integers(0, 12))
        out.append("s%d\t0\t%s\t%d\t60\t%dM%dS\t*\t0\t0\t%s\t%s\tAS:i:%d\tXS:i:%d"
                   % (i, c, a_pos + 1, kA, L - kA, read, q, kA, xs))
        out.append("s%d\t2048\t%s\t%d\t60\t%dH%dM\t*\t0\t0\t%s\t*\tAS:i:%d" % (i, c, b_pos + 1, kA, L - kA,
                                                                               read[kA:], L - kA))
    with open(path, "w") as f:
        f.write("\n".join(out) + "\n")


def counters(out):
    c = {}
    for l in open(os.path.join(out, "run.log")):
        m = re.search(r"\tfind_circ\t(\w+)=([0-9.]+)$", l.rstrip("\n"))
        if m:
            c[m.group(1)] = m.group(2)
    return c


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reads", type=int, default=1_000_000)
    ap.add_argument("--scale", type=float, default=1.0)
    ap.add_argument("--out", default="/tmp/fc2_scale")
    ap.add_argument("--only", default="", help="comma list of run tags (timing only; the identity check needs all)")
    a = ap.parse_args()
    # the runs share this process: the torch-based ones (--python-caller / --python-ingest, the Python
    # loop's Genome) and the default CLI's torch-free contexts must use one HIP runtime, so torch's is
    # brought up first (its libamdhip64 then serves libfc2.so too, as in the GPU tests)
    import torch
    torch.cuda.init()
    from find_circ2_amd import cli, sq_table
    rng = np.random.default_rng(2024)
    names, sizes = sq_table(os.path.join(ROOT, "tests", "golden", "test_norm.sam"))
    sizes = [max(1000, int(s * a.scale)) for s in sizes]
    os.makedirs(a.out, exist_ok=True)
    fa, sam = os.path.join(a.out, "genome.fa"), os.path.join(a.out, "reads.sam")
    for p in (fa + ".byo_index",):
        if os.path.exists(p):
            os.remove(p)
    t0 = time.time()
    seqs = make_genome(fa, names, sizes, rng)
    write_sam(sam, seqs, a.reads, rng)          # plants the junction signals into seqs
    write_fasta(fa, seqs)
    del seqs
    t_gen = time.time() - t0
    res = {"reads": a.reads, "bases": int(sum(sizes)), "gen_s": round(t_gen, 1)}
    outs = {}
    for tag, extra in (("native", []), ("native_gpus2", ["--gpus", "2"]), ("python_caller", ["--python-caller"]),
                       ("python_ingest", ["--python-ingest"]),
                       ("native_allhits", ["--all-hits", "--non-canonical"]),
                       ("python_caller_allhits", ["--python-caller", "--all-hits", "--non-canonical"])):
        if a.only and tag not in a.only.split(","):
            continue
        out = os.path.join(a.out, tag)
        t0 = time.time()
        rc = cli.main(["-G", fa, "-o", out, "-n", "scale", "-q"] + extra + [sam])
        res[tag + "_s"] = round(time.time() - t0, 2)
        res[tag + "_rc"] = rc
        log = open(os.path.join(out, "run.log")).read().splitlines()
        res[tag + "_log"] = [l.split("\t")[-1] for l in log if "processed" in l or "breakpoint search" in l
                             or "reading from" in l or "read loop stages" in l]
        outs[tag] = out
        print("done", tag, res[tag + "_s"], file=sys.stderr, flush=True)
    if a.only:
        print(json.dumps(res))
        return 0
    same = True
    for x, y in (("native", "python_caller"), ("native", "native_gpus2"), ("native", "python_ingest"),
                 ("native_allhits", "python_caller_allhits")):
        for f in ("circ_splice_sites.bed", "lin_splice_sites.bed", "multi_events.tsv"):
            if open(os.path.join(outs[x], f)).read() != open(os.path.join(outs[y], f)).read():
                same = False
                res["differs"] = "%s vs %s: %s" % (x, y, f)
        with gzip.open(os.path.join(outs[x], "spliced_reads.fastq.gz"), "rt") as p1, \
                gzip.open(os.path.join(outs[y], "spliced_reads.fastq.gz"), "rt") as p2:
            if p1.read() != p2.read():
                same = False
                res["differs"] = "%s vs %s: reads" % (x, y)
        if counters(outs[x]) != counters(outs[y]):
            same = False
            res["differs"] = "%s vs %s: counters" % (x, y)
    res["identical"] = same
    res["circ_rows"] = sum(1 for l in open(os.path.join(outs["native"], "circ_splice_sites.bed")) if l[0] != "#")
    res["lin_rows"] = sum(1 for l in open(os.path.join(outs["native"], "lin_splice_sites.bed")) if l[0] != "#")
    res["counters"] = counters(outs["native"])
    print(json.dumps(res))
    return 0 if same else 1


if __name__ == "__main__":
    sys.exit(main())
