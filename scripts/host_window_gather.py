#!/usr/bin/env python
"""Host side of north_star's window-carrying form: how fast can the CPU gather windows?

BASELINE.json's north_star streams "the two genome windows per pair from the
mmap'd FASTA" to the GPU.  fc2_pack_windows does that gather (get_data
semantics, find_circ.py:189-215) into the rows the window-carrying scan reads.
This times it on an hg19-sized FASTA (93 contigs of test_norm.sam, 3.137 Gbp,
50-nt lines; written once to --out) for random 100-bp anchor pairs, with 1 and
with all host threads, and prints one JSON line (pairs/s).  CPU only.

usage: python scripts/host_window_gather.py [--out DIR] [--pairs N] [--threads T]
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "scripts"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="/tmp/fc2_genome")
    ap.add_argument("--pairs", type=int, default=4_000_000)
    ap.add_argument("--threads", type=int, default=0, help="0: all CPUs this process may use")
    ap.add_argument("--scale", type=float, default=1.0)
    a = ap.parse_args()
    from find_circ2_amd import _native as N, sq_table
    from genome_load_time import write_fasta
    names, sizes = sq_table(os.path.join(ROOT, "tests", "golden", "test_norm.sam"))
    sizes = [max(1000, int(s * a.scale)) for s in sizes]
    os.makedirs(a.out, exist_ok=True)
    fa = os.path.join(a.out, "hg19_shaped.fa")
    if not os.path.exists(fa):
        print("writing", fa, file=sys.stderr, flush=True)
        write_fasta(fa, names, sizes)
        print("written", file=sys.stderr, flush=True)
    L = N.lib()
    h = ctypes.c_void_p()
    N.check(L.fc2_fasta_open(fa.encode(), 0, ctypes.byref(h)))
    p = N.Params(15, 2, 2, 0, 0, 0, 0)
    rng = np.random.default_rng(11)
    n = a.pairs
    sz = np.asarray(sizes, np.int64)
    chrom = rng.choice(len(sizes), n, p=sz / sz.sum())
    span = rng.integers(150, 20001, n)
    kA = rng.integers(15, 86, n)
    end = (rng.random(n) * (sz[chrom] - 200)).astype(np.int64) + 100
    start = np.maximum(0, end - span)
    hp = np.zeros(n, N.PAIR_DTYPE)
    hp["a_pos"] = end - kA
    hp["b_aend"] = start + (100 - kA)
    hp["chrom"] = chrom.astype(np.uint32)
    hp["read_len"] = 100
    hp["flags"] = N.PAIR_BACKSPLICE
    pw, ww, wnw = ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_uint32()
    N.check(L.fc2_window_geometry(ctypes.byref(p), 100, ctypes.byref(pw), ctypes.byref(ww), ctypes.byref(wnw)))
    words = np.zeros(ww.value * n, np.uint64)
    nwords = np.zeros(wnw.value * n, np.uint64)
    threads = a.threads or len(os.sched_getaffinity(0))
    out = {"pairs": n, "fasta_gbp": round(sum(sizes) / 1e9, 3), "cpu_model": None}
    try:
        out["cpu_model"] = [l for l in open("/proc/cpuinfo") if l.startswith("model name")][0].split(":", 1)[1].strip()
    except Exception:
        pass
    for T in sorted({1, 4, threads}):
        m = n if T > 1 else max(1, n // 8)
        t0 = time.perf_counter()
        N.check(L.fc2_pack_windows(ctypes.byref(p), h, m, hp.ctypes.data, words.ctypes.data, nwords.ctypes.data,
                                   pw.value, n, T))
        dt = time.perf_counter() - t0
        out["threads_%d" % T] = {"pairs": m, "seconds": round(dt, 3), "pairs_per_s": round(m / dt, 1)}
    out["bytes_per_pair_uploaded"] = 16 + 24 + 8 * ww.value
    print(json.dumps(out))
    L.fc2_fasta_close(h)


if __name__ == "__main__":
    main()
