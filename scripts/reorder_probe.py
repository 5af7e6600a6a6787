#!/usr/bin/env python
"""Time the device locality reorder against the read-order scan (bench workload).

Prints one JSON line per variant: ms per launch (HIP events, median of --reps)
for reorder alone, scan of the reordered batch (XCD swizzle off / on), the
read-order scan, and reorder + scan back to back.
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from find_circ2_amd import Genome, Options, PairBatch, SynthConfig, reorder, scan, sq_table  # noqa: E402
from find_circ2_amd import _native as N  # noqa: E402


def timeit(fn, reps, warm=2):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b))
    return float(np.median(ts)), float(np.min(ts))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pairs", type=int, default=50_000_000)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=8)
    a = ap.parse_args()
    dev = "cuda:0"
    names, sizes = sq_table(os.path.join(ROOT, "tests", "golden", "test_norm.sam"))
    g = Genome.synthetic(names, sizes, seed=4711, device=dev)
    opt = Options()
    b = PairBatch.synthetic(opt, g, a.pairs, SynthConfig(seed=1337, span_max=20000, p_backsplice=1.0))
    r = reorder(g, b)
    out_b = scan(opt, g, b)
    out_r = scan(opt, g, r)
    torch.cuda.synchronize()
    L = N.lib()
    rows = []
    for rounds in (32, 16, 8, 4, 2):
        for nt in (0, 1):
            L.fc2_set_tuning(4, rounds)
            L.fc2_set_tuning(5, nt)
            rr = reorder(g, b)
            rows.append(("reorder_r%d_nt%d" % (rounds, nt), timeit(lambda: reorder(g, b, into=rr), a.reps)))
            del rr
    L.fc2_set_tuning(4, a.rounds)
    L.fc2_set_tuning(5, 0)
    r = reorder(g, b)
    for sw in (0, 1, 2):
        L.fc2_set_tuning(N.TUNE_XCD_SWIZZLE if hasattr(N, "TUNE_XCD_SWIZZLE") else 3, sw)
        rows.append(("scan_reordered_sw%d" % sw, timeit(lambda: scan(opt, g, r, out=out_r), a.reps)))
        rows.append(("scan_readorder_sw%d" % sw, timeit(lambda: scan(opt, g, b, out=out_b), a.reps)))
    L.fc2_set_tuning(3, 2)

    def both():
        reorder(g, b, into=r)
        scan(opt, g, r, out=out_r)
    rows.append(("reorder+scan", timeit(both, a.reps)))
    for name, (med, mn) in rows:
        print(json.dumps({"variant": name, "ms_median": round(med, 4), "ms_min": round(mn, 4),
                          "Gpairs_per_s": round(a.pairs / med / 1e6, 2)}), flush=True)
    info = r.reorder_info
    print(json.dumps({"n_buckets": info.n_buckets, "shift": info.shift, "n_chunks": info.n_chunks,
                      "workspace_MB": round(info.workspace_bytes / 2**20, 1)}))


if __name__ == "__main__":
    main()
