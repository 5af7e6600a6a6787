#!/usr/bin/env python
"""Coarse genome bucketing in front of the scan: does it beat the read-order scan?

With ~1024 buckets the device reorder's scatter cost more than the scan saves
(profiles/r01/reorder_probe.jsonl).  Here the bucket size is raised
(FC2_TUNE_REORDER_SHIFT) so that (a) the scatter has only tens of write fronts and
(b) one bucket's slice of the word-pair table can stay in the 256 MiB Infinity
Cache while the scan works through it.  Per shift: reorder ms, scan ms of the
bucketed batch in two forms (LDS-staged + shifted copy; plain), and the sum,
next to the read-order scan -- all interleaved in one process.  Results of every
scan are checked against the read-order scan (through the slot map).
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


def ev_time(fn, reps):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pairs", type=int, default=50_000_000)
    ap.add_argument("--reps", type=int, default=4)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--shifts", default="0,24,26,27,28")
    a = ap.parse_args()
    dev = "cuda:0"
    names, sizes = sq_table(os.path.join(ROOT, "tests", "golden", "test_norm.sam"))
    g = Genome.synthetic(names, sizes, seed=4711, device=dev)
    opt = Options()
    b = PairBatch.synthetic(opt, g, a.pairs, SynthConfig(seed=1337, span_min=150, span_max=20000, p_backsplice=1.0,
                                                         p_planted=0.5, mut_rate=0.005, n_rate=0.0005))
    L = N.lib()
    out_b = scan(opt, g, b)
    torch.cuda.synchronize()
    ref = out_b.results[:b.n].clone()
    batches = {}
    for sh in [int(x) for x in a.shifts.split(",")]:
        N.check(L.fc2_set_tuning(12, sh))
        r = reorder(g, b)
        torch.cuda.synchronize()
        batches[sh] = (r, r.reorder_info.n_buckets, r.reorder_info.shift)
    N.check(L.fc2_set_tuning(12, 0))
    times = {}

    def rec(k, v):
        times.setdefault(k, []).append(v)

    forms = {"staged_twin": (1, 1), "plain": (0, 2)}   # (FC2_TUNE_STAGE, FC2_TUNE_TWIN)
    outs = {}
    for rnd in range(a.rounds):
        rec("scan_read_order", ev_time(lambda: scan(opt, g, b, out=out_b), a.reps))
        for sh, (r, nb, rs) in batches.items():
            N.check(L.fc2_set_tuning(12, sh))
            rec("reorder_s%d" % sh, ev_time(lambda: reorder(g, b, into=r), a.reps))
            for fname, (st, tw) in forms.items():
                N.check(L.fc2_set_tuning(7, st))
                N.check(L.fc2_set_tuning(6, tw))
                key = (sh, fname)
                if key not in outs:
                    outs[key] = scan(opt, g, r)
                    torch.cuda.synchronize()
                    # slot k holds input pair slot[k]: results[k] must equal ref[slot[k]]
                    assert torch.equal(outs[key].results[:b.n], ref[r.slot[:b.n].long()]), key
                o = outs[key]
                rec("scan_s%d_%s" % (sh, fname), ev_time(lambda: scan(opt, g, r, out=o), a.reps))
        N.check(L.fc2_set_tuning(7, 2))
        N.check(L.fc2_set_tuning(6, 2))
        N.check(L.fc2_set_tuning(12, 0))
    for k, v in times.items():
        line = {"variant": k, "median_ms": round(float(np.median(v)), 4), "min_ms": round(float(np.min(v)), 4)}
        if k.startswith("reorder_s"):
            sh = int(k[len("reorder_s"):])
            line["n_buckets"], line["shift"] = batches[sh][1], batches[sh][2]
        print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
