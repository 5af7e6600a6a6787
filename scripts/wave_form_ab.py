#!/usr/bin/env python
"""Same-process A/B: BASELINE north_star's kernel shape (one wavefront per pair, FC2_BATCH_FORM_WAVE,
bp_wave_kernel) against the shipped one-pair-per-lane scan, on the bench's configs[2] batch (50M
100-bp pairs, hg19-shaped genome) and the configs[4] shape (120-150 bp).  Interleaved rounds, HIP
events on the scan's stream; every wave-form result word must equal the shipped form's.
usage: python scripts/wave_form_ab.py [--rounds R] [--reps K] > out.jsonl"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=4)
    a = ap.parse_args()
    import torch
    import bench
    from find_circ2_amd import PairBatch, SynthConfig, scan
    from find_circ2_amd import _native as N
    dev = torch.device("cuda", 0)
    args = argparse.Namespace(workload="hg19", pairs=50_000_000, read_len=100, locus_ordered=False)
    opt, g, b = bench.build_workload(args, 0, dev)
    cases = [("configs[2]_100bp", b, 81)]
    b150 = PairBatch.synthetic(opt, g, 25_000_000, SynthConfig(seed=4242, len_min=120, len_max=150, span_max=20000))
    cases.append(("configs[4]_120_150bp_share", b150, 119))
    for name, bb, bpp in cases:
        ref = scan(opt, g, bb).results[:bb.n].clone()
        keep = bb.layout
        times = {"shipped": [], "wave": []}
        for _ in range(a.rounds):
            for form, hint in (("shipped", 0), ("wave", N.BATCH_FORM_WAVE)):
                bb.layout = keep | hint
                out = scan(opt, g, bb)                         # warm
                torch.cuda.synchronize()
                if form == "wave":
                    assert torch.equal(out.results[:bb.n], ref), "wave form differs"
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(a.reps):
                    scan(opt, g, bb, out=out)
                e.record()
                torch.cuda.synchronize()
                times[form].append(s.elapsed_time(e) / a.reps)
                del out
        bb.layout = keep
        for form, t in times.items():
            t = sorted(t)
            ms = t[len(t) // 2]
            print(json.dumps({"case": name, "form": form, "pairs": bb.n, "median_ms": round(ms, 4),
                              "min_ms": round(t[0], 4), "pairs_per_s": round(bb.n / ms * 1e3, 1),
                              "frac_hbm_8TBps": round(bb.n * bpp / (ms * 1e-3) / 8e12, 4),
                              "results_equal_shipped": True}), flush=True)


if __name__ == "__main__":
    main()
