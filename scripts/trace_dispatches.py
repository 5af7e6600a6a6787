#!/usr/bin/env python
"""Group a rocprofv3 kernel trace's dispatches of the scan / probe / compact kernels by grid size
(the bench runs the scan on batches of several sizes: the 50M-pair headline launches, the
strong-scaling sub-batches, the pipeline slices, ...), so the headline kernel's rocprof average
can be read next to bench.py's live HIP-event figure.

    python scripts/trace_dispatches.py gpurun_out/prof/kt_hg19/kt_kernel_trace.csv OUT.json
"""
import csv
import json
import re
import sys
from collections import defaultdict


def short(name):
    name = re.sub(r"\(anonymous namespace\)::", "", name)
    name = re.sub(r"^void ", "", name)
    return name.split("(")[0]


def main():
    src, out = sys.argv[1], sys.argv[2]
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 10      # the profiled bench's --steps
    groups = defaultdict(list)
    seq = []                                                    # (start, ms) of the 50M-pair scan launches
    for r in csv.DictReader(open(src)):
        n = r["Kernel_Name"]
        if not any(k in n for k in ("bp_scan32", "probe_pattern", "result_compact")):
            continue
        ms = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
        groups[(short(n), int(r["Grid_Size_X"]))].append(ms)
        if "bp_scan32" in n and int(r["Grid_Size_X"]) >= 50_000_000:
            seq.append((int(r["Start_Timestamp"]), ms))
    rows = [{"kernel": k, "grid_threads": g, "dispatches": len(v), "avg_ms": round(sum(v) / len(v), 4),
             "min_ms": round(min(v), 4), "max_ms": round(max(v), 4)}
            for (k, g), v in sorted(groups.items(), key=lambda kv: (kv[0][0], -kv[0][1]))]
    # bench.timed_scans launches the 8-byte reference scan, warmup - 1 compact scans (warmup 2), then the
    # `steps` timed compact scans: in launch order, dispatches [2, 2 + steps) of the 50M-pair grid are
    # the headline's timed launches (the rest: the access-pattern ceiling's 8-byte scans and others)
    seq.sort()
    timed = [ms for _, ms in seq[2:2 + steps]]
    head = ({"dispatches": len(timed), "avg_ms": round(sum(timed) / len(timed), 4), "min_ms": round(min(timed), 4),
             "max_ms": round(max(timed), 4)} if timed else None)
    json.dump({"source": "rocprofv3 --kernel-trace of the bench run (scripts/profile_round.sh): scan / probe / compact "
                         "dispatches grouped by grid size; the 50M-pair launches (grid 50000384) are the headline's "
                         "scan kernel, whose timed 2-byte-result launches are 'headline_timed_launches'",
               "trace": src, "headline_timed_launches": head, "dispatches": rows}, open(out, "w"), indent=1)
    print("headline timed launches:", head)
    for r in rows:
        print(r)


if __name__ == "__main__":
    main()
