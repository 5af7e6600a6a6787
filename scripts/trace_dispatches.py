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
    groups = defaultdict(list)
    for r in csv.DictReader(open(src)):
        n = r["Kernel_Name"]
        if not any(k in n for k in ("bp_scan32", "probe_pattern", "result_compact")):
            continue
        groups[(short(n), int(r["Grid_Size_X"]))].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    rows = [{"kernel": k, "grid_threads": g, "dispatches": len(v), "avg_ms": round(sum(v) / len(v), 4),
             "min_ms": round(min(v), 4), "max_ms": round(max(v), 4)}
            for (k, g), v in sorted(groups.items(), key=lambda kv: (kv[0][0], -kv[0][1]))]
    json.dump({"source": "rocprofv3 --kernel-trace of the default bench run itself (scripts/profile_r03.sh): scan / "
                         "probe / compact dispatches grouped by grid size; the 50M-pair launches (grid 50000384) are "
                         "the headline's", "trace": src, "dispatches": rows}, open(out, "w"), indent=1)
    for r in rows:
        print(r)


if __name__ == "__main__":
    main()
