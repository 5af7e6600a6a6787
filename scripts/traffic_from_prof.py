#!/usr/bin/env python
"""Build profiles/traffic_<round>.json from the rocprofv3 PMC passes of scripts/profile_r01.sh.

HBM bytes per launch of bp_scan_kernel = 2 x FETCH_SIZE x 1024 + WRITE_SIZE x 1024
(gfx950: FETCH_SIZE tallies 128-B requests at 64 B, MI355X_MICROARCH.md §HBM; the factor is
checked on the cdr1as run, whose reads are pure streaming because the genome is L2-resident).
"""
import collections
import csv
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def agg(prof, name, kern="bp_scan"):
    rows = list(csv.DictReader(open(os.path.join(prof, name, "pmc_counter_collection.csv"))))
    a = collections.defaultdict(list)
    for r in rows:
        if kern in r["Kernel_Name"]:
            a[r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in a.items()}


def kstats(prof, name, kern="bp_scan"):
    for r in csv.DictReader(open(os.path.join(prof, name, "kt_kernel_stats.csv"))):
        if kern in r["Name"]:
            return float(r["AverageNs"]), int(r["Calls"])
    return None, 0


def main():
    rnd = sys.argv[1] if len(sys.argv) > 1 else "r01"
    prof = os.path.join(ROOT, "gpurun_out", "prof")
    f, w, h, fc = agg(prof, "fetch_hg19"), agg(prof, "write_hg19"), agg(prof, "hit_hg19"), agg(prof, "fetch_cdr1as")
    ns, calls = kstats(prof, "kt_hg19")
    nsc, _ = kstats(prof, "kt_cdr1as")
    n = 50_000_000
    hbm = 2 * f["FETCH_SIZE"] * 1024 + w["WRITE_SIZE"] * 1024
    out = {
        "hg19": {"pairs_per_launch": n, "kernel": "bp_scan_kernel<2,NT>", "avg_kernel_ns_rocprof": ns,
                 "FETCH_SIZE_kB_raw": f["FETCH_SIZE"], "WRITE_SIZE_kB": w["WRITE_SIZE"],
                 "TCC_HIT_sum": h.get("TCC_HIT_sum"), "TCC_MISS_sum": h.get("TCC_MISS_sum"),
                 "hbm_bytes_per_launch": round(hbm), "hbm_bytes_per_pair": round(hbm / n, 1),
                 "moved_TBps": round(hbm / (ns * 1e-9) / 1e12, 3) if ns else None,
                 "correction": "reads = 2 x FETCH_SIZE x 1024 (gfx950), writes = WRITE_SIZE x 1024 (exact: 8 B x pairs)"},
        "cdr1as_50M_calibration": {"pairs_per_launch": n, "avg_kernel_ns_rocprof": nsc,
                                   "FETCH_SIZE_kB_raw": fc["FETCH_SIZE"],
                                   "reads_x2_bytes": round(2 * fc["FETCH_SIZE"] * 1024),
                                   "streamed_bytes_expected": n * 40,
                                   "note": "genome L2-resident: reads are the 16 B record + 24 B read row per pair "
                                           "plus N rows of READ_N pairs"},
        "source": "rocprofv3 --pmc passes (scripts/profile_r01.sh): bench.py --steps 10 --warmup 2; averages over "
                  "the bp_scan_kernel dispatches",
    }
    path = os.path.join(ROOT, "profiles", "traffic_%s.json" % rnd)
    json.dump(out, open(path, "w"), indent=1)
    dst = os.path.join(ROOT, "profiles", rnd)
    os.makedirs(dst, exist_ok=True)
    for d in ("kt_hg19", "kt_cdr1as"):
        shutil.copy(os.path.join(prof, d, "kt_kernel_stats.csv"), os.path.join(dst, d + "_kernel_stats.csv"))
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
