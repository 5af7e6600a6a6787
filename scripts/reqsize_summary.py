"""Summarise the r03 policy_probe runs (scripts/policy_probe.hip): per policy_probe variant, L2->fabric read requests per
random gather by size (TCC_EA0_RDREQ_32B/64B/128B) and those that went to DRAM.  The probe runs
3 allocations x 12 variants x 6 launches (one warm-up + five timed), in that order; the 4th launch of
each variant is the one reported.  Usage: python scripts/reqsize_summary.py gpurun_out/req_policy > summary.json"""
import collections
import csv
import json
import os
import sys


def load(p):
    by = collections.OrderedDict()
    for r in csv.DictReader(open(p)):
        if "probe" in r["Kernel_Name"]:
            by.setdefault(int(r["Dispatch_Id"]), {"k": r["Kernel_Name"]})[r["Counter_Name"]] = float(r["Counter_Value"])
    return list(by.values())


def main(d):
    s = load(os.path.join(d, "sizes", "pmc_counter_collection.csv"))
    dr = load(os.path.join(d, "dram", "pmc_counter_collection.csv"))
    allocs = ["coarse", "finegrained", "uncached"]
    pols = ["none", "nt", "sc0", "sc1", "sc0sc1", "sc0sc1nt"] * 2
    out = []
    for a in range(3):
        for v in range(12):
            i = (a * 12 + v) * 6 + 3
            x, y = s[i], dr[i]
            gathers = 256 * 32 * 256 * 64 / (2 if v >= 6 else 1)     # blocks x threads x iters (per pair: /2)
            out.append(dict(alloc=allocs[a], policy=pols[v], gather_bytes=32 if v >= 6 else 16, kernel=x["k"][:40],
                            rdreq_32B=x["TCC_EA0_RDREQ_32B_sum"] / gathers, rdreq_64B=x["TCC_EA0_RDREQ_64B_sum"] / gathers,
                            rdreq_128B=x["TCC_EA0_RDREQ_128B_sum"] / gathers, rdreq=y["TCC_EA0_RDREQ_sum"] / gathers,
                            rdreq_dram=y["TCC_EA0_RDREQ_DRAM_sum"] / gathers))
    json.dump(out, sys.stdout, indent=0)


if __name__ == "__main__":
    main(sys.argv[1])
