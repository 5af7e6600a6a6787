#!/usr/bin/env python
"""Build profiles/traffic_<round>.json from the rocprofv3 passes of scripts/profile_round.sh.

HBM bytes per launch of the scan kernel = 2 x FETCH_SIZE x 1024 + WRITE_SIZE x 1024
(gfx950 tallies 128-B line fills at 64 B, MI355X_MICROARCH.md §HBM; confirmed for this
kernel by the cdr1as run, whose reads are pure streaming because the genome is
L2-resident, and by scripts/gather_probe.hip for random 16-B gathers).
"""
import collections
import csv
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERN = "bp_scan"          # bp_scan32_kernel / bp_scan32_stage_bt_kernel / bp_scan_kernel
N_PAIRS = 50_000_000


PMC_KERNEL = {}      # pass name -> the scan kernel the PMC pass counted (its full name)


def dispatches(prof, name):
    """Per scan dispatch over the whole batch, in dispatch order: {counter: value}."""
    p = os.path.join(prof, name, "pmc_counter_collection.csv")
    if not os.path.exists(p):
        return []
    d = collections.OrderedDict()
    for r in csv.DictReader(open(p)):
        if KERN in r["Kernel_Name"] and int(float(r.get("Grid_Size") or N_PAIRS)) >= N_PAIRS:
            d.setdefault(int(r["Dispatch_Id"]), collections.defaultdict(list))[r["Counter_Name"]].append(
                float(r["Counter_Value"]))
            PMC_KERNEL[name] = r["Kernel_Name"]
    return [{k: sum(v) / len(v) for k, v in x.items()} for x in d.values()]


COMPACT = {}         # workload -> ordinals of the dispatches that wrote 2-B words (from the WRITE_SIZE pass)


def agg(prof, name, workload=None):
    """Counter means over the scan dispatches of a pass; for a workload whose WRITE_SIZE pass told the
    2-B compact launches (the headline) from the one 8-B reference scan, over those launches only --
    the passes run the same deterministic bench, so dispatch ordinals line up."""
    ds = dispatches(prof, name)
    if not ds:
        return {}
    keep = COMPACT.get(workload)
    if keep is not None and max(keep, default=-1) < len(ds):
        ds = [ds[i] for i in keep]
    a = collections.defaultdict(list)
    for x in ds:
        for k, v in x.items():
            a[k].append(v)
    return {k: sum(v) / len(v) for k, v in a.items()}


def kstats(prof, name, kernel=None):
    # the kernel trace, when present: only the dispatches of `kernel` (the one the PMC passes counted)
    # over the whole N_PAIRS batch (the bench's other legs launch it over sub-batches, which the stats
    # file averages in)
    t = os.path.join(prof, name, "kt_kernel_trace.csv")
    if os.path.exists(t):
        ns, kname = [], None
        for r in csv.DictReader(open(t)):
            if (r["Kernel_Name"] == kernel if kernel else KERN in r["Kernel_Name"]) and int(r["Grid_Size_X"]) >= N_PAIRS:
                ns.append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
                kname = r["Kernel_Name"].split("(fc2_params")[0].replace("void (anonymous namespace)::", "")
        if ns:
            return sum(ns) / len(ns), len(ns), kname
    p = os.path.join(prof, name, "kt_kernel_stats.csv")
    if not os.path.exists(p):
        return None, 0, None
    for r in csv.DictReader(open(p)):
        if KERN in r["Name"]:
            return float(r["AverageNs"]), int(r["Calls"]), r["Name"].split("(fc2_params")[0].replace(
                "void (anonymous namespace)::", "")
    return None, 0, None


def compact_ns(prof, name, keep):
    """Mean duration of the scan dispatches with the given ordinals (the 2-B compact launches) in the
    kernel trace: the launches the bench line's kernel_ms times, without the 8-B reference scans."""
    t = os.path.join(prof, name, "kt_kernel_trace.csv")
    if not keep or not os.path.exists(t):
        return None
    rows = sorted((r for r in csv.DictReader(open(t)) if KERN in r["Kernel_Name"] and int(r["Grid_Size_X"]) >= N_PAIRS),
                  key=lambda r: int(r["Dispatch_Id"]))
    ns = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows]
    sel = [ns[i] for i in keep if i < len(ns)]
    return sum(sel) / len(sel) if sel else None


def main():
    rnd = sys.argv[1] if len(sys.argv) > 1 else "r01"
    prof = os.path.join(ROOT, "gpurun_out", "prof")
    out = {}
    for w, key in (("hg19", "hg19"), ("hg19o", "hg19_locus_ordered"), ("cdr1as", "cdr1as_50M_calibration")):
        wd = dispatches(prof, "write_" + w)
        if wd:                        # the 2-B launches: under 4 B per pair written
            COMPACT[w] = [i for i, x in enumerate(wd) if x.get("WRITE_SIZE", 1e30) * 1024 < 4 * N_PAIRS]
        f, wr, h = agg(prof, "fetch_" + w, w), agg(prof, "write_" + w, w), agg(prof, "hit_" + w, w)
        rq = agg(prof, "req_" + w, w)
        ns, calls, kname = kstats(prof, "kt_" + w, PMC_KERNEL.get("fetch_" + w))
        if not f:
            continue
        hbm = 2 * f["FETCH_SIZE"] * 1024 + wr.get("WRITE_SIZE", 0) * 1024
        out[key] = {"pairs_per_launch": N_PAIRS, "kernel": kname,
                    "avg_kernel_ns_rocprof": ns,
                    "avg_kernel_ns_rocprof_compact_launches": compact_ns(prof, "kt_" + w, COMPACT.get(w)),
                    "FETCH_SIZE_kB_raw": f["FETCH_SIZE"], "WRITE_SIZE_kB": wr.get("WRITE_SIZE"),
                    "TCC_HIT_sum": h.get("TCC_HIT_sum"), "TCC_MISS_sum": h.get("TCC_MISS_sum"),
                    "TCC_EA0_RDREQ_sum": rq.get("TCC_EA0_RDREQ_sum"), "TCC_REQ_sum": rq.get("TCC_REQ_sum"),
                    "l2_requests_per_pair": round(rq["TCC_REQ_sum"] / N_PAIRS, 3) if rq.get("TCC_REQ_sum") else None,
                    "hbm_read_requests_per_pair": (round(rq["TCC_EA0_RDREQ_sum"] / N_PAIRS, 3)
                                                   if rq.get("TCC_EA0_RDREQ_sum") else None),
                    "hbm_bytes_per_launch": round(hbm), "hbm_bytes_per_pair": round(hbm / N_PAIRS, 1),
                    "moved_TBps": round(hbm / (ns * 1e-9) / 1e12, 3) if ns else None,
                    "pmc_dispatches": ("%d compact (2-B) launches of %d" % (len(COMPACT[w]), len(wd))
                                       if COMPACT.get(w) is not None else "all scan dispatches")}
    import subprocess
    try:
        commit = subprocess.check_output(["git", "-C", ROOT, "rev-parse", "HEAD"], text=True).strip()
    except Exception:
        commit = None
    for v in out.values():
        v["commit"] = commit        # the tree the passes ran on (stamped when the JSON is built, locally)
    out["correction"] = ("reads = 2 x FETCH_SIZE x 1024 (gfx950 128-B fills tallied at 64 B), writes = WRITE_SIZE x "
                         "1024 (exact: the result bytes x pairs -- the headline's 2-B compact words; the run's one 8-B "
                         "reference scan is left out by dispatch ordinal, pmc_dispatches)")
    out["source"] = ("rocprofv3 --kernel-trace --stats (r03: of the default bench run itself, averaged over the "
                     "dispatches on the whole 50M-pair batch) and separate --pmc passes of bench.py --steps 10 --warmup 2 "
                     "(scripts/profile_round.sh, scripts/profile_r03.sh); PMC averages over the scan-kernel dispatches")
    path = os.path.join(ROOT, "profiles", "traffic_%s.json" % rnd)
    json.dump(out, open(path, "w"), indent=1)
    dst = os.path.join(ROOT, "profiles", rnd)
    os.makedirs(dst, exist_ok=True)
    for w in ("hg19", "hg19o", "cdr1as"):
        src = os.path.join(prof, "kt_" + w, "kt_kernel_stats.csv")
        if os.path.exists(src):
            shutil.copy(src, os.path.join(dst, "kt_%s_kernel_stats.csv" % w))
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
