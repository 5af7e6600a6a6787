#!/usr/bin/env python
"""Interleaved A/B timing of bp_scan_kernel tuning knobs in ONE process (guide §5.4 rule 24), on A/B
builds of the library (-DFC2_AB_FORMS=1).

usage: python scripts/ab_kernel.py [--workload hg19|cdr1as] [--pairs N] [--rounds R] [--reps K]
Prints one JSON line per variant: median / min kernel ms over rounds, pairs/s.
"""
import argparse
import ctypes
import json
import re
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
# the knobs (fc2_set_tuning) exist only in A/B builds: libfc2_ab.so (make -C find_circ2_amd/csrc ab) unless
# FC2_LIB_VARIANT names another A/B build (scripts/ab_build.sh)
os.environ.setdefault("FC2_LIB_VARIANT", "ab")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="hg19")
    ap.add_argument("--pairs", type=int, default=50_000_000)
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--ordered", action="store_true", help="locus-ordered synthetic batch")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--read-len", type=int, default=100)
    ap.add_argument("--no-check", action="store_true", help="measurement-only libraries (ablations) change results")
    ap.add_argument("--second", default="",
                    help="NAME: also load find_circ2_amd/libfc2_NAME.so into THIS process; a variant prefixed "
                         "'2:' (e.g. 2:k32nt1) launches through that library on the same device buffers, so two "
                         "builds are compared without the between-process allocation spread")
    ap.add_argument("--variants", default="k32nt1,k64nt1",
                    help="comma list of k32|k64 + nt1|nt0 + sw0|sw1 + tw0|tw1 (FC2_TUNE_KERNEL32 / STREAM_NT / "
                         "XCD_SWIZZLE (default auto) / TWIN)")
    a = ap.parse_args()
    import torch
    import bench
    from find_circ2_amd import scan, _native as N
    dev = torch.device("cuda", 0)
    args = argparse.Namespace(workload=a.workload, pairs=a.pairs, read_len=a.read_len, locus_ordered=a.ordered)
    opt, g, b = bench.build_workload(args, 0, dev)
    out = scan(opt, g, b)
    torch.cuda.synchronize()
    ref = out.results[:b.n].clone()
    variants = a.variants.split(",")

    lib2 = None
    if a.second:
        lib2 = ctypes.CDLL(os.path.join(ROOT, "find_circ2_amd", "libfc2_%s.so" % a.second))
        lib2.fc2_bp_scan_launch.restype = ctypes.c_int
        lib2.fc2_bp_scan_launch.argtypes = [ctypes.POINTER(N.Params), ctypes.POINTER(N.GenomeView),
                                            ctypes.POINTER(N.BatchView), ctypes.c_void_p, ctypes.c_void_p,
                                            ctypes.c_uint32, ctypes.c_void_p]
        lib2.fc2_set_tuning.argtypes = [ctypes.c_int, ctypes.c_int]

    def apply(v):
        if v.startswith("2:"):
            set_knobs(lib2, v[2:])
        else:
            set_knobs(N.lib(), v)

    def set_knobs(L, v):
        L.fc2_set_tuning(1, 0 if "nt0" in v else 1)
        L.fc2_set_tuning(2, 0 if "k64" in v else 1)
        L.fc2_set_tuning(3, 0 if "sw0" in v else (1 if "sw1" in v else 2))
        L.fc2_set_tuning(6, 0 if "tw0" in v else (1 if "tw1" in v else 2))
        L.fc2_set_tuning(7, 0 if "st0" in v else (1 if "st1" in v else 2))
        L.fc2_set_tuning(9, 8192 if "lds8k" in v else (65536 if "lds64k" in v else 0))
        m = re.search(r"pe(A|\d+)", v)   # FC2_TUNE_PERSIST: peA = occupancy-sized grid, peK = K blocks/CU
        # knobs an older library (FC2_LIB_VARIANT) may not have: set unchecked, default when absent
        L.fc2_set_tuning(11, 0 if "wo0" in v else 1)                       # FC2_TUNE_WORDS
        mb = re.search(r"bt(\d+)", v)                                            # FC2_TUNE_STAGE_BLOCK
        L.fc2_set_tuning(13, int(mb.group(1)) if mb else 512)
        mt = re.search(r"tri(\d)", v)                                           # FC2_TUNE_TRI (default 3)
        L.fc2_set_tuning(14, int(mt.group(1)) if mt else 3)
        L.fc2_set_tuning(10, 0 if not m else (-1 if m.group(1) == "A" else int(m.group(1))))

    junk = torch.empty(b.n, dtype=torch.int64, device=dev)
    from find_circ2_amd import CompactResults
    from find_circ2_amd.hotpath import expand, scan_compact
    cres = {w: CompactResults(b.n, dev, cap=max(1 << 20, b.n // 64), width=w) for w in (2, 4)}
    cctr = torch.zeros(1, dtype=torch.int32, device=dev)

    win = {}

    def run(v):
        if v == "carried":        # window-carrying form: rows gathered once (untimed), sizes-only genome view
            if not win:
                b.carry_windows_from_device(g)
                win["gv"] = N.GenomeView(None, None, None, None, g.d_chrom_size.data_ptr(), 0, len(g.names), 0,
                                         None, None, 0, 0, None, 0, 0)
                win["bv"] = b.view()
                win["rows"] = (b.win_words, b.win_nwords)      # keep the rows alive
                b.win_words = b.win_nwords = None
                b.pw = 0
            pv = opt.params()
            N.check(N.lib().fc2_bp_scan_launch(ctypes.byref(pv), ctypes.byref(win["gv"]), ctypes.byref(win["bv"]),
                                               out.results.data_ptr(), None, b.tw,
                                               torch.cuda.current_stream(dev).cuda_stream))
            return
        if v.startswith("2:"):
            gv, bv, pv = g.view(), b.view(), opt.params()
            N.check(lib2.fc2_bp_scan_launch(ctypes.byref(pv), ctypes.byref(gv), ctypes.byref(bv),
                                            out.results.data_ptr(), None, b.tw,
                                            torch.cuda.current_stream(dev).cuda_stream))
            return
        mc = re.match(r"cmp(2|4)", v)
        if mc:                     # the same scan writing its results in a compact form (fc2_bp_scan_compact_launch)
            c = cres[int(mc.group(1))]
            scan_compact(opt, g, b, c.words.data_ptr(), c.width, c.esc.data_ptr(), c.cap, cctr.data_ptr(),
                         c.count.data_ptr())
            return
        if v.startswith("probe"):  # the scan's access pattern without its arithmetic (fc2_probe_pattern_launch)
            gv, bv, pv = g.view(), b.view(), opt.params()
            N.check(N.lib().fc2_probe_pattern_launch(ctypes.byref(pv), ctypes.byref(gv), ctypes.byref(bv),
                                                     junk.data_ptr(), torch.cuda.current_stream(dev).cuda_stream))
        else:
            scan(opt, g, b, out=out)

    times = {v: [] for v in variants}
    stream = torch.cuda.current_stream(dev)
    for r in range(a.rounds):
        for v in variants:
            apply(v)
            run(v)
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record(stream)
            for _ in range(a.reps):
                run(v)
            e.record(stream)
            torch.cuda.synchronize()
            times[v].append(s.elapsed_time(e) / a.reps)
            assert a.no_check or v.startswith(("probe", "cmp")) or torch.equal(out.results[:b.n], ref), \
                "variant %s changed results" % v
    for w in (2, 4):                               # the compact variants' words expand to the 8-byte results
        if "cmp%d" % w in variants and not a.no_check:
            c = cres[w]
            k = int(c.count.item())
            assert k <= c.cap
            esc = c.esc.cpu().numpy().view(N.ESCAPE_DTYPE)[:k]
            assert np.array_equal(expand(opt, c.words[:b.n].cpu().numpy(), esc), ref.cpu().numpy()), "cmp%d" % w
    for v in variants:
        t = np.array(times[v])
        print(json.dumps({"variant": v, "workload": a.workload + ("-ordered" if a.ordered else ""), "pairs": b.n, "median_ms": round(float(np.median(t)), 4),
                          "min_ms": round(float(t.min()), 4), "pairs_per_s": round(b.n / (np.median(t) * 1e-3), 1)}))


if __name__ == "__main__":
    main()
