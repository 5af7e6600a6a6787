#!/usr/bin/env python
"""Does the read-order scan's speed depend on where the word-pair table (Genome.wt) lives?

Builds the bench workload once, then rebuilds g.wt under several allocation
strategies and times the scan for each (interleaved rounds, one process):
  torch      -- torch.empty (the default path), address as the allocator gives it
  torch_2m   -- a slice of a larger torch tensor starting at a 2 MiB boundary
  hip        -- a dedicated hipMalloc through the HIP runtime (ctypes)
Prints one JSON line per strategy: median ms, the table's address modulo 2 MiB.
"""
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import argparse
    import torch
    import bench
    from find_circ2_amd import scan, _native as N
    dev = torch.device("cuda", 0)
    args = argparse.Namespace(workload="hg19", pairs=50_000_000, read_len=100, locus_ordered=False)
    opt, g, b = bench.build_workload(args, 0, dev)
    out = scan(opt, g, b)
    torch.cuda.synchronize()
    ref = out.results[:b.n].clone()
    stream = torch.cuda.current_stream(dev)
    hip = ctypes.CDLL("libamdhip64.so")
    nbytes = g.wt_bytes
    tables = {"torch": g.wt}
    for k in range(int(os.environ.get("WT_EXTRA", "0"))):      # more plain torch allocations
        tables["torch_%d" % k] = torch.empty(nbytes // 4, dtype=torch.int32, device=dev)
    big = torch.empty(nbytes // 4 + (4 << 20) // 4, dtype=torch.int32, device=dev)
    off = (-big.data_ptr()) % (2 << 20)
    tables["torch_2m"] = big[off // 4: off // 4 + nbytes // 4]
    ptr = ctypes.c_void_p()
    assert hip.hipMalloc(ctypes.byref(ptr), ctypes.c_size_t(nbytes)) == 0
    tables["hip"] = ptr.value
    for name, t in list(tables.items()):
        p = t if isinstance(t, int) else t.data_ptr()
        N.check(N.lib().fc2_wtab_launch(g.units.data_ptr(), g.n_units, p, stream.cuda_stream))
    torch.cuda.synchronize()
    base_view = g.view
    cur = {"ptr": None}

    def view():                      # the genome view with the table under test
        v = base_view()
        v.wt = cur["ptr"]
        return v
    g.view = view
    times = {k: [] for k in tables}
    for r in range(9):
        for name, t in tables.items():
            cur["ptr"] = t if isinstance(t, int) else t.data_ptr()
            scan(opt, g, b, out=out)
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record(stream)
            for _ in range(5):
                scan(opt, g, b, out=out)
            e.record(stream)
            torch.cuda.synchronize()
            times[name].append(s.elapsed_time(e) / 5)
            assert torch.equal(out.results[:b.n], ref), name
    for name, t in tables.items():
        p = t if isinstance(t, int) else t.data_ptr()
        print(json.dumps({"table": name, "addr_mod_2MiB": p % (2 << 20), "median_ms": round(float(np.median(times[name])), 4),
                          "min_ms": round(float(np.min(times[name])), 4)}))


if __name__ == "__main__":
    main()
