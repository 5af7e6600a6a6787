"""Why does the configs[3] merge overlap its copies with the scans on some runs and not on others?
Runs bench.strong_scaling (N = 1, 50M pairs, 8 batches) several times in ONE process with different
stream pairs for the scans and the D2H copies: the default (torch's current stream + a pool stream),
two fresh pool streams, a high-priority copier, and the default again after handing out 1..3 more
pool streams (HIP maps streams onto GPU_MAX_HW_QUEUES = 4 hardware queues; two streams on one queue
run one after the other).  Prints one JSON line per variant."""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from find_circ2_amd import scan  # noqa: E402

dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
a = argparse.Namespace(workload="hg19", pairs=None, read_len=100, locus_ordered=False)
opt, g, b = bench.build_workload(a, 0, dev)
ref = scan(opt, g, b).results[:b.n].cpu().numpy()
n0, kw0 = bench.workload_cfg(a, 0)


def run(label, streams):
    r = bench.strong_scaling(opt, g, b, ref, 1, 0, dev, 10, 3, n0, kw0, per_rank=8, streams=streams)
    print(json.dumps({"variant": label, "merge_ms": r["merge_ms_per_step"], "ms_per_step": r["ms_per_step"],
                      "scan_only_ms": r["scan_only"]["ms_per_step"],
                      "merge_4B_ms": r["merge_4B_words"]["merge_ms_per_step"],
                      "merge_8B_ms": r["merge_8B_words"]["merge_ms_per_step"],
                      "equal": r["merged_equals_single_rank"], "host": r.get("host_ms_per_batch_2B")}), flush=True)


cur = torch.cuda.current_stream(dev)
if os.environ.get("REPEAT"):                     # the same call again and again: which repetitions lose the overlap
    fixed = (cur, torch.cuda.Stream(dev)) if os.environ.get("FIXED") else None    # one copier for every call
    for k in range(int(os.environ["REPEAT"])):
        if os.environ.get("PAIRED"):              # scans and copies on two pool streams taken one after the other
            run("paired_%d" % k, (torch.cuda.Stream(dev), torch.cuda.Stream(dev)))
        else:
            run("%s_%d" % ("fixed" if fixed else "default", k), fixed)
    sys.exit(0)
run("default", None)
run("two_fresh_pool_streams", (torch.cuda.Stream(dev), torch.cuda.Stream(dev)))
run("high_priority_copier", (cur, torch.cuda.Stream(dev, priority=-1)))
for k in range(1, 4):
    for _ in range(k):
        torch.cuda.Stream(dev)
    run("default_after_%d_more_pool_streams" % k, None)
run("default_again", None)
