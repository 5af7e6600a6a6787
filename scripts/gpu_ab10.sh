set -o pipefail
mkdir -p gpurun_out
for r in 1 2 3; do WT_EXTRA=4 timeout -k 10 200 python scripts/wt_alloc_probe.py 2>/dev/null | sed "s/^/p$r /"; done > gpurun_out/wt_probe2.jsonl; cat gpurun_out/wt_probe2.jsonl
