set -o pipefail
mkdir -p gpurun_out
for r in 1 2 3 4; do timeout -k 10 150 python scripts/wt_alloc_probe.py 2>gpurun_out/wt_probe.err | sed "s/^/p$r /"; done > gpurun_out/wt_probe.jsonl; cat gpurun_out/wt_probe.jsonl; tail -3 gpurun_out/wt_probe.err
