set -o pipefail
mkdir -p gpurun_out/copyprobe
timeout -k 10 150 python -u scripts/probes/copy_engine_probe.py > gpurun_out/copyprobe/async_check.jsonl 2>&1 && echo PROBE_OK
