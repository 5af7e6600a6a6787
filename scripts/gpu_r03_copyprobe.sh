set -o pipefail
R=$(pwd)
mkdir -p gpurun_out/copyprobe
timeout -k 10 120 python -u scripts/probes/copy_engine_probe.py > gpurun_out/copyprobe/default.jsonl 2>&1 && echo DEFAULT_OK &&
export TMPDIR=/tmp && cd /tmp &&
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/copyprobe/kt -o kt --output-format csv -- python3 $R/scripts/probes/copy_engine_probe.py > $R/gpurun_out/copyprobe/kt.out 2>&1 && echo KT_OK
