set -o pipefail
# The copy-engine probe: default runtime, then the runtime's blit-engine selections, then one run with
# the runtime's copy log (which engine each hipMemcpyAsync took).
R=$(pwd)
mkdir -p gpurun_out/copyprobe
timeout -k 10 120 python -u scripts/probes/copy_engine_probe.py > gpurun_out/copyprobe/default.jsonl 2>&1 && echo DEFAULT_OK &&
GPU_BLIT_ENGINE_TYPE=2 timeout -k 10 120 python -u scripts/probes/copy_engine_probe.py > gpurun_out/copyprobe/blit_engine_2.jsonl 2>&1 && echo BE2_OK &&
GPU_BLIT_ENGINE_TYPE=3 timeout -k 10 120 python -u scripts/probes/copy_engine_probe.py > gpurun_out/copyprobe/blit_engine_3.jsonl 2>&1 && echo BE3_OK &&
AMD_LOG_LEVEL=3 timeout -k 10 150 python -u scripts/probes/copy_engine_probe.py > gpurun_out/copyprobe/log3.out 2>&1 && echo LOG_OK &&
(grep -c 'HSA Copy' gpurun_out/copyprobe/log3.out || true) &&
(grep -m 20 -E 'HSA Copy|copyBuffer|forceSDMA|engine' gpurun_out/copyprobe/log3.out || true) > gpurun_out/copyprobe/log3_copies.txt &&
gzip -f gpurun_out/copyprobe/log3.out &&
GPU_BLIT_ENGINE_TYPE=2 AMD_LOG_LEVEL=3 timeout -k 10 150 python -u scripts/probes/copy_engine_probe.py > gpurun_out/copyprobe/log3_be2.out 2>&1 && echo LOG_BE2_OK &&
(grep -m 20 -E 'HSA Copy|copyBuffer|forceSDMA|engine' gpurun_out/copyprobe/log3_be2.out || true) > gpurun_out/copyprobe/log3_be2_copies.txt &&
gzip -f gpurun_out/copyprobe/log3_be2.out &&
export TMPDIR=/tmp && cd /tmp &&
GPU_BLIT_ENGINE_TYPE=2 timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/copyprobe/kt_be2 -o kt --output-format csv -- python3 $R/scripts/probes/copy_engine_probe.py > $R/gpurun_out/copyprobe/kt_be2.out 2>&1 && echo KT_OK
