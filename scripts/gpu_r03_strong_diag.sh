# configs[3] merge diagnostics at N = 1: host seconds in the launch calls per batch (FC2_BENCH_HOST_TIMING)
set -o pipefail
mkdir -p gpurun_out/strong_diag
FC2_BENCH_HOST_TIMING=1 timeout -k 10 240 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-extra --no-config4 \
  > gpurun_out/strong_diag/host_timing.json 2> gpurun_out/strong_diag/host_timing.err && echo DIAG_OK
