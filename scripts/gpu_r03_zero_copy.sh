# The scan's compact epilogue (fc2_bp_scan_compact_launch): GPU tests, then configs[3] with the
# zero-copy merge next to the copy-based forms (N = 1, two processes).
set -o pipefail
mkdir -p gpurun_out/zc
timeout -k 10 600 python -u -m pytest tests/test_gpu_compact.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/zc/tests.log 2>&1 && echo TESTS_OK &&
for r in 1 2; do
  timeout -k 10 240 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-extra --no-config4 \
    > gpurun_out/zc/bench_r$r.json 2> gpurun_out/zc/bench_r$r.err || exit 1
done && echo BENCH_OK
