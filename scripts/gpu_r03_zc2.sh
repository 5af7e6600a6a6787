# zero-copy merge through the bench launch tests (two ranks on one GPU) and the default bench
set -o pipefail
mkdir -p gpurun_out/zc2
timeout -k 10 900 python -u -m pytest tests/test_bench_launch.py tests/test_gpu_compact.py -m gpu -x -v --timeout 600 --timeout-method thread > gpurun_out/zc2/tests.log 2>&1 && echo TESTS_OK &&
timeout -k 10 500 python -u bench.py > gpurun_out/zc2/bench_default.json 2> gpurun_out/zc2/bench_default.err && echo BENCH_OK
