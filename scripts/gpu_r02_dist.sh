set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_bench_launch.py -m gpu -x -v --timeout 250 --timeout-method thread > gpurun_out/launch_test.log 2>&1 && echo LAUNCH_TEST_OK &&
timeout -k 10 400 python -u bench.py --gpus 2 --steps 10 --warmup 2 --no-cpu-baseline --no-extra > gpurun_out/dist2.json 2> gpurun_out/dist2.err && echo DIST2_OK &&
timeout -k 10 400 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-extra > gpurun_out/bench1.json 2> gpurun_out/bench1.err && echo BENCH1_OK
