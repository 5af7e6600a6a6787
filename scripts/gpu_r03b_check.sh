# Round 3 (second session): the restored tree on the GPU -- suite, smoke, default bench.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 && echo TESTS_OK &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && echo SMOKE_OK &&
timeout -k 10 500 python -u bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err && echo BENCH_OK
