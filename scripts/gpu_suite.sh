# The GPU test suite, smoke and a short bench in one call (run through gpurun from the repo root).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 && echo TESTS_OK &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && echo SMOKE_OK &&
timeout -k 10 400 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-extra > gpurun_out/bench_short.json 2> gpurun_out/bench_short.err && echo BENCH_OK &&
timeout -k 10 300 python -u scripts/ab_kernel.py --variants k32nt1,k64nt1,k32nt1bt256,k32nt1peA --rounds 3 > gpurun_out/ab_smoke.jsonl 2> gpurun_out/ab_smoke.err && echo AB_OK
