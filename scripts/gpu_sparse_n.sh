set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 && echo TESTS_OK && tail -2 gpurun_out/gpu_tests.log &&
timeout -k 10 400 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err && echo BENCH_OK && python -c "
import json; d=json.load(open('gpurun_out/bench.json')); print(d['value'], d['roofline']['kernel_ms']); print(json.dumps(d['extra']['device_pipeline_pcie']))"
