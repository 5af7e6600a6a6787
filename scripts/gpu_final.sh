set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 && echo TESTS_OK &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && echo SMOKE_OK &&
timeout -k 10 400 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err && echo BENCH_OK && python -c "
import json; d=json.load(open('gpurun_out/bench.json')); r=d['roofline']
print(d['value'], r['kernel_ms'], r['frac'], r['access_pattern_ceiling']['scan_frac_of_ceiling'], d['extra']['device_pipeline_pcie']['value'])"
