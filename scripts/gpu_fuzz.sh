set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_fuzz.py -x -v --timeout 300 --timeout-method thread > gpurun_out/fuzz.log 2>&1 && echo FUZZ_OK; tail -15 gpurun_out/fuzz.log
