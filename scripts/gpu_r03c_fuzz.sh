# Round 3 (third session): a 2000-case GPU fuzz campaign on the final tree (options x kernel forms x
# the compact scan, every result and tie list against the oracle)
set -o pipefail
mkdir -p gpurun_out
FC2_FUZZ_CASES=2000 timeout -k 10 900 python -u -m pytest tests/test_gpu_fuzz.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_fuzz_2000.log 2>&1 && echo FUZZ_OK
