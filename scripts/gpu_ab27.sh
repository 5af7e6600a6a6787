set -o pipefail
mkdir -p gpurun_out
# best hit packed in one word vs HEAD: parity subset, then ordered / read order / 150 bp, one process each
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py tests/test_gpu_kernel_forms.py -x -q --timeout 300 --timeout-method thread > gpurun_out/ab27_tests.log 2>&1 && echo TESTS_OK &&
for r in 1 2; do
  timeout -k 10 200 python scripts/ab_kernel.py --ordered --second prev --variants k32nt1,2:k32nt1 --rounds 7 2>gpurun_out/ab27.err | sed "s/^/ord /"
  timeout -k 10 200 python scripts/ab_kernel.py --second prev --variants k32nt1,2:k32nt1 --rounds 7 2>>gpurun_out/ab27.err | sed "s/^/L100 /"
done > gpurun_out/ab27.jsonl; cat gpurun_out/ab27.jsonl; tail -2 gpurun_out/ab27_tests.log
