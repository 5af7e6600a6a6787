set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 && echo TESTS_OK &&
for r in 1 2; do for v in prev cur; do
  if [ $v = cur ]; then unset FC2_LIB_VARIANT; else export FC2_LIB_VARIANT=$v; fi
  timeout -k 10 150 python scripts/ab_kernel.py --variants k32nt1 --rounds 5 2>/dev/null | sed "s/^/$v /"
  timeout -k 10 150 python scripts/ab_kernel.py --variants k32nt1 --rounds 5 --ordered 2>/dev/null | sed "s/^/$v /"
done; done > gpurun_out/ab16.jsonl; cat gpurun_out/ab16.jsonl; tail -2 gpurun_out/gpu_tests.log
