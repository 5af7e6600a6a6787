set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 && echo TESTS_OK &&
for r in 1 2; do for v in prev cur; do
  if [ $v = cur ]; then unset FC2_LIB_VARIANT; V="k32nt1,k32nt1wo0"; else export FC2_LIB_VARIANT=$v; V=k32nt1; fi
  timeout -k 10 120 python scripts/ab_kernel.py --variants $V --rounds 5 2>/dev/null | sed "s/^/$v /"
  timeout -k 10 120 python scripts/ab_kernel.py --variants k32nt1 --rounds 5 --read-len 150 2>/dev/null | sed "s/^/$v L150 /"
done; done > gpurun_out/ab3.jsonl; cat gpurun_out/ab3.jsonl; tail -3 gpurun_out/gpu_tests.log
