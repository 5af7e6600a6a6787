set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernel_forms.py -x -v --timeout 240 --timeout-method thread > gpurun_out/forms.log 2>&1 && echo FORMS_OK &&
for r in 1 2; do for v in prev cur abl2; do
  if [ $v = cur ]; then unset FC2_LIB_VARIANT; else export FC2_LIB_VARIANT=$v; fi
  timeout -k 10 120 python scripts/ab_kernel.py --no-check --variants k32nt1 --rounds 5 2>/dev/null | sed "s/^/$v /"
done; done > gpurun_out/ab2.jsonl && cat gpurun_out/ab2.jsonl
