set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernel_forms.py -x -q --timeout 240 --timeout-method thread > gpurun_out/forms.log 2>&1 && echo FORMS_OK &&
for r in 1 2; do timeout -k 10 150 python scripts/ab_kernel.py --variants k32nt1pe0,k32nt1peA,k32nt1pe4,k32nt1pe3,probe --rounds 7 2>/dev/null; done > gpurun_out/ab11.jsonl; cat gpurun_out/ab11.jsonl
