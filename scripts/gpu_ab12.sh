set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernel_forms.py -x -q --timeout 300 --timeout-method thread > gpurun_out/forms.log 2>&1 && echo FORMS_OK &&
for r in 1 2; do timeout -k 10 150 python scripts/ab_kernel.py --variants k32nt1,k32nt1bt512,k32nt1bt1024,probe --rounds 7 2>/dev/null; done > gpurun_out/ab12.jsonl; cat gpurun_out/ab12.jsonl; tail -2 gpurun_out/forms.log
