set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernel_forms.py -x -v --timeout 240 --timeout-method thread > gpurun_out/forms.log 2>&1 && echo FORMS_OK &&
timeout -k 10 200 python -u scripts/ab_kernel.py --variants k32nt1pe0,k32nt1peA,k32nt1pe2,k32nt1pe3,k32nt1pe4 --rounds 7 > gpurun_out/ab_persist.jsonl 2>gpurun_out/ab_persist.err && cat gpurun_out/ab_persist.jsonl &&
for v in abl1 abl2 abl3; do FC2_LIB_VARIANT=$v timeout -k 10 200 python -u scripts/ab_kernel.py --no-check --variants k32nt1pe0,k32nt1peA --rounds 5 | sed "s/^/$v /" ; done > gpurun_out/ab_ablate.jsonl 2>gpurun_out/ab_ablate.err && cat gpurun_out/ab_ablate.jsonl
