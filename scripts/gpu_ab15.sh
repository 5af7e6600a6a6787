set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do for v in cur abl16; do
  if [ $v = cur ]; then unset FC2_LIB_VARIANT; else export FC2_LIB_VARIANT=$v; fi
  timeout -k 10 150 python scripts/ab_kernel.py --no-check --variants k32nt1 --rounds 5 2>/dev/null | sed "s/^/$v /"
done; done > gpurun_out/ab15.jsonl; cat gpurun_out/ab15.jsonl
