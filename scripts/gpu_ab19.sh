set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do for v in prev cur; do
  if [ $v = cur ]; then unset FC2_LIB_VARIANT; else export FC2_LIB_VARIANT=$v; fi
  timeout -k 10 150 python scripts/ab_kernel.py --variants k32nt1,probe --rounds 5 --read-len 150 2>/dev/null | sed "s/^/$v L150 /"
  timeout -k 10 150 python scripts/ab_kernel.py --variants k32nt1,probe --rounds 5 2>/dev/null | sed "s/^/$v L100 /"
done; done > gpurun_out/ab19.jsonl; cat gpurun_out/ab19.jsonl
