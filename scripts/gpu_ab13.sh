set -o pipefail
mkdir -p gpurun_out
for v in cur abl8; do
  if [ $v = cur ]; then unset FC2_LIB_VARIANT; else export FC2_LIB_VARIANT=$v; fi
  timeout -k 10 150 python scripts/ab_kernel.py --no-check --variants k32nt1,probe --rounds 5 --read-len 150 2>/dev/null | sed "s/^/$v /"
done > gpurun_out/ab13.jsonl; cat gpurun_out/ab13.jsonl
