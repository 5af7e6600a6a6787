set -o pipefail
mkdir -p gpurun_out
for v in cur abl4; do
  if [ $v = cur ]; then unset FC2_LIB_VARIANT; else export FC2_LIB_VARIANT=$v; fi
  for w in "" "--ordered"; do
    timeout -k 10 150 python scripts/ab_kernel.py --no-check --variants k32nt1,carried --rounds 5 $w 2>/dev/null | sed "s/^/$v /"
  done
done > gpurun_out/ab9.jsonl; cat gpurun_out/ab9.jsonl
