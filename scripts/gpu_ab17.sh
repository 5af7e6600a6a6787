set -o pipefail
mkdir -p gpurun_out
# 150 bp read order: where the time goes against the access-pattern probe (block size, no candidate walk)
for r in 1 2; do
  timeout -k 10 150 python scripts/ab_kernel.py --variants k32nt1,k32nt1bt256,k32nt1bt1024,probe --rounds 5 --read-len 150 2>/dev/null | sed "s/^/L150 /"
  FC2_LIB_VARIANT=abl4 timeout -k 10 150 python scripts/ab_kernel.py --no-check --variants k32nt1 --rounds 5 --read-len 150 2>/dev/null | sed "s/^/L150abl4 /"
done > gpurun_out/ab17.jsonl; cat gpurun_out/ab17.jsonl
