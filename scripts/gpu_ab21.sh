set -o pipefail
mkdir -p gpurun_out
# 150 bp: scan vs the access-pattern probe replaying the three-lane 48-B window loads
for r in 1 2; do
  timeout -k 10 150 python scripts/ab_kernel.py --second prev --variants k32nt1,2:k32nt1,probe --rounds 7 --read-len 150 2>gpurun_out/ab21.err | sed "s/^/L150 /"
done > gpurun_out/ab21.jsonl; cat gpurun_out/ab21.jsonl
