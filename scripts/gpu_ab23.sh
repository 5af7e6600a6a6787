set -o pipefail
mkdir -p gpurun_out
# 150 bp occupancy without spills: 7-slot exchange (libfc2.so) vs 4-slot exchange (libfc2_slot4.so), 512/256-pair blocks
for r in 1 2; do
  timeout -k 10 200 python scripts/ab_kernel.py --no-check --second slot4 --variants k32nt1,k32nt1bt256,2:k32nt1,2:k32nt1bt256,probe --rounds 7 --read-len 150 2>gpurun_out/ab23.err | sed "s/^/L150 /"
done > gpurun_out/ab23.jsonl; cat gpurun_out/ab23.jsonl
