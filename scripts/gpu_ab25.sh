set -o pipefail
mkdir -p gpurun_out
# read-order 100 bp: scan vs no candidate walk (abl4, timing only) vs probe, one process
for r in 1 2; do
  timeout -k 10 200 python scripts/ab_kernel.py --no-check --second abl4 --variants k32nt1,2:k32nt1,probe --rounds 7 2>gpurun_out/ab25.err | sed "s/^/L100 /"
done > gpurun_out/ab25.jsonl; cat gpurun_out/ab25.jsonl
