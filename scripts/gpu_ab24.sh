set -o pipefail
mkdir -p gpurun_out
# locus-ordered batch: scan vs no candidate walk (abl4, timing only) vs access-pattern probe, one process
for r in 1 2; do
  timeout -k 10 200 python scripts/ab_kernel.py --ordered --no-check --second abl4 --variants k32nt1,2:k32nt1,probe --rounds 7 2>gpurun_out/ab24.err | sed "s/^/ord /"
done > gpurun_out/ab24.jsonl; cat gpurun_out/ab24.jsonl
