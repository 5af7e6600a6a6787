set -o pipefail
mkdir -p gpurun_out
# same-process A/B: libfc2.so (working tree) vs libfc2_prev.so (HEAD) on the same device buffers
for r in 1 2; do
  timeout -k 10 150 python scripts/ab_kernel.py --second prev --variants k32nt1,2:k32nt1,probe --rounds 7 --read-len 150 2>gpurun_out/ab20.err | sed "s/^/L150 /"
  timeout -k 10 150 python scripts/ab_kernel.py --second prev --variants k32nt1,2:k32nt1,probe --rounds 7 2>>gpurun_out/ab20.err | sed "s/^/L100 /"
done > gpurun_out/ab20.jsonl; cat gpurun_out/ab20.jsonl
