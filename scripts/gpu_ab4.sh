set -o pipefail
mkdir -p gpurun_out
for r in 1 2 3; do
  timeout -k 10 150 python scripts/ab_kernel.py --variants k32nt1wo1,k32nt1wo0 --rounds 15 2>/dev/null | sed "s/^/p$r /"
  timeout -k 10 150 python scripts/ab_kernel.py --variants k32nt1wo0,k32nt1wo1 --rounds 15 2>/dev/null | sed "s/^/q$r /"
done > gpurun_out/ab4.jsonl; cat gpurun_out/ab4.jsonl
