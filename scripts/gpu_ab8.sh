set -o pipefail
mkdir -p gpurun_out
for w in "" "--ordered" "--workload cdr1as --pairs 50000000"; do
  timeout -k 10 150 python scripts/ab_kernel.py --variants k32nt1,probe --rounds 7 $w 2>/dev/null
done > gpurun_out/ab8.jsonl; cat gpurun_out/ab8.jsonl
SQ_WORKLOADS="hg19 hg19o cdr1as" bash scripts/sq_profile.sh > gpurun_out/sq.log 2>&1; tail -1 gpurun_out/sq.log
