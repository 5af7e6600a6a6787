set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 && echo TESTS_OK &&
for r in 1 2; do
  for w in "" "--ordered" "--workload cdr1as --pairs 50000000"; do
    timeout -k 10 150 python scripts/ab_kernel.py --variants k32nt1wo1,k32nt1wo0 --rounds 9 $w 2>/dev/null | sed "s/^/p$r /"
  done
done > gpurun_out/ab6.jsonl; cat gpurun_out/ab6.jsonl; tail -2 gpurun_out/gpu_tests.log
