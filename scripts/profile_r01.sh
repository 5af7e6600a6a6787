#!/bin/bash
# rocprofv3 passes for the bench kernel (run on the GPU box from the repo root).
# Kernel trace + stats in one pass; each PMC counter group in its own pass (no tracing domains mixed in).
# Workloads: hg19 read order (the headline), hg19 locus-ordered layout, cdr1as (genome L2-resident: calibration).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
B="python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-extra"
for W in hg19 hg19o cdr1as; do
  case $W in
    hg19)   A="$B" ;;
    hg19o)  A="$B --locus-ordered" ;;
    cdr1as) A="$B --workload cdr1as --pairs 50000000" ;;
  esac
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt_$W -o kt --output-format csv -- $A > $OUT/kt_$W.out 2>&1
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch_$W -o pmc --output-format csv -- $A > $OUT/fetch_$W.out 2>&1
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/write_$W -o pmc --output-format csv -- $A > $OUT/write_$W.out 2>&1
  timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d $OUT/hit_$W -o pmc --output-format csv -- $A > $OUT/hit_$W.out 2>&1
done
echo PROFILE_DONE
