#!/bin/bash
# rocprofv3 passes for the bench kernel (run on the GPU box from the repo root).
# Kernel trace + stats in one pass; each PMC counter group in its own pass (no tracing domains mixed in).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
B="python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-extra"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt_hg19 -o kt --output-format csv -- $B > $OUT/kt_hg19.out 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch_hg19 -o pmc --output-format csv -- $B > $OUT/fetch_hg19.out 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/write_hg19 -o pmc --output-format csv -- $B > $OUT/write_hg19.out 2>&1
timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d $OUT/hit_hg19 -o pmc --output-format csv -- $B > $OUT/hit_hg19.out 2>&1
C="python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-extra --workload cdr1as --pairs 50000000"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt_cdr1as -o kt --output-format csv -- $C > $OUT/kt_cdr1as.out 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch_cdr1as -o pmc --output-format csv -- $C > $OUT/fetch_cdr1as.out 2>&1
echo PROFILE_DONE
