#!/bin/bash
# rocprofv3 passes for the bench kernel (run on the GPU box from the repo root):
# kernel trace + stats in one pass; each PMC group in its own pass (no tracing domains mixed in).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
B="python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-extra --no-strong --no-config4"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt_hg19 -o kt --output-format csv -- $B > $OUT/kt_hg19.out 2>&1
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch_hg19 -o pmc --output-format csv -- $B > $OUT/fetch_hg19.out 2>&1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/write_hg19 -o pmc --output-format csv -- $B > $OUT/write_hg19.out 2>&1
timeout -s KILL 300 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_REQ_sum -d $OUT/req_hg19 -o pmc --output-format csv -- $B > $OUT/req_hg19.out 2>&1
O="$B --locus-ordered"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt_hg19o -o kt --output-format csv -- $O > $OUT/kt_hg19o.out 2>&1
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch_hg19o -o pmc --output-format csv -- $O > $OUT/fetch_hg19o.out 2>&1
echo PROFILE_DONE
