#!/bin/bash
# Round 3 measurement on the GPU box (from the repo root): the default bench line run UNDER
# rocprofv3 --kernel-trace --stats, so the bench's live HIP-event kernel time and rocprof's average
# come from the same process; then each PMC group in its own pass (no tracing domains mixed in)
# for profiles/traffic_r03.json (scripts/traffic_from_prof.py r03).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/kt_hg19 -o kt --output-format csv -- python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_under_rocprof.json 2> $OUT/kt_hg19.err && echo KT_OK &&
B="python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-extra --no-strong --no-config4" &&
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch_hg19 -o pmc --output-format csv -- $B > $OUT/fetch_hg19.out 2>&1 && echo FETCH_OK &&
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/write_hg19 -o pmc --output-format csv -- $B > $OUT/write_hg19.out 2>&1 && echo WRITE_OK &&
timeout -s KILL 300 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_REQ_sum -d $OUT/req_hg19 -o pmc --output-format csv -- $B > $OUT/req_hg19.out 2>&1 && echo REQ_OK &&
echo PROFILE_DONE
