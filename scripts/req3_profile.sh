#!/bin/bash
# L2 requests per lane of the paired-gather probe variants (coalescing check).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/req3
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
for C in TCC_REQ_sum TCC_EA0_RDREQ_sum; do
  timeout -k 10 200 rocprofv3 --pmc $C -d $OUT/pat_$C -o pmc --output-format csv -- $R/scripts/pattern_probe > $OUT/pat_$C.out 2>&1
done
echo REQ3_DONE
