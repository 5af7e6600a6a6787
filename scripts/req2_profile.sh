#!/bin/bash
# Per-launch L2 request / hit / miss / DRAM-request counts of the scan kernel (hg19 read order)
# and of scripts/pattern_probe (speed-of-light pattern); one counter per --pmc pass.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/req2
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
B="python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extra"
for C in TCC_EA0_RDREQ_sum TCC_REQ_sum TCC_HIT_sum TCC_MISS_sum; do
  timeout -k 10 200 rocprofv3 --pmc $C -d $OUT/scan_$C -o pmc --output-format csv -- $B > $OUT/scan_$C.out 2>&1
  timeout -k 10 200 rocprofv3 --pmc $C -d $OUT/pat_$C -o pmc --output-format csv -- $R/scripts/pattern_probe > $OUT/pat_$C.out 2>&1
done
echo REQ2_DONE
