#!/bin/bash
# L2->fabric read request sizes (TCC_EA0_RDREQ_32B/64B/128B) for the scan kernel
# (hg19 read order) and for the random-gather probe; one counter per --pmc pass.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/req
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
B="python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extra"
for C in TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_DRAM_sum; do
  timeout -k 10 200 rocprofv3 --pmc $C -d $OUT/scan_$C -o pmc --output-format csv -- $B > $OUT/scan_$C.out 2>&1
  timeout -k 10 200 rocprofv3 --pmc $C -d $OUT/probe_$C -o pmc --output-format csv -- $R/scripts/gather_probe > $OUT/probe_$C.out 2>&1
done
echo REQ_DONE
