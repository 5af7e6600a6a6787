#!/bin/bash
# 100 vs 150 bp read-order scan: L2 / HBM requests, LDS and instruction counters, one --pmc group per pass.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/pmc150
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
B="python3 $R/bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-extra"
for L in 100 150; do
  A="$B --read-len $L"
  timeout -s KILL 120 rocprofv3 --pmc TCC_REQ_sum TCC_EA0_RDREQ_sum -d $OUT/req_$L -o pmc --output-format csv -- $A > $OUT/req_$L.out 2>&1
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS -d $OUT/sq_$L -o pmc --output-format csv -- $A > $OUT/sq_$L.out 2>&1
  timeout -s KILL 120 rocprofv3 --pmc TA_TA_BUSY_sum -d $OUT/ta_$L -o pmc --output-format csv -- $A > $OUT/ta_$L.out 2>&1
done
echo PMC150_DONE
