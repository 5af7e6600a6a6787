#!/bin/bash
# SQ instruction/occupancy counters for the scan kernel (issue vs latency diagnosis).
# Each counter group in its own --pmc pass; run on the GPU box from the repo root.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/sq
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
B="python3 $R/bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-extra"
for W in ${SQ_WORKLOADS:-hg19 hg19o cdr1as}; do
  case $W in
    hg19)   A="$B" ;;
    hg19o)  A="$B --locus-ordered" ;;
    cdr1as) A="$B --workload cdr1as --pairs 50000000" ;;
  esac
  timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD -d $OUT/a_$W -o pmc --output-format csv -- $A > $OUT/a_$W.out 2>&1
  timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU -d $OUT/b_$W -o pmc --output-format csv -- $A > $OUT/b_$W.out 2>&1
  timeout -k 10 300 rocprofv3 --pmc SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM SQ_ACTIVE_INST_VMEM SQ_WAIT_ANY -d $OUT/c_$W -o pmc --output-format csv -- $A > $OUT/c_$W.out 2>&1
done
echo SQ_DONE
