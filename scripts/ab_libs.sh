#!/bin/bash
# Same-box A/B of find_circ2_amd/libfc2_prev.so vs libfc2.so on the three workloads, interleaved.
set -e
for r in 1 2; do
  for w in "" "--ordered" "--workload cdr1as"; do
    for v in prev cur; do
      if [ $v = cur ]; then unset FC2_LIB_VARIANT; else export FC2_LIB_VARIANT=$v; fi
      timeout -k 10 120 python scripts/ab_kernel.py --variants k32nt1 --rounds 5 $w 2>/dev/null | sed "s/^/$v /"
    done
  done
done
