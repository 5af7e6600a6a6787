#!/bin/bash
# Build libfc2.so of git revision $1 as find_circ2_amd/libfc2_$2.so (for same-box A/B:
# FC2_LIB_VARIANT=$2 python scripts/ab_kernel.py ...).  Uses a throw-away worktree under /tmp.
set -e
REV=$1; NAME=$2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
WT=/tmp/fc2_wt_$NAME
rm -rf $WT
git -C $ROOT worktree add --detach $WT $REV > /dev/null 2>&1
# A/B build (FC2_AB_FORMS=1 where the revision has it: fc2_set_tuning + every kernel form)
if grep -q "^ab:" $WT/find_circ2_amd/csrc/Makefile; then
  make -s -C $WT/find_circ2_amd/csrc ab > /dev/null
  cp $WT/find_circ2_amd/libfc2_ab.so $ROOT/find_circ2_amd/libfc2_$NAME.so
else
  make -s -C $WT/find_circ2_amd/csrc > /dev/null
  cp $WT/find_circ2_amd/libfc2.so $ROOT/find_circ2_amd/libfc2_$NAME.so
fi
git -C $ROOT worktree remove --force $WT
echo built $ROOT/find_circ2_amd/libfc2_$NAME.so from $REV
