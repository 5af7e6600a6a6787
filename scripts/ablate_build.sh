#!/bin/bash
# Measurement-only library variants: find_circ2_amd/libfc2_abl<N>.so built with -DFC2_ABLATE=<N>
# (fc2_scan32.hip: bit 0 = no third-unit loads, bit 1 = no N-plane loads).  Their results are
# WRONG by construction; they exist to price each memory request class in an A/B
# (FC2_LIB_VARIANT=abl<N> python scripts/ab_kernel.py ...).
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
for n in "$@"; do
  make -s -C $ROOT/find_circ2_amd/csrc -B OUT=../libfc2_abl$n.so \
    CXXFLAGS="-O3 -std=c++17 -fPIC -Wall -Wno-unused-result -I../../include -DFC2_ABLATE=$n"
  echo built libfc2_abl$n.so
done
make -s -C $ROOT/find_circ2_amd/csrc -B
