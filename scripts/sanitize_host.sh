#!/bin/bash
# Host-side sanitizer runs of the CPU test suite (no GPU): libfc2 rebuilt with ASan or UBSan on the
# host code only (-Xarch_host; GPU sanitizers are not available on the pool), loaded through
# FC2_LIB_VARIANT, the matching clang runtime preloaded into python.
#   bash scripts/sanitize_host.sh asan|ubsan|tsan [pytest args]   (tsan: the two-thread read loop)
set -e
KIND=${1:-asan}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
RT=$(ls -d /opt/rocm/lib/llvm/lib/clang/*/lib/linux | head -1)
case $KIND in
  asan)  SAN="-Xarch_host -fsanitize=address -Xarch_host -fno-omit-frame-pointer"
         PRE=$RT/libclang_rt.asan-x86_64.so; export ASAN_OPTIONS=detect_leaks=0:halt_on_error=1 ;;
  ubsan) SAN="-Xarch_host -fsanitize=undefined -Xarch_host -fno-sanitize-recover=undefined"
         PRE=$RT/libclang_rt.ubsan_standalone-x86_64.so; export UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1 ;;
  tsan)  SAN="-Xarch_host -fsanitize=thread"
         PRE=$RT/libclang_rt.tsan-x86_64.so; export TSAN_OPTIONS=${TSAN_OPTIONS:-halt_on_error=1:report_signal_unsafe=0} ;;
  *) echo "usage: $0 asan|ubsan|tsan"; exit 2 ;;
esac
cd $ROOT/find_circ2_amd/csrc
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O1 -g -std=c++17 -fPIC -Wall -Wno-unused-result -I../../include $SAN \
    -shared -o ../libfc2_$KIND.so fc2_kernels.hip fc2_scan32.hip fc2_reorder.hip fc2_inflate.hip fc2_host.cpp fc2_ingest.cpp \
    fc2_caller.cpp fc2_bamout.cpp fc2_ctx.cpp -lpthread -lz -ldl
cd $ROOT
shift || true
FC2_LIB_VARIANT=$KIND LD_PRELOAD="$PRE${LD_PRELOAD:+:$LD_PRELOAD}" python -m pytest ${@:-tests} -x -q -m "not gpu" -p no:xdist
rm -f find_circ2_amd/libfc2_$KIND.so
