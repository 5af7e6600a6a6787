# Same-box A/B of the sequential read loop: libfc2_<NAME>.so (e.g. scripts/ab_build.sh HEAD prev)
# against the tree's libfc2.so, alternating, $2 rounds (default 3).
set -o pipefail
mkdir -p gpurun_out
NAME=${1:-prev}; R=${2:-3}
for k in $(seq 1 $R); do
  for v in $NAME cur; do
    if [ $v = cur ]; then unset FC2_LIB_VARIANT; else export FC2_LIB_VARIANT=$v; fi
    timeout -k 10 300 python -u scripts/caller_cpu_profile.py 2000000 1.0 > gpurun_out/abc_$v.json 2>> gpurun_out/abc.err || exit 1
    echo "$v $(cat gpurun_out/abc_$v.json)"
  done
done
