# configs[3] strong scaling at N = 1: equal batches vs the last batch cut into halving pieces
# (bench.py --strong-tail, shard.round_bounds), alternating in separate processes on one box.
set -o pipefail
mkdir -p gpurun_out/strong_tail
for r in 1 2; do
  for t in 0 3 2; do
    timeout -k 10 240 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-extra --no-config4 --strong-tail $t \
      > gpurun_out/strong_tail/r${r}_t${t}.json 2> gpurun_out/strong_tail/r${r}_t${t}.err || exit 1
  done
done
echo TAIL_OK
