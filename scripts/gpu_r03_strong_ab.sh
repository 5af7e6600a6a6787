# configs[3] strong scaling at N = 1 with 4, 8 and 16 batches per rank (the last batch's copy is the
# merge's unhidden tail), one process each.
set -o pipefail
mkdir -p gpurun_out/strong_ab
i=0; for k in 4 8 16 4; do i=$((i+1))
  timeout -k 10 300 python -u bench.py --no-extra --no-cpu-baseline --no-config4 --no-cli --strong-batches $k > gpurun_out/strong_ab/r${i}_b$k.json 2> gpurun_out/strong_ab/r${i}_b$k.err || exit 1
  echo "k=$k done"
done
