# Rehearsal of the driver's N = 4 launch on the one-GPU box: four ranks share cuda:0 (the line's
# n_gpus says 4, its rates are one GPU's); checks the launcher, the per-rank shares and merges.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u bench.py --gpus 4 --no-cpu-baseline > gpurun_out/bench_4ranks_one_gpu.json 2> gpurun_out/bench_4ranks_one_gpu.err && echo BENCH4_OK
