set -o pipefail
mkdir -p gpurun_out/prof_r02
R=$(pwd)
timeout -k 10 500 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_full.json 2> gpurun_out/bench_full.err && echo BENCH_OK &&
timeout -k 10 300 python -u scripts/cli_scale_check.py --reads 1000000 > gpurun_out/cli_scale.json 2> gpurun_out/cli_scale.err && echo CLI_SCALE_OK &&
export TMPDIR=/tmp && cd /tmp &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r02/kt_hg19 -o kt --output-format csv -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-extra --no-strong > $R/gpurun_out/prof_r02/kt_hg19.out 2>&1 && echo PROF_OK
