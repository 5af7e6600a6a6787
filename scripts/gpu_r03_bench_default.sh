# The default bench line (what the driver runs), untraced.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err && echo BENCH_OK
