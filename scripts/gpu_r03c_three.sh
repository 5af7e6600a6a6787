set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py -m gpu -x -v --timeout 300 --timeout-method thread -k "three or configs4 or stream_share" > gpurun_out/three.log 2>&1 && echo THREE_OK &&
timeout -k 10 600 python -u bench.py --steps 10 --warmup 3 --no-cli > gpurun_out/bench_three.json 2> gpurun_out/bench_three.err && echo BENCH_OK
