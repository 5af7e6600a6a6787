set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_cli_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/cli_gpu.log 2>&1 && echo CLI_GPU_OK &&
timeout -k 10 600 python -u scripts/cli_scale_check.py --reads 2000000 > gpurun_out/cli_scale.json 2> gpurun_out/cli_scale.err && echo CLI_SCALE_OK
