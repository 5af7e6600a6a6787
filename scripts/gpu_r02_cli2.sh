set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u scripts/cli_scale_check.py --reads 2000000 --only native,native_gpus2,native_allhits > gpurun_out/cli_scale_quick.json 2> gpurun_out/cli_scale_quick.err && echo CLI_SCALE_OK
