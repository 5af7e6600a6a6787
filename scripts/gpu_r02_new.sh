set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_integration.py tests/test_read_limits.py tests/test_gpu_fullsize.py -m gpu -x -v -s --timeout 300 --timeout-method thread > gpurun_out/new_tests.log 2>&1 && echo NEW_TESTS_OK
