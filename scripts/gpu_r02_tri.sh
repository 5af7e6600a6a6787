set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernel_forms.py tests/test_gpu_fullsize.py tests/test_gpu_parity.py tests/test_gpu_fuzz.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/tri_tests.log 2>&1 && echo TESTS_OK &&
bash scripts/gpu_ab.sh tri150 "--read-len 150 --pairs 25000000 --second prev --variants k32nt1,2:k32nt1,probe --rounds 7" 3 0 &&
bash scripts/gpu_ab.sh tri100 "--second prev --variants k32nt1,2:k32nt1 --rounds 5" 1 0
