set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernel_forms.py tests/test_gpu_genomes.py "tests/test_gpu_parity.py::test_word_layout_vs_oracle" -x -q --timeout 300 --timeout-method thread > gpurun_out/tri_tests.log 2>&1 && echo TRI_TESTS_OK &&
for r in 1 2; do
  timeout -k 10 150 python scripts/ab_kernel.py --variants k32nt1,k32nt1tri0,probe --rounds 5 --read-len 150 2>/dev/null | sed "s/^/L150 /"
  timeout -k 10 150 python scripts/ab_kernel.py --variants k32nt1,k32nt1tri1 --rounds 5 2>/dev/null | sed "s/^/L100 /"
done > gpurun_out/ab14.jsonl; cat gpurun_out/ab14.jsonl; tail -2 gpurun_out/tri_tests.log
