set -o pipefail
mkdir -p gpurun_out
# three-lane exchange through 4 LDS slots (48 KB per 512-pair block, <= 80 VGPRs: 6 waves/SIMD)
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernel_forms.py "tests/test_gpu_parity.py::test_word_layout_vs_oracle" tests/test_gpu_parity.py::test_config5_shape_variable_length_150bp tests/test_gpu_parity.py::test_edge_lengths_and_long_reads -x -q --timeout 300 --timeout-method thread > gpurun_out/ab22_tests.log 2>&1 && echo TESTS_OK &&
for r in 1 2; do
  timeout -k 10 150 python scripts/ab_kernel.py --second prev --variants k32nt1,2:k32nt1,probe --rounds 7 --read-len 150 2>gpurun_out/ab22.err | sed "s/^/L150 /"
  timeout -k 10 150 python scripts/ab_kernel.py --second prev --variants k32nt1,2:k32nt1 --rounds 7 2>>gpurun_out/ab22.err | sed "s/^/L100 /"
done > gpurun_out/ab22.jsonl; cat gpurun_out/ab22.jsonl; tail -2 gpurun_out/ab22_tests.log
