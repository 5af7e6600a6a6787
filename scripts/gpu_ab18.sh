set -o pipefail
mkdir -p gpurun_out
# three-lane window loads: one offset permute per instruction where it serves one window class
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernel_forms.py "tests/test_gpu_parity.py::test_word_layout_vs_oracle" tests/test_gpu_parity.py::test_config5_shape_variable_length_150bp -x -q --timeout 300 --timeout-method thread > gpurun_out/ab18_tests.log 2>&1 && echo TESTS_OK &&
for r in 1 2; do for v in prev cur; do
  if [ $v = cur ]; then unset FC2_LIB_VARIANT; else export FC2_LIB_VARIANT=$v; fi
  timeout -k 10 150 python scripts/ab_kernel.py --variants k32nt1 --rounds 5 --read-len 150 2>/dev/null | sed "s/^/$v L150 /"
done; done > gpurun_out/ab18.jsonl; cat gpurun_out/ab18.jsonl; tail -2 gpurun_out/ab18_tests.log
