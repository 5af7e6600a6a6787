# After folding the escape count into the escape-slot block (one D2H copy per batch instead of two plus a
# 4-byte one): the repetitions that used to lose the copy/scan overlap, and the GPU tests of the forms.
set -o pipefail
mkdir -p gpurun_out
REPEAT=12 timeout -k 10 900 python -u scripts/probes/strong_streams_probe.py > gpurun_out/strong_single_block.jsonl 2> gpurun_out/strong_single_block.err && echo REPEAT_OK &&
timeout -k 10 900 python -u -m pytest tests/test_gpu_compact.py tests/test_gpu_fullsize.py tests/test_bench_launch.py -m gpu -x -v --timeout 600 --timeout-method thread > gpurun_out/single_block_tests.log 2>&1 && echo TESTS_OK
cut -c1-110 gpurun_out/strong_single_block.jsonl; tail -3 gpurun_out/single_block_tests.log
