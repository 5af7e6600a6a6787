# Same-process kernel A/B on the GPU box (run through gpurun from the repo root):
#   bash scripts/gpu_ab.sh NAME "<scripts/ab_kernel.py arguments>" [REPEATS] [TESTS]
# e.g. bash scripts/gpu_ab.sh tri "--read-len 150 --second prev --variants k32nt1,2:k32nt1" 2
# Builds nothing (build libfc2_ab.so / libfc2_<second>.so beforehand: make -C find_circ2_amd/csrc ab,
# scripts/ab_build.sh REV NAME).  TESTS=1 (default) first runs the GPU parity subset on the shipped
# library.  Each repeat runs ab_kernel.py once (one process: interleaved variants, medians) and
# appends its JSON lines to gpurun_out/ab_NAME.jsonl.
set -o pipefail
NAME=$1; ARGS=$2; REPEATS=${3:-2}; TESTS=${4:-1}
mkdir -p gpurun_out
if [ "$TESTS" = 1 ]; then
  timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py tests/test_gpu_kernel_forms.py \
    -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/ab_${NAME}_tests.log 2>&1 || exit 1
  echo TESTS_OK
fi
: > gpurun_out/ab_$NAME.jsonl
for r in $(seq 1 $REPEATS); do
  timeout -k 10 300 python -u scripts/ab_kernel.py $ARGS >> gpurun_out/ab_$NAME.jsonl 2>> gpurun_out/ab_$NAME.err || exit 1
done
cat gpurun_out/ab_$NAME.jsonl
