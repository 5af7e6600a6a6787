# Every GPU-box run of this repo, one parameterised runner (through gpurun, from the repo root):
#   bash scripts/gpu_run.sh suite                 GPU tests + smoke + a short bench line (the round-end trio)
#   bash scripts/gpu_run.sh tests ARGS...         pytest -m gpu on the given test files / -k expressions
#   bash scripts/gpu_run.sh cputests ARGS...      pytest -m "not gpu" on the box (as a non-root user)
#   bash scripts/gpu_run.sh bench [ARGS...]       bench.py with the driver's defaults (+ ARGS)
#   bash scripts/gpu_run.sh dist N [ARGS...]      bench.py --gpus N without a launcher (N ranks on the box's GPU)
#   bash scripts/gpu_run.sh torchrun N [ARGS...]  bench.py under torch.distributed.run with N ranks on the one GPU
#   bash scripts/gpu_run.sh cli                   GPU CLI tests + scripts/cli_scale_check.py (2M reads)
#   bash scripts/gpu_run.sh abcli [ARGS...]       scripts/prof/ab_cli.py (same-box CLI A/B)
#   bash scripts/gpu_run.sh ab NAME "ARGS" [REPS] same-process kernel A/B (scripts/ab_kernel.py)
#   bash scripts/gpu_run.sh rocprof [NAME]        rocprofv3 --kernel-trace --stats of the headline bench
#   bash scripts/gpu_run.sh pmc                   the HBM PMC passes of scripts/profile_round.sh
#   bash scripts/gpu_run.sh py SCRIPT [ARGS...]   any probe script under scripts/ (one process)
#   bash scripts/gpu_run.sh steady [ARGS...]      scripts/cli_steady.py (the CLI in anchor pairs/s, thread curve)
#   bash scripts/gpu_run.sh cliprof [N] [SITES]   rocprofv3 --kernel-trace --stats of the CLI on N reads
# Outputs land in gpurun_out/ (copy what should be kept into profiles/<round>/).  Every GPU step has
# its own time limit and the steps are chained with &&: a failure ends the call.
set -o pipefail
mkdir -p gpurun_out
R=$(pwd)
PYT="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
cmd=$1; shift
case $cmd in
  suite)
    timeout -k 10 1000 $PYT tests -m gpu > gpurun_out/gpu_tests.log 2>&1 && echo TESTS_OK &&
    timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && echo SMOKE_OK &&
    timeout -k 10 400 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-extra > gpurun_out/bench_short.json 2> gpurun_out/bench_short.err && echo BENCH_OK ;;
  tests)
    timeout -k 10 1000 $PYT -m gpu "$@" > gpurun_out/gpu_tests_part.log 2>&1 && echo TESTS_OK ;;
  cputests)
    timeout -k 10 900 $PYT -m "not gpu" "$@" > gpurun_out/cpu_tests_box.log 2>&1 && echo CPUTESTS_OK ;;
  bench)
    timeout -k 10 900 python -u bench.py "$@" > gpurun_out/bench.json 2> gpurun_out/bench.err && echo BENCH_OK ;;
  dist)
    n=$1; shift
    timeout -k 10 900 python -u bench.py --gpus $n "$@" > gpurun_out/bench_dist$n.json 2> gpurun_out/bench_dist$n.err && echo DIST_OK ;;
  torchrun)
    n=$1; shift
    timeout -k 10 900 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
      --master-port 29533 bench.py --gpus $n "$@" > gpurun_out/bench_torchrun$n.json 2> gpurun_out/bench_torchrun$n.err && echo TORCHRUN_OK ;;
  cli)
    timeout -k 10 600 $PYT tests/test_cli_gpu.py -m gpu > gpurun_out/cli_gpu.log 2>&1 && echo CLI_GPU_OK &&
    timeout -k 10 600 python -u scripts/cli_scale_check.py --reads 2000000 > gpurun_out/cli_scale.json 2> gpurun_out/cli_scale.err && echo CLI_SCALE_OK ;;
  abcli)
    timeout -k 10 900 python -u scripts/prof/ab_cli.py "$@" > gpurun_out/ab_cli.jsonl 2> gpurun_out/ab_cli.err && echo ABCLI_OK ;;
  ab)
    NAME=$1; ARGS=$2; REPS=${3:-2}
    timeout -k 10 600 $PYT tests/test_gpu_parity.py tests/test_gpu_fuzz.py tests/test_gpu_kernel_forms.py -m gpu \
      > gpurun_out/ab_${NAME}_tests.log 2>&1 || exit 1
    echo TESTS_OK
    : > gpurun_out/ab_$NAME.jsonl
    for r in $(seq 1 $REPS); do
      timeout -k 10 300 python -u scripts/ab_kernel.py $ARGS >> gpurun_out/ab_$NAME.jsonl 2>> gpurun_out/ab_$NAME.err || exit 1
    done
    cat gpurun_out/ab_$NAME.jsonl ;;
  rocprof)
    NAME=${1:-kt_hg19}
    mkdir -p gpurun_out/prof_kt && export TMPDIR=/tmp && cd /tmp &&
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_kt/$NAME -o kt --output-format csv -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extra --no-strong --no-config4 > $R/gpurun_out/prof_kt/$NAME.out 2>&1 && echo PROF_OK ;;
  pmc)
    bash scripts/profile_round.sh ;;
  steady)
    timeout -k 10 1000 python -u scripts/cli_steady.py "$@" > gpurun_out/steady.jsonl 2> gpurun_out/steady.err && echo STEADY_OK ;;
  cliprof)
    N=${1:-20000000}; S=${2:-0}
    mkdir -p gpurun_out/prof_cli && export TMPDIR=/tmp && cd /tmp &&
    timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_cli/cli_$N -o kt --output-format csv -- python3 $R/scripts/prof/cli_kernels.py $N $S > $R/gpurun_out/prof_cli/cli_$N.out 2>&1 && echo CLIPROF_OK ;;
  py)
    s=$1; shift
    timeout -k 10 900 python -u "$s" "$@" > gpurun_out/py_$(basename $s .py).out 2>&1 && echo PY_OK ;;
  *) sed -n 2,15p "$0"; exit 2 ;;
esac
