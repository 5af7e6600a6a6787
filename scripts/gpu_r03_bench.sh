# Round 3: the sort probe with its kernel trace and line counters, then the
# default bench line and its kernel-trace profile.
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out/prof_kt gpurun_out/prof_sort
timeout -k 10 120 ./scripts/sort_probe 50000000 > gpurun_out/sort_probe.jsonl 2> gpurun_out/sort_probe.err && echo PROBE_OK &&
export TMPDIR=/tmp && cd /tmp &&
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_sort/kt -o kt --output-format csv -- $R/scripts/sort_probe 50000000 > $R/gpurun_out/prof_sort/kt.out 2>&1 && echo PROBE_KT_OK &&
timeout -s KILL 180 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum -d $R/gpurun_out/prof_sort/req -o pmc --output-format csv -- $R/scripts/sort_probe 50000000 > $R/gpurun_out/prof_sort/req.out 2>&1 && echo PROBE_PMC_OK &&
cd $R &&
timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_full.json 2> gpurun_out/bench_full.err && echo BENCH_OK &&
cd /tmp &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_kt/kt_hg19 -o kt --output-format csv -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-extra --no-strong --no-config4 > $R/gpurun_out/prof_kt/kt_hg19.out 2>&1 && echo PROF_OK
