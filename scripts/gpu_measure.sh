# Measurement runs on the GPU box (through gpurun, from the repo root), one subcommand per call:
#   bash scripts/gpu_measure.sh bench      full bench.py line (N = 1, the driver's arguments)
#   bash scripts/gpu_measure.sh dist2      bench.py --gpus 2 without a launcher (two ranks on the box's GPU)
#   bash scripts/gpu_measure.sh cli        GPU CLI tests + scripts/cli_scale_check.py (2M reads, identity check)
#   bash scripts/gpu_measure.sh pipeline   host packer (scripts/pack_bench.py) + host pipeline at 2/4/8M chunks
#   bash scripts/gpu_measure.sh rocprof    rocprofv3 --kernel-trace --stats of bench.py --steps 10
# Outputs land in gpurun_out/ (copy what should be kept into profiles/<round>/).
set -o pipefail
mkdir -p gpurun_out
R=$(pwd)
case $1 in
  bench)
    timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_full.json 2> gpurun_out/bench_full.err && echo BENCH_OK ;;
  dist2)
    timeout -k 10 600 python -u bench.py --gpus 2 --steps 10 --warmup 2 --no-cpu-baseline --no-extra > gpurun_out/dist2.json 2> gpurun_out/dist2.err && echo DIST2_OK ;;
  cli)
    timeout -k 10 600 python -u -m pytest tests/test_cli_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/cli_gpu.log 2>&1 && echo CLI_GPU_OK &&
    timeout -k 10 600 python -u scripts/cli_scale_check.py --reads 2000000 > gpurun_out/cli_scale.json 2> gpurun_out/cli_scale.err && echo CLI_SCALE_OK ;;
  pipeline)
    timeout -k 10 120 python -u scripts/pack_bench.py 1 4 8 16 > gpurun_out/pack_bench.log 2>&1 && echo PACK_OK &&
    timeout -k 10 300 python -u -c "
import argparse, json, sys
sys.argv = ['bench.py']
import bench, torch
from find_circ2_amd import scan
a = argparse.Namespace(workload='hg19', pairs=50_000_000, read_len=100, locus_ordered=False)
opt, g, b = bench.build_workload(a, 0, torch.device('cuda', 0))
b._bench_ref_results = torch.from_numpy(scan(opt, g, b).results[:b.n].cpu().numpy().copy())
for ch in (2_000_000, 4_000_000, 8_000_000):
    print(json.dumps(bench.host_pipeline(opt, g, b, chunk=ch)), flush=True)
" > gpurun_out/host_pipe.log 2>&1 && echo PIPE_OK ;;
  rocprof)
    mkdir -p gpurun_out/prof_kt && export TMPDIR=/tmp && cd /tmp &&
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_kt/kt_hg19 -o kt --output-format csv -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-extra --no-strong --no-config4 > $R/gpurun_out/prof_kt/kt_hg19.out 2>&1 && echo PROF_OK ;;
  *) echo "usage: $0 bench|dist2|cli|pipeline|rocprof"; exit 2 ;;
esac
