set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 python -u scripts/pack_bench.py 1 4 8 16 > gpurun_out/pack_bench.log 2>&1 && echo PACK_OK &&
timeout -k 10 600 python -u -m pytest tests/test_cli_gpu.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/cli_gpu.log 2>&1 && echo CLI_GPU_OK &&
timeout -k 10 300 python -u -c "
import sys, json, time, argparse
sys.argv=['bench.py']
import bench, torch
a = argparse.Namespace(workload='hg19', pairs=50_000_000, read_len=100, locus_ordered=False)
dev = torch.device('cuda', 0)
opt, g, b = bench.build_workload(a, 0, dev)
from find_circ2_amd import scan
b._bench_ref_results = torch.from_numpy(scan(opt, g, b).results[:b.n].cpu().numpy().copy())
for ch in (2_000_000, 4_000_000, 8_000_000):
    r = bench.host_pipeline(opt, g, b, chunk=ch)
    print(json.dumps(r), flush=True)
" > gpurun_out/host_pipe.log 2>&1 && echo PIPE_OK
