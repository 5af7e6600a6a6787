set -o pipefail
mkdir -p gpurun_out
# device pipeline at 100 bp (narrow last row) and 150 bp (full last row)
timeout -k 10 300 python -u -c "
import argparse, json, torch, bench
for L in (100, 150):
    a = argparse.Namespace(workload='hg19', pairs=8_000_000, read_len=L, locus_ordered=False)
    opt, g, b = bench.build_workload(a, 0, torch.device('cuda', 0))
    from find_circ2_amd import scan
    b._bench_ref_results = scan(opt, g, b).results[:b.n].cpu()
    r = bench.device_pipeline(opt, g, b, reps=3)
    print(L, json.dumps(r))
    assert r['results_equal_device_resident_scan'], L
" > gpurun_out/pipe150.log 2>&1 && echo PIPE_OK; tail -4 gpurun_out/pipe150.log
