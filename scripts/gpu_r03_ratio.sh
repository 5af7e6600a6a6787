# Same box, same build: the 100-bp two-lane form and the 150-bp five-lane form against their probes.
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/ab_ratio.jsonl
timeout -k 10 300 python -u scripts/ab_kernel.py --pairs 50000000 --variants k32nt1,probe >> gpurun_out/ab_ratio.jsonl 2>> gpurun_out/ab_ratio.err &&
timeout -k 10 300 python -u scripts/ab_kernel.py --read-len 150 --pairs 25000000 --variants k32nt1,probe_tri3 >> gpurun_out/ab_ratio.jsonl 2>> gpurun_out/ab_ratio.err &&
timeout -k 10 300 python -u scripts/ab_kernel.py --pairs 50000000 --variants k32nt1,probe >> gpurun_out/ab_ratio.jsonl 2>> gpurun_out/ab_ratio.err &&
timeout -k 10 300 python -u scripts/ab_kernel.py --read-len 150 --pairs 25000000 --variants k32nt1,probe_tri3 >> gpurun_out/ab_ratio.jsonl 2>> gpurun_out/ab_ratio.err &&
cat gpurun_out/ab_ratio.jsonl
