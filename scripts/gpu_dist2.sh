set -o pipefail
mkdir -p gpurun_out
# two ranks sharing the box's one GPU: the N>1 bench path (gloo timing group, weak scaling)
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 > gpurun_out/dist2.json 2> gpurun_out/dist2.err && echo DIST2_OK && cat gpurun_out/dist2.json
