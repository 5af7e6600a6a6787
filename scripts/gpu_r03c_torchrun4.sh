# Round 3 (third session): the driver's N > 1 launch form on the one-GPU box (four ranks share cuda:0,
# so the rates are one GPU's): torch.distributed.run as the driver starts it, on the final tree
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 \
    --master-port 29531 bench.py --gpus 4 --steps 5 --warmup 2 > gpurun_out/torchrun4.json 2> gpurun_out/torchrun4.err && echo TORCHRUN_OK
