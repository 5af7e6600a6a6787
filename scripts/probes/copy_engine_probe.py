"""Which engine moves a D2H copy into pinned host memory on this box (blit kernel or SDMA), and what
a concurrent copy costs a running scan-sized kernel.  Prints JSON lines; run under rocprofv3
--kernel-trace to see __amd_rocclr_copyBuffer dispatches."""
import json
import os
import time

import torch

dev = torch.device("cuda", 0)
env = {k: v for k, v in os.environ.items() if any(s in k for s in ("SDMA", "HSA_", "GPU_", "ROC_", "HIP_", "AMD_"))}
print(json.dumps({"env": env}), flush=True)
src = torch.empty(100 << 20, dtype=torch.uint8, device=dev).fill_(7)
host = torch.empty(100 << 20, dtype=torch.uint8).pin_memory()
big = torch.randn(64 << 20, device=dev)
side = torch.cuda.Stream(dev)


def t_copy():
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    host.copy_(src, non_blocking=True)
    torch.cuda.synchronize(dev)
    return (time.perf_counter() - t0) * 1e3


def t_kernel(with_copy):
    torch.cuda.synchronize(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    if with_copy:
        with torch.cuda.stream(side):
            host.copy_(src, non_blocking=True)
    e0.record()
    for _ in range(4):
        big.mul_(1.0001)
    e1.record()
    torch.cuda.synchronize(dev)
    return e0.elapsed_time(e1)


for _ in range(2):
    t_copy(), t_kernel(False), t_kernel(True)
print(json.dumps({"d2h_100MB_ms": round(min(t_copy() for _ in range(5)), 3),
                  "kernel_ms_alone": round(min(t_kernel(False) for _ in range(5)), 3),
                  "kernel_ms_beside_copy": round(min(t_kernel(True) for _ in range(5)), 3)}), flush=True)
