"""Which engine moves a D2H copy into pinned host memory (blit kernel or a DMA engine), and what a
concurrent copy costs the breakpoint scan (12.5M hg19-shaped pairs, the strong-scaling batch size).
hipMemcpyAsync(..., hipMemcpyDeviceToHost) is run by the __amd_rocclr_copyBuffer shader on this
image; hipMemcpyDeviceToDeviceNoCU (HIP's "copy without compute units") is tried as the alternative,
with the pinned host buffer as the destination.  Prints JSON lines; run it under rocprofv3
--kernel-trace to see which copies became kernels."""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from find_circ2_amd import scan  # noqa: E402

hip = ctypes.CDLL("libamdhip64.so")
hip.hipMemcpyAsync.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p]
hip.hipMemcpyAsync.restype = ctypes.c_int
D2H, D2D_NOCU = 2, 1024

dev = torch.device("cuda", 0)
a = argparse.Namespace(workload="hg19", pairs=12_500_000, read_len=100, locus_ordered=False)
opt, g, b = bench.build_workload(a, 0, dev)
out = scan(opt, g, b)
torch.cuda.synchronize(dev)
MB = 100
src = torch.empty(MB << 20, dtype=torch.uint8, device=dev).fill_(7)
host = torch.empty(MB << 20, dtype=torch.uint8).pin_memory()
side = torch.cuda.Stream(dev)
main = torch.cuda.current_stream(dev)


DST = {"ptr": host.data_ptr()}


def copy(kind, nbytes):
    rc = hip.hipMemcpyAsync(DST["ptr"], src.data_ptr(), nbytes, kind, ctypes.c_void_p(side.cuda_stream))
    if rc != 0:
        raise RuntimeError("hipMemcpyAsync kind %d: error %d" % (kind, rc))


def t_copy(kind, nbytes):
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    copy(kind, nbytes)
    torch.cuda.synchronize(dev)
    return (time.perf_counter() - t0) * 1e3


def t_scan(kind=None, nbytes=0, both=False):
    """The scan's own span (events on its stream); with both=True the span from the common start to
    the later of scan and copy.  The copy's stream waits on an event the scan's stream records just
    before the scan, so the two start together, as a merge copy and the next batch's scan do."""
    torch.cuda.synchronize(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    with torch.cuda.stream(main):
        torch.cuda._sleep(4_000_000)       # hold the stream so every launch lands before e0 fires
    e0.record(main)
    if kind is not None:
        side.wait_event(e0)
        copy(kind, nbytes)
    scan(opt, g, b, out=out, stream=main.cuda_stream)
    if both and kind is not None:
        done = torch.cuda.Event()
        done.record(side)
        main.wait_event(done)
    e1.record(main)
    torch.cuda.synchronize(dev)
    return e0.elapsed_time(e1)


res = {"scan_ms_alone": None}
for _ in range(2):
    t_scan()
res["scan_ms_alone"] = round(float(np.median([t_scan() for _ in range(7)])), 4)
for name, kind in (("d2h", D2H), ("d2d_nocu", D2D_NOCU)):
    try:
        for nb in (25 << 20, 100 << 20):
            t_copy(kind, nb)
            res["%s_%dMB_copy_ms" % (name, nb >> 20)] = round(min(t_copy(kind, nb) for _ in range(5)), 4)
            res["%s_%dMB_scan_beside_ms" % (name, nb >> 20)] = round(float(np.median([t_scan(kind, nb)
                                                                                      for _ in range(7)])), 4)
            res["%s_%dMB_scan_and_copy_ms" % (name, nb >> 20)] = round(float(np.median(
                [t_scan(kind, nb, both=True) for _ in range(7)])), 4)
        host.zero_()
        copy(kind, 1 << 20)
        torch.cuda.synchronize(dev)
        res["%s_bytes_ok" % name] = bool((host[:1 << 20] == 7).all())
    except Exception as ex:
        res[name + "_error"] = repr(ex)

# Does a non_blocking copy_ return before the copy has run?  The strong-scaling merge copies into a
# /dev/shm segment page-locked with hipHostRegister (shard.SharedCompactResults); the probe above
# into hipHostMalloc memory.  The GPU is held busy by a spin kernel on the copy's stream while the
# host times the copy_ call itself: microseconds = asynchronous, the spin's length = synchronous.
from find_circ2_amd.shard import SharedResults  # noqa: E402

shm = SharedResults((25 << 20) // 8, create=True, pin=True)
dst = {"pinned_alloc": host[:25 << 20], "shm_registered": shm.tensor.view(torch.uint8)}
for name, d in dst.items():
    calls = []
    for _ in range(5):
        torch.cuda.synchronize(dev)
        with torch.cuda.stream(side):
            torch.cuda._sleep(8_000_000)
            t0 = time.perf_counter()
            d.copy_(src[:25 << 20], non_blocking=True)
            calls.append((time.perf_counter() - t0) * 1e3)
        t1 = time.perf_counter()
        torch.cuda.synchronize(dev)
        wait = (time.perf_counter() - t1) * 1e3
    res["copy_call_ms_%s" % name] = round(float(np.median(calls)), 4)
    res["sync_after_call_ms_%s" % name] = round(wait, 4)
    res["is_pinned_%s" % name] = bool(d.is_pinned())
# The scan beside copies into the hipHostRegister'ed /dev/shm segment (the merge's destination)
shm100 = SharedResults((100 << 20) // 8, create=True, pin=True)
DST["ptr"] = shm100.tensor.data_ptr()
for nb in (25 << 20, 100 << 20):
    t_copy(D2H, nb)
    res["shm_%dMB_copy_ms" % (nb >> 20)] = round(min(t_copy(D2H, nb) for _ in range(5)), 4)
    res["shm_%dMB_scan_beside_ms" % (nb >> 20)] = round(float(np.median([t_scan(D2H, nb) for _ in range(7)])), 4)
    res["shm_%dMB_scan_and_copy_ms" % (nb >> 20)] = round(float(np.median(
        [t_scan(D2H, nb, both=True) for _ in range(7)])), 4)
shm100.close()
shm.close()
print(json.dumps(res), flush=True)
