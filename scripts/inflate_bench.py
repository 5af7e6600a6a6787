"""GPU BGZF inflate (csrc/fc2_inflate.hip) against the CPU on the CLI's BAM input: the blocks of
scripts/gen_reads' BAM (fc2_sam_to_bam, zlib level 1) inflated by fc2_bgzf_inflate_launch in launches
of --batch blocks (the ingest's batch) and in one launch of all, timed with HIP events on the launch
stream, each block's CRC-32 checked on the device (and again here); the CPU leg is zlib on one core over the same blocks.  One JSON line.
Measurement infrastructure (not part of the product).

usage: python scripts/inflate_bench.py [--reads N] [--batch B] [--reps R]
"""
import argparse
import ctypes
import json
import os
import sys
import tempfile
import time
import zlib

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "scripts"))


def blocks(raw: bytes):
    """(payload offsets, payload lengths, isizes, crcs) of a BGZF file's blocks."""
    off, ln, isz, crc, pos = [], [], [], [], 0
    mv = memoryview(raw)
    while pos < len(raw):
        xlen = raw[pos + 10] | (raw[pos + 11] << 8)
        bsize = (raw[pos + 16] | (raw[pos + 17] << 8)) + 1
        off.append(pos + 12 + xlen)
        ln.append(bsize - 12 - xlen - 8)
        crc.append(int.from_bytes(mv[pos + bsize - 8:pos + bsize - 4], "little"))
        isz.append(int.from_bytes(mv[pos + bsize - 4:pos + bsize], "little"))
        pos += bsize
    return [np.array(x, np.uint32) for x in (off, ln, isz, crc)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reads", type=int, default=2_000_000)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    import torch
    from cli_steady import prepare
    from find_circ2_amd import _native as N
    d = tempfile.mkdtemp(prefix="fc2_inflate_")
    _, bams, _, _ = prepare(d, [a.reads])
    raw = open(bams[a.reads], "rb").read()
    off, ln, isz, crc = blocks(raw)
    n = len(off)
    dev = torch.device("cuda:0")
    src = torch.tensor(np.frombuffer(raw + bytes(64), np.uint8), device=dev)
    t_off, t_ln, t_isz, t_crc = (torch.tensor(x.view(np.int32), device=dev) for x in (off, ln, isz, crc))
    dst = torch.empty(n * 65536, dtype=torch.uint8, device=dev)
    st = torch.empty(n, dtype=torch.int32, device=dev)
    stream = torch.cuda.current_stream(dev)
    L = N.lib()

    def launch(i0, i1):
        N.check(L.fc2_bgzf_inflate_launch(src.data_ptr(), t_off[i0:].data_ptr(), t_ln[i0:].data_ptr(),
                                          t_isz[i0:].data_ptr(), t_crc[i0:].data_ptr(), dst[i0 * 65536:].data_ptr(),
                                          st[i0:].data_ptr(), i1 - i0, ctypes.c_void_p(stream.cuda_stream)))

    def timed(step):
        best = None
        for _ in range(a.reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for i0 in range(0, n, step):
                launch(i0, min(n, i0 + step))
            e1.record(stream)
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1)
            best = ms if best is None else min(best, ms)
        return best

    launch(0, n)
    torch.cuda.synchronize()
    s = st.cpu().numpy()
    out = dst.cpu().numpy()
    bad = sum(1 for i in range(n) if s[i] != 0 or zlib.crc32(out[i * 65536:i * 65536 + isz[i]].tobytes()) != crc[i])
    ms_all, ms_batch = timed(n), timed(a.batch)
    total = int(isz.sum())
    # CPU: zlib on one core, about 2 s of it
    t0, done, k = time.time(), 0, 0
    while time.time() - t0 < 2.0 and k < n:
        done += len(zlib.decompress(raw[off[k]:off[k] + ln[k]], -15))
        k += 1
    cpu_s = time.time() - t0
    print(json.dumps({
        "reads": a.reads, "blocks": n, "compressed_bytes": len(raw), "inflated_bytes": total,
        "bad_blocks": bad, "status_nonzero": int((s != 0).sum()),
        "gpu_one_launch_ms": round(ms_all, 3), "gpu_one_launch_GBps": round(total / ms_all / 1e6, 2),
        "gpu_batch": a.batch, "gpu_batched_ms": round(ms_batch, 3),
        "gpu_batched_GBps": round(total / ms_batch / 1e6, 2),
        "cpu_zlib_1core_GBps": round(done / cpu_s / 1e9, 3)}))


if __name__ == "__main__":
    main()
