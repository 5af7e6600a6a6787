"""Fuzz the GPU BGZF inflate (csrc/fc2_inflate.hip) with damaged real blocks: the blocks of a
gen_reads BAM (and of a level-6 / stored re-encoding) with random bit flips, byte runs overwritten,
cuts, appended garbage, wrong ISIZEs and pure noise, many thousands per launch.  Every launch must
complete; a block reported inflated must equal zlib's output of the same payload (its CRC-32 was
checked on the device).  One JSON line of counts.  Test infrastructure, not part of the product.

usage: python scripts/fuzz_inflate.py [--rounds R] [--blocks N] [--seed S]
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=8)
    ap.add_argument("--blocks", type=int, default=4000)
    ap.add_argument("--seed", type=int, default=99)
    a = ap.parse_args()
    import torch
    from cli_steady import prepare
    from inflate_bench import blocks
    from find_circ2_amd import _native as N
    d = tempfile.mkdtemp(prefix="fc2_fuzz_")
    _, bams, _, _ = prepare(d, [300000])
    raw = open(bams[300000], "rb").read()
    off, ln, isz, _ = blocks(raw)
    plain = [zlib.decompress(raw[o:o + n], -15) for o, n in zip(off, ln)]
    rng = np.random.default_rng(a.seed)
    forms = []                                  # (payload, isize) of valid blocks in three encodings
    for k, x in enumerate(plain):
        forms.append((raw[off[k]:off[k] + ln[k]], len(x)))
        if k % 4 == 0:
            for lv in (0, 6):
                c = zlib.compressobj(lv, zlib.DEFLATED, -15)
                forms.append((c.compress(x) + c.flush(), len(x)))
    dev = torch.device("cuda:0")
    L = N.lib()
    stream = torch.cuda.current_stream(dev).cuda_stream
    counts = {"launches": 0, "blocks": 0, "inflated": 0, "refused": 0, "wrong": 0, "status": {}}
    t0 = time.time()
    for r in range(a.rounds):
        pays, sizes, want = [], [], []
        for _ in range(a.blocks):
            p, n = forms[int(rng.integers(0, len(forms)))]
            b = bytearray(p)
            kind = int(rng.integers(0, 8))
            if kind == 0 and b:
                for _ in range(int(rng.integers(1, 6))):
                    k = int(rng.integers(0, len(b)))
                    b[k] ^= 1 << int(rng.integers(0, 8))
            elif kind == 1 and b:
                k = int(rng.integers(0, len(b)))
                b[k:k + 16] = rng.integers(0, 256, len(b[k:k + 16]), dtype=np.uint8).tobytes()
            elif kind == 2 and len(b) > 1:
                b = b[:int(rng.integers(0, len(b)))]
            elif kind == 3:
                b += rng.integers(0, 256, int(rng.integers(1, 64)), dtype=np.uint8).tobytes()
            elif kind == 4:
                n = int(rng.integers(0, 65537))
            elif kind == 5:
                b = bytearray(rng.integers(0, 256, int(rng.integers(0, 20000)), dtype=np.uint8).tobytes())
            # kind 6, 7: intact
            pays.append(bytes(b))
            sizes.append(n)
            want.append(zlib.decompress(p, -15) if len(p) else b"")
        o, buf = [], bytearray()
        for p in pays:
            buf += bytes(int(rng.integers(0, 4)))
            o.append(len(buf))
            buf += p
        buf += bytes(64)
        src = torch.tensor(np.frombuffer(bytes(buf), np.uint8), device=dev)
        t = [torch.tensor(np.array(x, np.uint32).view(np.int32), device=dev)
             for x in (o, [len(p) for p in pays], sizes, [zlib.crc32(w) for w in want])]
        dst = torch.zeros(a.blocks * 65536, dtype=torch.uint8, device=dev)
        st = torch.full((a.blocks,), -1, dtype=torch.int32, device=dev)
        N.check(L.fc2_bgzf_inflate_launch(src.data_ptr(), t[0].data_ptr(), t[1].data_ptr(), t[2].data_ptr(),
                                          t[3].data_ptr(), dst.data_ptr(), st.data_ptr(), a.blocks,
                                          ctypes.c_void_p(stream)))
        torch.cuda.synchronize(dev)
        s = st.cpu().numpy()
        out = dst.cpu().numpy()
        counts["launches"] += 1
        counts["blocks"] += a.blocks
        for i in range(a.blocks):
            counts["status"][int(s[i])] = counts["status"].get(int(s[i]), 0) + 1
            if s[i] == 0:
                counts["inflated"] += 1
                if out[i * 65536:i * 65536 + sizes[i]].tobytes() != want[i] or sizes[i] != len(want[i]):
                    counts["wrong"] += 1
            else:
                counts["refused"] += 1
        print("round %d: %s (%.0f s)" % (r, json.dumps(counts["status"]), time.time() - t0), file=sys.stderr, flush=True)
    counts["status"] = {str(k): v for k, v in sorted(counts["status"].items())}
    print(json.dumps(counts))
    return 1 if counts["wrong"] else 0


if __name__ == "__main__":
    sys.exit(main())
