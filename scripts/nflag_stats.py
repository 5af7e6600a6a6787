#!/usr/bin/env python
"""How often does a read-order window of the bench workload need the N plane?

For the bench's 50M-pair hg19-shaped workload: fraction of windows flagged by
the LDS super map (nsuper), by the 1024-base coarse map, and windows that
actually contain an 'N'; and the number of maximal N runs in the genome.
Prints one JSON line.  GPU (uses the device genome/batch builders).
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pairs", type=int, default=50_000_000)
    a = ap.parse_args()
    import torch
    import bench
    dev = torch.device("cuda", 0)
    args = argparse.Namespace(workload="hg19", pairs=a.pairs, read_len=100, locus_ordered=False)
    opt, g, b = bench.build_workload(args, 0, dev)
    e = opt.asize - opt.margin
    P = b.pairs[:16 * b.n].view(b.n, 16)
    i32 = P[:, :12].contiguous().view(torch.int32).view(b.n, 3)
    a_pos, b_aend, chrom = i32[:, 0].long(), i32[:, 1].long(), i32[:, 2].long()
    L = P[:, 12].long() | (P[:, 13].long() << 8)
    l = L - 2 * e
    W = l + 2
    cs = g.d_chrom_start[chrom]
    wsA = cs + a_pos + e
    wsB = cs + b_aend - e - W
    nsuper = g.nsuper.view(torch.int32).long() & 0xFFFFFFFF
    coarse = g.ncoarse.view(torch.int32).long() & 0xFFFFFFFF
    nplane = g.nplane

    def bit(words, k):
        return ((words[k >> 5] >> (k & 31)) & 1) != 0

    def flags(ws):
        hi = ws + W - 1
        s = g.nsuper_shift
        fs = bit(nsuper, ws >> s) | bit(nsuper, hi >> s)
        fc = bit(coarse, ws >> 10) | bit(coarse, hi >> 10)
        # exact: any N bit in [ws, ws+W)
        u0 = ws >> 6
        exact = torch.zeros_like(fs)
        for j in range(3):
            u = (u0 + j).clamp(max=g.n_units - 1)
            w = nplane[u]
            base = (u0 + j) * 64
            lo = (ws - base).clamp(0, 64)
            hi2 = (ws + W - base).clamp(0, 64)
            m = torch.where(hi2 > lo, ((torch.ones_like(w) << (hi2 - lo).clamp(max=63)) - 1) << lo, torch.zeros_like(w))
            m = torch.where(hi2 - lo >= 64, torch.full_like(w, -1), m)
            exact |= (w & m) != 0
        return fs, fc, exact

    out = {"pairs": b.n, "nsuper_shift": g.nsuper_shift}
    for name, ws in (("A", wsA), ("B", wsB)):
        fs, fc, ex = flags(ws)
        out[name] = {"nsuper_flagged": float(fs.float().mean()), "coarse_flagged": float(fc.float().mean()),
                     "contains_N": float(ex.float().mean())}
    # maximal N runs: starts = N bits whose predecessor is not N
    n = nplane
    prev_msb = torch.cat([torch.zeros(1, dtype=n.dtype, device=n.device), (n[:-1] >> 63) & 1])
    starts = n & ~((n << 1) | prev_msb)
    out["n_runs"] = sum(int(((starts >> k) & 1).sum()) for k in range(64))
    out["n_bases"] = sum(int(((n >> k) & 1).sum()) for k in range(64))
    print(json.dumps(out))


if __name__ == "__main__":
    main()
