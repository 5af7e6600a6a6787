#!/usr/bin/env python
"""Start-up cost of the CLI on an hg19-sized genome: index build, 2-bit packing, upload.

Writes an hg19-shaped synthetic FASTA (the 93 @SQ contigs of tests/golden/test_norm.sam,
3.137 Gbp, 50-nt lines, ~7 % of bases in N runs) and times
``Genome.from_fasta(write_index=True)`` twice: without and then with the .byo_index file
(the reference's find_circ.py:110-115 fast path).

usage: python scripts/genome_load_time.py [--out DIR] [--scale F]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def write_fasta(path, names, sizes, seed=7, width=50):
    rng = np.random.default_rng(seed)
    acgt = np.frombuffer(b"ACGT", np.uint8)
    with open(path, "wb") as f:
        for name, size in zip(names, sizes):
            f.write(b">" + name.encode() + b"\n")
            for s0 in range(0, size, 50_000_000):          # bounded memory per piece
                n = min(50_000_000, size - s0)
                seq = acgt[rng.integers(0, 4, n, dtype=np.uint8)]
                for _ in range(max(1, n // 2_000_000)):     # N runs (~7 %)
                    a = int(rng.integers(0, n))
                    seq[a:a + int(rng.integers(1000, 140_000))] = ord("N")
                if s0 + n < size:
                    assert n % width == 0
                full = n // width
                body = np.concatenate([seq[:full * width].reshape(full, width),
                                       np.full((full, 1), 10, np.uint8)], axis=1).tobytes()
                f.write(body)
                if n % width:
                    f.write(seq[full * width:].tobytes() + b"\n")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="/tmp/fc2_genome")
    ap.add_argument("--scale", type=float, default=1.0)
    a = ap.parse_args()
    from find_circ2_amd import Genome, sq_table
    names, sizes = sq_table(os.path.join(ROOT, "tests", "golden", "test_norm.sam"))
    sizes = [max(1000, int(s * a.scale)) // 50 * 50 if s * a.scale > 50_000_000 else max(1000, int(s * a.scale))
             for s in sizes]
    os.makedirs(a.out, exist_ok=True)
    fa = os.path.join(a.out, "hg19_synth.fa")
    for p in (fa, fa + ".byo_index"):
        if os.path.exists(p):
            os.remove(p)
    t0 = time.time()
    write_fasta(fa, names, sizes)
    t_write = time.time() - t0
    out = {"bases": int(sum(sizes)), "fasta_bytes": os.path.getsize(fa), "write_s": round(t_write, 1)}
    for tag in ("no_index", "with_index"):
        t0 = time.time()
        g = Genome.from_fasta(fa, device="cuda:0", write_index=True)
        import torch
        torch.cuda.synchronize()
        out[tag + "_s"] = round(time.time() - t0, 2)
        out["device_bytes"] = int(sum(t.numel() * t.element_size() for t in (g.units, g.units_twin, g.nplane,
                                                                             g.ncoarse) if t is not None))
        del g
        torch.cuda.empty_cache()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
