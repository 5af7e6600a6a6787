#!/usr/bin/env python
"""cProfile of the default CLI on the genome-scale input of cli_scale_check.py (dev tool)."""
import cProfile
import os
import pstats
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "scripts")]

from cli_scale_check import make_genome, write_fasta, write_sam  # noqa: E402


def main():
    reads = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
    scale = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
    from find_circ2_amd import cli, sq_table
    rng = np.random.default_rng(2024)
    names, sizes = sq_table(os.path.join(ROOT, "tests", "golden", "test_norm.sam"))
    sizes = [max(1000, int(s * scale)) for s in sizes]
    d = "/tmp/fc2_prof"
    os.makedirs(d, exist_ok=True)
    fa, sam = os.path.join(d, "genome.fa"), os.path.join(d, "reads.sam")
    seqs = make_genome(fa, names, sizes, rng)
    write_sam(sam, seqs, reads, rng)
    write_fasta(fa, seqs)
    del seqs
    for run in range(2):                  # the second run finds the .byo_index
        pr = cProfile.Profile()
        t0 = time.time()
        pr.enable()
        rc = cli.main(["-G", fa, "-o", os.path.join(d, "out%d" % run), "-q", sam])
        pr.disable()
        print("run", run, "rc", rc, "wall %.2f s" % (time.time() - t0), flush=True)
        pstats.Stats(pr).sort_stats("cumulative").print_stats(25)


if __name__ == "__main__":
    main()
