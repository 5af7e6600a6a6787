#!/usr/bin/env python
"""Same-box A/B of the whole CLI (two-thread loop, GPU search): libfc2_<NAME>.so against the tree's
libfc2.so on one generated hg19-sized input, alternating, one process per run (the library is chosen
at import through FC2_LIB_VARIANT).  usage: ab_cli.py NAME [rounds] [reads]"""
import os
import re
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "scripts")]


def main():
    name = sys.argv[1]
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    reads = int(sys.argv[3]) if len(sys.argv) > 3 else 2_000_000
    from cli_scale_check import make_genome, write_fasta, write_sam
    from find_circ2_amd import sq_table
    d = "/tmp/fc2_abcli"
    os.makedirs(d, exist_ok=True)
    fa, sam = os.path.join(d, "genome.fa"), os.path.join(d, "reads.sam")
    rng = np.random.default_rng(2024)
    names, sizes = sq_table(os.path.join(ROOT, "tests", "golden", "test_norm.sam"))
    seqs = make_genome(fa, names, sizes, rng)
    write_sam(sam, seqs, reads, rng)
    write_fasta(fa, seqs)
    del seqs
    for r in range(rounds + 1):                  # round 0 builds the .byo_index (not reported)
        for v in (name, "cur"):
            env = dict(os.environ)
            env.pop("FC2_LIB_VARIANT", None)
            if v != "cur":
                env["FC2_LIB_VARIANT"] = v
            out = os.path.join(d, "out_" + v)
            subprocess.run([sys.executable, "-c", "import sys; from find_circ2_amd import cli; "
                            "sys.exit(cli.main(['-G', %r, '-o', %r, '-q', %r]))" % (fa, out, sam)],
                           env=env, check=True, cwd=ROOT)
            log = open(os.path.join(out, "run.log")).read()
            rate = re.search(r"overall ([0-9.]+)k reads/second", log).group(1)
            st = re.search(r"read loop stages: (.*)", log).group(1)
            if r:
                print(v, rate, st, flush=True)


if __name__ == "__main__":
    main()
