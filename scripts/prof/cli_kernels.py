"""The CLI's GPU work under rocprofv3 (`rocprofv3 --kernel-trace --stats -- python3 scripts/prof/cli_kernels.py`):
cli_e2e's 2M-read input (hg19-shaped genome), the CLI run in this process (cli.main, the default
native loop and its ctxpipe search) so the process ends normally and the profiler writes its files
-- `python -m` ends with os._exit, which leaves no profile.  Prints the run.log phases as JSON."""
import json
import os
import re
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "scripts")]


def main():
    import numpy as np
    from cli_scale_check import make_genome, write_fasta, write_sam
    from find_circ2_amd import cli, sq_table
    reads = int(sys.argv[1]) if len(sys.argv) > 1 else 2_000_000
    d = tempfile.mkdtemp(prefix="fc2_cli_kernels_", dir="/tmp")
    fa, sam = os.path.join(d, "genome.fa"), os.path.join(d, "reads.sam")
    rng = np.random.default_rng(2024)
    names, sizes = sq_table(os.path.join(ROOT, "tests", "golden", "test_norm.sam"))
    seqs = make_genome(fa, names, sizes, rng)
    write_sam(sam, seqs, reads, rng)
    write_fasta(fa, seqs)
    del seqs
    out = os.path.join(d, "out")
    t0 = time.time()
    rc = cli.main(["-G", fa, "-o", out, "-q", sam])
    wall = time.time() - t0
    log = open(os.path.join(out, "run.log")).read()
    ph = re.search(r"process phases: (.*)", log)
    print(json.dumps({"rc": rc, "main_s": round(wall, 3), "reads": reads,
                      "phases": dict(re.findall(r"(\w+)=([0-9.naN]+)", ph.group(1))) if ph else None,
                      "search": [l.split("\t")[-1] for l in log.splitlines() if "breakpoint search" in l]}))


if __name__ == "__main__":
    main()
