#!/usr/bin/env python
"""Same-box A/B of the whole CLI (two-thread loop, GPU search): libfc2_<NAME>.so against the tree's
libfc2.so on one generated hg19-sized input, alternating, one process per run (the library is chosen
at import through FC2_LIB_VARIANT), in bench.py's two forms: BGZF BAM piped on stdin and SAM by path.
NAME may also be env:K=V[,K=V...] (the tree's library under those environment settings), and several
variants joined by '+'.  Every run's output files must equal the first run's.  One JSON line per run.
AB_TIMING=1: each run under FC2_CALLER_TIMING, its per-chunk phase times kept in
gpurun_out/abcli_timing/<variant>_<form>_<round>.txt.
usage: ab_cli.py NAME[+NAME...] [rounds] [reads]"""
import gzip
import json
import os
import re
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "scripts")]


def outputs(o):
    r = {}
    for f in ("circ_splice_sites.bed", "lin_splice_sites.bed", "multi_events.tsv"):
        r[f] = open(os.path.join(o, f), "rb").read()
    with gzip.open(os.path.join(o, "spliced_reads.fastq.gz"), "rb") as fh:
        r["reads"] = fh.read()
    return r


def main():
    name = sys.argv[1]
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    reads = int(sys.argv[3]) if len(sys.argv) > 3 else 2_000_000
    from cli_scale_check import make_genome, write_fasta, write_sam
    from find_circ2_amd import sq_table
    from find_circ2_amd.ingest import sam_to_bam
    d = "/tmp/fc2_abcli"
    os.makedirs(d, exist_ok=True)
    fa, sam, bam = os.path.join(d, "genome.fa"), os.path.join(d, "reads.sam"), os.path.join(d, "reads.bam")
    rng = np.random.default_rng(2024)
    names, sizes = sq_table(os.path.join(ROOT, "tests", "golden", "test_norm.sam"))
    seqs = make_genome(fa, names, sizes, rng)
    write_sam(sam, seqs, reads, rng)
    write_fasta(fa, seqs)
    del seqs
    sam_to_bam(sam, bam)
    ref = None
    for r in range(rounds + 1):                  # round 0 builds the .byo_index (not reported)
        for v in name.split("+") + ["cur"]:
            for form in ("bam_stdin", "sam_path"):
                env = dict(os.environ)
                env.pop("FC2_LIB_VARIANT", None)
                if v.startswith("env:"):
                    for kv in v[4:].split(","):
                        k, _, val = kv.partition("=")
                        env[k] = val
                elif v != "cur":
                    env["FC2_LIB_VARIANT"] = v
                out = os.path.join(d, "out_%s_%s" % (re.sub(r"[^A-Za-z0-9_]", "_", v), form))
                cmd = [sys.executable, "-m", "find_circ2_amd.cli", "-G", fa, "-o", out, "-q"]
                err = None
                if os.environ.get("AB_TIMING") == "1":
                    env["FC2_CALLER_TIMING"] = "1"
                    td = os.path.join(ROOT, "gpurun_out", "abcli_timing")
                    os.makedirs(td, exist_ok=True)
                    err = open(os.path.join(td, "%s_%s_%d.txt" % (re.sub(r"[^A-Za-z0-9_]", "_", v), form, r)), "w")
                from bench import _wait_blocking        # (one blocking waitpid: no 50-ms polling in the wall)
                t0 = time.time()
                if form == "bam_stdin":
                    feeder = subprocess.Popen(["cat", bam], stdout=subprocess.PIPE)
                    rc = _wait_blocking(subprocess.Popen(cmd, env=env, cwd=ROOT, stdin=feeder.stdout, stderr=err), 600)
                    wall = time.time() - t0
                    feeder.stdout.close()
                    feeder.wait()
                else:
                    rc = _wait_blocking(subprocess.Popen(cmd + [sam], env=env, cwd=ROOT, stderr=err), 600)
                    wall = time.time() - t0
                if rc != 0:
                    raise SystemExit("cli exit status %d (%s %s)" % (rc, v, form))
                if err is not None:
                    err.close()
                log = open(os.path.join(out, "run.log")).read()
                rate = float(re.search(r"overall ([0-9.]+)k reads/second", log).group(1)) * 1e3
                st = re.search(r"read loop stages: (.*)", log).group(1)
                o = outputs(out)
                if ref is None:
                    ref = o
                same = o == ref
                if r:
                    print(json.dumps({"variant": v, "form": form, "round": r, "reads_per_s": rate,
                                      "process_wall_s": round(wall, 2), "stages": st, "outputs_identical": same}),
                          flush=True)
                if not same:
                    raise SystemExit("outputs differ: %s %s" % (v, form))


if __name__ == "__main__":
    main()
