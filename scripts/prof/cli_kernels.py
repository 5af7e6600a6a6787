"""The CLI's GPU work under rocprofv3 (`rocprofv3 --kernel-trace --stats -- python3 scripts/prof/cli_kernels.py
[reads] [sites]`): scripts/cli_steady.py's input (scripts/gen_reads: hg19-shaped genome, bwa-mem-shaped
BAM), the CLI run in this process (cli.main, the default native loop and its ctxpipe search) so the
process ends normally and the profiler writes its files -- `python -m` ends with os._exit, which
leaves no profile.  Prints the run.log phases as JSON."""
import json
import os
import re
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "scripts")]


def main():
    from cli_steady import prepare
    from find_circ2_amd import cli
    reads = int(sys.argv[1]) if len(sys.argv) > 1 else 2_000_000
    sites = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    import shutil
    d = tempfile.mkdtemp(prefix="fc2_cli_kernels_", dir="/tmp")
    try:
        fa, bams, _, _ = prepare(d, [reads], sites=sites)
        out = os.path.join(d, "out")
        t0 = time.time()
        rc = cli.main(["-G", fa, "-o", out, "-q", bams[reads]])
        wall = time.time() - t0
        log = open(os.path.join(out, "run.log")).read()
    finally:
        shutil.rmtree(d, ignore_errors=True)
    ph = re.search(r"process phases: (.*)", log)
    print(json.dumps({"rc": rc, "main_s": round(wall, 3), "reads": reads, "sites": sites,
                      "phases": dict(re.findall(r"(\w+)=([0-9.naN]+)", ph.group(1))) if ph else None,
                      "search": [l.split("\t")[-1] for l in log.splitlines() if "breakpoint search" in l]}))


if __name__ == "__main__":
    main()
