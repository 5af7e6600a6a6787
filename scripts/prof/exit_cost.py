"""Where the CLI's process wall goes after main() returns (DESIGN.md §5 start-up): the CLI as its own
process on bench.cli_end_to_end's 2M-read input, main() run as `python -m` does (memory left
to the exit), then optionally the FASTA mapping dropped and the freed heap trimmed, each timed; each child writes its clock
and /proc/self/status memory lines just before os._exit, the parent notes when wait() returns.
One JSON line per run on stdout."""
import json
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "scripts"))

CHILD = r"""
import ctypes, os, sys, time
sys.argv = ["find_circ2_amd.cli"] + %r
import find_circ2_amd.cli as c
c.EXIT_AFTER_MAIN = True
rc = c.main()
variant = %r
libc = ctypes.CDLL("libc.so.6", use_errno=True)
t0 = time.time()
if "fasta" in variant:             # drop the FASTA mapping's page-table entries (the pages stay cached)
    libc.munmap.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    for l in open("/proc/self/maps"):
        if l.rstrip().endswith("genome.fa"):
            a, b = (int(x, 16) for x in l.split()[0].split("-"))
            libc.munmap(a, b - a)
t1 = time.time()
if "trim" in variant:              # hand freed heap back to the kernel
    libc.malloc_trim(0)
t2 = time.time()
mem = {l.split(":")[0]: l.split(":")[1].strip() for l in open("/proc/self/status") if l.startswith(("VmRSS", "RssAnon", "RssFile"))}
class MI(ctypes.Structure):
    _fields_ = [(k, ctypes.c_size_t) for k in ("arena", "ordblks", "smblks", "hblks", "hblkhd", "usmblks", "fsmblks",
                                                "uordblks", "fordblks", "keepcost")]
libc.mallinfo2.restype = MI
mi = libc.mallinfo2()
mem.update(malloc_heap_mb=mi.arena >> 20, malloc_inuse_mb=mi.uordblks >> 20, malloc_free_mb=mi.fordblks >> 20,
           malloc_mmapped_mb=mi.hblkhd >> 20, malloc_mmapped_n=mi.hblks)
open(%r, "w").write(repr((time.time(), c.process_age(), mem, t1 - t0, t2 - t1)))
sys.stdout.flush(); sys.stderr.flush()
os._exit(rc)
"""


def main():
    import numpy as np
    from cli_scale_check import make_genome, write_fasta, write_sam
    from find_circ2_amd import sq_table
    from find_circ2_amd.ingest import sam_to_bam
    reads = int(sys.argv[1]) if len(sys.argv) > 1 else 2_000_000
    d = tempfile.mkdtemp(prefix="fc2_exit_", dir="/tmp")
    fa, sam, bam = (os.path.join(d, x) for x in ("genome.fa", "reads.sam", "reads.bam"))
    rng = np.random.default_rng(2024)
    names, sizes = sq_table(os.path.join(ROOT, "tests", "golden", "test_norm.sam"))
    seqs = make_genome(fa, names, sizes, rng)
    write_sam(sam, seqs, reads, rng)
    write_fasta(fa, seqs)
    del seqs
    sam_to_bam(sam, bam)
    print(json.dumps({"prepared": d}), flush=True)
    for rep in range(2):
        for variant in ("none", "fasta", "fasta+trim"):
            out = os.path.join(d, "o%d%s" % (rep, variant))
            marker = os.path.join(d, "m")
            args = ["-G", fa, "-o", out, "-q", sam]
            t0 = time.time()
            env = dict(os.environ, FC2_CALLER_TIMING="1")
            pr = subprocess.run([sys.executable, "-c", CHILD % (args, variant, marker)], cwd=ROOT, env=env,
                                timeout=600, stderr=subprocess.PIPE, text=True)
            t1 = time.time()
            t_mark, age, mem, t_fasta, t_trim = eval(open(marker).read())
            print(json.dumps({"rep": rep, "variant": variant, "rc": pr.returncode, "wall_s": round(t1 - t0, 3),
                              "age_at_exit_s": round(age, 3), "exit_gap_s": round(t1 - t_mark, 3),
                              "unmap_fasta_s": round(t_fasta, 3), "malloc_trim_s": round(t_trim, 3),
                              "mem": mem}), flush=True)
    # bare processes: the interpreter alone, HIP initialised, one context with the genome resident
    for what, code in (("bare", "pass"),
                       ("hip_ctx", "from find_circ2_amd import ctxpipe as C, _native as N\n"
                                   "import ctypes\nh = ctypes.c_void_p()\nN.check(N.lib().fc2_ctx_create(0, ctypes.byref(h)))"),
                       ("hip_ctx_genome", "from find_circ2_amd import ctxpipe as C, _native as N\n"
                                          "import ctypes\nh = ctypes.c_void_p()\nN.check(N.lib().fc2_ctx_create(0, ctypes.byref(h)))\n"
                                          "g = C.FastaGenome(%r)\nN.check(N.lib().fc2_ctx_genome_load(h, g.fasta, 0))" % fa),
                       ("hip_ctx_genome_released", "from find_circ2_amd import ctxpipe as C, _native as N\n"
                                          "import ctypes\nh = ctypes.c_void_p()\nN.check(N.lib().fc2_ctx_create(0, ctypes.byref(h)))\n"
                                          "g = C.FastaGenome(%r)\nN.check(N.lib().fc2_ctx_genome_load(h, g.fasta, 0))\n"
                                          "N.lib().fc2_ctx_destroy(h)\ng.close()" % fa)):
        for rep in range(2):
            marker = os.path.join(d, "m")
            src = ("import os, sys, time\nsys.path.insert(0, %r)\n" % ROOT + code +
                   "\nopen(%r, 'w').write(repr(time.time()))\nos._exit(0)\n" % marker)
            t0 = time.time()
            rc = subprocess.run([sys.executable, "-c", src], cwd=ROOT, timeout=300).returncode
            t1 = time.time()
            t_mark = eval(open(marker).read())
            print(json.dumps({"what": what, "rep": rep, "rc": rc, "wall_s": round(t1 - t0, 3),
                              "exit_gap_s": round(t1 - t_mark, 3)}), flush=True)


if __name__ == "__main__":
    main()
