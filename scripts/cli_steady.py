#!/usr/bin/env python
"""The CLI at steady state, in the metric's unit (anchor pairs / s), with a host-thread curve.

VERDICT r05 "Next round" #2.  scripts/gen_reads (C; the model of scripts/cli_scale_check.py, see its
header) writes an hg19-shaped genome FASTA and a bwa-mem-shaped SAM of the largest size asked for;
the smaller sizes are its first reads.  fc2_sam_to_bam turns each into a BGZF BAM, and the shipped
CLI (``python -m find_circ2_amd.cli -G genome.fa -o out``, C++ read loop + HIP search) reads it from
a stdin pipe, as from samtools / an aligner.  Per (size, threads):

* the child process is pinned to `threads` CPUs (sched_setaffinity before exec) and its native pools
  are sized to them (FC2_PARSE_THREADS, FC2_INGEST_THREADS, FC2_NEXT_THREADS, FC2_CALLER_THREADS,
  OMP_NUM_THREADS);
* reported: reads/s and anchor pairs/s ("breakpoint search: N spans", i.e. JunctionSpans evaluated
  by find_breakpoints) of the read loop (run.log) and of the process wall, the loop's stage times
  and FC2_CALLER_TIMING's CPU seconds per stage (inflate, split, parse+group, consumer, next pool,
  submit pool, submit serial, gzip).

With --check the largest size also runs through the Python read loop (--python-caller, same HIP
search) and every output file must be byte-identical.  One JSON line on stdout; progress on stderr.

usage: python scripts/cli_steady.py [--sizes 2000000,20000000] [--threads 4,8,16,32] [--reps 1]
                                    [--check] [--out DIR] [--keep] [--sites K] [--variants K=V,...]
--sites K: the spliced reads cross K planted junctions (many reads per junction, as in a real
library) instead of one junction each (the junction tables then stay small).
Each run's record is printed as its own JSON line as soon as it is done; the summary comes last.
"""
import argparse
import gzip
import json
import os
import re
import shutil
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def cut_sam(src, dst, n_reads):
    """The first n_reads reads of src (records are 'u<i>' / 's<i>' in read order)."""
    import mmap
    with open(src, "rb") as f, mmap.mmap(f.fileno(), 0, access=mmap.ACCESS_READ) as m:
        end = len(m)
        for tag in (b"\nu%d\t" % n_reads, b"\ns%d\t" % n_reads):
            k = m.find(tag)
            if k >= 0:
                end = min(end, k + 1)
        with open(dst, "wb") as o:
            for p in range(0, end, 1 << 28):
                o.write(m[p:min(end, p + (1 << 28))])


def cpu_set(n):
    cpus = sorted(os.sched_getaffinity(0))
    return cpus[:n]


def quota():
    """The cgroup CPU quota (cpu.max) in CPUs, if one is set."""
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()
        return None if q == "max" else round(int(q) / int(p), 2)
    except (OSError, ValueError):
        return None


def run_cli(fa, bam, out, threads, extra=(), timeout=900, timing=False, by_path=False, env_extra=None):
    """One CLI process on `bam` (piped on stdin; by_path: given as the input path) -> its record."""
    env = dict(os.environ)
    env.update(env_extra or {})
    if timing:
        env["FC2_CALLER_TIMING"] = "1"
    if threads:
        for k in ("FC2_PARSE_THREADS", "FC2_INGEST_THREADS", "FC2_NEXT_THREADS", "FC2_CALLER_THREADS",
                  "OMP_NUM_THREADS"):
            env[k] = str(threads)
    cpus = cpu_set(threads) if threads else None
    cmd = [sys.executable, "-m", "find_circ2_amd.cli", "-G", fa, "-o", out, "-q"] + list(extra)
    err = open(out + ".stderr", "wb")
    t0 = time.time()
    feeder = None if by_path else subprocess.Popen(["cat", bam], stdout=subprocess.PIPE)
    p = subprocess.Popen(cmd + ([bam] if by_path else []), cwd=ROOT, stdin=feeder.stdout if feeder else None,
                         stderr=err, env=env, preexec_fn=(lambda: os.sched_setaffinity(0, cpus)) if cpus else None)
    if feeder:
        feeder.stdout.close()
    while True:                             # a heartbeat on stderr (a long run is not a hung one)
        try:
            rc = p.wait(timeout=30)
            break
        except subprocess.TimeoutExpired:
            if time.time() - t0 > timeout:
                p.kill()
                raise
            log("  ... %s running %.0f s" % (os.path.basename(out), time.time() - t0))
    wall = time.time() - t0
    if feeder:
        feeder.wait()
    err.close()
    if rc != 0:
        raise RuntimeError("cli exit status %d: %s" % (rc, open(out + ".stderr").read()[-2000:]))
    text = open(os.path.join(out, "run.log")).read()
    errt = open(out + ".stderr").read()
    m = re.search(r"processed ([0-9.]+)M .* reads in ([0-9.]+) minutes \(overall ([0-9.]+)k", text)
    sp = re.search(r"breakpoint search: (\d+) spans", text)
    st = re.search(r"read loop stages: (.*)", text)
    ph = re.search(r"process phases: (.*)", text)
    cpu = re.search(r"cpu s:(.*)", errt)
    phases = {k: float(v) for k, v in re.findall(r"(\w+)=([0-9.naN]+)", ph.group(1))} if ph else {}
    stages = {k: float(v) for k, v in re.findall(r"(\w+)=([0-9.]+)", st.group(1))} if st else {}
    cpu_s = {}
    if cpu:
        for name, v in re.findall(r"([a-z+ ]+?) ([0-9.]+)", cpu.group(1)):
            cpu_s[name.strip()] = float(v)
    reads = int(round(float(m.group(1)) * 1e6)) if m else None
    spans = int(sp.group(1)) if sp else None
    loop_s = phases.get("read_loop_s")
    net = loop_s - phases.get("genome_wait_s", 0.0) if loop_s else None
    subs = [l for l in errt.splitlines() if l.startswith("submit nf=")]
    sub_ms = {}
    for l in subs:
        for k, v in re.findall(r" ([A-D])=([0-9.]+)", l):
            sub_ms[k] = sub_ms.get(k, 0.0) + float(v)
    nxt = {}
    for l in errt.splitlines():
        if l.startswith("next nf="):
            for k, v in re.findall(r"(read|process|pairs)=([0-9.]+)", l):
                nxt[k] = nxt.get(k, 0.0) + float(v)
    sd = re.search(r"process shutdown: (.*)", text)
    if sd:
        phases.update({"shutdown_" + k: float(v) for k, v in re.findall(r"(\w+)=([0-9.naN]+)", sd.group(1))})
    return {
        "threads": threads, "cpus": len(cpus) if cpus else None, "process_wall_s": round(wall, 3),
        "reads": reads, "spans": spans,
        "loop_s": loop_s, "genome_wait_s": phases.get("genome_wait_s"),
        "loop_reads_per_s": round(reads / loop_s, 1) if loop_s else None,
        "loop_spans_per_s": round(spans / loop_s, 1) if loop_s else None,
        "loop_spans_per_s_after_genome": round(spans / net, 1) if net and net > 0 else None,
        "wall_reads_per_s": round(reads / wall, 1), "wall_spans_per_s": round(spans / wall, 1) if spans else None,
        "stages_s": stages, "cpu_s_per_stage": cpu_s, "phases_s": phases, "n_chunks": len(subs) or None,
        "gpu_inflate": (re.search(r"gpu inflate: (.*)", errt) or [None, None])[1],
        "upstream_ms": [round(sum(float(m[k]) for m in re.findall(
            r"upstream: inflate wait ([0-9.]+), splitter blocked ([0-9.]+), parsers idle ([0-9.]+)", errt)), 1)
            for k in range(3)],                 # inflate wait, splitter blocked, parsers idle (summed)
        "submit_phase_ms": {k: round(v, 1) for k, v in sub_ms.items()} or None,
        "next_phase_ms": {k: round(v, 1) for k, v in nxt.items()} or None,
    }


def prepare(d, sizes, keep_sam=False, keep_sam_sizes=(), sites=0):
    """genome.fa + reads_<n>.bam for every size in d (scripts/gen_reads for the largest, the smaller
    ones its first reads); returns (fasta, {n: bam}, {n: sam kept}, timings).  SAM files are deleted
    after conversion unless keep_sam (the largest) or n in keep_sam_sizes."""
    from find_circ2_amd import sq_table
    from find_circ2_amd.ingest import sam_to_bam
    gen = os.path.join(ROOT, "scripts", "gen_reads")
    if not os.path.exists(gen):
        subprocess.check_call(["gcc", "-O2", "-o", gen, gen + ".c"])
    info = {}
    names, lens = sq_table(os.path.join(ROOT, "tests", "golden", "test_norm.sam"))
    sq = os.path.join(d, "sq.tsv")
    open(sq, "w").write("".join("%s\t%d\n" % x for x in zip(names, lens)))
    fa, big = os.path.join(d, "genome.fa"), os.path.join(d, "reads_%d.sam" % max(sizes))
    t0 = time.time()
    subprocess.check_call([gen, sq, str(max(sizes)), "2024", fa, big] + ([str(sites)] if sites else []))
    info["gen_s"] = round(time.time() - t0, 1)
    log("generated", max(sizes), "reads in", info["gen_s"], "s")
    bams, sams = {}, {}
    for n in sorted(sizes):
        sam = big if n == max(sizes) else os.path.join(d, "reads_%d.sam" % n)
        if sam != big:
            cut_sam(big, sam, n)
        bam = os.path.join(d, "reads_%d.bam" % n)
        t0 = time.time()
        sam_to_bam(sam, bam)
        info["bam_%d" % n] = {"bytes": os.path.getsize(bam), "convert_s": round(time.time() - t0, 1)}
        if (sam == big and keep_sam) or n in keep_sam_sizes:
            sams[n] = sam
        elif sam != big:
            os.remove(sam)
        bams[n] = bam
        log("bam", n, info["bam_%d" % n])
    if max(sizes) not in sams:
        os.remove(big)
    return fa, bams, sams, info


def outputs(out):
    files = {}
    for f in ("circ_splice_sites.bed", "lin_splice_sites.bed", "multi_events.tsv"):
        files[f] = open(os.path.join(out, f), "rb").read()
    with gzip.open(os.path.join(out, "spliced_reads.fastq.gz")) as fh:
        files["spliced_reads.fastq"] = fh.read()
    return files


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="2000000,20000000")
    ap.add_argument("--threads", default="4,8,16,32")
    ap.add_argument("--reps", type=int, default=1)
    ap.add_argument("--check", action="store_true")
    ap.add_argument("--out", default="")
    ap.add_argument("--keep", action="store_true")
    ap.add_argument("--variants", default="",
                    help="comma-separated K=V environment settings, each run as well as the default "
                         "(e.g. FC2_GPU_INFLATE=0)")
    ap.add_argument("--sites", type=int, default=0,
                    help="junction sites the spliced reads cross (scripts/gen_reads.c); 0: one per read")
    a = ap.parse_args()
    sizes = [int(x) for x in a.sizes.split(",")]
    threads = [int(x) for x in a.threads.split(",") if x.strip() and x != "none"]
    import tempfile
    d = a.out or tempfile.mkdtemp(prefix="fc2_steady_", dir="/tmp")
    os.makedirs(d, exist_ok=True)
    res = {"cpus_visible": len(os.sched_getaffinity(0)), "cgroup_cpu_quota": quota(), "sizes": sizes,
           "cpu_model": next((l.split(":", 1)[1].strip() for l in open("/proc/cpuinfo") if l.startswith("model name")),
                             None)}
    try:
        fa, bams, _, info = prepare(d, sizes, keep_sam=a.check, sites=a.sites)
        res["sites"] = a.sites
        res.update(info)
        run_cli(fa, bams[min(sizes)], os.path.join(d, "warm"), 0)       # builds genome.fa.byo_index
        runs = []
        variants = [""] + [v for v in a.variants.split(",") if v]
        for n in sorted(sizes):
            for t, var in [(t, v) for t in [0] + threads for v in variants]:
                # the clean runs (what a user gets), then one with FC2_CALLER_TIMING's per-stage CPU
                # accounting (it also closes the caller at exit to print the totals)
                for r in list(range(a.reps)) + ["timing"]:
                    out = os.path.join(d, "o_%d_%d_%s%s" % (n, t, r, "_" + var.replace("=", "") if var else ""))
                    x = run_cli(fa, bams[n], out, t, timing=(r == "timing"),
                                env_extra=dict([var.split("=", 1)]) if var else None)
                    x["size"] = n
                    x["rep"] = r
                    x["variant"] = var or "default"
                    runs.append(x)
                    print(json.dumps(x), flush=True)
                    log("size %d threads %s %s rep %s: loop %.3f s, %.3g spans/s loop, %.3g spans/s wall, cpu %s" % (
                        n, t or "default", var, r, x["loop_s"], x["loop_spans_per_s"] or 0, x["wall_spans_per_s"] or 0,
                        x["cpu_s_per_stage"]))
                    if not a.keep and not (a.check and n == max(sizes) and t == 0 and r == 0):
                        shutil.rmtree(out, ignore_errors=True)
        res["runs"] = runs
        if a.check:
            n = max(sizes)
            o_py = os.path.join(d, "python_caller")
            t0 = time.time()
            x = run_cli(fa, bams[n], o_py, 0, extra=["--python-caller"], timeout=1500)
            res["python_caller_%d" % n] = {k: x[k] for k in ("process_wall_s", "loop_s", "loop_spans_per_s")}
            same = outputs(os.path.join(d, "o_%d_0_0" % n)) == outputs(o_py)
            res["identical_to_python_loop_at_%d" % n] = same
            log("python loop check:", same, round(time.time() - t0, 1), "s")
    finally:
        if not a.keep:
            shutil.rmtree(d, ignore_errors=True)
    print(json.dumps(res))
    return 0


if __name__ == "__main__":
    sys.exit(main())
