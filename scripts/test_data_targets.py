#!/usr/bin/env python
"""BASELINE configs[0]: the reference's own regression targets (test_data/Makefile) on the data at hand.

    python scripts/test_data_targets.py unit_test    [--gpu] [--out DIR]
    python scripts/test_data_targets.py cdr1as_test  [--gpu] [--out DIR]
    python scripts/test_data_targets.py rerun_test   [--gpu] [--out DIR]

No aligner is in the image, so the reads are "aligned" by tests/bwa_emul.py (exact-match segments in
bwa-mem's output shape: primary + supplementary records, clips, AS tags) and piped into the CLI on
stdin, as the Makefile pipes `bwa mem` into find_circ.py.  Without --gpu the breakpoint search is the
CPU oracle (the target is plumbing, as configs[0] says); with --gpu it is the shipped HIP scan.

* unit_test   (test_data/Makefile:10-19): test_reads.fa against test_ref.fa -> test_out/; prints the
  line counts of circ/lin_splice_sites.bed as the target does, and checks the truth encoded in the read
  names (--test: find_circ.py:1148-1273) -- every LIN_OK / CIRC_OK, nothing missed or spurious.
* cdr1as_test (test_data/Makefile:6-8): cdr1as_reads.fa against CDR1as_locus.fa, then cmp_bed against
  cdr1as_reference.bed (cmp_bed.py semantics: identical (chrom, start, end, strand) sets).
* rerun_test  (the procedure of test_data/Makefile:72-81, hek_test2, on data that exists here: the
  HEK293 blobs and hg19 are missing, .MISSING_LARGE_BLOBS): run 1 on a simulated read set over both
  golden genomes, then the reads run 1 wrote to spliced_reads.fastq.gz are aligned again and run
  through the CLI a second time; cmp_bed of the two circ_splice_sites.bed files must be identical.
Exit status 0 when the target's check holds.
"""
import argparse
import gzip
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TESTS = os.path.join(ROOT, "tests")
GOLDEN = os.path.join(TESTS, "golden")
for p in (ROOT, TESTS):
    if p not in sys.path:
        sys.path.insert(0, p)

from bwa_emul import read_fasta  # noqa: E402
from samgen import sam_text  # noqa: E402


def fasta_reads(path):
    names = [l[1:].strip() for l in open(path) if l.startswith(">")]
    seqs = read_fasta(path)
    return [(n.split()[0] if " " not in n else n, seqs[n.split()[0]]) for n in names]


def run_cli(genome_fa, reads, out, gpu, extra=()):
    """`aligner | find_circ -G genome -o out`: the emulated alignments on a stdin pipe."""
    sam = sam_text(read_fasta(genome_fa), reads).encode()
    cmd = [sys.executable, "-m", "find_circ2_amd.cli"] if gpu else [sys.executable,
                                                                        os.path.join(TESTS, "cli_oracle_main.py")]
    env = dict(os.environ, PYTHONPATH=os.pathsep.join([ROOT, TESTS]))
    r = subprocess.run(cmd + ["-G", genome_fa, "-o", out] + list(extra), input=sam, cwd=ROOT, env=env,
                       stdout=subprocess.PIPE, stderr=subprocess.PIPE, timeout=600)
    if r.returncode != 0:
        sys.stderr.write(r.stderr.decode()[-3000:])
        raise SystemExit("find_circ2_amd.cli failed (exit %d)" % r.returncode)
    return r.stdout.decode()


def wc_l(path):
    return sum(1 for _ in open(path))


def unit_test(out, gpu):
    o = os.path.join(out, "test_out")
    run_cli(os.path.join(GOLDEN, "test_ref.fa"), fasta_reads(os.path.join(GOLDEN, "test_reads.fa")), o, gpu,
            ["-n", "test", "--test"])
    for f in ("circ_splice_sites.bed", "lin_splice_sites.bed"):
        print("%8d %s" % (wc_l(os.path.join(o, f)), os.path.join(o, f)))
    rows = [l.rstrip("\n").split("\t") for l in open(os.path.join(o, "test_results.tsv")) if not l.startswith("#")]
    verdicts = [v for r in rows for v in r[1:] if v.isupper() and "_" in v]
    bad = [v for v in verdicts if v.startswith(("MISSED", "SPURIOUS"))]
    ok = [v for v in verdicts if v.endswith("_OK")]
    print("test_results.tsv: %d reads, %d *_OK, %d missed/spurious" % (len(rows), len(ok), len(bad)))
    return 0 if ok and not bad else 1


def cdr1as_test(out, gpu):
    from find_circ2_amd import cmp_bed
    o = os.path.join(out, "cdr1as_test_out")
    run_cli(os.path.join(GOLDEN, "CDR1as_locus.fa"), fasta_reads(os.path.join(GOLDEN, "cdr1as_reads.fa")), o, gpu,
            ["-n", "test"])
    print("\n>>> comparing to known CDR1as result.\n")
    same = cmp_bed.compare(os.path.join(GOLDEN, "cdr1as_reference.bed"), os.path.join(o, "circ_splice_sites.bed"))
    return 0 if same else 1


def simulated_reads(genome_fa, n, seed):
    from synth_small import load_genome, make_spans
    g = load_genome(genome_fa)
    spans = make_spans(g, n, seed=seed, L=(60, 150), p_readN=0.0, p_lower=0.0, p_clip=0.0, mut=0.0)
    return [("sim%05d" % i, s.read_part.decode().upper()) for i, s in enumerate(spans)]


def rerun_test(out, gpu):
    from find_circ2_amd import cmp_bed
    status = 0
    for fa_name, n, seed in (("CDR1as_locus.fa", 1500, 815), ("test_ref.fa", 1500, 110112)):
        fa = os.path.join(GOLDEN, fa_name)
        o1, o2 = os.path.join(out, fa_name + ".run1"), os.path.join(out, fa_name + ".run2")
        run_cli(fa, simulated_reads(fa, n, seed), o1, gpu, ["-n", "rerun"])
        with gzip.open(os.path.join(o1, "spliced_reads.fastq.gz"), "rt") as fh:
            lines = fh.read().splitlines()
        seen, again = set(), []
        for k in range(0, len(lines), 4):
            name, seq = lines[k][1:].split()[0], lines[k + 1]
            if name not in seen:                   # the reads file holds a mate once per junction set
                seen.add(name)
                again.append((name, seq))
        run_cli(fa, again, o2, gpu, ["-n", "rerun"])
        print("\n>>> %s: %d spliced reads of run 1 re-aligned and run again\n" % (fa_name, len(again)))
        if not cmp_bed.compare(os.path.join(o1, "circ_splice_sites.bed"), os.path.join(o2, "circ_splice_sites.bed")):
            status = 1
        if wc_l(os.path.join(o1, "circ_splice_sites.bed")) < 10:
            print("too few junctions in run 1 to mean anything", file=sys.stderr)
            status = 1
    return status


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("target", choices=["unit_test", "cdr1as_test", "rerun_test"])
    ap.add_argument("--gpu", action="store_true", help="the shipped HIP scan instead of the CPU oracle")
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "test_data_targets"))
    a = ap.parse_args()
    os.makedirs(a.out, exist_ok=True)
    sys.exit({"unit_test": unit_test, "cdr1as_test": cdr1as_test, "rerun_test": rerun_test}[a.target](a.out, a.gpu))


if __name__ == "__main__":
    main()
