"""Native ingest (include/fc2_ingest.h) == the Python reader + grouping, file for file.

The CLI is run twice on the same input -- ``--python-ingest`` (samio +
caller.group_alignments, the line-by-line restatement of find_circ.py:1450-1527)
and the default native ingest -- with the CPU oracle evaluator; every output
file and every N[...] counter in run.log must agree.  Inputs: the golden read
sets, and a larger synthetic single-end SAM/BAM mixing unspliced, linear and
backspliced reads, unmapped records, secondary hits and paired mates.
"""
import os
import re

import numpy as np
import pytest

from conftest import GOLDEN
from find_circ2_amd import cli
from oracle_engine import oracle_evaluator_factory
from samgen import sam_to_bam
from test_cli import _reads, run_cli

FILES = ("circ_splice_sites.bed", "lin_splice_sites.bed", "multi_events.tsv", "test_results.tsv")


def counters(out):
    c = {}
    for l in open(os.path.join(out, "run.log")):
        m = re.search(r"\tfind_circ\t(\w+)=([0-9.]+)$", l.rstrip("\n"))
        if m:
            c[m.group(1)] = float(m.group(2))
    return c


def same(o1, o2):
    for f in FILES:
        p1, p2 = os.path.join(o1, f), os.path.join(o2, f)
        assert os.path.exists(p1) == os.path.exists(p2), f
        if os.path.exists(p1):
            assert open(p1).read() == open(p2).read(), f
    import gzip
    with gzip.open(os.path.join(o1, "spliced_reads.fastq.gz"), "rt") as a, \
            gzip.open(os.path.join(o2, "spliced_reads.fastq.gz"), "rt") as b:
        assert a.read() == b.read()
    assert counters(o1) == counters(o2)


@pytest.mark.parametrize("fa,rf", [("test_ref.fa", "test_reads.fa"), ("CDR1as_locus.fa", "cdr1as_reads.fa")])
@pytest.mark.parametrize("bam", [False, True])
def test_native_equals_python_ingest_golden(tmp_path, fa, rf, bam):
    fa = os.path.join(GOLDEN, fa)
    rd = _reads(os.path.join(GOLDEN, rf))
    _, o1 = run_cli(tmp_path, fa, rd, extra=["--test", "--python-ingest"], bam=bam, tag="py")
    _, o2 = run_cli(tmp_path, fa, rd, extra=["--test"], bam=bam, tag="native")
    same(o1, o2)


def _mixed_sam(path, n, seed):
    """Synthetic bwa-mem-like SAM: single and paired reads, unmapped, secondary, spliced."""
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(__file__)), "scripts"))
    from cli_throughput import write_genome
    rng = np.random.default_rng(seed)
    fa = path + ".fa"
    seqs = write_genome(fa, 3, 60_000, rng)
    names = list(seqs)
    lines = ["@HD\tVN:1.5"] + ["@SQ\tSN:%s\tLN:%d" % (c, len(seqs[c])) for c in names]
    L = 100
    q = "I" * L
    for i in range(n):
        c = names[int(rng.integers(3))]
        g = seqs[c]
        kind = rng.random()
        paired = rng.random() < 0.3
        mates = [0x41, 0x81] if paired else [0]
        for mf in mates:
            qn = "q%d" % i
            if kind < 0.05 and mf != 0x81:
                lines.append("%s\t%d\t*\t0\t0\t*\t*\t0\t0\t%s\t%s" % (qn, 4 | mf, "A" * L, q))
                continue
            if kind < 0.5:
                p = int(rng.integers(0, len(g) - L))
                lines.append("%s\t%d\t%s\t%d\t60\t%dM\t*\t0\t0\t%s\t%s\tAS:i:%d\tXS:i:%d" %
                             (qn, mf | (16 if rng.random() < 0.3 else 0), c, p + 1, L, g[p:p + L], q, L,
                              int(rng.integers(0, L))))
                if rng.random() < 0.1:   # a secondary hit (SEQ '*') on another chromosome
                    lines.append("%s\t%d\t%s\t%d\t0\t%dM\t*\t0\t0\t*\t*\tAS:i:%d" %
                                 (qn, mf | 256, names[(names.index(c) + 1) % 3], 100, L, L - 5))
                continue
            kA = int(rng.integers(10, L - 10))
            kB = L - kA
            span = int(rng.integers(150, 3000))
            bs = kind < 0.75
            if bs:
                end = int(rng.integers(span + kA, len(g) - 10))
                st = end - span
                read = g[end - kA:end] + g[st:st + kB]
                a_pos, b_pos = end - kA, st
            else:
                d = int(rng.integers(kA, len(g) - span - kB - 10))
                read = g[d - kA:d] + g[d + span:d + span + kB]
                a_pos, b_pos = d - kA, d + span
            xs = int(rng.integers(0, 12))
            fl = mf | (16 if rng.random() < 0.2 else 0)
            lines.append("%s\t%d\t%s\t%d\t60\t%dM%dS\t*\t0\t0\t%s\t%s\tAS:i:%d\tXS:i:%d" %
                         (qn, fl, c, a_pos + 1, kA, kB, read, q, kA, xs))
            lines.append("%s\t%d\t%s\t%d\t60\t%dH%dM\t*\t0\t0\t%s\t*\tAS:i:%d" %
                         (qn, fl | 2048, c, b_pos + 1, kA, kB, read[kA:], kB))
    open(path, "w").write("\n".join(lines) + "\n")
    return fa


@pytest.mark.parametrize("extra", [[], ["--no-linear"], ["--noop"], ["--chunk-size", "7", "--all-hits"]])
def test_native_equals_python_ingest_mixed(tmp_path, extra):
    sam = str(tmp_path / "mixed.sam")
    fa = _mixed_sam(sam, 1500, seed=815)
    bam = str(tmp_path / "mixed.bam")
    sam_to_bam(open(sam).read(), bam)
    outs = []
    for tag, inp, ing in (("py", sam, ["--python-ingest"]), ("nat", sam, []), ("natbam", bam, [])):
        out = str(tmp_path / tag)
        rc = cli.main(["-G", fa, "-o", out, "-n", "mix", "-q"] + extra + ing + [inp],
                      evaluator_factory=oracle_evaluator_factory)
        assert rc == 0
        outs.append(out)
    same(outs[0], outs[1])
    same(outs[0], outs[2])
    if not extra:
        c = counters(outs[0])
        # random junctions rarely sit on GT/AG: most evaluated spans end in *_no_bp
        assert c["circ_spliced"] + c["circ_no_bp"] > 300 and c["lin_spliced"] + c["lin_no_bp"] > 200
        assert c["circ_spliced"] > 5 and c["unmapped_reads"] > 10


def test_single_record_input_fails_like_reference(tmp_path):
    fa = os.path.join(GOLDEN, "test_ref.fa")
    sam = tmp_path / "one.sam"
    sam.write_text("@SQ\tSN:testbed_plus\tLN:720\nr\t0\ttestbed_plus\t10\t60\t20M\t*\t0\t0\t%s\t*\tAS:i:20\n"
                   % ("A" * 20))
    for ing in ([], ["--python-ingest"]):
        rc = cli.main(["-G", fa, "-o", str(tmp_path / ("o%d" % len(ing))), "-q"] + ing + [str(sam)],
                      evaluator_factory=oracle_evaluator_factory)
        assert rc == 1       # UnboundLocalError at find_circ.py:1486 -> exit 1
