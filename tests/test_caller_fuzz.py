"""Differential fuzzing of the three read loops (native C++, --python-caller, --python-ingest).

The "rich" SAM of test_native_caller.py is mutated record by record: flag bits (strand,
secondary, supplementary, unmapped, mate bits), CIGAR variants (I/D/N/=/X ops, clips moved,
hard for soft), AS/XS changes (XS > AS, XS dropped, AS dropped), SEQ/QUAL '*', lower case,
N and IUPAC bytes in reads, an RNAME that the header lists but the FASTA lacks, POS shifts.
For every seed the three loops must agree on the exit status and, when it is 0, on every
output file and counter; when it is 1, on the exception type the log reports.
"""
import os
import re

import numpy as np
import pytest

from find_circ2_amd import cli
from oracle_engine import oracle_evaluator_factory
from test_ingest import same
from test_native_caller import _rich_sam


def _mutate_cigar(cig, rng):
    ops = re.findall(r"(\d+)([MIDNSHP=X])", cig)
    ops = [[int(n), o] for n, o in ops]
    r = rng.random()
    ms = [k for k, (n, o) in enumerate(ops) if o == "M" and n > 8]
    if r < 0.3 and ms:                          # split an M by an I / D / N / =X
        k = ms[int(rng.integers(len(ms)))]
        n = ops[k][0]
        a = int(rng.integers(2, n - 2))
        mid = ["I", "D", "N", "=", "X"][int(rng.integers(5))]
        ins = [[a, "M"], [int(rng.integers(1, 3)) if mid in "IDN" else 2, mid], [n - a - (2 if mid in "=X" else 0), "M"]]
        if mid == "I":
            ins[2][0] = n - a - ins[1][0]
        ops[k:k + 1] = [x for x in ins if x[0] > 0]
    elif r < 0.45:                              # soft <-> hard clips
        ops = [[n, {"S": "H", "H": "S"}.get(o, o)] for n, o in ops]
    elif r < 0.55 and ms:                       # an M as "="
        ops[ms[0]][1] = "="
    return "".join("%d%s" % (n, o) for n, o in ops)


def _mutate(lines, rng, rate, fatal=True):
    """fatal=False leaves out the mutations on which the reference raises (AS dropped,
    SEQ '*', an RNAME outside the FASTA)."""
    out = []
    for l in lines:
        if l.startswith("@"):
            out.append(l)
            continue
        f = l.split("\t")
        flag = int(f[1])
        if rng.random() < rate:
            flag ^= [0x10, 0x100, 0x800, 0x4, 0x40, 0x80, 0x2][int(rng.integers(7))]
        if rng.random() < rate:
            f[5] = _mutate_cigar(f[5], rng) if f[5] != "*" else f[5]
        if rng.random() < rate:
            f[3] = str(max(0, int(f[3]) + int(rng.integers(-3, 4))))
        tags = f[11:]
        if rng.random() < rate:
            tags = [t for t in tags if not t.startswith("XS:")]
        if rng.random() < rate:
            as_ = [int(t[5:]) for t in tags if t.startswith("AS:i:")]
            if as_:
                tags = [t for t in tags if not t.startswith("XS:")] + ["XS:i:%d" % (as_[0] + int(rng.integers(-2, 5)))]
        if fatal and rng.random() < rate * 0.1:
            tags = [t for t in tags if not t.startswith("AS:")]          # fatal when the segment is used
        if f[9] != "*" and rng.random() < rate:
            s = list(f[9])
            k = int(rng.integers(len(s)))
            s[k] = "NRYacgtn"[int(rng.integers(8))]
            f[9] = "".join(s)
        if f[9] != "*" and rng.random() < rate * 0.5:
            f[9] = f[9].lower()
        if fatal and rng.random() < rate * 0.05:
            f[9] = "*"
        if rng.random() < rate * 0.1 or f[9] == "*":
            f[10] = "*"                                                   # SEQ '*' needs QUAL '*' (SAM spec)
        if fatal and rng.random() < rate * 0.05:
            f[2] = "chrU"                                                 # in the header, not in the FASTA
        f[1] = str(flag)
        out.append("\t".join(f[:11] + tags))
    return out


def _exc_type(out):
    log = open(os.path.join(out, "run.log")).read()
    m = re.findall(r"\n(\w+(?:Error|Exception))\b", log)
    return m[-1] if m else None


@pytest.mark.parametrize("seed", list(range(12)))
@pytest.mark.parametrize("extra", [[], ["--all-hits", "--non-canonical", "--half-unique"], ["--chunk-size", "5"]],
                         ids=["default", "allhits", "chunk5"])
def test_three_loops_agree_on_mutated_input(tmp_path, seed, extra):
    sam0 = str(tmp_path / "base.sam")
    fa = _rich_sam(sam0, 400, seed=1000 + seed)
    lines = open(sam0).read().splitlines()
    hdr = [l for l in lines if l.startswith("@")]
    hdr.append("@SQ\tSN:chrU\tLN:5000")
    rng = np.random.default_rng(seed)
    body = _mutate([l for l in lines if not l.startswith("@")], rng, rate=0.02 if seed % 3 else 0.08)
    sam = str(tmp_path / "mut.sam")
    open(sam, "w").write("\n".join(hdr + body) + "\n")
    rcs, outs = [], []
    for tag, mode in (("py", ["--python-ingest"]), ("pyc", ["--python-caller"]), ("nat", [])):
        out = str(tmp_path / tag)
        rcs.append(cli.main(["-G", fa, "-o", out, "-n", "fz", "-q"] + extra + mode + [sam],
                            evaluator_factory=oracle_evaluator_factory))
        outs.append(out)
    assert rcs[0] == rcs[1] == rcs[2], rcs
    if rcs[0] == 0:
        same(outs[0], outs[1])
        same(outs[0], outs[2])
    else:
        assert _exc_type(outs[0]) == _exc_type(outs[1]) == _exc_type(outs[2])
        # what the reference writes before it fails: every fragment ahead of the failing one
        assert _partial(outs[0]) == _partial(outs[1]) == _partial(outs[2])


def _partial(out):
    import gzip
    with gzip.open(os.path.join(out, "spliced_reads.fastq.gz"), "rt") as f:
        reads = f.read()
    return reads, open(os.path.join(out, "multi_events.tsv")).read()


def _frag_sam(tmp_path, recs):
    fa = os.path.join(os.path.dirname(__file__), "golden", "test_ref.fa")
    sam = str(tmp_path / "r.sam")
    open(sam, "w").write("@SQ\tSN:testbed_plus\tLN:720\n@SQ\tSN:testbed_minus\tLN:720\n" + "\n".join(recs) + "\n")
    return fa, sam


def _agree(tmp_path, fa, sam, extra):
    rcs, outs = [], []
    for tag, mode in (("py", ["--python-ingest"]), ("pyc", ["--python-caller"]), ("nat", [])):
        out = str(tmp_path / tag)
        rcs.append(cli.main(["-G", fa, "-o", out, "-q"] + extra + mode + [sam], evaluator_factory=oracle_evaluator_factory))
        outs.append(out)
    assert rcs[0] == rcs[1] == rcs[2], rcs
    return rcs[0], outs


def test_clips_longer_than_seq_are_an_empty_query(tmp_path):
    """Found by the fuzzer: a supplementary record whose soft clips exceed its SEQ has
    query == '' (Python slice), a too-short segment, not len(None)."""
    seq = "ACGT" * 25
    fa, sam = _frag_sam(tmp_path, [
        "r1\t0\ttestbed_plus\t100\t60\t60M40S\t*\t0\t0\t%s\t*\tAS:i:60" % seq,
        "r1\t2048\ttestbed_plus\t300\t60\t60S40M\t*\t0\t0\t%s\t*\tAS:i:40" % seq[60:],
        "r2\t0\ttestbed_plus\t10\t60\t100M\t*\t0\t0\t%s\t*\tAS:i:100" % seq])
    rc, outs = _agree(tmp_path, fa, sam, [])
    assert rc == 0
    same(outs[0], outs[2])


def test_missing_as_raises_under_no_linear(tmp_path):
    """Found by the fuzzer: JunctionSpan.__init__ computes uniqness for linear spans too, so a
    missing AS raises even with --no-linear (find_circ.py:809-819, 1566-1569)."""
    seq = "ACGT" * 25
    fa, sam = _frag_sam(tmp_path, [
        "r1\t0\ttestbed_plus\t100\t60\t60M40S\t*\t0\t0\t%s\t*\tAS:i:60" % seq,
        "r1\t2048\ttestbed_plus\t300\t60\t60H40M\t*\t0\t0\t%s\t*" % seq[60:],
        "r2\t0\ttestbed_plus\t10\t60\t100M\t*\t0\t0\t%s\t*\tAS:i:100" % seq])
    rc, outs = _agree(tmp_path, fa, sam, ["--no-linear"])
    assert rc == 1 and _exc_type(outs[2]) == "KeyError"


@pytest.mark.parametrize("seed", list(range(6)))
def test_sam_and_bam_inputs_agree_on_mutated_input(tmp_path, seed):
    """The same mutated records as SAM text, as BGZF / plain-gzip BAM (native reader) and as BAM
    through the Python reader (reads upper-cased: BAM stores 4-bit bases)."""
    from samgen import sam_to_bam
    sam0 = str(tmp_path / "base.sam")
    fa = _rich_sam(sam0, 300, seed=9000 + seed)
    lines = open(sam0).read().splitlines()
    hdr = [l for l in lines if l.startswith("@")] + ["@SQ\tSN:chrU\tLN:5000"]
    rng = np.random.default_rng(seed)
    body = _mutate([l for l in lines if not l.startswith("@")], rng, rate=[0.01, 0.05, 0.1][seed % 3])
    body = ["\t".join(f[:9] + [f[9].upper()] + f[10:]) for f in (l.split("\t") for l in body)]
    txt = "\n".join(hdr + body) + "\n"
    sam, bam = str(tmp_path / "m.sam"), str(tmp_path / "m.bam")
    open(sam, "w").write(txt)
    sam_to_bam(txt, bam, bgzf=bool(seed % 2))
    rcs, outs = [], []
    for tag, inp, mode in (("sam", sam, []), ("bam", bam, []), ("pybam", bam, ["--python-ingest"])):
        out = str(tmp_path / tag)
        rcs.append(cli.main(["-G", fa, "-o", out, "-q"] + mode + [inp], evaluator_factory=oracle_evaluator_factory))
        outs.append(out)
    assert rcs[0] == rcs[1] == rcs[2], rcs
    if rcs[0] == 0:
        same(outs[0], outs[1])
        same(outs[0], outs[2])


def test_rev_comp_keyerror_names_first_bad_byte(tmp_path):
    """Hit.add's rev_comp (find_circ.py:54-58, :573/:582) complements the read forward, so a read
    with two bytes outside the table raises KeyError for the first one.  The breakpoint search
    compares bytes (the pair takes the byte path) and still finds the junction, so the failure
    comes from Hit.add, in all three loops."""
    from samgen import sam_text
    from test_cli import _reads
    from find_circ2_amd.caller import rev_comp
    with pytest.raises(KeyError) as e:
        rev_comp("AC=GT.A")
    assert e.value.args[0] == "="
    fa = os.path.join(os.path.dirname(__file__), "golden", "CDR1as_locus.fa")
    reads = _reads(os.path.join(os.path.dirname(__file__), "golden", "cdr1as_reads.fa"))
    from bwa_emul import read_fasta
    lines = sam_text(read_fasta(fa), reads).splitlines()
    out, hit = [], False
    for l in lines:
        f = l.split("\t")
        if not hit and not l.startswith("@") and re.match(r"^\d+M\d+S$", f[5]) and int(f[1]) & 0x900 == 0:
            # the primary of a spliced read: two of its first bases become bytes outside the table
            f[9] = "=" + f[9][1:4] + "." + f[9][5:]
            hit = True
        out.append("\t".join(f))
    assert hit
    sam = str(tmp_path / "junk.sam")
    open(sam, "w").write("\n".join(out) + "\n")
    rc, outs = _agree(tmp_path, fa, sam, [])
    logs = [open(os.path.join(o, "run.log")).read() for o in outs]
    assert rc == 1 and all("KeyError: '='" in l for l in logs), [l[-300:] for l in logs]


@pytest.mark.parametrize("chunk", ["2", "3", "7"])
def test_failure_inside_a_flushed_chunk_records_each_fragment_once(tmp_path, chunk):
    """A fragment whose span raises at record time (its chromosome is in the SAM header but not in
    the FASTA: KeyError at find_circ.py:193) in the middle of a chunk: the fragments before it are
    recorded once, nothing after it, in all three loops (the reference stops there, :1578-1583)."""
    sam0 = str(tmp_path / "base.sam")
    fa = _rich_sam(sam0, 200, seed=77)
    lines = open(sam0).read().splitlines()
    hdr = [l for l in lines if l.startswith("@")] + ["@SQ\tSN:chrU\tLN:500000"]
    body = [l for l in lines if not l.startswith("@")]
    # the 12th read with a supplementary record (a split read) moves to chrU, all its records
    split = []
    for l in body:
        f = l.split("\t")
        if int(f[1]) & 0x800 and f[0] not in split:
            split.append(f[0])
    victim = split[11]
    body = ["\t".join(f[:2] + ["chrU"] + f[3:]) if f[0] == victim else "\t".join(f)
            for f in (l.split("\t") for l in body)]
    sam = str(tmp_path / "u.sam")
    open(sam, "w").write("\n".join(hdr + body) + "\n")
    rc, outs = _agree(tmp_path, fa, sam, ["--chunk-size", chunk])
    assert rc == 1
    assert _exc_type(outs[0]) == _exc_type(outs[1]) == _exc_type(outs[2]) == "KeyError"
    parts = [_partial(o) for o in outs]
    assert parts[0] == parts[1] == parts[2]
    # fragments in input order, each once (a paired fragment writes its two mates)
    from collections import Counter
    ids = [int(l.split()[0][2:]) for l in parts[0][0].splitlines()[::4]]
    assert ids and ids == sorted(ids) and max(Counter(ids).values()) <= 2
