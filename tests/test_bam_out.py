"""-B/--bam: spliced_alignments.bam (find_circ.py:479-483, 1134-1140).

The reference hands pysam every mate's anchor alignments while
adjacent_segment_pairs runs: seg_a of each adjacent pair that passes the
anchor-length filter, then the last pair's seg_b, for every mate with two or
more proper segments (unique or not, with or without a junction, --no-linear
or not; nothing under --noop).  The expected records come from a restatement
of that rule on the Python reader's records (samio + caller.group_alignments);
the written BAM is decoded by the independent reader below.  SAM lines are
encoded the way htslib's sam_parse1 does (smallest integer tag type, '='
RNEXT, reg2bin bin): checked against hand-built bytes.
pysam itself is absent, so byte identity with a pysam-written file is
unpinned; the decoded records and BAM-input byte copies are what is checked.
"""
import gzip
import os
import struct
from collections import defaultdict

import pytest

from find_circ2_amd import cli
from find_circ2_amd.caller import _aligned_start, group_alignments
from find_circ2_amd.samio import AlignmentFile
from oracle_engine import oracle_evaluator_factory
from samgen import sam_to_bam
from test_native_caller import _rich_sam


def read_bam(path):
    """(header text, [(name, len)], [record body bytes]) of a BAM file."""
    data = gzip.open(path, "rb").read()
    assert data[:4] == b"BAM\1"
    lt, = struct.unpack_from("<i", data, 4)
    text = data[8:8 + lt].decode()
    o = 8 + lt
    nref, = struct.unpack_from("<i", data, o)
    o += 4
    refs = []
    for _ in range(nref):
        ln, = struct.unpack_from("<i", data, o)
        name = data[o + 4:o + 4 + ln - 1].decode()
        lref, = struct.unpack_from("<i", data, o + 4 + ln)
        refs.append((name, lref))
        o += 8 + ln
    recs = []
    while o < len(data):
        bs, = struct.unpack_from("<i", data, o)
        recs.append(data[o + 4:o + 4 + bs])
        o += 4 + bs
    return text, refs, recs


def key(body):
    """(qname, flag, tid, pos, cigar words) of a BAM record body."""
    ref, pos, lname, _mq, _bin, ncig, flag = struct.unpack_from("<iiBBHHH", body, 0)
    qn = body[32:32 + lname - 1].decode()
    cig = struct.unpack_from("<%dI" % ncig, body, 32 + lname)
    return qn, flag, ref, pos, tuple(cig)


def expected_keys(path, mode, asize=15):
    recs = list(AlignmentFile(path, mode))
    out = []
    for _, m1, m2 in group_alignments(recs, defaultdict(float)):
        for m in (m1, m2):
            if not m or len(m.proper_segs) < 2:
                continue
            segs = sorted(m.proper_segs, key=_aligned_start)
            for a, b in zip(segs, segs[1:]):
                if len(a.query) < asize or len(b.query) < asize:
                    continue
                out.append(a)
            out.append(segs[-1])
    return [(a.qname, a.flag, a.tid, a.pos, tuple((n << 4) | op for op, n in a.cigar)) for a in out]


@pytest.fixture(scope="module")
def rich(tmp_path_factory):
    d = tmp_path_factory.mktemp("bamout")
    sam = str(d / "rich.sam")
    fa = _rich_sam(sam, 1500, seed=31)
    bam = str(d / "rich.bam")
    sam_to_bam(open(sam).read(), bam)
    return fa, sam, bam


def _run(tmp_path, fa, inp, extra, tag):
    out = str(tmp_path / tag)
    rc = cli.main(["-G", fa, "-o", out, "-q", "-B"] + extra + [inp], evaluator_factory=oracle_evaluator_factory)
    return rc, out


@pytest.mark.parametrize("extra", [[], ["--python-caller"], ["--no-linear", "-a", "20"], ["--chunk-size", "7"]])
def test_bam_out_records_follow_reference_rule(tmp_path, rich, extra):
    fa, sam, bam = rich
    rc, out = _run(tmp_path, fa, sam, extra, "sam")
    assert rc == 0
    text, refs, recs = read_bam(os.path.join(out, "spliced_alignments.bam"))
    sam_text = open(sam).read()
    assert text == "".join(l + "\n" for l in sam_text.splitlines() if l.startswith("@"))
    assert refs == [("chr1", 90000), ("chr2", 90000), ("chr3", 90000)]
    asize = 20 if "-a" in extra else 15
    want = expected_keys(sam, "r", asize)
    assert len(want) > 1000
    assert [key(r) for r in recs] == want
    # BAM input: the same records, copied byte for byte from the input
    rc, out2 = _run(tmp_path, fa, bam, extra, "bam")
    assert rc == 0
    _, refs2, recs2 = read_bam(os.path.join(out2, "spliced_alignments.bam"))
    _, _, inrecs = read_bam(bam)
    assert refs2 == refs and [key(r) for r in recs2] == want
    assert set(recs2) <= set(inrecs)
    # SAM-encoded records have the BAM-input copies' fixed fields (samgen leaves bin 0 and writes
    # integer tags as 'i', htslib computes the bin and picks the smallest integer type)
    for a, b in zip(recs, recs2):
        assert a[:10] == b[:10] and a[12:32] == b[12:32]


def test_bam_out_nothing_under_noop(tmp_path, rich):
    fa, sam, _ = rich
    rc, out = _run(tmp_path, fa, sam, ["--noop"], "noop")
    assert rc == 0
    _, _, recs = read_bam(os.path.join(out, "spliced_alignments.bam"))
    assert recs == []


def test_bam_out_rejected_with_python_ingest(tmp_path, rich):
    fa, sam, _ = rich
    rc, _ = _run(tmp_path, fa, sam, ["--python-ingest"], "py")
    assert rc == 1


def test_sam_line_encoding_matches_htslib_rules(tmp_path):
    """One spliced read whose anchor lines carry every tag type; bytes built from the spec."""
    sam = tmp_path / "t.sam"
    hdr = "@HD\tVN:1.5\n@SQ\tSN:c1\tLN:1000\n@SQ\tSN:c2\tLN:500\n"
    seqA = "ACGTNacgtRYACGTACGTACGTA"
    l1 = ("r1\t0\tc1\t101\t60\t24M16S\t=\t300\t-55\t%s%s\t%s\tAS:i:24\tXS:i:-3\tNM:i:70000\tXA:Z:c2,+5,3M,0\t"
          "YA:A:x\tYF:f:1.5\tYB:B:s,-2,7\tYH:H:1AE3\tYN:i:-200\tYL:i:-40000\tYU:i:300" % (seqA, "G" * 16, "I" * 40))
    l2 = "r1\t2048\tc1\t201\t7\t24H16M\tc2\t9\t0\t%s\t*\tAS:i:16" % ("G" * 16)
    l3 = "r2\t4\t*\t0\t0\t*\t*\t0\t0\tACGT\t####"
    sam.write_text(hdr + l1 + "\n" + l2 + "\n" + l3 + "\n")
    fa = tmp_path / "g.fa"
    fa.write_text(">c1\n" + "A" * 1000 + "\n>c2\n" + "C" * 500 + "\n")
    out = str(tmp_path / "o")
    rc = cli.main(["-G", str(fa), "-o", out, "-q", "-B", str(sam)], evaluator_factory=oracle_evaluator_factory)
    assert rc == 0
    _, _, recs = read_bam(os.path.join(out, "spliced_alignments.bam"))
    assert len(recs) == 2

    def nt16(s):
        t = "=ACMGRSVTWYHKDBN"
        codes = [t.index(c.upper()) if c.upper() in t else 15 for c in s]
        codes += [0] * (len(codes) % 2)
        return bytes((codes[k] << 4) | codes[k + 1] for k in range(0, len(codes), 2))

    seq1 = seqA + "G" * 16
    body = struct.pack("<iiBBHHHiiii", 0, 100, 3, 60, 4681 + (100 >> 14), 2, 0, 40, 0, 299, -55)
    body += b"r1\0" + struct.pack("<II", (24 << 4) | 0, (16 << 4) | 4) + nt16(seq1) + bytes([40] * 40)
    body += b"ASC" + bytes([24]) + b"XSc" + struct.pack("<b", -3) + b"NMI" + struct.pack("<I", 70000)
    body += b"XAZc2,+5,3M,0\0" + b"YAAx" + b"YFf" + struct.pack("<f", 1.5)
    body += b"YBBs" + struct.pack("<ihh", 2, -2, 7) + b"YHH1AE3\0" + b"YNs" + struct.pack("<h", -200)
    body += b"YLi" + struct.pack("<i", -40000) + b"YUS" + struct.pack("<H", 300)
    assert recs[0] == body
    body2 = struct.pack("<iiBBHHHiiii", 0, 200, 3, 7, 4681 + (200 >> 14), 2, 2048, 16, 1, 8, 0)
    body2 += b"r1\0" + struct.pack("<II", (24 << 4) | 5, (16 << 4) | 0) + nt16("G" * 16) + b"\xff" * 16
    body2 += b"ASC" + bytes([16])
    assert recs[1] == body2
