"""The reference's own bwa-mem records through every reader of the repo.

``tests/golden/test_norm.sam`` is ``test_data/test_norm.sam`` of the reference: 93 hg19 ``@SQ``
lines and three reads, each a primary (``56M20S`` / ``54M22S`` / ``42M34S``) plus a hard-clipped
supplementary (``52H24M`` / ``50H26M`` / ``38H38M``) carrying ``SA``, ``AS`` and ``XS``.  It is the
only bwa-mem output the reference holds, so it is the one reference-held pin of pair formation
(SURVEY.md §8(c)): ``aligned_start_from_cigar`` (find_circ.py:1086-1097), ``q_start`` / ``q_end``
(:1100-1101, :1130-1131), ``JunctionSpan`` (:821-852) and ``uniqness`` (:809-819).

Three readers form the pairs and each is checked against the table below, which is derived by hand
from the SAM text (not computed by any code of the repo):

* the Python ``samio`` reader + ``caller.MateSegments`` (the ``--python-ingest`` loop);
* the native ingest (``fc2_ingest_next``, SAM and BAM) + ``caller.MateSegments`` (``--python-caller``);
* the native read loop's pair formation (``fc2_caller_next``, SAM and BAM), the shipped path.

Breakpoints need hg19 chr22, which is absent.  ``planted_chr22`` rebuilds the bases the records
themselves state: a FASTA with chr22 at its ``@SQ`` length (51,304,566 bp, 50-nt lines) holding, at
every aligned position, the read base the alignment puts there (NM:0 records first; the one NM:1
record, read 3's supplementary, must disagree with them at exactly one position), 'N' everywhere no
record aligns.  The three reads then cross one donor/acceptor pair that the data itself carries: the
primaries end in ...GG|AGGT and the supplementaries start AGGT..., a 4-base microhomology in which
``GT`` (read bases 54-55 of read 1) is the donor and ``AG`` the acceptor.  The expected junction row
is derived by hand from that below and checked for every reader; the GPU CLI is compared with the
oracle CLI on this genome, on a dummy genome and on a random-filled variant in test_cli_gpu-style
tests at the bottom (``-m gpu``).
"""
import ctypes
import gzip
import os
import shutil

import numpy as np
import pytest

from conftest import GOLDEN

NORM = os.path.join(GOLDEN, "test_norm.sam")
CHR22_LEN = 51304566          # test_norm.sam @SQ SN:chr22 LN:51304566
QN = ["hek_test_norm_000012_hek_test_norm_000011_s_8_1_00%s_qseq_%s" % s
      for s in (("21", "146360_583"), ("57", "101659_584"), ("76", "124611_585"))]

# --------------------------------------------------------------------------------------------------
# The hand-derived table.  SAM POS is 1-based; pysam's pos is POS - 1.  aend = pos + the M ops.
#   q_start of a segment = leading S/H clips before its first M (:1092-1096); q_end = q_start +
#   len(query) (:1101), query = SEQ without soft clips (hard-clipped bases are not in SEQ).
#   Segments sorted by q_start (:1106): A = primary (q_start 0), B = supplementary.
#   JunctionSpan q_start/q_end = min/max over the two (:1130-1131); read_part = primary.seq[q_start:
#   q_end] (:843-844); dist = B.pos - A.aend (:842), backsplice iff < 0 (:851-852); uniq_X = AS - XS
#   (:814-819); uniq = min (:831); weight = 1/(n_proper - 1) = 1.0 for two segments (:1084).
#
# read 1: primary  POS 50647092 56M20S -> pos 50647091, aend 50647147, q 0..56,  AS 56 - XS 17 = 39
#         suppl.   POS 50648608 52H24M -> pos 50648607, aend 50648631, q 52..76, AS 24 - XS 18 = 6
#         q_start 0, q_end 76, dist 50648607 - 50647147 = 1460 > 0: linear, uniq min(39, 6) = 6
# read 2: primary  POS 50647094 54M22S -> pos 50647093, aend 50647147, q 0..54,  54 - 17 = 37
#         suppl.   POS 50648608 50H26M -> pos 50648607, aend 50648633, q 50..76, 26 - 18 = 8
#         q_start 0, q_end 76, dist 1460: linear, uniq 8
# read 3: primary  POS 50647106 42M34S -> pos 50647105, aend 50647147, q 0..42,  42 - 17 = 25
#         suppl.   POS 50648608 38H38M -> pos 50648607, aend 50648645, q 38..76, 33 - 18 = 15
#         q_start 0, q_end 76, dist 1460: linear, uniq 15
# --------------------------------------------------------------------------------------------------
EXPECTED = [
    dict(qname=QN[0], q_start=0, q_end=76, a_pos=50647091, a_aend=50647147, b_pos=50648607, b_aend=50648631,
         uniq_A=39, uniq_B=6, uniq=6, weight=1.0, backsplice=False, strand="+"),
    dict(qname=QN[1], q_start=0, q_end=76, a_pos=50647093, a_aend=50647147, b_pos=50648607, b_aend=50648633,
         uniq_A=37, uniq_B=8, uniq=8, weight=1.0, backsplice=False, strand="+"),
    dict(qname=QN[2], q_start=0, q_end=76, a_pos=50647105, a_aend=50647147, b_pos=50648607, b_aend=50648645,
         uniq_A=25, uniq_B=15, uniq=15, weight=1.0, backsplice=False, strand="+"),
]

# Breakpoints on planted_chr22 (defaults: asize 15, margin 2 -> e = 13; L = 76 -> l = 50, windows of
# 52 bases).  Af[i] = G[A.pos + 13 + i], Bf[j] = G[B.aend - 13 - 52 + j] (:900-902).  Af is planted
# below G[50647147] (all three primaries end there), Bf from G[50648607] on (all supplementaries
# start there).  The dinucleotides Af[x:x+2] and Bf[x:x+2] are both free of 'N' at exactly one x, the
# x with A.pos + 13 + x = 50647145 and B.aend - 65 + x = 50648607:
#   read 1: x = 50647145 - 50647104 = 41 (and 50648607 - 50648566 = 41), gtag G[50647145:+2] +
#           G[50648607:+2] = 'GT' + 'AG'; dist 0
#   read 2: x = 50647145 - 50647106 = 39 (50648607 - 50648568 = 39); dist 0
#   read 3: x = 50647145 - 50647118 = 27 (50648607 - 50648580 = 27); dist 1 (its NM:1 base, at
#           G[50648631], read base 62 = internal index 49, right of x, compared against Bf)
# Coordinates (:929-945, linear): start = min(B.aend - e - l + x, A.pos + e + x + 1) - 1, end = max:
#   read 1: (50648631 - 63 + 41, 50647091 + 14 + 41) = (50648609, 50647146) -> (50647145, 50648609)
#   read 2: (50648633 - 63 + 39, 50647093 + 14 + 39) -> the same;  read 3: (50648645 - 63 + 27,
#   50647105 + 14 + 27) -> the same.  One linear junction, chr22:50647145-50648609 '+', GTAG.
BP = [dict(x=41, dist=0), dict(x=39, dist=0), dict(x=27, dist=1)]
JUNCTION = ("chr22", 50647145, 50648609, "+")
# Its lin_splice_sites.bed row with -n test (store_list :722-729, Hit :486-654): 3 fragments, weight
# 1.0 each, 3 distinct read sequences, every qA/qB non-zero -> uniq_bridges 3.0, best quals
# max(39, 37, 25) / max(6, 8, 15), edits min(0, 0, 1), overlap 0, n_hits 1, no categories (GTAG,
# 1464 nt between the short and huge thresholds, no fragment flags on a linear junction).
LIN_ROW = ["chr22", "50647145", "50648609", "test_lin_000001", "3", "+", "3.0", "3", "3", "3.0", "39", "15",
           "test", "3.0", "0", "0", "1", "GTAG", "N/A", "", "N/A", "0"]


def _records():
    return [l.rstrip("\n").split("\t") for l in open(NORM) if not l.startswith("@")]


def planted_chr22(path, fill=None, seed=0):
    """chr22 at its hg19 length with the bases test_norm.sam's alignments state (see module doc);
    `fill` None: 'N' elsewhere, else random ACGT (seeded) elsewhere."""
    if fill is None:
        g = np.full(CHR22_LEN, ord("N"), np.uint8)
    else:
        g = np.frombuffer(b"ACGT", np.uint8)[np.random.default_rng(seed).integers(0, 4, CHR22_LEN)].copy()
    planted = np.zeros(CHR22_LEN, bool)
    recs = sorted(_records(), key=lambda f: [t for t in f[11:] if t.startswith("NM:i:")][0])   # NM:0 first
    conflicts = {}
    for f in recs:
        from find_circ2_amd.samio import parse_cigar
        pos, seq, q = int(f[3]) - 1, f[9], 0
        nm = int([t for t in f[11:] if t.startswith("NM:i:")][0][5:])
        bad = 0
        for op, n in parse_cigar(f[5]):
            if op == 0:
                for k in range(n):
                    b = ord(seq[q + k])
                    if planted[pos + k] and g[pos + k] != b:
                        bad += 1
                        conflicts[pos + k] = chr(b)
                    elif not planted[pos + k]:
                        g[pos + k], planted[pos + k] = b, True
                pos += n
                q += n
            elif op == 4:
                q += n
        assert bad == nm, (f[0], f[5], bad, nm)      # the records agree with one genome up to their NM
    assert conflicts == {50648631: "C"}              # read 3's one mismatch (read 2 has 'T' there)
    with open(path, "wb") as fh:
        fh.write(b">chr22\n")
        body = g.tobytes()
        fh.write(b"\n".join(body[i:i + 50] for i in range(0, len(body), 50)) + b"\n")
    return path


@pytest.fixture(scope="module")
def chr22(tmp_path_factory):
    d = tmp_path_factory.mktemp("chr22")
    return planted_chr22(str(d / "chr22.fa"))


@pytest.fixture(scope="module")
def norm_bam(tmp_path_factory):
    from find_circ2_amd.ingest import sam_to_bam
    p = str(tmp_path_factory.mktemp("bam") / "test_norm.bam")
    sam_to_bam(NORM, p)
    return p


def _check_span(sp, exp, read_seq):
    assert sp.primary.qname == exp["qname"]
    assert (sp.q_start, sp.q_end) == (exp["q_start"], exp["q_end"])
    assert (sp.align_A.pos, sp.align_A.aend, sp.align_B.pos, sp.align_B.aend) == \
        (exp["a_pos"], exp["a_aend"], exp["b_pos"], exp["b_aend"])
    assert (sp.uniq_A, sp.uniq_B, sp.uniq) == (exp["uniq_A"], exp["uniq_B"], exp["uniq"])
    assert sp.weight == exp["weight"] and sp.is_backsplice == exp["backsplice"] and sp.strand == exp["strand"]
    assert sp.read_part == read_seq[exp["q_start"]:exp["q_end"]] and len(sp.read_part) == 76


def _primary_seqs():
    return [f[9] for f in _records() if int(f[1]) & 0x800 == 0]


def _spans_from_records(records, refs):
    from collections import defaultdict

    from find_circ2_amd.caller import CallerOptions, group_alignments
    opts, counters = CallerOptions(), defaultdict(float)
    out = []
    for _, m1, m2 in group_alignments(records, counters):
        for m in (m1, m2):
            if m:
                out += m.spans(opts, counters, lambda a: refs[a.tid])
    return out, counters


def test_hand_table_matches_the_sam_text():
    """The table's inputs are the file's: three primaries of 76 bases, unpaired, forward strand."""
    recs = _records()
    assert [f[0] for f in recs] == [q for q in QN for _ in (0, 1)]
    assert [f[1] for f in recs] == ["0", "2048"] * 3
    assert [f[5] for f in recs] == ["56M20S", "52H24M", "54M22S", "50H26M", "42M34S", "38H38M"]
    assert all(len(s) == 76 for s in _primary_seqs())
    # the microhomology the junction derivation rests on: primaries end ...AGGT, supplementaries start AGGT
    seqs = _primary_seqs()
    assert seqs[0][52:56] == "AGGT" and seqs[0][54:56] == "GT"
    assert [f[9][:4] for f in recs if f[1] == "2048"] == ["AGGT"] * 3


@pytest.mark.parametrize("fmt", ["sam", "bam"])
def test_python_samio_spans(fmt, norm_bam):
    from find_circ2_amd.samio import AlignmentFile
    f = AlignmentFile(NORM if fmt == "sam" else norm_bam)
    assert f.format == fmt and len(f.references) == 93 and f.references[f.references.index("chr22")] == "chr22"
    spans, counters = _spans_from_records(list(f), f.references)
    f.close()
    assert len(spans) == 3
    for sp, exp, seq in zip(spans, EXPECTED, _primary_seqs()):
        _check_span(sp, exp, seq)
        assert sp.chrom == "chr22"
    assert counters["total_mates"] == 3 and counters["seg_too_short_skip"] == 0


@pytest.mark.parametrize("fmt", ["sam", "bam"])
def test_native_ingest_spans(fmt, norm_bam):
    """fc2_ingest_next hands back the three fragments (every one carries an anchor pair)."""
    from find_circ2_amd.ingest import NativeIngest
    ing = NativeIngest(NORM if fmt == "sam" else norm_bam, fmt == "bam")
    assert ing.format()[0] == fmt
    frags = []
    while not ing.eof:
        frags += ing.next_chunk(15, False, False, 100)
    assert [len(fr) for fr in frags] == [2, 2, 2]
    spans = []
    for fr in frags:
        s, _ = _spans_from_records(fr, ing.references)
        spans += s
    c = ing.counts
    assert (c.n_reads, c.total_mates, c.records, c.handed_back) == (3, 3, 6, 3)
    ing.close()
    for sp, exp, seq in zip(spans, EXPECTED, _primary_seqs()):
        _check_span(sp, exp, seq)


def _native_pairs(path, is_bam, **kw):
    """The pairs fc2_caller_next hands out for evaluation (the shipped read loop)."""
    from find_circ2_amd import _native as N
    from find_circ2_amd.caller import CallerOptions
    from find_circ2_amd.native_caller import NativeCaller
    nc = NativeCaller(path, is_bam, CallerOptions(**kw), ["chr22"], write_reads=False, write_multi=False)
    nc.open()
    out = []
    try:
        L = N.lib()
        while True:
            b, eof = N.CallerBatch(), ctypes.c_int(0)
            N.check(L.fc2_caller_next(nc.h, ctypes.byref(b), ctypes.byref(eof)))
            n = int(b.n)
            assert int(b.n_long) == 0
            if n:
                pairs = np.frombuffer(ctypes.string_at(b.pairs, 16 * n), N.PAIR_DTYPE)
                offs = np.frombuffer(ctypes.string_at(b.read_off, 8 * n), np.uint64)
                end = int((offs + pairs["read_len"]).max())
                reads = ctypes.string_at(b.reads, end)
                for p, o in zip(pairs, offs):
                    out.append(dict(a_pos=int(p["a_pos"]), b_aend=int(p["b_aend"]), chrom=int(p["chrom"]),
                                    flags=int(p["flags"]),
                                    read_part=reads[int(o):int(o) + int(p["read_len"])].decode()))
            while L.fc2_caller_queued(nc.h) > 0:          # (a chunk may hold no eligible pair: n = 0)
                res = np.zeros(max(n, 1), N.RESULT_DTYPE)
                res["best_x"] = -1
                N.check(L.fc2_caller_submit(nc.h, res.ctypes.data, None, 0, n))
            if eof.value:
                break
        counters = nc.counters()
    finally:
        nc.close()
    return out, counters


@pytest.mark.parametrize("fmt", ["sam", "bam"])
def test_native_caller_pairs(fmt, norm_bam):
    """fc2_caller_next's pair records: A.pos, B.aend, chromosome, read part (= seq[q_start:q_end]),
    backsplice / primary-strand flags; with the default --min-uniq-qual 2 all three are evaluated."""
    pairs, counters = _native_pairs(NORM if fmt == "sam" else norm_bam, fmt == "bam")
    assert len(pairs) == 3
    for p, exp, seq in zip(pairs, EXPECTED, _primary_seqs()):
        assert (p["a_pos"], p["b_aend"], p["chrom"]) == (exp["a_pos"], exp["b_aend"], 0)
        assert p["read_part"] == seq[exp["q_start"]:exp["q_end"]]
        assert p["flags"] & 0x13 == 0     # FC2_PAIR_BACKSPLICE | _PRIMARY_REV | _SKIP (include/fc2_bp.h)
    # every result was "no breakpoint": three linear spans without a hit (:1358-1361)
    assert counters["lin_no_bp"] == 3 and counters["total_mates"] == 3


@pytest.mark.parametrize("fmt", ["sam", "bam"])
@pytest.mark.parametrize("q", [6, 7, 8, 9, 15, 16])
def test_native_caller_uniq_threshold(fmt, q, norm_bam):
    """uniq = min(AS - XS) of each span, seen through the native path's only use of it: a span is
    evaluated iff uniq >= --min-uniq-qual (:846-848, :1351-1353).  Uniq 6 / 8 / 15 (the table)."""
    pairs, counters = _native_pairs(NORM if fmt == "sam" else norm_bam, fmt == "bam", min_uniq_qual=q)
    kept = [e["a_pos"] for e in EXPECTED if e["uniq"] >= q]
    assert [p["a_pos"] for p in pairs] == kept
    assert counters.get("lin_junc_not_unique", 0) == 3 - len(kept)


def test_planted_genome_breakpoints_match_hand_derivation(chr22):
    """The literal oracle (find_breakpoints, find_circ.py:854-974) on the three spans over the planted
    chr22: one hit each, at the hand-derived x, dist, coordinates and signal."""
    from oracle.bp_oracle import Options, RefGenomeTrack, RefIndexedFasta, Span, find_breakpoints
    g = RefGenomeTrack(RefIndexedFasta(chr22))
    for exp, bp, seq in zip(EXPECTED, BP, _primary_seqs()):
        sp = Span("chr22", exp["a_pos"], exp["a_aend"], exp["b_pos"], exp["b_aend"], seq.encode())
        for nc in (False, True):
            hits = find_breakpoints(sp, g, Options(noncanonical=nc))
            best = hits[0]
            assert (best.x, best.dist, best.ov, best.gtag, best.strand) == (bp["x"], bp["dist"], 0, "GTAG", "+")
            assert best.coord == JUNCTION and best.n_hits == 1
            assert len(hits) == 1


def _run(tmp, fa, inp, extra=(), mode=(), evaluator="oracle", tag="o"):
    from find_circ2_amd import cli
    from oracle_engine import oracle_evaluator_factory
    out = str(tmp / tag)
    ev = oracle_evaluator_factory if evaluator == "oracle" else None
    rc = cli.main(["-G", fa, "-o", out, "-n", "test", "-q"] + list(mode) + list(extra) + [inp], evaluator_factory=ev)
    return rc, out


def _rows(out, f):
    return [l.rstrip("\n").split("\t") for l in open(os.path.join(out, f)) if not l.startswith("#")]


READERS = [("sam", []), ("sam", ["--python-caller"]), ("sam", ["--python-ingest"]),
           ("bam", []), ("bam", ["--python-caller"]), ("bam", ["--python-ingest"])]


@pytest.mark.parametrize("fmt,mode", READERS)
def test_cli_every_reader_writes_the_hand_derived_row(tmp_path, chr22, norm_bam, fmt, mode):
    """Every read loop (native, --python-caller, --python-ingest) on SAM and BAM, with the CPU oracle as
    the breakpoint search: the one linear junction row, the three reads in spliced_reads.fastq.gz,
    no circular row, no multi-event."""
    fa = str(tmp_path / "chr22.fa")
    shutil.copy(chr22, fa)
    rc, out = _run(tmp_path, fa, NORM if fmt == "sam" else norm_bam, mode=mode)
    assert rc == 0
    assert _rows(out, "lin_splice_sites.bed") == [LIN_ROW]
    assert _rows(out, "circ_splice_sites.bed") == []
    assert _rows(out, "multi_events.tsv") == []
    # write_read (:1442-1447): "@qname junctions flags" with an empty flag list, qual '*' -> None
    with gzip.open(os.path.join(out, "spliced_reads.fastq.gz"), "rt") as fh:
        fq = fh.read()
    want = "".join("@{0} test_lin_000001 \n{1}\n+{0} test_lin_000001 \nNone\n".format(q, s)
                   for q, s in zip(QN, _primary_seqs()))
    assert fq == want
    from test_ingest import counters
    c = counters(out)
    assert c["lin_spliced"] == 3 and c["total_mates"] == 3


@pytest.mark.parametrize("extra,row", [
    # -d 0: simple_match's bool (:865-871); read 3 (dist 1) no longer qualifies -> 2 reads,
    # best_qual_right max(6, 8), edits False
    (["-d", "0"], ["chr22", "50647145", "50648609", "test_lin_000001", "2", "+", "2.0", "2", "2", "2.0", "39",
                   "8", "test", "2.0", "False", "0", "1", "GTAG", "N/A", "", "N/A", "0"]),
    # --min-uniq-qual 9: read 1 (uniq 6) and read 2 (uniq 8) are not evaluated (:1351-1353); read 3
    # alone has edits 1, overlap 0 -> WARN_EXT_1MM (:619-622)
    (["--min-uniq-qual", "9"], ["chr22", "50647145", "50648609", "test_lin_000001", "1", "+", "1.0", "1", "1",
                                "1.0", "25", "15", "test", "1.0", "1", "0", "1", "GTAG", "N/A", "WARN_EXT_1MM",
                                "N/A", "0"]),
    # --strand-pref adds 100 to '+' hits of '+' primaries; nothing changes for one hit per read
    (["--strand-pref", "--non-canonical", "--all-hits"], LIN_ROW),
])
@pytest.mark.parametrize("mode", [[], ["--python-ingest"]])
def test_cli_options_on_the_planted_genome(tmp_path, chr22, extra, row, mode):
    fa = str(tmp_path / "chr22.fa")
    shutil.copy(chr22, fa)
    rc, out = _run(tmp_path, fa, NORM, extra=extra, mode=mode)
    assert rc == 0
    assert _rows(out, "lin_splice_sites.bed") == [row]


def test_cli_dummy_genome_has_no_breakpoint(tmp_path):
    """No FASTA: dummy mode (all-N windows, find_circ.py:340-345) -- every x mismatches all 50 internal
    bases, so the three spans end in lin_no_bp and no row is written, in every read loop."""
    from test_ingest import counters
    for k, mode in enumerate(([], ["--python-ingest"], ["--python-caller"])):
        rc, out = _run(tmp_path, str(tmp_path / "absent.fa"), NORM, mode=mode, tag="dummy%d" % k)
        assert rc == 0
        assert _rows(out, "lin_splice_sites.bed") == [] and _rows(out, "circ_splice_sites.bed") == []
        assert counters(out)["lin_no_bp"] == 3


# ---------------------------------------------------------------------------------------------- GPU
def _files_equal(o1, o2):
    from test_ingest import same
    same(o1, o2)


@pytest.mark.gpu
@pytest.mark.parametrize("genome", ["planted", "random", "dummy"])
@pytest.mark.parametrize("extra", [[], ["--non-canonical", "--all-hits"], ["-d", "0"]])
@pytest.mark.parametrize("fmt", ["sam", "bam"])
def test_gpu_cli_on_test_norm_equals_oracle_cli(tmp_path, chr22, norm_bam, genome, extra, fmt):
    """The shipped CLI (native read loop + HIP search) on the reference's bwa-mem records writes the
    files the Python loop + CPU oracle writes: on the planted chr22, on a random-filled chr22 with the
    same planted bases, and on a dummy genome."""
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    if genome == "planted":
        fa = str(tmp_path / "chr22.fa")
        shutil.copy(chr22, fa)
    elif genome == "random":
        fa = planted_chr22(str(tmp_path / "chr22r.fa"), fill="random", seed=110112)
    else:
        fa = str(tmp_path / "absent.fa")
    inp = NORM if fmt == "sam" else norm_bam
    rc1, o1 = _run(tmp_path, fa, inp, extra=extra, mode=["--python-ingest"], tag="oracle")
    rc2, o2 = _run(tmp_path, fa, inp, extra=extra, evaluator=None, tag="gpu")
    assert rc1 == rc2 == 0
    _files_equal(o1, o2)
    if genome == "planted" and not extra:
        assert _rows(o2, "lin_splice_sites.bed") == [LIN_ROW]
