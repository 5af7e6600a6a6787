"""Pin the CPU oracle to the reference's own known answers.

* tests/golden/test_reads.fa: truth strings after ``___`` in the read names
  (format find_circ.py:1148-1191, produced like simulate_reads.py:100-144).
* tests/golden/cdr1as_reference.bed row 2: CDR1as_locus 728 2213 +, edits 0,
  anchor_overlap 0, breakpoints 1, signal GTAG, 3 reads.

Inputs are bwa-mem-shaped anchor pairs from tests/bwa_emul.py (no aligner in
this image).  Both the literal Python oracle and the C oracle are checked.
"""
import os

import numpy as np
import pytest

import oracle
from oracle.bp_oracle import Options, RefIndexedFasta, Span, find_breakpoints
from bwa_emul import emulate_pairs, read_fasta, truth_from_name
from conftest import GOLDEN


def _reads(path):
    names = [l[1:].strip() for l in open(path) if l.startswith('>')]
    seqs = read_fasta(path)
    return [(n, seqs[n.split()[0]]) for n in names]


def _calls(fa, reads_fa, shift=0):
    g = RefIndexedFasta(fa)
    genome = read_fasta(fa)
    out = []
    for name, seq in _reads(reads_fa):
        for p in emulate_pairs(name, seq, genome, shift=shift):
            sp = Span(p.chrom, p.a_pos, p.a_aend, p.b_pos, p.b_aend, p.read_part.encode(), p.primary_reverse)
            hits = find_breakpoints(sp, g, Options())
            out.append((name, sp, hits))
    return out


@pytest.mark.parametrize("shift", [0, -2, 3])
def test_test_reads_truth(shift):
    calls = _calls(os.path.join(GOLDEN, "test_ref.fa"), os.path.join(GOLDEN, "test_reads.fa"), shift)
    by_read = {}
    for name, sp, hits in calls:
        d = by_read.setdefault(name, (set(), set()))
        for h in hits[:1]:                                  # first tie (find_circ.py:1316-1317)
            (d[1] if sp.is_backsplice else d[0]).add(h.coord)
    n_checked = 0
    for name, (lin, circ) in by_read.items():
        t = truth_from_name(name)
        if t is None:
            continue
        assert lin == t[0], (name, lin, t[0])
        assert circ == t[1], (name, circ, t[1])
        n_checked += 1
    assert n_checked == 3


def test_minus_strand_reads_mirror_plus():
    calls = _calls(os.path.join(GOLDEN, "test_ref.fa"), os.path.join(GOLDEN, "test_reads.fa"))
    minus = {(h.coord, h.gtag) for name, sp, hits in calls if 'minus' in name for h in hits}
    assert (('testbed_minus', 160, 240, '-'), 'GTAG') in minus
    assert (('testbed_minus', 240, 320, '-'), 'GTAG') in minus


def test_cdr1as_reference_bed_row():
    calls = _calls(os.path.join(GOLDEN, "CDR1as_locus.fa"), os.path.join(GOLDEN, "cdr1as_reads.fa"))
    row = open(os.path.join(GOLDEN, "cdr1as_reference.bed")).read().splitlines()[1].split('\t')
    chrom, start, end, strand = row[0], int(row[1]), int(row[2]), row[5]
    n_reads, edits, ov, bps, signal = int(row[4]), int(row[14]), int(row[15]), int(row[16]), row[17]
    support = [hits[0] for _, sp, hits in calls if hits and sp.is_backsplice]
    assert {h.coord for h in support} == {(chrom, start, end, strand)}
    assert len(support) == n_reads == 3
    assert min(h.dist for h in support) == edits == 0
    assert min(h.ov for h in support) == ov == 0
    assert min(h.n_hits for h in support) == bps == 1
    assert {h.gtag for h in support} == {signal}


def test_c_oracle_matches_python_on_known_answers():
    for fa, rf in [("test_ref.fa", "test_reads.fa"), ("CDR1as_locus.fa", "cdr1as_reads.fa")]:
        calls = _calls(os.path.join(GOLDEN, fa), os.path.join(GOLDEN, rf))
        of = oracle.OracleFasta(os.path.join(GOLDEN, fa))
        spans = [sp for _, sp, _ in calls]
        for fast in (False, True):
            r = oracle.scan_fasta(oracle.params(), of, [s.read_part for s in spans],
                                  [of.names.index(s.chrom) for s in spans], [s.a_pos for s in spans],
                                  [s.b_aend for s in spans], [s.is_backsplice for s in spans],
                                  [s.primary_reverse for s in spans], use_fast=fast)
            for i, (_, sp, hits) in enumerate(calls):
                assert r.n_ties[i] == len(hits)
                if hits:
                    f = r.first[i]
                    assert (f['x'], f['start'], f['end'], f['strand'].decode(), f['gtag'].decode()) == \
                           (hits[0].x, hits[0].start, hits[0].end, hits[0].strand, hits[0].gtag)


def test_ref_track_chain_equals_indexed_fasta(tmp_path):
    """oracle.bp_oracle.RefGenomeTrack (Track.get -> GenomeAccessor.get_data -> indexed_fasta.get_data,
    find_circ.py:274-312, 362-368, 189-215), the chain bench.py's CPU baseline times, over an mmap'd
    FASTA with its .byo_index: the same windows as RefIndexedFasta itself, and the same
    find_breakpoints results on the CDR1as known answer; a chromosome missing from the index raises
    KeyError('chrom') from get_data (:193), not from the accessor cache."""
    import ctypes
    import shutil
    from find_circ2_amd import _native as N
    from oracle.bp_oracle import Options, RefGenomeTrack, RefIndexedFasta, Span, find_breakpoints
    fa = str(tmp_path / "c.fa")
    shutil.copy(os.path.join(GOLDEN, "CDR1as_locus.fa"), fa)
    h = ctypes.c_void_p()
    N.check(N.lib().fc2_fasta_open(fa.encode(), 1, ctypes.byref(h)))
    N.lib().fc2_fasta_close(h)
    plain = RefIndexedFasta(fa)
    track = RefGenomeTrack(RefIndexedFasta(fa, use_existing_index=True, use_mmap=True))
    rng = np.random.default_rng(3)
    for _ in range(300):
        a = int(rng.integers(-100, 3000))
        e = a + int(rng.integers(0, 200))
        assert track.get("CDR1as_locus", a, e, "+") == plain.get_data("CDR1as_locus", a, e, "+")
    with pytest.raises(KeyError) as ex:
        track.get("chrX", 10, 20, "+")
    assert ex.value.args[0] == "chrX"
    genome = read_fasta(os.path.join(GOLDEN, "CDR1as_locus.fa"))
    reads = read_fasta(os.path.join(GOLDEN, "cdr1as_reads.fa"))
    n = 0
    for name, seq in reads.items():
        for s in emulate_pairs(name, seq, genome):
            sp = Span(s.chrom, s.a_pos, s.a_aend, s.b_pos, s.b_aend, s.read_part.encode(), s.primary_reverse)
            h1 = find_breakpoints(sp, track, Options())
            h2 = find_breakpoints(sp, plain, Options())
            assert [(t.x, t.coord) for t in h1] == [(t.x, t.coord) for t in h2]
            n += bool(h1)
    assert n >= 3


def test_literal_rate_pool_matches_direct_calls(tmp_path):
    """bench.py's multi-process literal CPU baseline (oracle.bp_oracle.literal_rate on spawned workers,
    disjoint slices): every span's first tie equals a direct find_breakpoints call on the same span."""
    import multiprocessing as mp
    import shutil
    from oracle.bp_oracle import literal_rate
    fa = str(tmp_path / "CDR1as_locus.fa")
    shutil.copy(os.path.join(GOLDEN, "CDR1as_locus.fa"), fa)
    calls = _calls(fa, os.path.join(GOLDEN, "cdr1as_reads.fa")) + \
        _calls(fa, os.path.join(GOLDEN, "cdr1as_reads.fa"), shift=2)
    spans = [(sp.chrom, sp.a_pos, sp.a_aend, sp.b_pos, sp.b_aend, sp.read_part, sp.primary_reverse)
             for _, sp, _ in calls]
    want = [(h[0].x, h[0].n_hits) if h else (-1, 0) for _, _, h in calls]
    P = 2
    sl = [spans[len(spans) * i // P:len(spans) * (i + 1) // P] for i in range(P)]
    with mp.get_context("spawn").Pool(P) as pool:
        outs = pool.starmap(literal_rate, [(fa, x, 60.0) for x in sl])
    assert sum(o[0] for o in outs) == len(spans)
    assert [t for o in outs for t in o[2]] == want
    assert (39, 1) in want
