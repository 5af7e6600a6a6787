"""Cross-check the three CPU restatements against each other on seeded pairs.

literal Python (oracle/bp_oracle.py, O(l^2) numpy idiom of find_circ.py:906-908)
== C naive O(l^2) == C fast O(l), over every option the hot path reads
(find_circ.py:393-404): margin, maxdist (incl. the bool quirk at 0),
--non-canonical, --strand-pref, --all-hits; N-padded windows at chromosome
ends; N and lower-case bytes in reads; short reads with l <= 0.
"""
import os

import pytest

import oracle
from oracle.bp_oracle import Options, RefIndexedFasta, Span, find_breakpoints, ReferenceKeyError
from synth_small import load_genome, make_spans
from conftest import GOLDEN

OPTS = [
    dict(),
    dict(maxdist=0),
    dict(maxdist=4, margin=0),
    dict(noncanonical=True),
    dict(strandpref=True),
    dict(allhits=True, noncanonical=True),
    dict(asize=20, margin=5, maxdist=3),
    dict(asize=10, margin=1, maxdist=1, strandpref=True, noncanonical=True),
]


@pytest.mark.parametrize("fa", ["CDR1as_locus.fa", "test_ref.fa"])
@pytest.mark.parametrize("oi", range(len(OPTS)))
def test_python_vs_c(fa, oi):
    o = OPTS[oi]
    opt = Options(**o)
    path = os.path.join(GOLDEN, fa)
    genome = load_genome(path)
    spans = make_spans(genome, 150, seed=1337 + oi, asize=opt.asize)
    ref = RefIndexedFasta(path)
    of = oracle.OracleFasta(path)
    p = oracle.params(**o)
    args = ([s.read_part for s in spans], [s.chrom_idx for s in spans], [s.a_pos for s in spans],
            [s.b_aend for s in spans], [s.is_backsplice for s in spans], [s.primary_reverse for s in spans])
    rn = oracle.scan_fasta(p, of, *args, use_fast=False, all_ties=True)
    rf = oracle.scan_fasta(p, of, *args, use_fast=True, all_ties=True)
    n_hit = 0
    for i, s in enumerate(spans):
        sp = Span(s.chrom, s.a_pos, s.a_aend, s.b_pos, s.b_aend, s.read_part, s.primary_reverse)
        try:
            hits = find_breakpoints(sp, ref, opt)
        except ReferenceKeyError:
            assert rn.n_ties[i] == -oracle.ORC_ERR_KEY
            continue
        assert rn.n_ties[i] == len(hits), i
        assert rf.n_ties[i] == len(hits), i
        for r in (rn, rf):
            got = [(t['x'], t['start'], t['end'], t['strand'].decode(), t['gtag'].decode(), int(t['dist']),
                    t['ov'], t['score'], t['n_hits']) for t in r.ties_of(i)]
            exp = [(h.x, h.start, h.end, h.strand, h.gtag, int(h.dist), h.ov, h.score, h.n_hits) for h in hits]
            assert got == exp, (i, got, exp)
        n_hit += bool(hits)
    assert n_hit > 10
