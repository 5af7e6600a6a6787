"""Test-only evaluator: the CPU oracle behind the caller's ``evaluate(spans)`` hook.

Lets the whole CLI (grouping, record_hits, aggregation, writers) run on CPU
with the oracle's breakpoint search, so that (a) the host logic is tested
without a GPU and (b) on a GPU box the outputs of the GPU evaluator can be
compared file-for-file with this one.
"""
import oracle
from find_circ2_amd.hotpath import Splice


def oracle_evaluator_factory(options, hp):
    of = oracle.OracleFasta(options.genome)
    p = oracle.params(hp.asize, hp.margin, hp.maxdist, hp.noncanonical, hp.strandpref, hp.allhits)

    def evaluate(spans):
        idx = [of.names.index(s.chrom) if s.chrom in of.names else -1 for s in spans]
        r = oracle.scan_fasta(p, of, [s.read_part.encode("latin-1") for s in spans], idx,
                              [s.align_A.pos for s in spans], [s.align_B.aend for s in spans],
                              [s.is_backsplice for s in spans], [s.strand == '-' for s in spans],
                              use_fast=False, all_ties=True)
        for i, s in enumerate(spans):
            nt = int(r.n_ties[i])
            if nt == -oracle.ORC_ERR_KEY:
                s.result = KeyError("gtag")
            elif nt == -oracle.ORC_ERR_CHROM:
                s.result = KeyError(s.chrom)
            elif nt < 0:
                s.result = RuntimeError("shape")
            else:
                out = []
                for t in r.ties_of(i):
                    sp = Splice(s, s.chrom, int(t["start"]), int(t["end"]), t["strand"].decode(),
                                False if hp.maxdist == 0 else int(t["dist"]), int(t["ov"]), t["gtag"].decode())
                    sp.n_hits = int(t["n_hits"])
                    sp._score = int(t["score"])
                    out.append(sp)
                s.result = out
    return evaluate
