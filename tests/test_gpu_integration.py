"""The drop-in binding exactly as INTEGRATION.md prints it (§1 one span per call, §2 the batched
``flush``), run against a stand-in of the reference's module globals: ``options``, ``Splice``
(find_circ.py:766-806), ``JunctionSpan`` (:821-852, the package mirror), ``fast_chrom_lookup``
(:471-477) and a ``record_hits`` that calls ``find_breakpoints()`` span by span in input order
(:1276-1439).  Spans are pysam-shaped records (``pos``, ``aend``, ``seq``, ``is_reverse``,
``AS``/``XS`` tags).  Every span's result -- the ties, or the exception -- must be the oracle's
(oracle/bp_oracle.py, find_circ.py:854-974): KeyError for a chromosome missing from the FASTA
(:193) and for a non-ACGTN splice signal (:927), the ``-d 0`` bool, all ties under --all-hits.
"""
import os
import re
import types

import numpy as np
import pytest

from conftest import GOLDEN
from synth_small import load_genome, make_spans

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

import find_circ2_amd as fc2  # noqa: E402
from oracle.bp_oracle import Options as ROptions, RefIndexedFasta, Span as RSpan, find_breakpoints as ref_fb  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _blocks():
    text = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    blocks = re.findall(r"```python\n(.*?)```", text, re.S)
    one = [b for b in blocks if "def find_breakpoints(self)" in b]
    two = [b for b in blocks if "def flush(pending)" in b]
    assert len(one) == 1 and len(two) == 1
    return one[0], two[0]


class Rec:
    """pysam.AlignedSegment fields the path reads."""

    def __init__(self, tid, pos, aend, seq=None, is_reverse=False, AS=None, XS=None):
        self.tid, self.pos, self.aend, self.seq, self.is_reverse = tid, pos, aend, seq, is_reverse
        self._tags = {"AS": AS}
        if XS is not None:
            self._tags["XS"] = XS

    def get_tag(self, k):
        return self._tags[k]

    def has_tag(self, k):
        return k in self._tags


class RefSplice:
    """The reference's Splice constructor (find_circ.py:766-776)."""

    def __init__(self, junc_span, chrom, start, end, strand, dist, ov, gtag):
        self.junc_span, self.chrom, self.start, self.end = junc_span, chrom, start, end
        self.strand, self.dist, self.ov, self.gtag = strand, dist, ov, gtag
        self.n_hits = 1


def _env(path, opt, names):
    """Module globals of find_circ.py the printed snippets use."""
    options = types.SimpleNamespace(genome=path, asize=opt.asize, margin=opt.margin, maxdist=opt.maxdist,
                                    noncanonical=opt.noncanonical, strandpref=opt.strandpref,
                                    allhits=opt.allhits, min_uniq_qual=2, chunksize=100000)
    JS = type("JunctionSpan", (fc2.JunctionSpan,), {})          # a class of its own: the snippets patch it
    written = []
    calls = []

    def fast_chrom_lookup(align):
        return names[align.tid]

    def record_hits(frag_name, circ, lin, unspliced, broken):
        # the evaluation order of find_circ.py:1295-1303, 1346-1355 (circ spans first)
        for span in circ + lin:
            if not span.is_uniq:
                continue
            calls.append((span, span.find_breakpoints()))
        return ({"j"} if any(r for _, r in calls[-len(circ + lin):]) else set()), set()

    def write_read(mate, junctions, flags):
        written.append(mate)

    ns = dict(options=options, Splice=RefSplice, JunctionSpan=JS, fast_chrom_lookup=fast_chrom_lookup,
              record_hits=record_hits, write_read=write_read)
    return ns, calls, written


def _spans_from_small(JS, sp, names, extra_names):
    out = []
    for s in sp:
        tid = names.index(s.chrom) if s.chrom in names else extra_names.index(s.chrom) + len(names)
        seq = s.read_part.decode("latin-1") if isinstance(s.read_part, bytes) else s.read_part
        A = Rec(tid, s.a_pos, s.a_aend, AS=30)
        B = Rec(tid, s.b_pos, s.b_aend, AS=30, XS=(29 if len(out) % 17 == 5 else None))  # some not unique
        prim = Rec(tid, min(s.a_pos, s.b_pos), None, seq=seq, is_reverse=s.primary_reverse, AS=30)
        out.append(JS(A, B, prim, 0, len(seq), 1.0))
    return out


def _expected(span, path, opt, fasta):
    rs = RSpan(span.chrom, span.align_A.pos, span.align_A.aend, span.align_B.pos, span.align_B.aend,
               span.read_part.encode("latin-1"), span.strand == '-')
    try:
        hits = ref_fb(rs, fasta, ROptions(opt.asize, opt.margin, opt.maxdist, opt.noncanonical, opt.strandpref,
                                          opt.allhits))
    except KeyError:
        return KeyError
    except AttributeError:                   # ReferenceShapeError: windows outside get_data's range
        return "shape"
    if not opt.allhits:
        hits = hits[:1]
    return [(h.start, h.end, h.strand, h.gtag, h.dist, h.ov, h.n_hits) for h in hits]


def _got(r):
    if isinstance(r, fc2.BreakpointError):
        return "shape"
    if isinstance(r, BaseException):
        return type(r)
    return [(s.start, s.end, s.strand, s.gtag, s.dist, s.ov, s.n_hits) for s in r]


def _key_genome(tmp_path):
    """A locus whose planted GT..AG site carries an IUPAC byte in the donor dinucleotide: the
    qualifying breakpoint's gtag is outside ACGTN, so the reference raises KeyError (:927)."""
    rng = np.random.default_rng(5)
    g = list(rng.choice(list("ACGT"), 3000))
    g[1000:1002] = list("RT")           # donor dinucleotide with an IUPAC byte
    g[2000:2002] = list("AG")
    seq = "".join(g)
    path = str(tmp_path / "key.fa")
    with open(path, "w") as f:
        f.write(">keylocus\n")
        for i in range(0, len(seq), 50):
            f.write(seq[i:i + 50] + "\n")
    return path, seq


OPTS = [dict(), dict(maxdist=0), dict(allhits=True, noncanonical=True), dict(strandpref=True, maxdist=3),
        dict(asize=20, margin=5, allhits=True)]


@pytest.mark.parametrize("oi", range(len(OPTS)))
def test_integration_snippets_vs_oracle(oi, tmp_path):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    opt = fc2.Options(**OPTS[oi])
    path = os.path.join(GOLDEN, "CDR1as_locus.fa")
    kpath, kseq = _key_genome(tmp_path)
    # one FASTA holding the CDR1as locus and the KeyError locus
    both = str(tmp_path / "both.fa")
    with open(both, "w") as f:
        f.write(open(path).read().rstrip("\n") + "\n" + open(kpath).read())
    names = ["CDR1as_locus", "keylocus"]
    gen = load_genome(both)
    small = make_spans({"CDR1as_locus": gen["CDR1as_locus"]}, 3000, seed=31 + oi, asize=opt.asize, L=(40, 160),
                       p_readN=0.05)
    # the KeyError span: linear junction G[900:1000] + G[2000:2060] read forward, breakpoint at 1000
    from synth_small import SmallSpan
    e = opt.asize - opt.margin
    rp = kseq[1000 - 40:1000] + kseq[2002:2002 + 40]
    key_span = SmallSpan("keylocus", 1, 1000 - 40, 1000 - 40 + 30, 2002 + 10, 2002 + 40, rp.encode(), False)
    missing = SmallSpan("chrMissing", 9, 100, 160, 300, 360, b"ACGT" * 20, False)
    small[100:100] = [key_span]
    small[7:7] = [missing]

    fasta = RefIndexedFasta(both)
    one, two = _blocks()

    # §1: one span per call
    ns, calls, _ = _env(both, opt, names + ["chrMissing"])
    exec(compile(one, "INTEGRATION.md#1", "exec"), ns)
    spans = _spans_from_small(ns["JunctionSpan"], small, names, ["chrMissing"])
    n_err = 0
    for k, s in enumerate(spans[:400] + [spans[7], spans[101]]):
        s.chrom = names[s.align_A.tid] if s.align_A.tid < 2 else "chrMissing"
        exp = _expected(s, both, opt, fasta)
        try:
            got = _got(s.find_breakpoints())
        except KeyError:
            got = KeyError
        except fc2.BreakpointError:
            got = "shape"
        n_err += got is KeyError
        assert got == exp, (k, got, exp)
    assert n_err >= 2 or opt.maxdist == 0 and n_err >= 1

    # §2: the batched flush; record_hits raises at the first failing span, after the earlier ones
    ns, calls, written = _env(both, opt, names + ["chrMissing"])
    exec(compile(one, "INTEGRATION.md#1", "exec"), ns)
    exec(compile(two, "INTEGRATION.md#2", "exec"), ns)
    spans = _spans_from_small(ns["JunctionSpan"], small, names, ["chrMissing"])
    pending = [("frag%d" % i, [s] if s.is_backsplice else [], [] if s.is_backsplice else [s], [], [],
                types.SimpleNamespace(name="m1"), None) for i, s in enumerate(spans)]
    first_bad = None
    for i, s in enumerate(spans):
        s.chrom = names[s.align_A.tid] if s.align_A.tid < 2 else "chrMissing"
        if s.is_uniq and _expected(s, both, opt, fasta) is KeyError:
            first_bad = i
            break
    assert first_bad is not None
    with pytest.raises(KeyError):
        ns["flush"](pending)
    # every span before the failing one was evaluated, in order, with the oracle's result
    evaluated = [s for s in spans[:first_bad] if s.is_uniq]
    assert [c[0] for c in calls] == evaluated
    for s, r in calls:
        assert _got(r) == _expected(s, both, opt, fasta)
    # spans after the failing one, one flush per fragment: the rest of the chunk matches too
    for i in range(first_bad + 1, min(len(spans), first_bad + 600)):
        calls.clear()
        try:
            ns["flush"]([pending[i]])
        except KeyError:
            assert _expected(spans[i], both, opt, fasta) is KeyError
            continue
        except fc2.BreakpointError:
            assert _expected(spans[i], both, opt, fasta) == "shape"
            continue
        for s, r in calls:
            assert _got(r) == _expected(s, both, opt, fasta), i
