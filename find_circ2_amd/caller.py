"""Host side of the caller around the GPU hot path (find_circ.py 1.99 semantics).

SURVEY.md §8(f) rows 1, 3 and 4: alignment grouping and anchor-pair formation
(find_circ.py:976-1140, 1450-1527), per-fragment junction logic
(``record_hits``, :1276-1439), junction aggregation and the output tables with
Python-2 formatting (``Hit``/``SpliceSiteStorage``/``MultiEventRecorder``,
:486-763; ``write_read`` :1442-1447), and the ``--test`` validator (:1148-1273).

What differs from the reference, by design: the breakpoint search is evaluated
for a whole chunk of fragments in one GPU launch before the chunk's
``record_hits`` calls run (it is a pure function of the span), and any error
the reference would raise inside ``find_breakpoints`` is re-raised at the same
call.  Rows of the BED tables are written in first-appearance order (the
reference iterates a Python 2 dict, an order its own ``cmp_bed.py`` ignores);
comma-joined sets in ``multi_events.tsv`` / ``--test`` output are sorted.
"""
from __future__ import annotations

import gzip
import logging
import sys
import time
from collections import defaultdict
from typing import Dict, List, Optional, Sequence

from .hotpath import Splice, _py2_min, uniq_ok

_COMP = {'a': 't', 't': 'a', 'c': 'g', 'g': 'c', 'k': 'm', 'm': 'k', 'r': 'y', 'y': 'r', 's': 's', 'w': 'w',
         'b': 'v', 'v': 'b', 'h': 'd', 'd': 'h', 'n': 'n', 'A': 'T', 'T': 'A', 'C': 'G', 'G': 'C', 'K': 'M',
         'M': 'K', 'R': 'Y', 'Y': 'R', 'S': 'S', 'W': 'W', 'B': 'V', 'V': 'B', 'H': 'D', 'D': 'H', 'N': 'N'}


def rev_comp(seq: str) -> str:
    """find_circ.py:54-58: complement() walks the sequence forward, so the KeyError names the first
    byte outside the IUPAC table."""
    return "".join([_COMP[c] for c in seq])[::-1]


def py2_str(v) -> str:
    """``str(v)`` as Python 2 prints it: floats via '%.12g' (+ '.0'), bools as True/False."""
    if isinstance(v, bool):
        return "True" if v else "False"
    if isinstance(v, float):
        if v != v:
            return "nan"
        if v in (float("inf"), float("-inf")):
            return "inf" if v > 0 else "-inf"
        r = "%.12g" % v
        if not any(c in r for c in ".en"):
            r += ".0"
        return r
    return str(v)


# ---------------------------------------------------------------------------
# options (find_circ.py:383-413)
# ---------------------------------------------------------------------------
class CallerOptions:
    def __init__(self, **kw):
        self.name = "unknown"
        self.min_uniq_qual = 2
        self.asize = 15
        self.margin = 2
        self.maxdist = 2
        self.short_threshold = 100
        self.huge_threshold = 100000
        self.noncanonical = False
        self.allhits = False
        self.stranded = False
        self.strandpref = False
        self.halfunique = False
        self.report_nobridges = False
        self.throughput = False
        self.chunksize = 100000
        self.noop = False
        self.test = False
        self.nolinear = False
        self.multi_events = True
        self.debug = False
        for k, v in kw.items():
            if not hasattr(self, k):
                raise TypeError("unknown option %s" % k)
            setattr(self, k, v)


# ---------------------------------------------------------------------------
# alignment grouping (find_circ.py:976-1140, 1450-1486)
# ---------------------------------------------------------------------------
class MateSegments:
    """All alignments bwa-mem reported for one mate (primary + supplementary)."""

    def __init__(self, primary, counters):
        counters['total_mates'] += 1
        self.primary = primary
        self.full_seq = primary.seq
        self.proper_segs = [primary]
        self.other_chrom_segs = []
        self.other_strand_segs = []

    def belongs(self, align) -> bool:          # is_segment (:1025-1030)
        return align.is_read1 == self.primary.is_read1 and align.qname == self.primary.qname

    def is_other_mate(self, align) -> bool:    # :1032-1037
        return align.is_read1 != self.primary.is_read1 and align.qname == self.primary.qname

    def add(self, align):                      # add_segment (:1039-1056)
        if align.tid != self.primary.tid:
            self.other_chrom_segs.append(align)
        elif align.is_reverse != self.primary.is_reverse:
            self.other_strand_segs.append(align)
        else:
            self.proper_segs.append(align)

    def spans(self, opts: CallerOptions, counters, chrom_of):
        """Adjacent segment pairs in query order (adjacent_segment_pairs, :1058-1140)."""
        if len(self.proper_segs) < 2:
            return []
        weight = 1. / (len(self.proper_segs) - 1.)
        starts = [_aligned_start(s) for s in self.proper_segs]
        ends = [st + len(s.query) for st, s in zip(starts, self.proper_segs)]
        order = sorted(range(len(self.proper_segs)), key=lambda k: starts[k])   # stable, like sorted()
        out = []
        for a, b in zip(order, order[1:]):
            if ends[a] - starts[a] < opts.asize or ends[b] - starts[b] < opts.asize:
                counters['seg_too_short_skip'] += 1
                continue
            sa, sb = self.proper_segs[a], self.proper_segs[b]
            out.append(Span(sa, sb, self.primary, min(starts[a], starts[b]), max(ends[a], ends[b]), weight,
                            chrom_of(sa)))
        return out


def _aligned_start(seg) -> int:
    """Leading soft/hard clips before the first M (aligned_start_from_cigar, :1086-1097)."""
    s = 0
    for op, n in seg.cigar:
        if op in (4, 5):
            s += n
        elif op == 0:
            break
    return s


def group_alignments(records, counters):
    """(line_num, other_mate, current_mate) per read (collected_bwa_mem_segments, :1450-1486)."""
    it = enumerate(records)
    try:
        _, first = next(it)
    except StopIteration:          # a Python 2 generator ends silently here
        return
    current = MateSegments(first, counters)
    other = None
    line_num = None
    for line_num, align in it:
        if align.is_unmapped:
            counters['unmapped_reads'] += 1
        elif current.belongs(align):
            current.add(align)
        elif current.is_other_mate(align):
            other, current = current, MateSegments(align, counters)
        else:
            yield line_num, other, current
            other = None
            current = MateSegments(align, counters)
    if line_num is None:
        # the reference raises UnboundLocalError on single-record input (:1486)
        raise UnboundLocalError("local variable 'line_num' referenced before assignment")
    yield line_num, other, current


class Span:
    """JunctionSpan (find_circ.py:821-852) plus the result of its GPU evaluation."""

    __slots__ = ("primary", "align_A", "align_B", "q_start", "q_end", "weight", "uniq_A", "uniq_B", "uniq",
                 "strand", "dist", "read_part", "chrom", "result")

    def __init__(self, align_A, align_B, primary, q_start, q_end, weight, chrom):
        self.primary = primary
        self.align_A = align_A
        self.align_B = align_B
        self.q_start = q_start
        self.q_end = q_end
        self.weight = weight
        self.uniq_A = _uniqness(align_A)
        self.uniq_B = _uniqness(align_B)
        self.uniq = _py2_min(self.uniq_A, self.uniq_B)
        self.strand = '-' if primary.is_reverse else '+'
        self.dist = align_B.pos - align_A.aend
        self.read_part = primary.seq[q_start:q_end]
        self.chrom = chrom
        self.result = None

    @property
    def is_backsplice(self):
        return self.dist < 0

    def find_breakpoints(self):
        """The precomputed GPU result; raises what the reference raises (:927, :193)."""
        if isinstance(self.result, BaseException):
            raise self.result
        if self.result is None:
            raise RuntimeError("span was not evaluated")
        return self.result


def _uniqness(align):                        # :809-819 (an int, a float, or a str / array AS as it is)
    u = align.get_tag('AS')
    if align.has_tag('XS'):
        u -= align.get_tag('XS')
    return u


# ---------------------------------------------------------------------------
# aggregation (find_circ.py:486-730)
# ---------------------------------------------------------------------------
class Hit:
    """Evidence for one junction coordinate (find_circ.py:486-654)."""

    def __init__(self, name, splice, opts: CallerOptions):
        self.opts = opts
        self.name = name
        self.reads = []
        self.readnames = []
        self.uniq = set()
        self.mapquals_A = []
        self.mapquals_B = []
        self.n_weighted = 0.
        self.n_spanned = 0
        self.n_uniq_bridges = 0.
        self.edits = []
        self.overlaps = []
        self.n_hits = []
        self.signal = "NNNN"
        self.strand_plus = 0
        self.strand_minus = 0
        self.strandmatch = 'NA'
        self.flags = defaultdict(int)
        self.read_flags = defaultdict(set)
        self.tissues = defaultdict(float)
        self.coord = splice.coord
        self.add(splice)

    def add_flag(self, flag, frag_name):
        self.flags[flag] += 1
        self.read_flags[frag_name].add(flag)

    def add(self, splice):
        self.signal = splice.gtag
        self.strandmatch = 'N/A'
        if self.opts.stranded:   # Splice has no strandmatch attribute (:532-533)
            raise AttributeError("'Splice' object has no attribute 'strandmatch'")
        self.edits.append(splice.dist)
        self.overlaps.append(splice.ov)
        self.n_hits.append(splice.n_hits)
        span = splice.junc_span
        if not span:
            return
        self.n_spanned += 1
        self.n_weighted += span.weight
        A, B = span.align_A, span.align_B
        if span.is_backsplice:
            A, B = B, A
        ta, tb = dict(A.tags), dict(B.tags)
        qA = ta.get('AS') - ta.get('XS', 0)
        qB = tb.get('AS') - tb.get('XS', 0)
        if qA and qB:
            self.n_uniq_bridges += span.weight
        self.mapquals_A.append(qA)
        self.mapquals_B.append(qB)
        self.readnames.append(span.primary.qname)
        read = span.primary.seq
        if A.is_reverse:
            self.strand_minus += span.weight
            self.reads.append(rev_comp(read))
        else:
            self.strand_plus += span.weight
            self.reads.append(read)
        self.tissues[self.opts.name] += span.weight
        self.uniq.add((read, self.opts.name))
        self.uniq.add((rev_comp(read), self.opts.name))

    @property
    def n_frags(self):
        return len(set(self.readnames))

    @property
    def n_uniq(self):
        return len(self.uniq) // 2

    def best_anchor_quals(self):
        return max(self.mapquals_A), max(self.mapquals_B)

    def categories(self) -> List[str]:           # :601-654
        o = self.opts
        cats = []
        if self.signal != "GTAG":
            cats.append("NON_CANONICAL")
        qa, qb = self.best_anchor_quals()
        if qa == 0 or qb == 0:
            cats.append("WARN_NON_UNIQUE_ANCHOR")
        if self.n_uniq_bridges == 0:
            cats.append("WARN_NO_UNIQ_BRIDGES")
        if min(self.n_hits) > 1:
            cats.append("WARN_AMBIGUOUS_BP")
        mov, med = min(self.overlaps), min(self.edits)
        if mov == 0 and med == 0:
            pass
        elif mov < 2 and med < 2:
            cats.append("WARN_EXT_1MM")
        elif mov >= 2 or med >= 2:
            cats.append("WARN_EXT_2MM+")
        _, start, end, _ = self.coord
        if end - start < o.short_threshold:
            cats.append("SHORT")
        elif end - start > o.huge_threshold:
            cats.append("HUGE")
        unbroken = unwarned = 0
        total = 0.
        for frag, fl in self.read_flags.items():
            total += 1.
            if 'BROKEN_SEGMENTS' not in fl:
                unbroken += 1
            for w in fl:
                if not w.startswith('WARN'):
                    unwarned += 1
        if total:
            if not unbroken:
                cats.append('WARN_ALWAYS_BROKEN')
            if not unwarned:
                cats.append('WARN_ALWAYS_WARN')
        return cats


BED_HEADER = "#" + "\t".join(['chrom', 'start', 'end', 'name', 'n_frags', 'strand', 'n_weight', 'n_spanned', 'n_uniq',
                              'uniq_bridges', 'best_qual_left', 'best_qual_right', 'tissues', 'tiss_counts', 'edits',
                              'anchor_overlap', 'breakpoints', 'signal', 'strandmatch', 'category', 'flags',
                              'flag_counts']) + "\n"


class SpliceSiteStorage:
    """Junctions of one kind ('circ' / 'lin'), named by first appearance (:657-730)."""

    def __init__(self, prefix: str, opts: CallerOptions, counters, known: str = ""):
        self.prefix = prefix
        self.opts = opts
        self.counters = counters
        self.sites: Dict[tuple, Hit] = {}
        self.novel_count = 0
        if known:
            self._load_known(known)

    def _load_known(self, path):
        n = 0
        with open(path, encoding="latin-1") as f:
            for line in f:
                if line.startswith('#'):
                    continue
                chrom, start, end, name, score, sense = line.rstrip().split('\t')[:6]
                sp = Splice(None, chrom, int(start), int(end), sense, 10, 10, 'NNNN')
                self.sites[sp.coord] = Hit(name, sp, self.opts)
                n += 1
        logging.getLogger('find_circ').info("loaded {0} known splice sites from '{1}'".format(n, path))

    def add(self, splice) -> Hit:
        coord = splice.coord
        hit = self.sites.get(coord)
        if hit is None:
            self.novel_count += 1
            hit = Hit("{0}_{1}_{2:06d}".format(self.opts.name, self.prefix, self.novel_count), splice, self.opts)
            self.sites[coord] = hit
        else:
            hit.add(splice)
        return hit

    def __getitem__(self, coord):
        return self.sites[coord]

    def rows(self) -> List[str]:
        o, N = self.opts, self.counters
        out = []
        for (chrom, start, end, sense), hit in self.sites.items():
            if not hit.reads:
                continue
            qa, qb = hit.best_anchor_quals()
            if o.halfunique:
                if qa < o.min_uniq_qual and qb < o.min_uniq_qual:
                    N['anchor_not_uniq'] += 1
                    continue
            elif qa < o.min_uniq_qual or qb < o.min_uniq_qual:
                N['anchor_not_uniq'] += 1
                continue
            if hit.n_uniq_bridges == 0 and not o.report_nobridges:
                N['no_uniq_bridges'] += 1
                continue
            tissues = sorted(hit.tissues)
            tiss_counts = [py2_str(hit.tissues[k]) for k in tissues]
            if hit.flags:
                flags = sorted(hit.flags)
                flag_counts = [hit.flags[f] for f in flags]
            else:
                flags, flag_counts = ["N/A"], [0]
            cols = [chrom, start, end, hit.name, hit.n_frags, sense, hit.n_weighted, hit.n_spanned, hit.n_uniq,
                    hit.n_uniq_bridges, qa, qb, ",".join(tissues), ",".join(tiss_counts), min(hit.edits),
                    min(hit.overlaps), min(hit.n_hits), hit.signal, hit.strandmatch, ",".join(sorted(hit.categories())),
                    ",".join(flags), ",".join(str(c) for c in flag_counts)]
            out.append("\t".join(py2_str(c) for c in cols) + "\n")
        return out

    def store(self, fh):
        fh.write(BED_HEADER)
        for r in self.rows():
            fh.write(r)


MULTI_HEADER = "#" + "\t".join(['chrom', 'start', 'end', 'name', 'score', 'strand', 'fragment_name', 'lin_cons',
                                'lin_incons', 'unspliced_cons', 'unspliced_incons']) + "\n"


def multi_event_row(frag_name, circ_hit, lin_cons, lin_incons, un_cons, un_incons) -> str:   # :733-763
    score = len(lin_cons) - 10 * len(lin_incons) + len(un_cons) - 10 * len(un_incons)
    chrom, start, end, sense = circ_hit.coord
    cols = [chrom, str(start), str(end), "ME:" + circ_hit.name, str(score), sense, frag_name]
    cols.append(",".join("%d-%d" % (s, e) for _, s, e, _ in sorted(lin_cons)) if lin_cons else "NO_LIN_CONS")
    cols.append(",".join("[%s:%d-%d]" % (c, s, e) for c, s, e, _ in sorted(lin_incons)) if lin_incons
                else "NO_LIN_INCONS")
    cols.append(",".join("%d-%d" % (s, e) for _, s, e, _ in sorted(un_cons)) if un_cons else "NO_UNSPLICED_CONS")
    cols.append(",".join("[%s:%d-%d]" % (c, s, e) for c, s, e, _ in sorted(un_incons)) if un_incons
                else "NO_UNSPLICED_INCONS")
    return "\t".join(cols) + "\n"


# ---------------------------------------------------------------------------
# --test validator (find_circ.py:1148-1273)
# ---------------------------------------------------------------------------
def parse_truth(align_str: str, stranded: bool):
    lin, circ, unspliced = set(), set(), set()
    for mate_str in align_str.split('|'):
        spliced = False
        chrom = strand = None
        start = end = None
        for code in mate_str.split(';'):
            parts = code.split(':')
            op = parts[0]
            if op == 'O':
                chrom, start, strand = parts[1], int(parts[2]), parts[3]
                end = start
            elif op == 'M':
                end += int(parts[1])
            elif op == 'LS':
                left, right = int(parts[1]) + start, int(parts[2]) + start
                lin.add((chrom, left, right, strand))
                spliced = True
                end = right
            elif op == 'CS':
                left, right = int(parts[1]) + start, int(parts[2]) + start
                circ.add((chrom, left, right, strand))
                spliced = True
                end = left
        if not spliced and chrom:
            unspliced.add((chrom, start, end, strand if stranded else "*"))
    return lin, circ, unspliced


def _flag_set(kind, ref, got):
    flags = set()
    if ref - got:
        flags.add('MISSED_%s:%s' % (kind, ','.join(str(j) for j in sorted(ref - got))))
    if got - ref:
        flags.add('SPURIOUS_%s:%s' % (kind, ','.join(str(j) for j in sorted(got - ref))))
    return flags


def test_row(frag_name, lin_coords, circ_coords, unspliced_coords, broken_coords, stranded) -> str:
    if '___' not in frag_name:
        return "\t".join([frag_name, "N/A", "N/A", "N/A", "N/A"]) + "\n"
    lin_ref, circ_ref, un_ref = parse_truth(frag_name.split("___")[-1], stranded)
    cols = [frag_name]
    for kind, ok, ref, got in (("LINEAR_JUNCTIONS", "LIN_OK", lin_ref, lin_coords),
                               ("CIRCULAR_JUNCTIONS", "CIRC_OK", circ_ref, circ_coords),
                               ("UNSPLICED", "UNSPLICED_OK", un_ref, set(unspliced_coords))):
        fl = _flag_set(kind, ref, got)
        cols.append(";".join(sorted(fl)) if fl else (ok if ref else "N/A"))
    cols.append('BROKEN_SEGMENTS:%s' % ";".join(str(b) for b in sorted(broken_coords)) if broken_coords else "N/A")
    return "\t".join(cols) + "\n"


# ---------------------------------------------------------------------------
# the per-fragment logic (find_circ.py:1276-1439) and the driver (:1490-1597)
# ---------------------------------------------------------------------------
class Fragment:
    __slots__ = ("name", "mate1", "mate2", "circ", "lin", "unspliced", "broken")

    def __init__(self, name, mate1, mate2):
        self.name, self.mate1, self.mate2 = name, mate1, mate2
        self.circ, self.lin, self.unspliced, self.broken = [], [], [], []


class Caller:
    """Runs find_circ's read loop with the breakpoint search batched on the GPU."""

    def __init__(self, opts: CallerOptions, evaluate, chrom_of, outputs, known_circ="", known_lin=""):
        self.o = opts
        self.evaluate = evaluate          # callable(list[Span]) -> fills span.result
        self.chrom_of = chrom_of          # fast_chrom_lookup (:471-477)
        self.out = outputs                # dict: circs, lins, reads, multi, test (file objects or None)
        self.N = defaultdict(float)
        self.circ_splices = SpliceSiteStorage("circ", opts, self.N, known_circ)
        self.linear_splices = SpliceSiteStorage("lin", opts, self.N, known_lin)
        if self.out.get("multi") is not None:
            self.out["multi"].write(MULTI_HEADER)
        self.n_reads = 0
        self.n_spans_evaluated = 0
        self.gpu_seconds = 0.0

    # -- per mate (process_mate, :1492-1527)
    def _process_mate(self, mate, frag: Fragment):
        o = self.o
        if len(mate.proper_segs) < 2:
            self.N['unspliced_mates'] += 1
            frag.unspliced.append(mate.primary)
            return
        L = len(mate.full_seq)
        min_s, max_e = L, 0
        for sp in mate.spans(o, self.N, self.chrom_of):
            (frag.circ if sp.is_backsplice else frag.lin).append(sp)
            min_s = min(min_s, sp.q_start)
            max_e = max(max_e, sp.q_end)
        if max_e < L - o.asize or min_s > o.asize:
            frag.broken.extend(mate.other_chrom_segs)
            frag.broken.extend(mate.other_strand_segs)

    def record_hits(self, frag: Fragment):
        o, N = self.o, self.N
        warns, junctions = set(), set()
        circ_coords = set()
        circ = None
        for span in frag.circ:
            if not uniq_ok(span.uniq, o.min_uniq_qual):
                N['circ_junc_not_unique'] += 1
                continue
            splices = span.find_breakpoints()
            if not splices:
                N['circ_no_bp'] += 1
                warns.add('WARN_UNRESOLVED_EXTRA_BACKSPLICE')
                continue
            N['circ_spliced'] += 1
            for splice in (splices if o.allhits else splices[:1]):
                circ = self.circ_splices.add(splice)
                circ_coords.add(circ.coord)
                junctions.add(circ)
        if len(circ_coords) > 1:
            for coord in circ_coords:
                warns.add('WARN_MULTI_BACKSPLICE')
                h = self.circ_splices[coord]
                h.add_flag('WARN_MULTI_BACKSPLICE', frag.name)
                junctions.add(h)
            return junctions, warns
        if not circ_coords and o.nolinear:
            return junctions, warns
        if circ_coords:
            _, circ_start, circ_end, _ = circ.coord
            circ_span = frag.circ[0]
            if len(frag.circ) > 1:
                warns.add('SUPPORT_CLOSURE')
        lin_cons, lin_incons, lin_coords = set(), set(), set()
        for span in frag.lin:
            if not uniq_ok(span.uniq, o.min_uniq_qual):
                N['lin_junc_not_unique'] += 1
                continue
            splices = span.find_breakpoints()
            if not splices:
                N['lin_no_bp'] += 1
                warns.add('WARN_UNRESOLVED_LINSPLICE')
                continue
            N['lin_spliced'] += 1
            for splice in (splices if o.allhits else splices[:1]):
                lin = self.linear_splices.add(splice)
                junctions.add(lin)
                lin_coords.add(lin.coord)
                if circ_coords:
                    if splice.start <= circ_start or splice.end >= circ_end:
                        warns.add('WARN_OUTSIDE_SPLICE_JUNCTION')
                        lin_incons.add(splice.coord)
                    else:
                        lin_cons.add(splice.coord)
                        warns.add('SUPPORT_INSIDE_SPLICE_JUNCTION')
        if o.test and self.out.get("test") is not None:
            def coords(a):
                s = ('-' if a.is_reverse else '+') if o.stranded else '*'
                return (self.chrom_of(a), a.pos, a.aend, s)
            self.out["test"].write(test_row(frag.name, lin_coords, circ_coords,
                                            {coords(m) for m in frag.unspliced}, {coords(b) for b in frag.broken},
                                            o.stranded))
        if circ_coords:
            un_cons, un_incons = set(), set()
            for a in frag.unspliced:
                coord = (self.chrom_of(a), a.pos, a.aend, '*')
                if circ_span.primary.tid != a.tid:
                    warns.add('WARN_OTHER_CHROM_MATE')
                    un_incons.add(coord)
                elif a.pos + o.asize <= circ_start or a.aend - o.asize >= circ_end:
                    warns.add('WARN_OUTSIDE_MATE')
                    un_incons.add(coord)
                else:
                    warns.add('SUPPORT_INSIDE_MATE')
                    un_cons.add(coord)
            if frag.broken:
                warns.add('BROKEN_SEGMENTS')
            if (un_cons or un_incons or lin_cons or lin_incons) and o.multi_events and self.out.get("multi"):
                self.out["multi"].write(multi_event_row(frag.name, circ, lin_cons, lin_incons, un_cons, un_incons))
            for w in warns:
                circ.add_flag(w, frag.name)
        return junctions, warns

    def _write_read(self, mate, junctions, flags):      # :1442-1447
        fh = self.out.get("reads")
        if fh is None:
            return
        name = "%s %s %s" % (mate.primary.qname, ",".join(sorted(j.name for j in junctions)),
                             ",".join(sorted(flags)))
        fh.write("@%s\n%s\n+%s\n%s\n" % (name, mate.primary.seq, name, mate.primary.qual))

    def _flush(self, pending: List[Fragment]):
        # the chunk leaves `pending` before anything runs: if evaluate or record_hits raises, the
        # fragments recorded so far stay recorded exactly once and nothing after the failing one
        # is recorded (the reference stops at the fragment that raises, find_circ.py:1578-1583)
        frags = list(pending)
        pending.clear()
        spans = [s for f in frags for s in f.circ + f.lin if uniq_ok(s.uniq, self.o.min_uniq_qual)]
        if spans:
            t0 = time.perf_counter()
            self.evaluate(spans)
            self.gpu_seconds += time.perf_counter() - t0
            self.n_spans_evaluated += len(spans)
        for f in frags:
            junctions, flags = self.record_hits(f)
            if f.mate1 and junctions:
                self._write_read(f.mate1, junctions, flags)
            if f.mate2 and junctions:
                self._write_read(f.mate2, junctions, flags)

    def run(self, records, stderr=sys.stderr):
        o = self.o
        t0 = time.time()
        pending: List[Fragment] = []
        try:
            self._run_loop(records, stderr, pending, t0)
        except BaseException:
            # the reference records every fragment before it reads the next: those of this chunk
            # are recorded before the failure propagates (a failure of their own comes first)
            self._flush(pending)
            raise
        self._flush(pending)
        if o.throughput:
            stderr.write('\n')
        return time.time() - t0

    def _run_loop(self, records, stderr, pending, t0):
        o = self.o
        t_last = t0
        for line_num, mate1, mate2 in group_alignments(records, self.N):
            self.n_reads += 1
            if o.throughput and not (self.n_reads % o.chunksize):
                t1 = time.time()
                stderr.write("\rprocessed {0:.1f}M (paired-end) reads in {1:.1f} minutes ({2:.2f}k reads/second)"
                             "       \r".format(self.n_reads / 1e6, (t1 - t0) / 60.,
                                                float(o.chunksize) / float(t1 - t_last) / 1000.))
                t_last = t1
            if o.noop:
                continue
            frag = Fragment(mate2.primary.qname, mate1, mate2)
            if mate1:
                self._process_mate(mate1, frag)
            if mate2:
                self._process_mate(mate2, frag)
            if not frag.circ and o.nolinear:
                continue
            if frag.circ or frag.lin:
                pending.append(frag)
                if len(pending) >= o.chunksize:
                    self._flush(pending)

    def run_native(self, ingest, stderr=sys.stderr):
        """Same loop with the native ingest (include/fc2_ingest.h): only fragments carrying
        anchor pairs come back as records; the grouping counters of the others come from C++."""
        o = self.o
        t0 = time.time()
        t_last = t0
        scratch = defaultdict(float)      # grouping counters of handed-back fragments are counted natively
        pending: List[Fragment] = []
        try:
            self._run_native_loop(ingest, stderr, pending, scratch, t0)
        except BaseException:
            self._flush(pending)        # as in run(): the fragments before the failure are recorded
            raise
        self._flush(pending)
        c = ingest.counts
        return self._finish_native(c, stderr, t0)

    def _run_native_loop(self, ingest, stderr, pending, scratch, t0):
        o = self.o
        t_last = t0
        last_reads = 0
        while not ingest.eof:
            for recs in ingest.next_chunk(o.asize, o.nolinear, o.noop, o.chunksize):
                for _, mate1, mate2 in group_alignments(recs, scratch):
                    frag = Fragment(mate2.primary.qname, mate1, mate2)
                    if mate1:
                        self._process_mate(mate1, frag)
                    if mate2:
                        self._process_mate(mate2, frag)
                    if not frag.circ and o.nolinear:
                        continue
                    if frag.circ or frag.lin:
                        pending.append(frag)
                if len(pending) >= o.chunksize:
                    self._flush(pending)
            self.n_reads = int(ingest.counts.n_reads)
            if o.throughput and self.n_reads // o.chunksize > last_reads // o.chunksize:
                t1 = time.time()
                stderr.write("\rprocessed {0:.1f}M (paired-end) reads in {1:.1f} minutes ({2:.2f}k reads/second)"
                             "       \r".format(self.n_reads / 1e6, (t1 - t0) / 60.,
                                                (self.n_reads - last_reads) / max(t1 - t_last, 1e-9) / 1000.))
                t_last, last_reads = t1, self.n_reads

    def _finish_native(self, c, stderr, t0):
        for key, v in (("total_mates", c.total_mates), ("unmapped_reads", c.unmapped_reads),
                       ("unspliced_mates", c.unspliced_mates), ("seg_too_short_skip", c.seg_too_short_skip)):
            if v:
                self.N[key] += float(v)
        self.n_reads = int(c.n_reads)
        if self.o.throughput:
            stderr.write('\n')
        return time.time() - t0
