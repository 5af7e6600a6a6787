"""CPU oracle for the breakpoint-search hot path -- TEST INFRASTRUCTURE ONLY.

This is a deliberately literal, pure-Python restatement of the reference's
per-anchor-pair breakpoint search and of the genome window fetch that feeds it.
It exists to CHECK the HIP product path; nothing in ``find_circ2_amd/`` may
import it.  Only ``tests/``, ``__graft_entry__.smoke()`` and the ``cpu_baseline``
leg of ``bench.py`` use it.

Reference (read-only, Python 2.7, /root/reference):
  * ``indexed_fasta.index``       find_circ.py:120-155
  * ``indexed_fasta.store_index`` find_circ.py:157-179 (format line 167)
  * ``indexed_fasta.load_index``  find_circ.py:182-187
  * ``indexed_fasta.get_data``    find_circ.py:189-215
  * ``GenomeAccessor`` dummy mode find_circ.py:338-345, 370-371
  * ``fast_4mer_RC``              find_circ.py:21-74
  * ``Splice.score / coord``      find_circ.py:791-806
  * ``JunctionSpan`` fields       find_circ.py:821-852
  * ``find_breakpoints``          find_circ.py:854-974

Python-2 semantics that matter and how they are kept:
  * integer ``/`` on ints is floor division            -> ``//`` (find_circ.py:204-205)
  * ``str`` is a byte string; slicing / ``replace`` / ``upper`` act on bytes
                                                        -> ``bytes`` throughout
  * ``mmap[a:b]`` slices like a string (negative indices wrap)
                                                        -> slicing a ``bytes`` copy
  * ``(fromstring(a) != fromstring(b)).sum()`` on equal-length byte strings
                                                        -> count of differing bytes
    (unequal lengths: the reference's numpy comparison fails; we raise)
  * ``simple_match`` for ``maxdist == 0`` returns a bool  (find_circ.py:865-871)
  * ``sorted(..., reverse=True)`` is stable            (find_circ.py:966)

Parity status: pinned by the reference's own known answers
(tests/golden/cdr1as_reference.bed row 2 and the truth strings embedded in
tests/golden/test_reads.fa); see tests/test_oracle_known_answers.py.
"""
from __future__ import annotations

import os
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple

import numpy as np

# ---------------------------------------------------------------------------
# splice-signal table (find_circ.py:21-74)
# ---------------------------------------------------------------------------
_COMPLEMENT = {
    'a': 't', 't': 'a', 'c': 'g', 'g': 'c', 'k': 'm', 'm': 'k', 'r': 'y', 'y': 'r',
    's': 's', 'w': 'w', 'b': 'v', 'v': 'b', 'h': 'd', 'd': 'h', 'n': 'n',
    'A': 'T', 'T': 'A', 'C': 'G', 'G': 'C', 'K': 'M', 'M': 'K', 'R': 'Y', 'Y': 'R',
    'S': 'S', 'W': 'W', 'B': 'V', 'V': 'B', 'H': 'D', 'D': 'H', 'N': 'N',
}


def complement(s: str) -> str:
    return "".join(_COMPLEMENT[c] for c in s)


def rev_comp(s: str) -> str:
    return complement(s)[::-1]


def _kmers(k, alphabet):
    prefix = [""] if k == 1 else list(_kmers(k - 1, alphabet))
    for pre in prefix:
        for a in alphabet:
            yield pre + a


# find_circ.py:72-74 -- only 4-mers over ACGTN have an entry; any other byte
# in a qualifying gtag raises KeyError in the reference (find_circ.py:927).
FAST_4MER_RC = {m: rev_comp(m) for m in _kmers(4, ['A', 'C', 'G', 'T', 'N'])}


class ReferenceKeyError(KeyError):
    """The reference would raise KeyError here (fatal, find_circ.py:1578-1583)."""


class ReferenceShapeError(AttributeError):
    """The reference's numpy comparison would fail (window of wrong length)."""


# ---------------------------------------------------------------------------
# indexed FASTA (find_circ.py:103-215)
# ---------------------------------------------------------------------------
class RefIndexedFasta:
    """Byte-exact restatement of ``indexed_fasta`` (find_circ.py:103-215).

    ``data`` is the whole FASTA file as bytes (the reference mmaps it).
    The index maps chrom -> (ofs, ldata, skip, skipchar, size).
    """

    def __init__(self, fname: str, use_existing_index: bool = False, use_mmap: bool = False):
        self.fname = fname
        with open(fname, 'rb') as f:
            if use_mmap:                    # as the reference does (find_circ.py:104-118): slices copy out
                import mmap
                self.data = mmap.mmap(f.fileno(), 0, access=mmap.ACCESS_READ)
            else:
                self.data = f.read()
        self.chrom_stats: Dict[str, tuple] = {}
        ipath = fname + '.byo_index'
        if use_existing_index and os.access(ipath, os.R_OK):
            self.load_index(ipath)          # find_circ.py:110-112
        else:
            self.index()                    # find_circ.py:114

    # find_circ.py:120-155
    def index(self):
        ofs = 0
        chrom = b"undef"
        chrom_ofs = 0
        size = 0
        stats: Dict[bytes, list] = {}
        for line in _py2_file_lines(self.data):
            ofs += len(line)
            if line.startswith(b'>'):
                if size:
                    stats[chrom].append(size)
                chrom = line[1:].split()[0].strip()
                chrom_ofs = ofs
            else:
                if chrom not in stats:
                    size = 0
                    lline = len(line)
                    ldata = len(line.strip())
                    nl_char = lline - ldata
                    stats[chrom] = [chrom_ofs, ldata, nl_char, line[ldata:]]
                size += len(line.strip())
        if size:
            stats[chrom].append(size)
        self.chrom_stats = {k.decode('latin-1'): tuple(v) for k, v in stats.items()}

    # find_circ.py:157-179 (line format 167: "%s\t%d\t%d\t%d\t%r\t%d\n")
    def index_text(self) -> str:
        out = []
        for chrom in sorted(self.chrom_stats):
            ofs, ldata, skip, skipchar, size = self.chrom_stats[chrom]
            out.append("%s\t%d\t%d\t%d\t%s\t%d\n" % (chrom, ofs, ldata, skip, _py2_repr_bytes(skipchar), size))
        return "".join(out)

    # find_circ.py:182-187
    def load_index(self, ipath: str):
        self.chrom_stats = {}
        with open(ipath, 'r') as f:
            for line in f:
                chrom, ofs, ldata, skip, skipchar, size = line.rstrip().split('\t')
                sc = skipchar[1:-1].encode('latin-1').decode('unicode_escape').encode('latin-1')
                self.chrom_stats[chrom] = (int(ofs), int(ldata), int(skip), sc, int(size))

    # find_circ.py:189-215
    def get_data(self, chrom: str, start: int, end: int, sense: str = '+') -> bytes:
        ofs, ldata, skip, skip_char, size = self.chrom_stats[chrom]   # KeyError like 193
        pad_start = 0
        pad_end = 0
        if start < 0:
            pad_start = -start
            start = 0
        if end > size:
            pad_end = end - size
            end = size
        l_start = start // ldata
        l_end = end // ldata
        ofs_start = l_start * skip + start + ofs
        ofs_end = l_end * skip + end + ofs
        s = self.data[ofs_start:ofs_end]
        if skip_char:
            s = s.replace(skip_char, b"")
        if pad_start or pad_end:
            s = b"N" * pad_start + s + b"N" * pad_end
        if sense == '-':
            s = rev_comp(s.decode('latin-1')).encode('latin-1')
        return s


class RefGenomeTrack:
    """``genome = Track(options.genome, accessor=GenomeAccessor)`` (find_circ.py:435-436) as
    ``find_breakpoints`` calls it per window (``genome.get(chrom, start, end, '+')``, :900-902):
    ``Track.get`` -> ``Track.load`` (accessor cache keyed by chrom + sense, :274-297, :310-312) ->
    ``GenomeAccessor.get_data`` (:362-368) -> ``indexed_fasta.get_data`` (:189-215).  The CPU
    baseline times this chain; ``get_data`` is ``get`` under the name this module's
    ``find_breakpoints`` calls."""

    def __init__(self, fasta: "RefIndexedFasta"):
        self.fasta = fasta
        self.acc_cache: Dict[str, object] = {}
        self.auto_flush = False              # Track's default (:253)
        self.last_chrom = ""

    class _Accessor:                         # GenomeAccessor (:329-368)
        def __init__(self, data):
            self.data = data

        def get_data(self, chrom, start, end, sense):
            seq = self.data.get_data(chrom, start, end, "+")
            if sense == "-":
                seq = complement(seq.decode("latin-1")).encode("latin-1")
            return seq

    def load(self, chrom, sense):
        if self.auto_flush and chrom != self.last_chrom:
            self.acc_cache = {}
        self.last_chrom = chrom
        ID = chrom + sense
        if ID not in self.acc_cache:
            acc = RefGenomeTrack._Accessor(self.fasta)
            covered = [c + '+' for c in self.fasta.chrom_stats] + [c + '-' for c in self.fasta.chrom_stats]   # :348
            for ID in covered:               # the loop rebinds ID, as at :294-295: a chromosome missing
                self.acc_cache[ID] = acc     # from the index gets an accessor and fails in get_data (:193)
        return self.acc_cache[ID]

    def get(self, chrom, start, end, sense):
        acc = self.load(chrom, sense)
        return acc.get_data(chrom, start, end, sense)

    get_data = get


def _py2_file_lines(data: bytes):
    """Python 2 ``for line in file(...)``: split after every b'\\n' only."""
    i = 0
    n = len(data)
    while i < n:
        j = data.find(b'\n', i)
        if j < 0:
            yield data[i:]
            return
        yield data[i:j + 1]
        i = j + 1


def _py2_repr_bytes(b: bytes) -> str:
    """Python 2 ``repr(str)`` for the short newline strings a FASTA index holds."""
    body = []
    for c in b:
        ch = chr(c)
        if ch == '\n':
            body.append('\\n')
        elif ch == '\r':
            body.append('\\r')
        elif ch == '\t':
            body.append('\\t')
        elif ch == "'":
            body.append("\\'")
        elif ch == '\\':
            body.append('\\\\')
        elif 32 <= c < 127:
            body.append(ch)
        else:
            body.append('\\x%02x' % c)
    return "'" + "".join(body) + "'"


class DummyGenome:
    """``GenomeAccessor.get_dummy`` (find_circ.py:340-345, 370-371): all-N windows."""

    def get_data(self, chrom, start, end, sense='+'):
        return b"N" * int(end - start)


# ---------------------------------------------------------------------------
# hot path (find_circ.py:766-974)
# ---------------------------------------------------------------------------
@dataclass
class Options:
    """The ``options.*`` the hot path reads (find_circ.py:393-404)."""
    asize: int = 15
    margin: int = 2
    maxdist: int = 2
    noncanonical: bool = False
    strandpref: bool = False
    allhits: bool = False


@dataclass
class Span:
    """The ``JunctionSpan`` fields ``find_breakpoints`` reads (find_circ.py:821-852)."""
    chrom: str
    a_pos: int
    a_aend: int
    b_pos: int
    b_aend: int
    read_part: bytes
    primary_reverse: bool = False

    @property
    def strand(self) -> str:                 # find_circ.py:834-837
        return '-' if self.primary_reverse else '+'

    @property
    def is_backsplice(self) -> bool:         # find_circ.py:842, 851-852
        return (self.b_pos - self.a_aend) < 0


@dataclass
class Hit:
    """One ``Splice`` (find_circ.py:766-806) plus the breakpoint index x."""
    x: int
    chrom: str
    start: int
    end: int
    strand: str
    dist: object          # int, or bool when maxdist == 0 (find_circ.py:865-871)
    ov: int
    gtag: str
    score: int
    n_hits: int = 1

    @property
    def coord(self):                          # find_circ.py:801-806
        if self.start < self.end:
            return (self.chrom, self.start, self.end, self.strand)
        return (self.chrom, self.end, self.start, self.strand)


def _mismatches(a: bytes, b: bytes) -> int:
    """find_circ.py:861-863 -- numpy byte compare + sum, with numpy's broadcasting: equal lengths
    compare elementwise, a 1-byte operand is broadcast against the other (0 against 1 bytes is an
    empty comparison)."""
    if len(a) != len(b) and len(a) != 1 and len(b) != 1:
        # numpy 1.x (Python 2): `!=` of shapes it cannot broadcast returns the scalar True
        # (DeprecationWarning), and True.sum() raises AttributeError (find_circ.py:861-863)
        raise ReferenceShapeError("'bool' object has no attribute 'sum'")
    return int((np.frombuffer(a, dtype=np.int8) != np.frombuffer(b, dtype=np.int8)).sum())


def _simple_match(a: bytes, b: bytes) -> bool:
    """find_circ.py:865-866 -- used when maxdist == 0 (returns a bool)."""
    return a != b


def find_breakpoints(span: Span, genome, opt: Options) -> List[Hit]:
    """Literal restatement of ``JunctionSpan.find_breakpoints`` (find_circ.py:854-974).

    Keeps the reference's O(l^2) shape: for each breakpoint x it builds the
    spliced string and compares it byte-by-byte with the internal read part.
    """
    mismatches = _simple_match if opt.maxdist == 0 else _mismatches   # 868-870
    read = span.read_part
    L = len(read)
    margin = opt.margin
    maxdist = opt.maxdist
    is_backsplice = span.is_backsplice
    eff_a = opt.asize - opt.margin                                      # 882
    hits: List[Hit] = []
    internal = read[eff_a:-eff_a].upper()                               # 895
    chrom = span.chrom
    flank = L - 2 * eff_a + 2                                           # 900
    A_flank = genome.get_data(chrom, span.a_pos + eff_a, span.a_pos + eff_a + flank, '+').upper()   # 901
    B_flank = genome.get_data(chrom, span.b_aend - eff_a - flank, span.b_aend - eff_a, '+').upper() # 902
    l = L - 2 * eff_a                                                   # 904
    for x in range(l + 1):                                              # 906
        spliced = A_flank[:x] + B_flank[x + 2:]                         # 907
        dist = mismatches(spliced, internal)                            # 908
        if dist <= maxdist:                                             # 915
            ov = 0
            if margin:
                if x < margin:
                    ov = margin - x
                if l - x < margin:
                    ov = margin - (l - x)
            gt = A_flank[x:x + 2]
            ag = B_flank[x:x + 2]
            gtag = (gt + ag).decode('latin-1')
            try:
                rc_gtag = FAST_4MER_RC[gtag]                            # 927
            except KeyError:
                raise ReferenceKeyError(gtag)
            start, end = span.b_aend - eff_a - l + x, span.a_pos + eff_a + x + 1   # 929
            start, end = min(start, end), max(start, end)
            if is_backsplice:                                           # 941-945
                end -= 1
            else:
                start -= 1
            if opt.noncanonical:                                        # 947-949
                hits.append(_mk(x, chrom, start, end, '+', dist, ov, gtag, span, opt))
                hits.append(_mk(x, chrom, start, end, '-', dist, ov, rc_gtag, span, opt))
            else:
                if gtag == 'GTAG':
                    hits.append(_mk(x, chrom, start, end, '+', dist, ov, gtag, span, opt))
                elif gtag == 'CTAC':
                    hits.append(_mk(x, chrom, start, end, '-', dist, ov, rc_gtag, span, opt))
    if len(hits) < 2:                                                   # 961-963
        return hits
    hits = sorted(hits, key=lambda h: h.score, reverse=True)            # 966 (stable)
    best_score = hits[0].score
    ties = [h for h in hits if h.score == best_score]
    n_hits = len(ties)
    for h in hits:
        h.n_hits = n_hits
    return ties


def _mk(x, chrom, start, end, strand, dist, ov, gtag, span: Span, opt: Options) -> Hit:
    # Splice.score, find_circ.py:791-799 (bool dist multiplies like 0/1)
    s = (gtag == 'GTAG') * 20 - int(dist) * 10 - ov
    if opt.strandpref:
        s += 100 * (strand == span.strand)
    return Hit(x=x, chrom=chrom, start=start, end=end, strand=strand, dist=dist, ov=ov, gtag=gtag, score=s)


def first_tie(hits: List[Hit], opt: Options) -> List[Hit]:
    """What ``record_hits`` keeps from the ties (find_circ.py:1312-1317, 1364-1378)."""
    if not hits:
        return []
    return list(hits) if opt.allhits else [hits[0]]


def literal_rate(fasta_path: str, spans: List[tuple], budget_s: float, cycle: bool = False):
    """The literal path timed on one core, for the bench's CPU baseline run over a process pool: per
    span (chrom, a_pos, a_aend, b_pos, b_aend, read_part, primary_reverse) both windows through the
    Track.get chain of the mmap'd FASTA (its .byo_index loaded) and find_breakpoints with the default
    options, until `budget_s` seconds have passed (cycle: over the spans again until then).  Returns
    (spans done, seconds, first ties of the first pass) with a first tie = (x, n_hits), (-1, 0) for no
    hit, None where the reference raises."""
    import time
    track = RefGenomeTrack(RefIndexedFasta(fasta_path, use_existing_index=True, use_mmap=True))
    opt = Options()
    out = []
    done = 0
    t0 = time.perf_counter()
    while spans:
        for t in spans:
            try:
                ties = find_breakpoints(Span(*t), track, opt)
                r = (ties[0].x, ties[0].n_hits) if ties else (-1, 0)
            except Exception:
                r = None
            if len(out) < len(spans):
                out.append(r)
            done += 1
            if time.perf_counter() - t0 > budget_s:
                return done, time.perf_counter() - t0, out
        if not cycle:
            break
    return done, time.perf_counter() - t0, out
