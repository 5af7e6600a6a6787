"""Tiny bwa-mem-shaped split-alignment emulator for the golden read sets.

No aligner exists in this image, so the reference's regression inputs
(``test_reads.fa`` / ``cdr1as_reads.fa``, which the reference's Makefile pipes
through ``bwa mem -k 15 -T 1``, test_data/Makefile:12-19) are turned into
anchor pairs here by greedy maximal exact matching.  The output mirrors what
``MateSegments.adjacent_segment_pairs`` (find_circ.py:1058-1140) yields for a
bwa-mem record group: segments in query order, read_part = union of two
adjacent segments' query ranges, ``A``/``B`` = earlier/later segment in the
read, all coordinates on the forward genome strand (SAM SEQ orientation).

The breakpoint search is designed so the called junction does not depend on
where exactly the aligner splits the read; tests vary the split (``shift``) to
check that, too.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, List, Optional, Tuple

_COMP = {'A': 'T', 'C': 'G', 'G': 'C', 'T': 'A', 'N': 'N'}


def revcomp(s: str) -> str:
    return "".join(_COMP[c] for c in reversed(s.upper()))


def read_fasta(path: str) -> Dict[str, str]:
    seqs: Dict[str, List[str]] = {}
    order = []
    name = None
    with open(path) as f:
        for line in f:
            line = line.rstrip('\r\n')
            if not line:
                continue
            if line.startswith('>'):
                name = line[1:].split()[0]
                seqs[name] = []
                order.append(name)
            else:
                seqs[name].append(line)
    return {k: "".join(seqs[k]) for k in order}


@dataclass
class Segment:
    q_start: int
    q_end: int
    chrom: str
    pos: int
    aend: int


@dataclass
class PairSpec:
    qname: str
    chrom: str
    a_pos: int
    a_aend: int
    b_pos: int
    b_aend: int
    read_part: str
    primary_reverse: bool
    q_start: int
    q_end: int

    @property
    def is_backsplice(self) -> bool:
        return self.b_pos - self.a_aend < 0


def _longest_match(seq: str, i: int, genome: Dict[str, str], min_len: int) -> Optional[Segment]:
    best = None
    for chrom, g in genome.items():
        gu = g.upper()
        # extend every seed occurrence of seq[i:i+min_len]
        seed = seq[i:i + min_len]
        if len(seed) < min_len:
            return None
        p = gu.find(seed)
        while p >= 0:
            k = min_len
            while i + k < len(seq) and p + k < len(gu) and seq[i + k] == gu[p + k]:
                k += 1
            if best is None or k > best.q_end - best.q_start:
                best = Segment(i, i + k, chrom, p, p + k)
            p = gu.find(seed, p + 1)
    return best


def segment_read(seq: str, genome: Dict[str, str], min_len: int = 12) -> List[Segment]:
    segs = []
    i = 0
    while i < len(seq):
        s = _longest_match(seq, i, genome, min_len)
        if s is None:
            i += 1
            continue
        segs.append(s)
        i = s.q_end
    return segs


def emulate_pairs(qname: str, read: str, genome: Dict[str, str], asize: int = 15,
                  shift: int = 0) -> List[PairSpec]:
    """Anchor pairs for one read, trying forward then reverse strand.

    ``shift`` moves every internal segment boundary ``shift`` bases later in the
    query (A keeps ``shift`` more bases, B starts ``shift`` later), emulating a
    different aligner clip choice on the same read.
    """
    best = None
    for rev in (False, True):
        seq = revcomp(read) if rev else read.upper()
        segs = segment_read(seq, genome)
        covered = sum(s.q_end - s.q_start for s in segs)
        if best is None or covered > best[2]:
            best = (rev, seq, covered, segs)
    rev, seq, _, segs = best
    out: List[PairSpec] = []
    for a, b in zip(segs, segs[1:]):
        if a.chrom != b.chrom:
            continue
        a_q_end, a_aend = a.q_end + shift, a.aend + shift
        b_q_start, b_pos = b.q_start + shift, b.pos + shift
        if (a_q_end - a.q_start) < asize or (b.q_end - b_q_start) < asize:   # find_circ.py:1125
            continue
        r_start = min(a.q_start, b_q_start)
        r_end = max(a_q_end, b.q_end)
        out.append(PairSpec(qname, a.chrom, a.pos, a_aend, b_pos, b.aend,
                            seq[r_start:r_end], rev, r_start, r_end))
    return out


def truth_from_name(name: str):
    """Parse the ``O:..;M:..;LS:..;CS:..`` truth (find_circ.py:1148-1191)."""
    lin, circ = set(), set()
    if '___' not in name:
        return None
    for mate_str in name.split('___')[-1].split('|'):
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
                end = right
            elif op == 'CS':
                left, right = int(parts[1]) + start, int(parts[2]) + start
                circ.add((chrom, left, right, strand))
                end = left
    return lin, circ
