"""Small seeded anchor-pair generator for CPU-side parity tests.

Follows SURVEY.md §8(d)'s recipe at toy scale: junctions planted at GT..AG /
CT..AC sites half of the time, uniform otherwise; backsplice reads are
``G[end-kA:end] + G[start:start+L-kA]``, linear reads ``G[d-kA:d] + G[a:a+L-kA]``;
per-base substitutions; optional read ends clipped (emulating bwa local
alignment), N bases and lower-case bytes in reads; some pairs placed at the
chromosome ends so the genome windows get N-padded (find_circ.py:194-211).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, List

import numpy as np

from bwa_emul import read_fasta


@dataclass
class SmallSpan:
    chrom: str
    chrom_idx: int
    a_pos: int
    a_aend: int
    b_pos: int
    b_aend: int
    read_part: bytes
    primary_reverse: bool

    @property
    def is_backsplice(self):
        return self.b_pos - self.a_aend < 0


def _find_site(g: str, p: int, motif: str, step: int, limit: int = 400):
    for k in range(limit):
        q = p + k * step
        if 0 <= q and q + 2 <= len(g) and g[q:q + 2].upper() == motif:
            return q
    return None


def make_spans(genome: Dict[str, str], n: int, seed: int, L=(60, 160), asize=15, mut=0.01,
               p_planted=0.5, p_backsplice=0.6, p_edge=0.05, p_readN=0.05, p_lower=0.05,
               p_clip=0.2, p_short=0.02) -> List[SmallSpan]:
    rng = np.random.default_rng(seed)
    names = list(genome)
    out: List[SmallSpan] = []
    while len(out) < n:
        ci = int(rng.integers(len(names)))
        chrom = names[ci]
        g = genome[chrom]
        G = len(g)
        Lr = int(rng.integers(L[0], L[1] + 1))
        if rng.random() < p_short:
            Lr = int(rng.integers(2 * asize - 6, 2 * asize + 3))
        kA = int(rng.integers(asize, max(asize + 1, Lr - asize + 1)))
        kB = Lr - kA
        bs = rng.random() < p_backsplice
        planted = rng.random() < p_planted
        minus = rng.random() < 0.3
        if bs:
            # exon [start, end): A = G[end-kA:end], B = G[start:start+kB]
            span = int(rng.integers(max(kA, kB) + 1, max(max(kA, kB) + 2, min(G, 1500))))
            end = int(rng.integers(kA, G + 1))
            if planted:
                q = _find_site(g, end, "CT" if minus else "GT", 1)
                if q is not None:
                    end = q
            start = end - span
            if planted and start >= 2:
                q = _find_site(g, start - 2, "AC" if minus else "AG", -1)
                if q is not None:
                    start = q + 2
            if rng.random() < p_edge:   # touch a chromosome end -> N padded windows
                if rng.random() < 0.5:
                    start = int(rng.integers(0, 6))
                else:
                    end = G - int(rng.integers(0, 6))
                    start = min(start, end - max(kA, kB) - 1)
            if start < 0 or end - kA < 0 or start + kB > G or end > G or start >= end:
                continue
            read = g[end - kA:end] + g[start:start + kB]
            a_pos, a_aend, b_pos, b_aend = end - kA, end, start, start + kB
        else:
            # intron [d, a): A = G[d-kA:d], B = G[a:a+kB]
            d = int(rng.integers(kA, G))
            if planted:
                q = _find_site(g, d, "CT" if minus else "GT", 1)
                if q is not None:
                    d = q
            a = d + int(rng.integers(30, 1200))
            if planted:
                q = _find_site(g, a - 2, "AC" if minus else "AG", 1)
                if q is not None:
                    a = q + 2
            if d - kA < 0 or a + kB > G:
                continue
            read = g[d - kA:d] + g[a:a + kB]
            a_pos, a_aend, b_pos, b_aend = d - kA, d, a, a + kB
        r = np.frombuffer(read.upper().encode(), dtype=np.uint8).copy()
        # substitutions
        m = rng.random(len(r)) < mut
        if m.any():
            alph = np.frombuffer(b"ACGT", dtype=np.uint8)
            r[m] = alph[rng.integers(0, 4, m.sum())]
        if rng.random() < p_readN:
            k = int(rng.integers(1, 4))
            r[rng.integers(0, len(r), k)] = ord('N')
        if rng.random() < p_lower:
            lo = rng.random(len(r)) < 0.3
            r[lo] = r[lo] + 32
        c0 = c1 = 0
        if rng.random() < p_clip:
            c0, c1 = int(rng.integers(0, 4)), int(rng.integers(0, 4))
            if kA - c0 < 2 or kB - c1 < 2:
                c0 = c1 = 0
        read_b = bytes(r[c0:len(r) - c1])
        out.append(SmallSpan(chrom, ci, a_pos + c0, a_aend, b_pos, b_aend - c1, read_b,
                             bool(rng.random() < 0.5)))
    return out


def load_genome(path: str) -> Dict[str, str]:
    return read_fasta(path)


def make_odd_spans(genome: Dict[str, str], n: int, seed: int, asize=15, margin=2) -> List[SmallSpan]:
    """Spans at the edges of find_breakpoints' input domain (find_circ.py:854-974): read parts of
    0..4 bases and of 2e-2 .. 2e+3 bases (e = asize - margin, so the internal part read[e:-e] is
    empty or one base long), windows that start past a chromosome's end or end before its start
    (get_data pads them with 'N' to more than the requested length, :194-211), next to ordinary
    spans.  Reads are genome text around a random junction, so some candidates qualify."""
    rng = np.random.default_rng(seed)
    names = list(genome)
    e = asize - margin
    out: List[SmallSpan] = []
    while len(out) < n:
        ci = int(rng.integers(len(names)))
        chrom = names[ci]
        g = genome[chrom]
        G = len(g)
        u = rng.random()
        if u < 0.35:
            L = int(rng.integers(0, 5))
        elif u < 0.7:
            L = int(rng.integers(max(0, 2 * e - 2), max(1, 2 * e + 4)))
        else:
            L = int(rng.integers(max(1, 2 * e), max(2, 2 * e + 60)))
        # each window from its own bucket, so a short window (past the end) meets a long one (before
        # the start) as often as two of a kind: the byte kernel's slots must hold either
        v, w = rng.random(), rng.random()
        if v < 0.25:                                       # A's window past the chromosome's end
            a_pos = G + int(rng.integers(-5, 40))
        elif v < 0.5:                                      # ... or before its start
            a_pos = int(rng.integers(-40, 8))
        else:
            a_pos = int(rng.integers(0, max(1, G - 1)))
        if w < 0.25:                                       # B's window past the end
            b_aend = G + int(rng.integers(-5, 80))
        elif w < 0.5:                                      # ... or before the start
            b_aend = int(rng.integers(-20, 30))
        else:
            b_aend = int(rng.integers(0, max(1, G)))
        kA = L // 2
        src = rng.random() < 0.6
        if src and 0 <= a_pos and a_pos + kA <= G and b_aend - (L - kA) >= 0 and b_aend <= G:
            read = g[a_pos:a_pos + kA] + g[b_aend - (L - kA):b_aend]
        else:
            read = "".join("ACGTN"[int(c)] for c in rng.integers(0, 5, L))
        bs = rng.random() < 0.5
        a_aend = a_pos + kA
        b_pos = b_aend - (L - kA)
        if bs and b_pos >= a_aend:                         # is_backsplice = b_pos < a_aend (:842)
            b_pos = a_aend - 1 - int(rng.integers(0, 50))
        elif not bs and b_pos < a_aend:
            b_pos = a_aend + int(rng.integers(0, 50))
        out.append(SmallSpan(chrom, ci, int(a_pos), int(a_aend), int(b_pos), int(b_aend), read.encode(),
                             bool(rng.random() < 0.5)))
    return out


def truncated_fasta(tmp_path):
    """A FASTA cut short after it was indexed: its .byo_index (which the reference reads instead of
    indexing, find_circ.py:110-112) claims 60 more bases for the last chromosome than the file holds,
    so get_data returns windows shorter than asked near that end and padded longer before the start
    (:194-211).  Returns (path, {chrom: text})."""
    rng = np.random.default_rng(8)
    seqs = {c: bytes(rng.choice(np.frombuffer(b"ACGT", np.uint8), n).tobytes()) for c, n in (("u1", 300), ("u2", 240))}
    for c in seqs:                                   # splice signals to qualify some breakpoints
        b = bytearray(seqs[c])
        for k in range(5, len(b) - 5, 37):
            b[k:k + 2] = b"GT" if k % 2 else b"AG"
        seqs[c] = bytes(b)
    path = str(tmp_path / "trunc.fa")
    body, idx, ofs = b"", [], 0
    for c, sq in seqs.items():
        head = b">" + c.encode() + b"\n"
        ofs += len(head)
        lines = b"".join(sq[k:k + 60] + b"\n" for k in range(0, len(sq), 60))
        idx.append("%s\t%d\t60\t1\t'\\n'\t%d\n" % (c, ofs, len(sq) + (60 if c == "u2" else 0)))
        body += head + lines
        ofs += len(lines)
    open(path, "wb").write(body)
    open(path + ".byo_index", "w").write("".join(idx))
    return path, {c: sq.decode() for c, sq in seqs.items()}
