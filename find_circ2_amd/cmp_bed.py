"""Compare two splice-site BED files as sets of (chrom, start, end, strand) -- cmp_bed.py semantics.

    python -m find_circ2_amd.cmp_bed reference.bed result.bed [names]

The reference's own notion of parity (cmp_bed.py:6-62): rows are keyed by
their first six BED columns' coordinates, order is ignored; shared rows are
printed (or "name1<TAB>name2" with a third argument), rows only in the first
file as "MISSING<TAB>row", counters on stderr, and "files contain identical
splice sites!" when both sets are equal.  Output rows are sorted by key here
(the reference prints them in Python 2 dict order).
"""
from __future__ import annotations

import sys
from collections import defaultdict
from typing import Dict, Tuple


def read_sites(path: str, ds: int = 0, de: int = 0, flank: int = 0) -> Dict[Tuple, str]:
    """cmp_bed.read_to_hash (cmp_bed.py:6-25)."""
    pos: Dict[Tuple, str] = {}
    with open(path) as f:
        for line in f:
            if line.startswith("#"):
                continue
            line = line.strip()
            chrom, start, end, name, score, sense = line.split("\t")[:6]
            start, end = int(start) + ds, int(end) + de
            pos[(chrom, start, end, sense)] = line
            for x in range(flank):
                for key in ((chrom, start - x, end, sense), (chrom, start + x, end, sense),
                            (chrom, start, end - x, sense), (chrom, start, end + x, sense)):
                    pos[key] = line
    return pos


def compare(path1: str, path2: str, names: bool = False, out=sys.stdout, err=sys.stderr) -> bool:
    N = defaultdict(int)
    bed1 = read_sites(path1)
    N['unique_input1'] = len(bed1)
    bed2 = read_sites(path2)
    N['unique_input2'] = len(bed2)
    for key in sorted(bed2):
        line = bed2[key]
        if key in bed1:
            if names:
                out.write("%s\t%s\n" % (bed1[key].split('\t')[3], line.split('\t')[3]))
            else:
                out.write(bed1[key] + "\n")
            N['overlap'] += 1
            del bed1[key]
        else:
            N['input2_not_in_input1'] += 1
    for key in sorted(bed1):
        out.write("MISSING\t%s\n" % bed1[key])
        N['input1_not_in_input2'] += 1
    for k in sorted(N):
        err.write("%s\t%d\n" % (k, N[k]))
    identical = N['overlap'] == N['unique_input1'] == N['unique_input2']
    if identical:
        err.write("files contain identical splice sites!\n")
    return identical


def main(argv=None) -> int:
    argv = sys.argv[1:] if argv is None else argv
    if len(argv) < 2:
        sys.stderr.write("usage: cmp_bed.py <bed1> <bed2> [names]\n")
        return 2
    compare(argv[0], argv[1], names=len(argv) > 2)
    return 0


if __name__ == "__main__":
    sys.exit(main())
