"""Damaged genomes: FASTA text and .byo_index entries (the index the reference writes next to the
FASTA, find_circ.py:110-179, and trusts when it exists).  The reference's Python slices clip or wrap
on nonsense offsets and fail on impossible sizes; the native indexer, packer and window reader must
either follow it or return an error -- never read outside the mapped file or abort.  Seeded cases;
scripts/sanitize_host.sh runs them under ASan / UBSan.
"""
import ctypes
import os
import random

import numpy as np
import pytest

from conftest import GOLDEN
from find_circ2_amd import _native as N

GOLD = ("CDR1as_locus.fa", "test_ref.fa")


def _damage_fasta(rng, b: bytes) -> bytes:
    b = bytearray(b)
    k = rng.randrange(5)
    if k == 0:
        return bytes(b[:rng.randrange(len(b) + 1)])
    if k == 1:
        for _ in range(rng.randint(1, 6)):
            b[rng.randrange(len(b))] = rng.choice(b"ACGTNacgtn>\r\n \tRYK#\x00\xff")
        return bytes(b)
    if k == 2:
        i = rng.randrange(len(b))
        return bytes(b[:i]) + bytes(rng.randrange(256) for _ in range(rng.randint(1, 40))) + bytes(b[i:])
    if k == 3:
        lines = bytes(b).split(b"\n")
        i = rng.randrange(len(lines))
        lines[i] = lines[i][:rng.randrange(len(lines[i]) + 1)]
        return b"\n".join(lines)
    return bytes(rng.randrange(256) for _ in range(rng.randint(0, 200)))


def _set_index_field(text: bytes, line: int, field: int, value: bytes) -> bytes:
    lines = text.split(b"\n")
    parts = lines[line].split(b"\t")
    parts[field] = value
    lines[line] = b"\t".join(parts)
    return b"\n".join(lines)


def _exercise(path, rng):
    """open -> layout -> pack -> random windows; returns the first failing step or 'ok'."""
    L = N.lib()
    h = ctypes.c_void_p()
    if L.fc2_fasta_open(path.encode(), 0, ctypes.byref(h)) != 0:
        return "open"
    try:
        nu, ncw = ctypes.c_uint64(), ctypes.c_uint64()
        nch = L.fc2_fasta_n_chrom(h)
        cs = np.zeros(max(1, nch), np.uint64)
        if L.fc2_fasta_layout(h, ctypes.byref(nu), ctypes.byref(ncw), cs.ctypes.data) != 0:
            return "layout"
        if nu.value > 50_000_000:
            return "huge"
        units = np.empty(2 * nu.value, np.uint64)
        npl = np.empty(nu.value, np.uint64)
        nc = np.zeros(max(1, ncw.value), np.uint32)
        ne = ctypes.c_uint64()
        if L.fc2_fasta_pack(h, units.ctypes.data, npl.ctypes.data, nc.ctypes.data, ctypes.byref(ne), 2) != 0:
            return "pack"
        buf = np.zeros(4096, np.uint8)
        ln = ctypes.c_int64()
        for _ in range(20):
            a = rng.randrange(-3000, 5000)
            L.fc2_fasta_get_upper(h, rng.randrange(-1, nch + 1), a, a + rng.randrange(-10, 300), buf.ctypes.data,
                                  4096, ctypes.byref(ln))
        return "ok"
    finally:
        L.fc2_fasta_close(h)


def _write_index(tmp_path, name):
    fa = str(tmp_path / name)
    with open(fa, "wb") as fh:
        fh.write(open(os.path.join(GOLDEN, name), "rb").read())
    h = ctypes.c_void_p()
    N.check(N.lib().fc2_fasta_open(fa.encode(), 1, ctypes.byref(h)))
    N.lib().fc2_fasta_close(h)
    idx = fa + ".byo_index"
    os.chmod(idx, 0o644)
    return fa, idx


def test_damaged_fasta_text(tmp_path):
    rng = random.Random(110112)
    seen = set()
    for k in range(60):
        name = GOLD[k % 2]
        fa = str(tmp_path / ("d%d_%s" % (k, name)))
        with open(fa, "wb") as fh:
            fh.write(_damage_fasta(rng, open(os.path.join(GOLDEN, name), "rb").read()))
        seen.add(_exercise(fa, rng))
    assert "ok" in seen


@pytest.mark.parametrize("field,value", [(1, b"-5"), (1, b"-999999999999"), (1, b"999999999"), (2, b"0"),
                                         (2, b"-7"), (3, b"-1"), (5, b"-999999999999"), (5, b"9223372036854775807"),
                                         (4, b"'\\x'"), (4, b"x")])
def test_damaged_index_entries(tmp_path, field, value):
    """One field of a .byo_index line set to nonsense: open fails, or every later step either
    succeeds or reports an error (a negative offset once made the packer read before the mapping, a
    negative size made the window reader try a 1 TB allocation)."""
    rng = random.Random(field * 31 + len(value))
    for name in GOLD:
        fa, idx = _write_index(tmp_path, name)
        with open(idx, "rb") as fh:
            text = fh.read()
        with open(idx, "wb") as fh:
            fh.write(_set_index_field(text, 0, field, value))
        assert _exercise(fa, rng) in ("ok", "open", "layout", "pack", "huge")
