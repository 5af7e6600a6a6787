"""fc2_fasta_pack (the device genome's 2-bit planes, N plane and coarse N map) against a numpy
restatement of the reference's window bytes (find_circ.py:189-215 get_data over the .byo_index
layout, upper-cased at :901-902): bit j of unit u = base 64u + j of the chromosome's slot; A/C/G/T
-> (lo, hi) = 00/10/01/11 with the N plane clear, 'N' and every other byte -> N plane set (the
others counted as exotic), bases past a chromosome's end N.  Line lengths below, at and above the
packer's 64-base segments, CRLF lines, lower case, a file without its last newline, chromosomes
longer than one work item (2^20 bases), one irregular chromosome (all N), 1 and 8 threads."""
import ctypes

import numpy as np
import pytest

from find_circ2_amd import _native as N


def _expected(seqs, regular):
    """units [2*nu], nplane [nu], ncoarse, n_exotic for chromosomes laid out back to back in 64-base
    slots (fc2_fasta_layout)."""
    slots = [(len(s) + 63) // 64 for s in seqs]
    nu = max(1, sum(slots))
    units = np.zeros(2 * nu, np.uint64)
    nplane = np.full(nu, ~np.uint64(0), np.uint64)
    n_exotic = 0
    u0 = 0
    for s, k, reg in zip(seqs, slots, regular):
        if k == 0:
            continue
        if reg:
            b = np.frombuffer(s, np.uint8) & 0xDF
            a, c, g, t, n = (b == ord(x) for x in "ACGTN")
            acgt = a | c | g | t
            n_exotic += int((~(acgt | n)).sum())
            pad = np.ones(k * 64 - len(b), bool)          # past the chromosome's end: N
            bits = lambda m: np.packbits(m.reshape(-1, 64)[:, ::-1], axis=1).view(">u8").astype(np.uint64).ravel()
            units[2 * u0:2 * (u0 + k):2] = bits(np.concatenate([c | t, ~pad]))
            units[2 * u0 + 1:2 * (u0 + k):2] = bits(np.concatenate([g | t, ~pad]))
            nplane[u0:u0 + k] = bits(np.concatenate([~acgt, pad]))
        u0 += k
    nb = (nu + 15) >> 4
    blk = np.zeros(nb * 16, np.uint64)
    blk[:nu] = nplane
    anyn = (blk.reshape(nb, 16) != 0).any(axis=1)
    nw = (nb + 31) >> 5
    bitsc = np.zeros(nw * 32, bool)
    bitsc[:nb] = anyn
    ncoarse = (bitsc.reshape(nw, 32) * (np.uint64(1) << np.arange(32, dtype=np.uint64))).sum(axis=1).astype(np.uint32)
    return units, nplane, ncoarse, n_exotic


def _write(path, chroms, eol=b"\n", last_newline=True):
    out = []
    for name, s, width in chroms:
        out.append(b">" + name + eol)
        if isinstance(width, int):
            lines = [s[i:i + width] for i in range(0, len(s), width)]
        else:                                   # irregular: the given line lengths
            lines, i = [], 0
            for w in width:
                lines.append(s[i:i + w])
                i += w
        out.append(eol.join(lines) + eol)
    data = b"".join(out)
    if not last_newline:
        data = data[:-len(eol)]
    open(path, "wb").write(data)


def _pack(path, threads):
    L = N.lib()
    h = ctypes.c_void_p()
    N.check(L.fc2_fasta_open(path.encode(), 0, ctypes.byref(h)))
    try:
        nu, ncw = ctypes.c_uint64(), ctypes.c_uint64()
        cs = np.zeros(max(1, L.fc2_fasta_n_chrom(h)), np.uint64)
        N.check(L.fc2_fasta_layout(h, ctypes.byref(nu), ctypes.byref(ncw), cs.ctypes.data))
        units = np.full(2 * nu.value, 0x5A5A5A5A5A5A5A5A, np.uint64)      # every word must be written
        nplane = np.full(nu.value, 0x5A5A5A5A5A5A5A5A, np.uint64)
        ncoarse = np.zeros(max(1, ncw.value), np.uint32)
        exo = ctypes.c_uint64()
        N.check(L.fc2_fasta_pack(h, units.ctypes.data, nplane.ctypes.data, ncoarse.ctypes.data,
                                 ctypes.byref(exo), threads))
        return units, nplane, ncoarse[:ncw.value], exo.value
    finally:
        L.fc2_fasta_close(h)


def _seq(rng, n, alphabet=b"ACGT", p_low=0.1, p_n=0.02, p_exotic=0.001):
    s = np.frombuffer(alphabet, np.uint8)[rng.integers(0, len(alphabet), n)].copy()
    low = rng.random(n) < p_low
    s[low] |= 0x20
    s[rng.random(n) < p_n] = ord("N")
    ex = rng.random(n) < p_exotic
    s[ex] = np.frombuffer(b"RYKMSWnx#*-", np.uint8)[rng.integers(0, 11, int(ex.sum()))]
    if n > 5000:
        a = int(rng.integers(0, n - 3000))
        s[a:a + int(rng.integers(1, 3000))] = ord("N")
    return s.tobytes()


@pytest.mark.parametrize("width", [1, 7, 50, 60, 63, 64, 65, 100, 127, 200, 10 ** 7])
@pytest.mark.parametrize("eol", [b"\n", b"\r\n"], ids=["lf", "crlf"])
def test_pack_equals_numpy_restatement(tmp_path, width, eol):
    rng = np.random.default_rng(width * 7 + len(eol))
    sizes = [1, 63, 64, 65, 1000, 4097, 2_200_000 if width >= 50 else 70_000, 129, 5]
    chroms = [(b"c%d" % i, _seq(rng, n), width) for i, n in enumerate(sizes)]
    path = str(tmp_path / "g.fa")
    _write(path, chroms, eol=eol, last_newline=width % 2 == 0)
    exp = _expected([s for _, s, _ in chroms], [True] * len(chroms))
    for threads in (1, 8):
        got = _pack(path, threads)
        for name, a, b in zip(("units", "nplane", "ncoarse"), got[:3], exp[:3]):
            assert np.array_equal(a, b), (name, threads, np.flatnonzero(a != b)[:5])
        assert got[3] == exp[3]


def test_pack_irregular_chromosome_is_all_n(tmp_path):
    rng = np.random.default_rng(5)
    s0, s1, s2 = _seq(rng, 3000), _seq(rng, 500), _seq(rng, 777)
    chroms = [(b"reg", s0, 60), (b"irr", s1, [60, 60, 59, 60, 60, 60, 60, 60, 21]), (b"tail", s2, 61)]
    path = str(tmp_path / "g.fa")
    _write(path, chroms)
    exp = _expected([s0, s1, s2], [True, False, True])
    got = _pack(path, 4)
    for a, b in zip(got[:3], exp[:3]):
        assert np.array_equal(a, b)
    assert got[3] == exp[3]


@pytest.mark.parametrize("damage", ["long_row", "short_row", "lf_in_crlf", "last_row_long"])
def test_pack_row_damage_deep_inside_is_all_n(tmp_path, damage):
    """A row of the wrong length (or a missing '\\r') past the first work item of a 2.2-Mbase
    chromosome: the row check of the planes pass makes the whole chromosome irregular (all N, no
    exotic bases counted), its neighbours unchanged."""
    rng = np.random.default_rng(17)
    s0, s1, s2 = _seq(rng, 5000), _seq(rng, 2_200_000), _seq(rng, 3333)
    eol = b"\r\n" if damage == "lf_in_crlf" else b"\n"
    rows = [s1[i:i + 50] for i in range(0, len(s1), 50)]
    k = 1_600_000 // 50 if damage != "last_row_long" else len(rows) - 2
    if damage in ("long_row", "last_row_long"):
        rows[k], rows[k + 1] = rows[k] + rows[k + 1][:1], rows[k + 1][1:]
    elif damage == "short_row":
        rows[k], rows[k + 1] = rows[k][:-1], rows[k][-1:] + rows[k + 1]
    body1 = eol.join(rows) + eol
    if damage == "lf_in_crlf":
        body1 = body1.replace(rows[k] + b"\r\n", rows[k] + b"\n", 1)
    path = str(tmp_path / "g.fa")
    with open(path, "wb") as f:
        f.write(b">a" + eol + eol.join(s0[i:i + 60] for i in range(0, len(s0), 60)) + eol)
        f.write(b">b" + eol + body1)
        f.write(b">c" + eol + eol.join(s2[i:i + 70] for i in range(0, len(s2), 70)) + eol)
    exp = _expected([s0, s1, s2], [True, False, True])
    for threads in (1, 8):
        got = _pack(path, threads)
        for a, b in zip(got[:3], exp[:3]):
            assert np.array_equal(a, b)
        assert got[3] == exp[3]


def test_prepack_then_pack_and_close(tmp_path):
    """fc2_fasta_prepack (the CLI's start-up packs beside HIP init; fc2_ctx_genome_load takes the planes
    over): the FASTA handle is packed as by fc2_fasta_pack (a later pack gives the same planes), a
    second prepack replaces the first, and planes no context took are freed with the handle."""
    rng = np.random.default_rng(23)
    chroms = [(b"c%d" % i, _seq(rng, n), w) for i, (n, w) in enumerate(((70_000, 60), (5, 50), (3000, 61)))]
    path = str(tmp_path / "g.fa")
    _write(path, chroms)
    exp = _expected([s for _, s, _ in chroms], [True] * 3)
    L = N.lib()
    for k in range(2):
        h = ctypes.c_void_p()
        N.check(L.fc2_fasta_open(path.encode(), 0, ctypes.byref(h)))
        try:
            N.check(L.fc2_fasta_prepack(h, 4))
            if k:
                N.check(L.fc2_fasta_prepack(h, 1))
            nu, ncw = ctypes.c_uint64(), ctypes.c_uint64()
            N.check(L.fc2_fasta_layout(h, ctypes.byref(nu), ctypes.byref(ncw), None))
            units, nplane = np.zeros(2 * nu.value, np.uint64), np.zeros(nu.value, np.uint64)
            ncoarse, exo = np.zeros(max(1, ncw.value), np.uint32), ctypes.c_uint64()
            N.check(L.fc2_fasta_pack(h, units.ctypes.data, nplane.ctypes.data, ncoarse.ctypes.data,
                                     ctypes.byref(exo), 2))
            for a, b in zip((units, nplane, ncoarse[:ncw.value]), exp[:3]):
                assert np.array_equal(a, b)
            assert exo.value == exp[3]
        finally:
            L.fc2_fasta_close(h)
    assert L.fc2_fasta_prepack(None, 0) == N.FC2_E_PARAM
