"""Read-length limit of the boundary: fc2_result.best_x is 16-bit, so read parts longer
than FC2_MAX_READ_LEN = 32767 bases are refused with FC2_E_RANGE instead of wrapping; the longest
accepted reads (byte path) are checked against the oracle with the breakpoint near the end."""
import ctypes
import os

import numpy as np
import pytest

import oracle
from find_circ2_amd import _native as N


def _fasta(tmp_path, seq, name="big"):
    path = str(tmp_path / "g.fa")
    with open(path, "w") as f:
        f.write(">%s\n" % name)
        for i in range(0, len(seq), 60):
            f.write(seq[i:i + 60] + "\n")
    return path


def _long_pair(seq, L, x_frac=0.95):
    """A linear junction read of length L: G[d-k:d] + G[a:a+L-k], donor GT at d, acceptor AG at a-2."""
    k = int(L * x_frac)
    d = 1000 + k
    a = d + 5000
    read = seq[d - k:d] + seq[a:a + L - k]
    return read, d - k, a + L - k, k


def _genome_seq(L):
    rng = np.random.default_rng(3)
    g = list(rng.choice(list("ACGT"), 2 * L + 20000))
    return g


def test_pack_refuses_reads_longer_than_limit(tmp_path):
    assert N.MAX_READ_LEN == 32767
    g = _genome_seq(40000)
    path = _fasta(tmp_path, "".join(g))
    h = ctypes.c_void_p()
    N.check(N.lib().fc2_fasta_open(path.encode(), 0, ctypes.byref(h)))
    try:
        nu, ncw = ctypes.c_uint64(), ctypes.c_uint64()
        cs = np.zeros(1, np.uint64)
        N.check(N.lib().fc2_fasta_layout(h, ctypes.byref(nu), ctypes.byref(ncw), cs.ctypes.data))
        units = np.zeros(2 * nu.value, np.uint64)
        nplane = np.zeros(nu.value, np.uint64)
        ncoarse = np.zeros(max(1, ncw.value), np.uint32)
        exo = ctypes.c_uint64()
        N.check(N.lib().fc2_fasta_pack(h, units.ctypes.data, nplane.ctypes.data, ncoarse.ctypes.data,
                                       ctypes.byref(exo), 0))
        p = N.Params(15, 2, 2, 0, 0, 0, 0)
        for L, ok in ((32767, True), (32768, False), (40000, False)):
            buf = np.frombuffer(("A" * L).encode() + b"\0" * 16, np.uint8)
            off = np.zeros(1, np.uint64)
            hp = np.zeros(1, N.PAIR_DTYPE)
            hp["a_pos"], hp["b_aend"], hp["read_len"] = 100, 30000, L
            rw, nw, tw = ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_uint32()
            N.check(N.lib().fc2_batch_geometry(ctypes.byref(p), L, ctypes.byref(rw), ctypes.byref(nw), ctypes.byref(tw)))
            words = np.zeros(rw.value, np.uint64)
            nwords = np.zeros(nw.value, np.uint64)
            nbp = ctypes.c_uint64()
            rc = N.lib().fc2_pack_pairs(ctypes.byref(p), h, 1, buf.ctypes.data, off.ctypes.data, hp.ctypes.data,
                                        words.ctypes.data, rw.value, nwords.ctypes.data, nw.value, 1,
                                        ctypes.byref(nbp), 1)
            if ok:
                assert rc == N.FC2_OK and nbp.value == 1          # l > 510: byte path
            else:
                assert rc == N.FC2_E_RANGE
                assert b"32767" in N.lib().fc2_last_error()
    finally:
        N.lib().fc2_fasta_close(h)


@pytest.mark.gpu
def test_longest_reads_vs_oracle(tmp_path):
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from find_circ2_amd import Genome, Options, PairBatch, decode_splices, scan
    L = 32767
    g = _genome_seq(L + 8000)
    reads, a_pos, b_aend = [], [], []
    for frac in (0.95, 0.5, 0.999):
        k = int(L * frac)
        d, a = 1000 + k, 1000 + k + 5000
        g[d:d + 2] = list("GT")
        g[a - 2:a] = list("AG")
    seq = "".join(g)
    for frac in (0.95, 0.5, 0.999):
        r, ap, be, k = _long_pair(seq, L, frac)
        reads.append(r.encode())
        a_pos.append(ap)
        b_aend.append(be)
    path = _fasta(tmp_path, seq)
    opt = Options()
    gen = Genome.from_fasta(path, device="cuda:0")
    b = PairBatch.pack(opt, gen, reads, a_pos, b_aend, [0] * 3, [0] * 3)
    assert b.m_bytepath == 3
    got = decode_splices(opt, gen, b, scan(opt, gen, b))
    of = oracle.OracleFasta(path)
    r = oracle.scan_fasta(oracle.params(), of, reads, [0] * 3, a_pos, b_aend, [False] * 3, [False] * 3,
                          use_fast=True)
    for i in range(3):
        assert r.n_ties[i] >= 1
        f = r.first[i]
        assert got[i] and (got[i][0].start, got[i][0].end, got[i][0].n_hits) == \
            (int(f["start"]), int(f["end"]), int(r.n_ties[i])), i
    assert int(r.first[0]["x"]) > 30000 and int(r.first[2]["x"]) > 32000
