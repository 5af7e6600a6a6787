"""CPU tests of the C ABI library (no GPU needed): load, exports, host-side FASTA
semantics vs the oracle, genome/pair packing round trips, byte-path arena."""
import ctypes
import os
import re
import shutil

import numpy as np
import pytest

import oracle
from conftest import GOLDEN, ROOT
from find_circ2_amd import _native as N
from oracle.bp_oracle import RefIndexedFasta
from planes import decode_genome, decode_read
from synth_small import load_genome, make_spans


@pytest.fixture(scope="module")
def L():
    N.build()
    return N.lib()


def test_exports_every_declared_symbol(L):
    import glob
    hdr = "".join(open(h).read() for h in sorted(glob.glob(os.path.join(ROOT, "include", "*.h"))))
    declared = set(re.findall(r"\b(fc2_[a-z0-9_]+)\s*\(", hdr))
    assert declared, "no declarations parsed"
    assert declared == set(N.EXPORTED), declared ^ set(N.EXPORTED)
    for name in declared:
        assert hasattr(L, name), name


def test_info_calls(L):
    assert L.fc2_abi_version() == 1
    c = ctypes.c_int(-1)
    assert L.fc2_device_count(ctypes.byref(c)) == 0 and c.value >= 0
    assert L.fc2_max_fast_l() == 510
    p = N.Params(15, 2, 2, 0, 0, 0, 0)
    rw, nw, tw = ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_uint32()
    assert L.fc2_batch_geometry(ctypes.byref(p), 100, ctypes.byref(rw), ctypes.byref(nw), ctypes.byref(tw)) == 0
    assert (rw.value, nw.value, tw.value) == (3, 2, 4)      # l=74: 148 bits, 74 bits, 75 x-bits
    assert L.fc2_batch_geometry(ctypes.byref(p), 150, ctypes.byref(rw), ctypes.byref(nw), ctypes.byref(tw)) == 0
    assert (rw.value, nw.value, tw.value) == (4, 2, 4)      # l=124
    # l = 63 / 127: the kernels write (l + 2 + 63) // 64 tie words per strand (r2 fix: was l + 1)
    for L_, t in ((26 + 62, 2), (26 + 63, 4), (26 + 127, 6), (26 + 126, 4)):
        assert L.fc2_batch_geometry(ctypes.byref(p), L_, ctypes.byref(rw), ctypes.byref(nw), ctypes.byref(tw)) == 0
        assert tw.value == t, (L_, tw.value)
    # asize <= margin is the reference's own (degenerate) search (find_circ.py:895), not an error
    e0 = N.Params(2, 2, 2, 0, 0, 0, 0)
    assert L.fc2_batch_geometry(ctypes.byref(e0), 100, ctypes.byref(rw), ctypes.byref(nw), ctypes.byref(tw)) == 0
    assert tw.value == 2 * ((100 + 2 + 63) // 64)
    bad = N.Params(2, 70000, 2, 0, 0, 0, 0)
    assert L.fc2_batch_geometry(ctypes.byref(bad), 100, None, None, None) == N.FC2_E_RANGE
    assert b"asize - margin" in L.fc2_last_error()


def _open(path, write_index=0):
    h = ctypes.c_void_p()
    rc = N.lib().fc2_fasta_open(path.encode(), write_index, ctypes.byref(h))
    return rc, h


def _chroms(h):
    L = N.lib()
    out = []
    for i in range(L.fc2_fasta_n_chrom(h)):
        nm, sz, of, ld, sk, rg = (ctypes.c_char_p(), ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64(),
                                  ctypes.c_int64(), ctypes.c_int())
        assert L.fc2_fasta_chrom(h, i, ctypes.byref(nm), ctypes.byref(sz), ctypes.byref(of), ctypes.byref(ld),
                                 ctypes.byref(sk), ctypes.byref(rg)) == 0
        out.append((nm.value.decode(), of.value, ld.value, sk.value, sz.value, rg.value))
    return out


def _pack(h):
    L = N.lib()
    nu, ncw = ctypes.c_uint64(), ctypes.c_uint64()
    n = L.fc2_fasta_n_chrom(h)
    cs = np.zeros(max(1, n), np.uint64)
    assert L.fc2_fasta_layout(h, ctypes.byref(nu), ctypes.byref(ncw), cs.ctypes.data) == 0
    units = np.zeros(2 * nu.value, np.uint64)
    npl = np.zeros(nu.value, np.uint64)
    nco = np.zeros(max(1, ncw.value), np.uint32)
    ne = ctypes.c_uint64()
    assert L.fc2_fasta_pack(h, units.ctypes.data, npl.ctypes.data, nco.ctypes.data, ctypes.byref(ne), 2) == 0
    return units, npl, nco, cs, ne.value


WEIRD_FASTA = (b">c1 some description\n"
               b"ACGTNacgtn\nRYKMacgtAC\nGT\n"
               b">c2\n"
               b"AAAAACCCCC\r\nGGGGGTTTTT\r\nNNNNNACGTA\r\nAC\r\n"
               b">c3\n"
               b"ACGTACGTAC\nACG\nTACGTAC\n"          # irregular: short middle line
               b">c4\n"
               b"acgtacgtacgtacgtacgtacgtacgtacgtacgtacgtacgtacgtacgtacgtacgtacgtacgtacgt")  # no newline


@pytest.mark.parametrize("fa", ["CDR1as_locus.fa", "test_ref.fa", "weird"])
def test_fasta_index_and_get_match_oracle(L, fa, tmp_path):
    if fa == "weird":
        path = str(tmp_path / "weird.fa")
        open(path, "wb").write(WEIRD_FASTA)
    else:
        path = str(tmp_path / fa)
        shutil.copy(os.path.join(GOLDEN, fa), path)
    rc, h = _open(path)
    assert rc == 0, L.fc2_last_error()
    ref = RefIndexedFasta(path)
    of = oracle.OracleFasta(path)
    got = _chroms(h)
    assert [g[0] for g in got] == of.names
    for name, ofs, ldata, skip, size, _ in got:
        r = ref.chrom_stats[name]
        assert (ofs, ldata, skip, size) == (r[0], r[1], r[2], r[4]), name
    rng = np.random.default_rng(7)
    buf = np.zeros(400, np.uint8)
    ln = ctypes.c_int64()
    for ci, (name, _, _, _, size, _) in enumerate(got):
        for _ in range(200):
            s = int(rng.integers(-30, size + 30))
            e = s + int(rng.integers(0, 90))
            assert L.fc2_fasta_get_upper(h, ci, s, e, buf.ctypes.data, 400, ctypes.byref(ln)) == 0
            mine = bytes(buf[:ln.value])
            assert mine == ref.get_data(name, s, e).upper(), (name, s, e)
            assert mine == of.get_upper(ci, s, e)
    L.fc2_fasta_close(h)


def test_index_file_roundtrip(L, tmp_path):
    path = str(tmp_path / "t.fa")
    open(path, "wb").write(WEIRD_FASTA)
    rc, h = _open(path, write_index=1)
    assert rc == 0
    L.fc2_fasta_close(h)
    written = open(path + ".byo_index").read()
    assert written == RefIndexedFasta(path).index_text()
    # a present index is used as is (find_circ.py:110-112)
    rc, h2 = _open(path)
    assert rc == 0
    ref = RefIndexedFasta(path)
    loaded = _chroms(h2)
    for name, ofs, ldata, skip, size, _ in loaded:
        r = ref.chrom_stats[name]
        assert (ofs, ldata, skip, size) == (r[0], r[1], r[2], r[4])
    # chromosome indices keep FASTA order whether or not the index file was there (the file
    # itself lists them by name)
    os.rename(path + ".byo_index", path + ".moved")
    rc, h3 = _open(path)
    assert rc == 0 and [c[0] for c in _chroms(h3)] == [c[0] for c in loaded]
    assert [c[1] for c in loaded] == sorted(c[1] for c in loaded)
    L.fc2_fasta_close(h2)
    L.fc2_fasta_close(h3)


def test_index_file_keeps_fasta_order(L, tmp_path):
    """The .byo_index lists chromosomes by name; indices must still follow the FASTA."""
    path = str(tmp_path / "u.fa")
    open(path, "wb").write(b">zeta\nACGTACGT\n>alpha\nGGGG\n>mid\nTTTTTT\n")
    rc, h = _open(path, write_index=1)
    built = [c[0] for c in _chroms(h)]
    L.fc2_fasta_close(h)
    assert built == ["zeta", "alpha", "mid"]
    assert [l.split("\t")[0] for l in open(path + ".byo_index")] == ["alpha", "mid", "zeta"]
    rc, h = _open(path)
    assert rc == 0 and [c[0] for c in _chroms(h)] == built
    L.fc2_fasta_close(h)


def test_malformed_fasta_errors(L, tmp_path):
    p = str(tmp_path / "dup.fa")
    open(p, "wb").write(b">a\nACGT\n>a\nACGT\n")
    rc, h = _open(p)
    assert rc == N.FC2_E_FORMAT
    p = str(tmp_path / "empty.fa")
    open(p, "wb").write(b">a\n>b\nACGT\n")
    rc, h = _open(p)
    assert rc == 0          # header without sequence before a header with none pending is fine
    rc, h = _open(str(tmp_path / "missing.fa"))
    assert rc == N.FC2_E_IO


@pytest.mark.parametrize("fa", ["CDR1as_locus.fa", "test_ref.fa", "weird"])
def test_genome_pack_roundtrip(L, fa, tmp_path):
    if fa == "weird":
        path = str(tmp_path / "weird.fa")
        open(path, "wb").write(WEIRD_FASTA)
    else:
        path = os.path.join(GOLDEN, fa)
    rc, h = _open(path)
    assert rc == 0
    units, npl, nco, cs, n_exo = _pack(h)
    ref = RefIndexedFasta(path)
    chroms = _chroms(h)
    exo_expected = 0
    for ci, (name, _, _, _, size, regular) in enumerate(chroms):
        want = ref.get_data(name, 0, size).upper()
        if regular == 1:
            got = decode_genome(units, npl, int(cs[ci]), size)
            exp = bytes(c if c in b"ACGTN" else ord('N') for c in want)
            assert got == exp, name
            exo_expected += sum(c not in b"ACGTN" for c in want)
        else:
            assert name == "c3"
            assert decode_genome(units, npl, int(cs[ci]), size) == b"N" * size
    assert n_exo == exo_expected
    # coarse map consistent with the N plane
    for blk in range((len(npl) + 15) // 16):
        anyn = bool(np.bitwise_or.reduce(npl[blk * 16:blk * 16 + 16]))
        assert bool((nco[blk >> 5] >> (blk & 31)) & 1) == anyn
    L.fc2_fasta_close(h)


def _pack_pairs(L, p, h, spans, chrom_idx):
    reads = [s.read_part for s in spans]
    lens = np.array([len(r) for r in reads], np.int64)
    off = np.zeros(len(reads), np.uint64)
    off[1:] = np.cumsum(lens[:-1])
    buf = np.frombuffer(b"".join(reads) + b"\0" * 16, np.uint8)
    hp = np.zeros(len(spans), N.PAIR_DTYPE)
    hp["a_pos"] = [s.a_pos for s in spans]
    hp["b_aend"] = [s.b_aend for s in spans]
    hp["chrom"] = chrom_idx
    hp["read_len"] = lens
    hp["flags"] = [(1 if s.is_backsplice else 0) | (2 if s.primary_reverse else 0) for s in spans]
    rw, nw, tw = ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_uint32()
    assert L.fc2_batch_geometry(ctypes.byref(p), int(lens.max()), ctypes.byref(rw), ctypes.byref(nw),
                                ctypes.byref(tw)) == 0
    stride = len(spans) + 3
    words = np.zeros(rw.value * stride, np.uint64)
    nwords = np.zeros(nw.value * stride, np.uint64)
    nbp = ctypes.c_uint64()
    rc = L.fc2_pack_pairs(ctypes.byref(p), h, len(spans), buf.ctypes.data, off.ctypes.data, hp.ctypes.data,
                          words.ctypes.data, rw.value, nwords.ctypes.data, nw.value, stride, ctypes.byref(nbp), 3)
    return rc, hp, words, nwords, stride, nbp.value, buf, off


def test_pair_pack_roundtrip(L):
    path = os.path.join(GOLDEN, "CDR1as_locus.fa")
    rc, h = _open(path)
    _pack(h)
    genome = load_genome(path)
    spans = make_spans(genome, 300, seed=5, p_readN=0.3, p_lower=0.3)
    # exotic bytes in a few reads
    for k in (3, 17, 101):
        s = spans[k]
        rp = bytearray(s.read_part)
        rp[len(rp) // 2] = ord('R')
        s.read_part = bytes(rp)
    p = N.Params(15, 2, 2, 0, 0, 0, 0)
    rc, hp, words, nwords, stride, nbp, _, _ = _pack_pairs(L, p, h, spans, [0] * len(spans))
    assert rc == 0, L.fc2_last_error()
    e = 13
    n_bp = 0
    for i, s in enumerate(spans):
        l = len(s.read_part) - 2 * e
        internal = s.read_part[e:len(s.read_part) - e].upper()
        flags = int(hp["flags"][i])
        if l < 0:
            assert flags & N.PAIR_BYTEPATH == 0
            continue
        exotic = any(c not in b"ACGTN" for c in internal)
        assert bool(flags & N.PAIR_BYTEPATH) == exotic, i
        if exotic:
            n_bp += 1
            continue
        assert bool(flags & N.PAIR_READ_N) == (b"N" in internal), i
        # a single 'N' travels in the record (FC2_PAIR_READ_N1 + npos); the N row is filled all the same
        single = internal.count(b"N") == 1 and internal.index(b"N") < 256
        assert bool(flags & N.PAIR_READ_N1) == single, i
        assert int(hp["npos"][i]) == (internal.index(b"N") if single else 0), i
        assert decode_read(words, nwords, stride, i, l, bool(flags & N.PAIR_READ_N)) == internal, i
    assert n_bp == nbp == 3
    L.fc2_fasta_close(h)


def test_pack_unknown_chrom_is_key_error(L):
    path = os.path.join(GOLDEN, "CDR1as_locus.fa")
    rc, h = _open(path)
    _pack(h)
    spans = make_spans(load_genome(path), 5, seed=9)
    p = N.Params(15, 2, 2, 0, 0, 0, 0)
    rc, *_ = _pack_pairs(L, p, h, spans, [0, 0, 7, 0, 0])
    assert rc == N.FC2_E_KEY and b"KeyError" in L.fc2_last_error()
    L.fc2_fasta_close(h)


def test_bytepath_arena_matches_reference_windows(L, tmp_path):
    path = str(tmp_path / "weird.fa")
    open(path, "wb").write(WEIRD_FASTA * 1)
    rc, h = _open(path)
    _pack(h)
    ref = RefIndexedFasta(path)
    chroms = _chroms(h)
    # pairs on every chrom, short reads (asize 5, margin 1 -> e 4)
    p = N.Params(5, 1, 2, 0, 0, 0, 0)
    from synth_small import SmallSpan
    spans, cidx = [], []
    rng = np.random.default_rng(3)
    for ci, (name, _, _, _, size, regular) in enumerate(chroms):
        for _ in range(6):
            L_ = int(rng.integers(8, 20))
            a = int(rng.integers(-2, size))
            b = int(rng.integers(0, size + 3))
            spans.append(SmallSpan(name, ci, a, a + 5, b - 5, b, bytes(rng.choice(list(b"ACGTNR"), L_)), False))
            cidx.append(ci)
        # both windows outside the chromosome: A's past its end, B's before its start (padded long)
        L_ = int(rng.integers(10, 20))
        spans.append(SmallSpan(name, ci, size + 2, size + 7, -40, -35, bytes(rng.choice(list(b"ACGT"), L_)), True))
        cidx.append(ci)
    rc, hp, words, nwords, stride, nbp, buf, off = _pack_pairs(L, p, h, spans, cidx)
    assert rc == 0, L.fc2_last_error()
    m, nb = ctypes.c_uint64(), ctypes.c_uint64()
    assert L.fc2_bytepath_size(ctypes.byref(p), len(spans), hp.ctypes.data, ctypes.byref(m), ctypes.byref(nb)) == 0
    assert m.value == nbp > 0
    idx = np.zeros(m.value, np.uint64)
    bp = np.zeros(m.value, N.PAIR_DTYPE)
    offs = np.zeros(m.value, np.uint64)
    arena = np.zeros(nb.value, np.uint8)
    assert L.fc2_bytepath_fill(ctypes.byref(p), h, len(spans), buf.ctypes.data, off.ctypes.data, hp.ctypes.data,
                               idx.ctypes.data, bp.ctypes.data, offs.ctypes.data, arena.ctypes.data) == 0
    e = 4
    for k in range(m.value):
        i = int(idx[k])
        s = spans[i]
        o = int(offs[k])
        lenI, lenA, lenB = np.frombuffer(arena[o:o + 12].tobytes(), np.int32)
        l = len(s.read_part) - 2 * e
        assert lenI == max(0, l)
        I = arena[o + 16:o + 16 + lenI].tobytes()
        assert I == s.read_part[e:len(s.read_part) - e].upper()
        if l >= 0:
            # header: the windows' full lengths; body: slots of l + 3 (A) and 2l + 3 (B) bytes holding
            # their first bytes
            sa, sb = l + 3, 2 * l + 3
            A = arena[o + 16 + lenI:o + 16 + lenI + min(lenA, sa)].tobytes()
            B = arena[o + 16 + lenI + sa:o + 16 + lenI + sa + min(lenB, sb)].tobytes()
            ra = ref.get_data(s.chrom, s.a_pos + e, s.a_pos + e + l + 2).upper()
            rb = ref.get_data(s.chrom, s.b_aend - e - l - 2, s.b_aend - e).upper()
            assert (lenA, lenB) == (len(ra), len(rb))
            assert A == ra[:sa] and B == rb[:sb]
    L.fc2_fasta_close(h)


def test_bytepath_arena_truncated_fasta(L, tmp_path):
    """A FASTA cut short after indexing (its .byo_index claims more bases, find_circ.py:110-112):
    windows near that end come back shorter than l + 2, windows before the start longer.  The arena's
    slots hold what the reference's string form can read (A[:l+3], B[:2l+3]), against the Python
    restatement reading the same index, and the C oracle honours the index as well."""
    from synth_small import SmallSpan, truncated_fasta
    path, gen = truncated_fasta(tmp_path)
    rc, h = _open(path)
    assert rc == 0
    _pack(h)
    ref = RefIndexedFasta(path, use_existing_index=True)
    of = oracle.OracleFasta(path)
    assert of.sizes == [len(gen["u1"]), len(gen["u2"]) + 60]
    p = N.Params(6, 1, 2, 0, 0, 0, 0)
    e = 5
    rng = np.random.default_rng(5)
    spans, cidx = [], []
    for _ in range(200):
        L_ = int(rng.integers(2 * e, 2 * e + 30))
        a = int(rng.integers(len(gen["u2"]) - 30, len(gen["u2"]) + 70)) - e
        b = int(rng.integers(-40, 20)) + e
        spans.append(SmallSpan("u2", 1, a, a + 3, b - 3, b, bytes(rng.choice(list(b"ACGT"), L_)), False))
        cidx.append(1)
    rc, hp, words, nwords, stride, nbp, buf, off = _pack_pairs(L, p, h, spans, cidx)
    assert rc == 0, L.fc2_last_error()
    m, nb = ctypes.c_uint64(), ctypes.c_uint64()
    assert L.fc2_bytepath_size(ctypes.byref(p), len(spans), hp.ctypes.data, ctypes.byref(m), ctypes.byref(nb)) == 0
    assert m.value == len(spans)
    idx = np.zeros(m.value, np.uint64)
    bp = np.zeros(m.value, N.PAIR_DTYPE)
    offs = np.zeros(m.value, np.uint64)
    arena = np.zeros(nb.value, np.uint8)
    assert L.fc2_bytepath_fill(ctypes.byref(p), h, len(spans), buf.ctypes.data, off.ctypes.data, hp.ctypes.data,
                               idx.ctypes.data, bp.ctypes.data, offs.ctypes.data, arena.ctypes.data) == 0
    n_short = 0
    for k in range(m.value):
        s = spans[int(idx[k])]
        o = int(offs[k])
        lenI, lenA, lenB = np.frombuffer(arena[o:o + 12].tobytes(), np.int32)
        l = len(s.read_part) - 2 * e
        sa, sb = l + 3, 2 * l + 3
        ra = ref.get_data("u2", s.a_pos + e, s.a_pos + e + l + 2).upper()
        rb = ref.get_data("u2", s.b_aend - e - l - 2, s.b_aend - e).upper()
        assert ra == of.get_upper(1, s.a_pos + e, s.a_pos + e + l + 2)
        assert (lenA, lenB) == (len(ra), len(rb))
        assert arena[o + 16 + lenI:o + 16 + lenI + min(lenA, sa)].tobytes() == ra[:sa]
        assert arena[o + 16 + lenI + sa:o + 16 + lenI + sa + min(lenB, sb)].tobytes() == rb[:sb]
        n_short += len(ra) < l + 2 < len(rb)
    assert n_short > 20
    L.fc2_fasta_close(h)


def test_shipped_library_has_no_tuning_state():
    """The shipped libfc2.so keeps no process-global knobs: fc2_set_tuning fails,
    fc2_get_tuning reports the fixed defaults; forms are chosen per call (FC2_BATCH_FORM_*)."""
    L = N.lib()
    for key in (1, 2, 3, 6, 7, 9, 10, 11, 13, 14):
        assert L.fc2_set_tuning(key, 0) == N.FC2_E_PARAM
    assert b"A/B builds" in L.fc2_last_error()
    defaults = {1: 1, 2: 1, 3: 2, 6: 2, 7: 2, 9: 0, 10: 0, 11: 1, 13: 512, 14: 3}
    for key, v in defaults.items():
        assert N.get_tuning(key) == v, key


def test_ctx_arguments_without_a_device(L):
    """fc2_ctx (include/fc2_ctx.h) checks its arguments before touching a device, and fails with
    FC2_E_HIP, not a crash, where no MI355X is visible (this container)."""
    c = ctypes.c_void_p()
    assert L.fc2_ctx_create(-1, ctypes.byref(c)) == N.FC2_E_PARAM
    assert L.fc2_ctx_create(0, None) == N.FC2_E_PARAM
    n = ctypes.c_int(0)
    assert L.fc2_device_count(ctypes.byref(n)) == 0
    if n.value == 0:
        assert L.fc2_ctx_create(0, ctypes.byref(c)) == N.FC2_E_HIP
        assert not c.value
    assert L.fc2_ctx_sync(None) == N.FC2_E_PARAM
    assert L.fc2_ctx_genome_load(None, None, 0) == N.FC2_E_PARAM
    assert L.fc2_ctx_last_error(None) == b""
    L.fc2_ctx_destroy(None)


def test_compact_scan_arguments_without_a_device(L):
    """fc2_bp_scan_compact_launch / fc2_host_device_pointer check their arguments before any HIP call:
    the compact forms are canonical-mode only, without --all-hits, width 2 or 4."""
    gv, bv = N.GenomeView(), N.BatchView()
    co = N.CompactOut(2, 0, None, None, None, None)
    assert L.fc2_bp_scan_compact_launch(ctypes.byref(N.Params(15, 2, 2, 0, 0, 0, 0)), None, ctypes.byref(bv),
                                        ctypes.byref(co), None) == N.FC2_E_PARAM
    for nc, ah in ((1, 0), (0, 1)):
        p = N.Params(15, 2, 2, nc, 0, ah, 0)
        assert L.fc2_bp_scan_compact_launch(ctypes.byref(p), ctypes.byref(gv), ctypes.byref(bv), ctypes.byref(co),
                                            None) == N.FC2_E_PARAM
    p = N.Params(15, 2, 2, 0, 0, 0, 0)
    for width in (0, 3, 8):
        bad = N.CompactOut(width, 0, None, None, None, None)
        assert L.fc2_bp_scan_compact_launch(ctypes.byref(p), ctypes.byref(gv), ctypes.byref(bv), ctypes.byref(bad),
                                            None) == N.FC2_E_PARAM
    assert L.fc2_bp_scan_compact_launch(ctypes.byref(p), ctypes.byref(gv), ctypes.byref(bv), ctypes.byref(co),
                                        None) == N.FC2_E_PARAM     # no esc_count
    d = ctypes.c_void_p()
    assert L.fc2_host_device_pointer(None, ctypes.byref(d)) == N.FC2_E_PARAM
