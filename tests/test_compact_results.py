"""The 4- and 2-byte transfer forms of the results (include/fc2_bp.h "compact results").

CPU: fc2_result_expand against a numpy restatement of the packing rules, on words of every shape
the scan writes (no hit, '+' GTAG and '-' CTAC hits, error bits, ties) plus words that must escape
(4 B: x > 254, n_ties > 255, dist / ov > 15, a no-hit word with a strand bit; 2 B also x > 125,
n_ties > 16, dist / ov > 3, any error bit), and its refusal of escape lists that do not match the
escaped words.  GPU (tests/test_gpu_fullsize.py): the device packer on all 50M results of the bench
batch, both widths, expanded back bit for bit; tests/test_gpu_compact.py: the device words and escapes
equal these restatements word for word, on words that escape and on real results with escapes.
"""
import numpy as np
import pytest

from find_circ2_amd import Options, expand
from find_circ2_amd import _native as N

GTAG = 2 | 3 << 3 | 0 << 6 | 2 << 9
CTAC = 1 | 3 << 3 | 0 << 6 | 1 << 9


def words8(x, dist, ov, nt, info):
    return ((x.astype(np.int64) & 0xFFFF) | (dist.astype(np.int64) << 16) | (ov.astype(np.int64) << 24) |
            (nt.astype(np.int64) << 32) | (info.astype(np.int64) << 48))


def pack_restated(w):
    """numpy restatement of fc2::r32_pack + the round-trip test of fc2_result_compact_launch."""
    w = w.astype(np.uint64)
    x = (w & 0xFFFF).astype(np.uint16).view(np.int16).astype(np.int64)
    dist, ov = (w >> 16) & 0xFF, (w >> 24) & 0xFF
    nt, info = (w >> 32) & 0xFFFF, (w >> 48) & 0xFFFF
    c = (((x + 1) & 0xFF).astype(np.uint64) | ((nt & 0xFF) << 8) | ((dist & 0xF) << 16) | ((ov & 0xF) << 20) |
         (((info & 1) != 0).astype(np.uint64) << 24) | (((info & 0x2000) != 0).astype(np.uint64) << 25) |
         (((info & 0x4000) != 0).astype(np.uint64) << 26) | (((info & 0x8000) != 0).astype(np.uint64) << 27))
    # unpack
    cx = (c & 0xFF).astype(np.int64) - 1
    ui = (((c >> 25) & 1) * 0x2000) | (((c >> 26) & 1) * 0x4000) | (((c >> 27) & 1) * 0x8000)
    minus = (c >> 24) & 1
    hit_info = ui | minus | (np.where(minus == 1, CTAC, GTAG).astype(np.uint64) << 1)
    back = np.where(cx < 0, np.uint64(0xFFFF) | (ui << 48),
                    (cx.astype(np.uint64) & 0xFFFF) | (((c >> 16) & 0xF) << 16) | (((c >> 20) & 0xF) << 24) |
                    (((c >> 8) & 0xFF) << 32) | (hit_info << 48))
    esc = back != w
    c = np.where(esc, np.uint64(N.R32_ESCAPE), c).astype(np.uint32)
    idx = np.nonzero(esc)[0]
    e = np.zeros(len(idx), N.ESCAPE_DTYPE)
    e["index"] = idx
    e["result"] = w[idx].astype(np.int64).view(N.RESULT_DTYPE)
    return c, e


def pack16_restated(w):
    """numpy restatement of fc2::r16_pack / r16_unpack + the escape rule (width 2)."""
    w = w.astype(np.uint64)
    x = (w & 0xFFFF).astype(np.uint16).view(np.int16).astype(np.int64)
    dist, ov = (w >> 16) & 0xFF, (w >> 24) & 0xFF
    nt, info = (w >> 32) & 0xFFFF, (w >> 48) & 0xFFFF
    minus = (info & 1)
    c = np.where(x < 0, 0, ((x + 1) & 0x7F).astype(np.uint64) | (minus << 7) | ((dist & 3) << 8) | ((ov & 3) << 10) |
                 (((nt - 1) & 15) << 12)).astype(np.uint64)
    x1 = c & 0x7F
    m = (c >> 7) & 1
    hit = ((x1 - 1) & 0xFFFF) | (((c >> 8) & 3) << 16) | (((c >> 10) & 3) << 24) | ((((c >> 12) & 15) + 1) << 32) | \
        ((np.uint64(0x8000) | m | (np.where(m == 1, CTAC, GTAG).astype(np.uint64) << 1)) << 48)
    back = np.where(x1 == 0, np.uint64(0xFFFF) | (np.uint64(0x8000) << 48), hit)
    esc = (back != w) | (x1 == 0x7F)
    c = np.where(esc, np.uint64(N.R16_ESCAPE), c).astype(np.uint16)
    idx = np.nonzero(esc)[0]
    e = np.zeros(len(idx), N.ESCAPE_DTYPE)
    e["index"] = idx
    e["result"] = w[idx].astype(np.int64).view(N.RESULT_DTYPE)
    return c, e


def pack(w, width):
    return pack16_restated(w) if width == 2 else pack_restated(w)


def sample_words(n, seed):
    rng = np.random.default_rng(seed)
    kind = rng.integers(0, 10, n)
    x = rng.integers(0, 125, n)
    dist = rng.integers(0, 3, n)
    ov = rng.integers(0, 3, n)
    nt = rng.integers(1, 40, n)
    minus = rng.integers(0, 2, n)
    err = rng.choice([0, 0, 0, 0x2000, 0x4000], n)
    info = 0x8000 | err | minus | (np.where(minus == 1, CTAC, GTAG) << 1)
    w = words8(x, dist, ov, nt, info)
    nohit = kind < 4
    w[nohit] = words8(np.full(nohit.sum(), -1), np.zeros(nohit.sum()), np.zeros(nohit.sum()),
                      np.zeros(nohit.sum()), 0x8000 | err[nohit])
    # words that must escape
    odd = kind == 9
    k = np.nonzero(odd)[0]
    which = rng.integers(0, 5, len(k))
    x2, d2, o2, t2, i2 = x[k].copy(), dist[k].copy(), ov[k].copy(), nt[k].copy(), info[k].copy()
    x2[which == 0] = rng.integers(255, 32000, (which == 0).sum())
    t2[which == 1] = rng.integers(256, 60000, (which == 1).sum())
    d2[which == 2] = rng.integers(16, 255, (which == 2).sum())
    o2[which == 3] = rng.integers(16, 255, (which == 3).sum())
    i2[which == 4] = 0x8000 | 0x1 | (GTAG << 1)          # '-' with a '+' signal (--non-canonical only)
    w[k] = words8(x2, d2, o2, t2, i2)
    return w


@pytest.mark.parametrize("width", [4, 2])
@pytest.mark.parametrize("n,seed", [(0, 1), (1, 2), (1000, 3), (300_001, 4)])
def test_expand_restores_every_word(n, seed, width):
    w = sample_words(n, seed)
    c, e = pack(w, width)
    assert n < 1000 or 0 < len(e) < (n // 5 if width == 4 else n)
    rng = np.random.default_rng(seed)
    e = e[rng.permutation(len(e))]                     # escapes arrive in no particular order
    for threads in (1, 0):
        out = expand(Options(), c, e, n_threads=threads)
        assert np.array_equal(out, w)


@pytest.mark.parametrize("width", [4, 2])
def test_expand_refuses_mismatched_escapes(width):
    w = sample_words(5000, 9)
    c, e = pack(w, width)
    assert len(e) > 2
    with pytest.raises(Exception, match="escape"):
        expand(Options(), c, e[:-1])                    # an escaped word without its escape
    dup = e.copy()
    dup[1] = dup[0]
    with pytest.raises(Exception, match="escape"):
        expand(Options(), c, dup)                       # one word escaped twice, another not at all
    bad = e.copy()
    flagged = (c & 0x7F) == N.R16_ESCAPE if width == 2 else (c & N.R32_ESCAPE) != 0
    bad["index"][0] = np.nonzero(~flagged)[0][0]
    with pytest.raises(Exception, match="escape"):
        expand(Options(), c, bad)                       # an escape for a word that was not escaped
    with pytest.raises(Exception, match="canonical"):
        expand(Options(noncanonical=True), c, e)


def test_two_byte_form_holds_the_default_options_words():
    """Default options (margin 2, maxdist 2) at l <= 124: every canonical hit with n_ties <= 16 and
    every error-free miss fits 2 bytes; only error bits and ties beyond 16 escape."""
    rng = np.random.default_rng(5)
    n = 20000
    x = rng.integers(0, 125, n)
    minus = rng.integers(0, 2, n)
    info = 0x8000 | minus | (np.where(minus == 1, CTAC, GTAG) << 1)
    w = words8(x, rng.integers(0, 3, n), rng.integers(0, 3, n), rng.integers(1, 17, n), info)
    w[:5000] = words8(np.full(5000, -1), np.zeros(5000), np.zeros(5000), np.zeros(5000), np.full(5000, 0x8000))
    c, e = pack16_restated(w)
    assert len(e) == 0
    assert np.array_equal(expand(Options(), c, e), w)
