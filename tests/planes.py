"""Test-side decoders for the device layouts of include/fc2_bp.h (independent of libfc2)."""
import numpy as np

CODE = np.frombuffer(b"ACGT", np.uint8)


def decode_genome(units: np.ndarray, nplane: np.ndarray, gstart: int, size: int) -> bytes:
    """Bases [0, size) of a chromosome starting at global base ``gstart``."""
    if size <= 0:
        return b""
    g = np.arange(gstart, gstart + size, dtype=np.uint64)
    u = (g >> np.uint64(6)).astype(np.int64)
    b = (g & np.uint64(63)).astype(np.uint64)
    lo = (units[2 * u] >> b) & np.uint64(1)
    hi = (units[2 * u + 1] >> b) & np.uint64(1)
    nn = (nplane[u] >> b) & np.uint64(1)
    out = CODE[(lo | (hi << np.uint64(1))).astype(np.int64)].copy()
    out[nn.astype(bool)] = ord('N')
    return out.tobytes()


def window(units, nplane, gstart, size, start, end) -> bytes:
    """get_data(start, end).upper() on a decoded chromosome, N outside [0, size)."""
    out = bytearray(b"N" * (end - start))
    a, b = max(start, 0), min(end, size)
    if b > a:
        out[a - start:b - start] = decode_genome(units, nplane, gstart + a, b - a)
    return bytes(out)


def _bits(words: np.ndarray, stride: int, n: int) -> np.ndarray:
    """[n, nwords*64] bit matrix of column-major u64 rows."""
    nwords = len(words) // stride
    m = np.ascontiguousarray(words.reshape(nwords, stride)[:, :n].T)      # [n, nwords]
    return np.unpackbits(m.view(np.uint8).reshape(n, nwords * 8), axis=1, bitorder="little")


def decode_reads_vec(words, nwords, stride, n, ls, has_n):
    """All internal read parts at once -> (uint8 [n, lmax] bytes matrix, lengths)."""
    ls = np.maximum(np.asarray(ls, np.int64), 0)
    lmax = int(ls.max()) if n else 0
    out = np.full((n, max(lmax, 1)), ord('N'), np.uint8)
    if lmax == 0:
        return out[:, :0], ls
    B = _bits(words, stride, n)
    j = np.arange(lmax)[None, :]
    valid = j < ls[:, None]
    lo = np.take_along_axis(B, np.minimum(j, B.shape[1] - 1).repeat(n, 0), axis=1)
    hi_idx = np.minimum(ls[:, None] + j, B.shape[1] - 1)
    hi = np.take_along_axis(B, hi_idx, axis=1)
    out = CODE[(lo | (hi << 1)).astype(np.int64)]
    NB = _bits(nwords, stride, n)[:, :lmax] if NB_needed(has_n) else None
    if NB is not None:
        nmask = NB.astype(bool) & np.asarray(has_n, bool)[:, None]
        out[nmask] = ord('N')
    out[~valid] = 0
    return out, ls


def NB_needed(has_n):
    return bool(np.any(has_n))


def decode_read(words: np.ndarray, nwords: np.ndarray, stride: int, i: int, l: int, has_n: bool) -> bytes:
    """Internal read part of pair i from its column-major tight bit rows."""
    if l <= 0:
        return b""
    rw = len(words) // stride
    bits = np.zeros(rw * 64, np.uint8)
    for j in range(rw):
        w = int(words[j * stride + i])
        bits[j * 64:(j + 1) * 64] = [(w >> k) & 1 for k in range(64)]
    lo = bits[:l]
    hi = bits[l:2 * l]
    out = CODE[(lo | (hi << 1)).astype(np.int64)].copy()
    if has_n:
        nw = len(nwords) // stride
        nb = np.zeros(nw * 64, np.uint8)
        for j in range(nw):
            w = int(nwords[j * stride + i])
            nb[j * 64:(j + 1) * 64] = [(w >> k) & 1 for k in range(64)]
        out[nb[:l].astype(bool)] = ord('N')
    return out.tobytes()
