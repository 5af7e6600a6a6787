"""Helpers that put GPU results and oracle results side by side as numpy arrays."""
import numpy as np

import oracle
from find_circ2_amd import first_tie_arrays
from find_circ2_amd import _native as N

_RC = str.maketrans("ACGTN", "TGCAN")


def _gtag_strings(g12: np.ndarray) -> np.ndarray:
    codes = np.frombuffer(b"ACGTN???", np.uint8)
    g12 = g12.astype(np.int64)
    chars = np.stack([codes[(g12 >> (3 * k)) & 7] for k in range(4)], axis=1)
    return chars.copy().view("S4").ravel()


def gpu_arrays(options, host_pairs, res):
    a = first_tie_arrays(options, host_pairs, res)
    g = _gtag_strings(a["gtag12"])
    # the Splice signal of a '-' hit is rev_comp(gtag) (find_circ.py:949, 954)
    sig = np.array([s.decode()[::-1].translate(_RC) if m else s.decode() for s, m in zip(g, a["minus"])],
                   dtype=object)
    n_t = np.where(a["hit"], a["n_ties"], 0)
    return dict(n_ties=n_t, x=np.where(a["hit"], a["x"], -1), start=a["start"], end=a["end"],
                strand=np.where(a["minus"], "-", "+"), dist=a["dist"], ov=a["ov"], sig=sig,
                err_key=a["err_key"], err_win=a["err_win"], done=a["done"])


def oracle_arrays(r: oracle.OracleResult):
    f = r.first
    hit = r.n_ties > 0
    return dict(n_ties=np.where(hit, r.n_ties, 0), x=np.where(hit, f["x"], -1), start=f["start"], end=f["end"],
                strand=np.array([s.decode() for s in f["strand"]], dtype=object), dist=f["dist"], ov=f["ov"],
                sig=np.array([s.decode() for s in f["gtag"]], dtype=object),
                err_key=r.n_ties == -oracle.ORC_ERR_KEY, err_shape=r.n_ties == -oracle.ORC_ERR_SHAPE)


def assert_same(gpu, orc, mask=None, label=""):
    n = len(gpu["n_ties"])
    m = np.ones(n, bool) if mask is None else mask
    keyerr = orc["err_key"] & m
    assert np.array_equal(gpu["err_key"][m], orc["err_key"][m]), label + " KeyError flags differ"
    shape = orc.get("err_shape", np.zeros(n, bool)) & m
    assert np.array_equal(gpu["err_win"][m], shape[m]), label + " window/shape error flags differ"
    ok = m & ~keyerr & ~shape
    assert np.array_equal(gpu["n_ties"][ok], orc["n_ties"][ok]), _first_diff(gpu, orc, ok, "n_ties", label)
    hit = ok & (orc["n_ties"] > 0)
    for k in ("x", "start", "end", "dist", "ov"):
        assert np.array_equal(np.asarray(gpu[k])[hit], np.asarray(orc[k])[hit]), _first_diff(gpu, orc, hit, k, label)
    for k in ("strand", "sig"):
        a = np.asarray(gpu[k])[hit].astype(str)
        b = np.asarray(orc[k])[hit].astype(str)
        assert np.array_equal(a, b), _first_diff(gpu, orc, hit, k, label)
    return int(hit.sum())


def _first_diff(gpu, orc, m, k, label):
    idx = np.nonzero(m)[0]
    a = np.asarray(gpu[k])[idx]
    b = np.asarray(orc[k])[idx]
    bad = idx[np.nonzero(a.astype(str) != b.astype(str))[0]]
    if len(bad) == 0:
        return label + " " + k
    i = int(bad[0])
    return "%s field %s differs at pair %d: gpu=%s oracle=%s (gpu n_ties=%s x=%s; oracle n_ties=%s x=%s)" % (
        label, k, i, gpu[k][i], orc[k][i], gpu["n_ties"][i], gpu["x"][i], orc["n_ties"][i], orc["x"][i])
