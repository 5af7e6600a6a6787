"""Sparse upload of the read N rows (hotpath.sparse_nrows / upload_nrows): the device rows must be
byte-identical to the dense rows fc2_pack_pairs writes, whose rows are zero for every pair without
FC2_PAIR_READ_N (CPU only: torch CPU tensors stand in for the device)."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

from find_circ2_amd import _native as N  # noqa: E402
from find_circ2_amd.hotpath import sparse_nrows, upload_nrows  # noqa: E402


@pytest.mark.parametrize("n,nw,p", [(0, 2, 0.1), (1, 1, 1.0), (1000, 2, 0.04), (777, 3, 0.5), (64, 8, 0.0)])
def test_sparse_rows_rebuild_dense_rows(n, nw, p):
    rng = np.random.default_rng(n * 7 + nw)
    stride = max(n, 1)
    hp = np.zeros(n, N.PAIR_DTYPE)
    flagged = rng.random(n) < p
    hp["flags"] = np.where(flagged, N.PAIR_READ_N, 0) | rng.choice([0, N.PAIR_BACKSPLICE], n)
    dense = rng.integers(0, 2**63, size=(nw, stride), dtype=np.int64)
    dense[:, :n][:, ~flagged] = 0                     # the packer's rows for pairs without an 'N'
    if n < stride:
        dense[:, n:] = 0
    idx, rows = sparse_nrows(hp, dense.view(np.uint64).ravel(), nw, stride)
    assert np.array_equal(idx, np.nonzero(flagged)[0])
    assert rows.shape == (nw, len(idx))
    got = upload_nrows(hp, dense.view(np.uint64).ravel(), nw, stride, "cpu")
    assert torch.equal(got, torch.from_numpy(dense.ravel()))


@pytest.mark.parametrize("rw,stride,tail_bits", [(3, 1000, 20), (3, 5, 32), (2, 17, 33), (1, 9, 10), (4, 1, 0)])
def test_read_rows_narrow_tail(rw, stride, tail_bits):
    """upload_read_rows sends the last row as uint32 only when every value fits, and the device
    rows equal the packed rows either way."""
    from find_circ2_amd.hotpath import narrow_tail, upload_read_rows
    rng = np.random.default_rng(rw * 100 + stride)
    w = rng.integers(0, 2**63, size=(rw, stride), dtype=np.int64).view(np.uint64)
    w[rw - 1] &= np.uint64((1 << tail_bits) - 1) if tail_bits < 64 else np.uint64(2**64 - 1)
    words = w.ravel()
    assert narrow_tail(words, rw, stride) == (rw > 1 and tail_bits <= 32 and True)
    got = upload_read_rows(words, rw, stride, "cpu")
    assert torch.equal(got, torch.from_numpy(words.view(np.int64)))
