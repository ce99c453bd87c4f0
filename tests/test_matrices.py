"""Matrix generators and layout helpers (CPU)."""
import os

import numpy as np
import pytest


@pytest.mark.parametrize("N", [1, 2, 5, 9])
def test_laplacians_match_oracle_kron(cal, ref, N):
    for mine, theirs in ((cal.matrices.laplacian_2d(N), ref.laplacian_2d(N)),
                         (cal.matrices.laplacian_3d(N), ref.laplacian_3d(N))):
        assert np.array_equal(mine.indptr, theirs.indptr)
        assert np.array_equal(mine.indices, theirs.indices)
        assert np.array_equal(mine.data, theirs.data)


def test_config_sizes(cal):
    # 3-D 215^3 has n = 9,938,375 and nnz = 69,291,275 (check via counts only)
    N = 215
    n = N ** 3
    nnz = 7 * n - 6 * N * N
    assert n == 9938375 and nnz == 69291275
    A = cal.matrices.laplacian_2d(1000)
    assert A.shape[0] == 1000000 and A.nnz == 4996000


def test_row_slabs(cal):
    A = cal.matrices.laplacian_3d(9)
    b = cal.matrices.slab_bounds(A.shape[0], 4, 81)
    assert b[0] == 0 and b[-1] == A.shape[0] and all(x % 81 == 0 for x in b)
    for r0, r1 in zip(b[:-1], b[1:]):
        rp, col, val = cal.matrices.laplacian_rows(3, 9, r0, r1)
        assert np.array_equal(col, A.indices[A.indptr[r0]:A.indptr[r1]])
        assert np.array_equal(val, A.data[A.indptr[r0]:A.indptr[r1]])
        assert np.array_equal(rp, A.indptr[r0:r1 + 1] - A.indptr[r0])


def test_matrix_market_roundtrip(cal, tmp_path):
    A = cal.matrices.laplacian_2d(6)
    p = os.path.join(tmp_path, "a.mtx")
    from scipy.io import mmwrite
    import scipy.sparse as sp
    mmwrite(p, sp.tril(A).tocoo(), symmetry="symmetric")
    B = cal.matrices.read_matrix_market(p)
    assert (A != B).nnz == 0


def test_diagonal_config1(cal):
    A = cal.matrices.diagonal(np.arange(1.0, 1001.0))
    assert A.nnz == 1000 and A[999, 999] == 1000.0
