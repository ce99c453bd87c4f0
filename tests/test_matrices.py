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


def test_matrix_market_general_gz_pattern(cal, tmp_path):
    import gzip
    p = os.path.join(tmp_path, "g.mtx.gz")
    with gzip.open(p, "wt") as f:
        f.write("%%MatrixMarket matrix coordinate pattern general\n% comment\n3 3 4\n1 1\n2 3\n3 2\n3 3\n")
    B = cal.matrices.load_matrix(p)
    assert B.indices.dtype == np.int32
    assert np.array_equal(B.toarray(), [[1, 0, 0], [0, 0, 1], [0, 1, 1]])


def test_suitesparse_mat_problem_struct(cal, tmp_path):
    """load(...); A = Problem.A (test_restarted_ca_lanczos_all_matrices.m:25-26)."""
    import scipy.io
    import scipy.sparse as sp
    A = cal.matrices.laplacian_2d(7).tocsc()
    p = os.path.join(tmp_path, "lap.mat")
    scipy.io.savemat(p, {"Problem": {"A": A, "name": "lap7", "kind": "2D/3D problem"}})
    B = cal.matrices.load_matrix(p)
    assert (sp.csr_matrix(A) != B).nnz == 0 and B.has_sorted_indices
    with pytest.raises(ValueError):
        scipy.io.savemat(os.path.join(tmp_path, "x.mat"), {"B": np.eye(3)})
        cal.matrices.load_matrix(os.path.join(tmp_path, "x.mat"))
    with pytest.raises(ValueError):
        cal.matrices.load_matrix(os.path.join(tmp_path, "x.txt"))


def test_matrix_market_values_roundtrip_exactly(cal, tmp_path):
    import scipy.sparse as sp
    A = cal.matrices.circuit_like(12, seed=5)
    L = sp.tril(A).tocoo()
    p = os.path.join(tmp_path, "c.mtx")
    with open(p, "w") as f:
        f.write("%%%%MatrixMarket matrix coordinate real symmetric\n%d %d %d\n" % (A.shape[0], A.shape[1], L.nnz))
        np.savetxt(f, np.column_stack([L.row + 1, L.col + 1, L.data]), fmt="%d %d %.17g")
    B = cal.matrices.load_matrix(p)
    assert np.array_equal(A.indptr, B.indptr) and np.array_equal(A.indices, B.indices)
    assert np.array_equal(A.data, B.data)
