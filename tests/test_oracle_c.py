"""The C/OpenMP restatement (oracle/c/ca_lanczos_omp.c: the bench's CPU
baseline) against the NumPy oracle and the analytic known answers.  CPU only."""
import numpy as np
import pytest


@pytest.fixture(scope="module")
def omp():
    from oracle import omp as o
    o.build()
    return o


@pytest.mark.parametrize("basis,tol", [("newton", 1e-12), ("monomial", 1e-8)])
def test_omp_matches_numpy_oracle(ref, omp, basis, tol):
    A = ref.laplacian_2d(32)
    r = ref.matlab_rand(1024)
    T, flags = omp.ca_lanczos(A, r, 8, 48, basis)
    exp = ref.ca_lanczos(A, r, 8, 48, basis, "local", diagnostics=False)
    assert flags == list(exp.reorth)
    # the s = 8 monomial basis amplifies rounding (kappa ~ 8^8)
    assert np.max(np.abs(T - exp.T)) <= tol * 8.0


def test_omp_lap3d_and_config1(ref, omp):
    A = ref.laplacian_3d(12)
    r = ref.matlab_rand(A.shape[0])
    T, flags = omp.ca_lanczos(A, r, 8, 40, "newton")
    exp = ref.ca_lanczos(A, r, 8, 40, "newton", "local", diagnostics=False)
    assert flags == list(exp.reorth) and np.max(np.abs(T - exp.T)) <= 1e-11 * 12.0
    # BASELINE config 1: diag(1:1000), r = ones, s = 4 monomial, 120 iterations
    import scipy.sparse as sp
    D = sp.csr_matrix(sp.diags(np.arange(1.0, 1001.0)))
    T, _ = omp.ca_lanczos(D, np.ones(1000), 4, 120, "monomial")
    exp = ref.ca_lanczos(D, np.ones(1000), 4, 120, "monomial", "local", diagnostics=False)
    w, we = np.sort(np.linalg.eigvals(T).real), np.sort(np.linalg.eigvals(exp.T).real)
    assert abs(w[-1] - we[-1]) < 1e-8 * 1000 and abs(w[0] - we[0]) < 1e-8 * 1000
    assert abs(w[-1] - 1000.0) < 1e-5 and abs(w[0] - 1.0) < 1e-5


def test_omp_multi_tile_tsqr_and_loop_timer(ref, omp):
    """n = 5041: three TSQR row tiles (2048, 2048, 945 rows), so the stacked-R
    tree and the ragged last tile of the out-of-place TSQR are exercised; the
    loop timer reports the outer loop of the last call."""
    A = ref.laplacian_2d(71)
    r = ref.matlab_rand(A.shape[0])
    T, flags = omp.ca_lanczos(A, r, 8, 56, "newton")
    exp = ref.ca_lanczos(A, r, 8, 56, "newton", "local", diagnostics=False)
    assert flags == list(exp.reorth)
    assert np.max(np.abs(T - exp.T)) <= 1e-12 * 8.0
    assert omp.loop_seconds() > 0.0
