"""Householder TSQR on the device (tsqr.m:7-12) against the oracle's
``ref.tsqr`` (LAPACK QR + the sign fix), across conditioning.

Bars (tolerances written per test):
  * R: |R - R_ref| <= 20 m kappa u ||X|| (first-order perturbation bound of
    the unique positive-diagonal R);
  * Q: ||Q'Q - I|| <= 1e-13 for every kappa (Householder is unconditionally
    orthogonal -- CholQR2 is not beyond kappa ~ 1e8);
  * ||QR - X|| <= 1e-13 ||X||.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu
U = 2.0 ** -53


def _block(n, m, cond, seed):
    rng = np.random.RandomState(seed)
    A = rng.randn(n, m)
    Q, _ = np.linalg.qr(A)
    V, _ = np.linalg.qr(rng.randn(m, m))
    s = np.logspace(0, -np.log10(cond), m) if m > 1 else np.ones(1)
    return np.asfortranarray((Q * s) @ V.T)


def _check(cal, ref, X, cond):
    n, m = X.shape
    Q, R = cal.tsqr(X)
    Qr, Rr = ref.tsqr(X)
    nx = np.linalg.norm(X, 2)
    assert np.all(np.diag(R) >= 0) and np.allclose(R, np.triu(R), atol=0)
    assert np.linalg.norm(Q.T @ Q - np.eye(m), 2) <= 1e-13
    assert np.linalg.norm(Q @ R - X, 2) <= 1e-13 * nx
    assert np.max(np.abs(R - Rr)) <= 20 * m * cond * U * nx
    return Q, R


@pytest.mark.parametrize("cond", [1.0, 1e4, 1e8, 1e11, 1e14])
@pytest.mark.parametrize("m", [8, 16])
def test_tsqr_conditioning(cal, ref, m, cond):
    X = _block(50000, m, cond, seed=int(np.log10(cond)) + m)
    _check(cal, ref, X, cond)


# shapes: one tile, ragged last tile, several tree levels (m = 8: 512-row
# tiles -> n = 300001 takes 586 -> 10 -> 1 tiles), every register width
@pytest.mark.parametrize("n,m", [(1, 1), (7, 7), (100, 3), (511, 8), (513, 8), (300001, 8), (4096, 9),
                                 (100000, 12), (257, 16), (70001, 17), (20000, 24), (129, 32), (50000, 32)])
def test_tsqr_shapes(cal, ref, n, m):
    X = _block(n, m, 1e3, seed=n + m) if n >= m else None
    _check(cal, ref, X, 1e3)


def test_tsqr_zero_column_sign(cal, ref):
    """sign(0) = 0 (tsqr.m:9): an exactly zero column gets R(j,j) = 0, a zero
    row of R and a zero Q column.  The rows below are not unique for a
    rank-deficient X (any QR may route row j's content elsewhere), so only the
    leading rows are compared."""
    X = _block(3000, 6, 10.0, seed=5)
    X[:, 3] = 0.0
    Q, R = cal.tsqr(X)
    Qr, Rr = ref.tsqr(X)
    assert R[3, 3] == 0.0 and Rr[3, 3] == 0.0
    assert np.all(Q[:, 3] == 0.0) and np.all(R[3, :] == 0.0)
    assert np.max(np.abs(R[:3] - Rr[:3])) <= 1e-12 * np.linalg.norm(X, 2)


def test_tsqr_deterministic(cal):
    X = _block(200000, 8, 1e6, seed=9)
    Q1, R1 = cal.tsqr(X)
    Q2, R2 = cal.tsqr(X)
    assert np.array_equal(Q1, Q2) and np.array_equal(R1, R2)


def test_normalize_tsqr_rank(cal, ref):
    """normalize.m:13-24 on top of the Householder TSQR: the rank from svd(R)."""
    X = _block(20000, 8, 1e3, seed=11)
    X[:, 5] = X[:, 1] * 2.0 - X[:, 2]
    Q, R, rank = cal.normalize(X)
    Qr, Rr, rank_r = ref.normalize(X)
    assert rank == rank_r == 7
    assert np.linalg.norm(Q @ R - X, 2) <= 1e-13 * np.linalg.norm(X, 2)


@pytest.mark.parametrize("backend", ["tsqr", "cholqr2", "auto"])
def test_ca_lanczos_normalize_backends(cal, ref, backend):
    """The whole CA-Lanczos run with each normalize backend matches the oracle."""
    A = cal.matrices.laplacian_2d(32)
    r = ref.matlab_rand(A.shape[0])
    ctx = cal.Context(normalize=backend).set_matrix(A)
    out = cal.ca_lanczos_ex(A, r, 8, 80, "newton", "local", diagnostics=True, ctx=ctx)
    exp = ref.ca_lanczos(A, r, 8, 80, "newton", "local", diagnostics=True)
    nA = 8.0
    assert list(out.reorth) == list(exp.reorth)
    assert np.max(np.abs(out.T - exp.T)) <= 1e-9 * nA
    w = np.sort(np.linalg.eigvals(out.T).real)
    we = np.sort(np.linalg.eigvals(exp.T).real)
    assert abs(w[-1] - we[-1]) <= 1e-10 * nA and abs(w[0] - we[0]) <= 1e-10 * nA
    ctx.close()


@pytest.mark.parametrize("orth,tol", [("local", 0.0), ("full", -1.0)])
def test_tsqr_fold_declined_fallback(cal, ref, orth, tol):
    """The fused TSQR projectAndNormalize's fallback (blockorth.cpp pn_tsqr:
    a declined fold redoes the block on the explicit-Z path, i.e.
    projectAndNormalize.m:25-26,63-64 literally), forced through
    cal_set_tsqr_fold_tol: 0 declines every block that takes the second
    projection, a negative value every block.  'full' includes the in-place
    re-projection against all of Q (ca_lanczos.m:197, whose output aliases
    its input X) at k = 2, where the fold applies: the declined fold must not
    have stored its stale Q over X before the fallback reads X.  Same bars as
    the backend test, plus 'full''s orthogonality."""
    A = cal.matrices.laplacian_2d(32)
    r = ref.matlab_rand(A.shape[0])
    ctx = cal.Context(normalize="tsqr").set_matrix(A).set_tsqr_fold_tol(tol)
    f0 = ctx.tsqr_fold_stats()
    out = cal.ca_lanczos_ex(A, r, 8, 80, "newton", orth, diagnostics=True, ctx=ctx)
    f1 = ctx.tsqr_fold_stats()
    ctx.close()
    exp = ref.ca_lanczos(A, r, 8, 80, "newton", orth, diagnostics=True)
    runs, declined = f1["runs"] - f0["runs"], f1["declined"] - f0["declined"]
    if orth == "local":
        assert runs == 9 and declined == sum(out.reorth) > 0
    else:
        assert runs > 0 and declined == runs
    nA = 8.0
    assert list(out.reorth) == list(exp.reorth)
    assert np.max(np.abs(out.T - exp.T)) <= 1e-9 * nA
    w = np.sort(np.linalg.eigvals(out.T).real)
    we = np.sort(np.linalg.eigvals(exp.T).real)
    assert abs(w[-1] - we[-1]) <= 1e-10 * nA and abs(w[0] - we[0]) <= 1e-10 * nA
    if orth == "full":
        assert np.max(out.orth_err) < 1e-12


def test_tsqr_fold_tol_cannot_be_raised(cal):
    """the fold's acceptance threshold may only be lowered (more
    declines, each redone on the explicit-Z path); a tol above the default
    1e-14 would accept folds the default declines and is rejected."""
    ctx = cal.Context(normalize="tsqr")
    ctx.set_tsqr_fold_tol(1e-15)
    ctx.set_tsqr_fold_tol(1e-14)
    for bad in (1e-13, 1.0, float("inf"), float("nan")):
        with pytest.raises(cal.CalError):
            ctx.set_tsqr_fold_tol(bad)
    ctx.close()
