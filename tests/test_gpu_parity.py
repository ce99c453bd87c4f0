"""GPU parity tests: the HIP path through the C ABI vs the oracle restatement.

Bars:
  * SpMV / matrix powers: bit-identical to the oracle's sequential CSR SpMV
    (same summation order, no FMA contraction);
  * tsqr/normalize/cholqr/project/projectAndNormalize: same R up to
    |dR| <= 1e-12 * ||X|| * kappa-scaled tolerance, Q orthonormal to 1e-13;
  * CA-Lanczos: identical reorthogonalisation flags, Newton shifts within
    1e-9 * ||A||, converged Ritz values within 1e-10 * ||A||, residual norms
    above 1e-10 within a factor 2 of the oracle's.
"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _lap2d(cal, N):
    return cal.matrices.laplacian_2d(N)


# ---------------------------------------------------------------- a1 - a4
@pytest.mark.parametrize("N", [1, 7, 32, 100])
def test_spmv_bitexact_lap2d(cal, ref, N):
    A = cal.matrices.laplacian_2d(N)
    v = ref.matlab_rand(N * N, seed=3) - 0.5
    assert np.array_equal(cal.SpMV(A, v), ref.SpMV(A, v))


def test_spmv_bitexact_lap3d(cal, ref):
    A = cal.matrices.laplacian_3d(20)
    v = ref.matlab_rand(A.shape[0], seed=4)
    assert np.array_equal(cal.SpMV(A, v), ref.SpMV(A, v))


def test_spmv_irregular_and_long_rows(cal, ref):
    import scipy.sparse as sp
    rng = np.random.RandomState(1)
    n = 3000
    B = sp.random(n, n, density=0.002, random_state=rng, format="csr")
    B = B + B.T
    # a few dense rows/cols (> 2048 nonzeros: the long-row path) and empty rows
    D = sp.lil_matrix((n, n))
    for r in (5, 1500):
        D[r, :] = rng.rand(n)
        D[:, r] = D[r, :].T
    A = (B + D.tocsr()).tocsr()
    A[17, :] = 0
    A[:, 17] = 0
    A.eliminate_zeros()
    A.sort_indices()
    v = rng.randn(n)
    assert np.array_equal(cal.SpMV(A, v), ref.SpMV(A, v))


@pytest.mark.parametrize("fmt", ["csr", "pattern"])
@pytest.mark.parametrize("kind,N", [("2d", 1), ("2d", 33), ("3d", 17), ("diag", 1000)])
def test_spmv_both_formats_bitexact(cal, ref, fmt, kind, N):
    A = {"2d": cal.matrices.laplacian_2d, "3d": cal.matrices.laplacian_3d}.get(kind, None)
    A = A(N) if A else cal.matrices.diagonal(np.arange(1.0, N + 1.0))
    ctx = cal.Context(spmv_format=fmt).set_matrix(A)
    assert ctx.spmv_format()[0] == fmt
    v = ref.matlab_rand(A.shape[0], seed=13) - 0.25
    assert np.array_equal(ctx.spmv(v), ref.SpMV(A, v))
    ctx.close()


@pytest.mark.parametrize("n", [401, 4000])
def test_spmv_pattern_pairs_irregular(cal, ref, n):
    """Row-pattern SpMV on a small-integer-valued irregular matrix (<= 8 per
    row, empty rows, odd n): pair patterns with merged entries and split
    pairs; non-finite values outside the rows' own entries must not leak."""
    import scipy.sparse as sp
    rng = np.random.RandomState(n)
    rows, cols = [], []
    for r in range(n):
        k = rng.randint(0, 5)
        for c in rng.randint(max(0, r - 40), min(n, r + 40), size=k):
            rows += [r, c]
            cols += [c, r]
    vals = rng.randint(-3, 4, size=len(rows)).astype(float)
    A = sp.csr_matrix((vals, (rows, cols)), shape=(n, n))
    A.sum_duplicates()
    A.data[A.data == 0] = 1.0
    A.sort_indices()
    if A.getnnz(axis=1).max() > 8:
        keep = A.getnnz(axis=1) <= 8
        A = sp.diags(keep.astype(float)) @ A @ sp.diags(keep.astype(float))
        A = A.tocsr()
        A.eliminate_zeros()
        A.sort_indices()
    ctx = cal.Context(spmv_format="pattern").set_matrix(A)
    assert ctx.spmv_format()[0] == "pattern"
    v = rng.randn(n)
    assert np.array_equal(ctx.spmv(v), ref.SpMV(A, v))
    # an inf in x only reaches the rows that reference it
    v[7] = np.inf
    got, exp = ctx.spmv(v), ref.SpMV(A, v)
    assert np.array_equal(np.isnan(got), np.isnan(exp))
    fin = np.isfinite(exp)
    assert np.array_equal(got[fin], exp[fin])
    ctx.close()


def test_pattern_format_falls_back_to_csr(cal):
    import scipy.sparse as sp
    A = sp.random(500, 500, density=0.1, random_state=np.random.RandomState(0), format="csr")
    A = (A + A.T).tocsr()  # rows of ~100 entries (> 32): no pattern table
    ctx = cal.Context().set_matrix(A)
    assert ctx.spmv_format()[0] == "csr"
    with pytest.raises(cal.CalError):
        cal.Context(spmv_format="pattern").set_matrix(A)


def test_ca_lanczos_format_invariant(cal, ref):
    """Bit-identical SpMV => the whole run is identical in both formats."""
    A = cal.matrices.laplacian_3d(12)
    r = ref.matlab_rand(A.shape[0])
    outs = []
    for fmt in ("csr", "pattern"):
        ctx = cal.Context(spmv_format=fmt).set_matrix(A)
        outs.append(cal.ca_lanczos_ex(A, r, 8, 40, "newton", "local", diagnostics=False, ctx=ctx))
        ctx.close()
    assert np.array_equal(outs[0].T, outs[1].T)
    assert np.array_equal(outs[0].Q, outs[1].Q)


def test_spmv_diag_config1(cal, ref):
    A = cal.matrices.diagonal(np.arange(1.0, 1001.0))
    v = np.ones(1000)
    assert np.array_equal(cal.SpMV(A, v), np.arange(1.0, 1001.0))


def test_matrix_powers_monomial_bitexact(cal, ref):
    A = cal.matrices.laplacian_2d(30)
    q = ref.matlab_rand(900)
    q = q / np.linalg.norm(q)
    assert np.array_equal(cal.matrix_powers_monomial(A, q, 8), ref.matrix_powers_monomial(A, q, 8))


def test_matrix_powers_newton_bitexact(cal, ref):
    A = cal.matrices.laplacian_3d(10)
    v = ref.matlab_rand(1000)
    lam = np.array([11.5, 0.3, 6.1, 2.2, 9.0, 4.4, 1.1, 7.7])
    for modifiedp in (0, 1):
        assert np.array_equal(cal.matrix_powers_newton(A, v, 8, lam, modifiedp),
                              ref.matrix_powers_newton(A, v, 8, lam, modifiedp))


def test_matrix_powers_newton_complex_modified(cal, ref):
    A = cal.matrices.laplacian_2d(12)
    v = ref.matlab_rand(144)
    lam = np.array([7.0, 3 + 0.5j, 3 - 0.5j, 1.0])
    assert np.array_equal(cal.matrix_powers_newton(A, v, 4, lam, 1), ref.matrix_powers_newton(A, v, 4, lam, 1))


# ---------------------------------------------------------------- a5 - a9
def _rand_block(n, m, seed, cond=1e3):
    rng = np.random.RandomState(seed)
    U, _ = np.linalg.qr(rng.randn(n, m))
    V, _ = np.linalg.qr(rng.randn(m, m))
    s = np.logspace(0, -np.log10(cond), m)
    return (U * s) @ V.T


@pytest.mark.parametrize("n,m,cond", [(1000, 8, 1e2), (5000, 9, 1e5), (777, 1, 1.0), (20000, 16, 1e6)])
def test_tsqr_normalize(cal, ref, n, m, cond):
    X = _rand_block(n, m, 5, cond)
    Q, R = cal.tsqr(X)
    Qr, Rr = ref.tsqr(X)
    assert np.all(np.diag(R) > 0)
    assert np.allclose(np.triu(R), R)
    assert np.max(np.abs(Q.T @ Q - np.eye(m))) < 1e-13
    assert np.max(np.abs(R - Rr)) <= 1e-13 * cond * np.linalg.norm(X, 2)
    assert np.max(np.abs(Q @ R - X)) <= 1e-13 * np.linalg.norm(X, 2)
    Qn, Rn, rank = cal.normalize(X)
    assert rank == ref.normalize(X)[2]


def test_cholqr(cal, ref):
    X = _rand_block(4000, 8, 2, 1e2)
    Q, R = cal.cholqr(X)
    Qr, Rr = ref.cholqr(X)
    assert np.max(np.abs(R - Rr)) < 1e-12
    assert np.max(np.abs(Q - Qr)) < 1e-11


def test_project_blocks(cal, ref):
    rng = np.random.RandomState(9)
    n = 3000
    Q1, _ = np.linalg.qr(rng.randn(n, 5))
    Q2, _ = np.linalg.qr(rng.randn(n, 3))
    X = rng.randn(n, 4)
    for doreorth in (False, True):
        Xg, Rg = cal.project([Q1, np.zeros((n, 0)), Q2], X, doreorth)
        Xr, Rr = ref.project([Q1, np.zeros((n, 0)), Q2], X, doreorth)
        assert np.max(np.abs(Xg - Xr)) < 1e-12
        assert np.max(np.abs(Rg[0] - Rr[0])) < 1e-12 and np.max(np.abs(Rg[2] - Rr[2])) < 1e-12
        assert Rg[1].shape == (0, 4)


@pytest.mark.parametrize("frac", [0.9, 0.1])
def test_project_and_normalize_one_block(cal, ref, frac):
    """frac = share of X inside span(Qp): 0.9 triggers the second pass."""
    rng = np.random.RandomState(11)
    n, w, m = 6000, 9, 8
    Qp, _ = np.linalg.qr(rng.randn(n, w))
    X = frac * Qp @ rng.randn(w, m) + (1 - frac) * rng.randn(n, m) / np.sqrt(n) * 3
    QZ, RZ, re, rank = cal.projectAndNormalize_ex([Qp], X)
    QZr, RZr, info = ref.projectAndNormalize_ex([Qp], X)
    assert re == info.reorth
    assert np.max(np.abs(RZ[0] - RZr[0])) < 1e-12
    assert np.max(np.abs(RZ[1] - RZr[1])) < 1e-11
    assert np.max(np.abs(QZ - QZr)) < 1e-10
    assert np.max(np.abs(QZ.T @ Qp)) < 1e-13


@pytest.mark.parametrize("n,w,m,frac", [(70001, 9, 8, 0.9), (1200001, 9, 8, 0.9), (1200001, 5, 4, 0.9),
                                        (300001, 9, 8, 0.1), (1200001, 3, 2, 0.1), (10001, 9, 8, 0.9),
                                        (257, 9, 8, 0.9)])
def test_project_and_normalize_fused_tsqr_tree(cal, ref, n, w, m, frac):
    """The fused TSQR projectAndNormalize (blockorth.cpp pn_tsqr_fold,
    tsqr_fold.hip) with several tiles on every tree level: 70001 rows = 274
    level-0 tiles, 5 level-1 tiles; 1.2 M rows = 4688 / 74 / 2 level tiles
    under the root; 10001 and 257 rows: 40 and 2 level-0 tiles under a root
    that stacks level 0 directly (k_fold_root on the first level); m < 8
    pads the stacked R factors.  Against the oracle's
    projectAndNormalize (explicit Z, Householder QR): RZ to 1e-11 (C) and
    1e-12 ||X|| (R), QZ orthonormal to 1e-13 and to Qp like the oracle's, the
    reorth flag identical; the fold ran and was not declined."""
    rng = np.random.RandomState(n % 1000 + m)
    Qp, _ = np.linalg.qr(rng.randn(n, w))
    X = frac * Qp @ rng.randn(w, m) + (1 - frac) * rng.randn(n, m) / np.sqrt(n) * 3
    ctx = cal.default_context()
    f0 = ctx.tsqr_fold_stats()
    QZ, RZ, re, rank = cal.projectAndNormalize_ex([Qp], X)
    f1 = ctx.tsqr_fold_stats()
    assert f1["runs"] == f0["runs"] + 1 and f1["declined"] == f0["declined"]
    QZr, RZr, info = ref.projectAndNormalize_ex([Qp], X)
    assert re == info.reorth
    assert np.max(np.abs(RZ[0] - RZr[0])) < 1e-11
    assert np.max(np.abs(RZ[1] - RZr[1])) <= 1e-12 * np.linalg.norm(X, 2)
    assert np.linalg.norm(QZ.T @ QZ - np.eye(m), 2) <= 1e-13
    assert np.max(np.abs(QZ.T @ Qp)) <= 10 * np.max(np.abs(QZr.T @ Qp)) + 1e-13
    assert np.max(np.abs(QZ - QZr)) < 1e-10


def test_project_and_normalize_two_blocks(cal, ref):
    rng = np.random.RandomState(12)
    n = 2000
    Q1, _ = np.linalg.qr(rng.randn(n, 6))
    Q2, _ = np.linalg.qr(rng.randn(n, 6))
    Q2 = Q2 - Q1 @ (Q1.T @ Q2)
    Q2, _ = np.linalg.qr(Q2)
    X = Q1 @ rng.randn(6, 4) * 5 + rng.randn(n, 4)
    QZ, RZ, re, _ = cal.projectAndNormalize_ex([Q1, Q2], X)
    QZr, RZr, info = ref.projectAndNormalize_ex([Q1, Q2], X)
    assert re == info.reorth
    for a, b in zip(RZ, RZr):
        assert np.max(np.abs(a - b)) < 1e-11


@pytest.mark.parametrize("n,widths,m", [(2000, (9, 9, 9), 8), (600001, (9, 9, 12, 5), 8),
                                          (300007, (20, 9, 16), 12), (70001, (16, 7), 16)])
def test_project_and_normalize_blocks_fused(cal, ref, n, widths, m):
    """Block MGS over several blocks (project.m): the update of block i and
    the Gram of block i + 1 run as one pass (k_apply_gram: [Q{i} | X] up to
    32 columns, X up to 16, Q{i+1} up to 16); heights past one grid stride of
    the kernel (262144 rows) and not a multiple of 64, the 8- and 16-column X
    layouts, 24- and 32-column P.  R blocks within 1e-11 of the oracle's,
    QZ within 1e-10, the same reorth decision."""
    rng = np.random.RandomState(len(widths) * 7 + m)
    Qs = []
    for w in widths:
        Q = rng.randn(n, w)
        for P in Qs:
            Q = Q - P @ (P.T @ Q)
        Qs.append(np.linalg.qr(Q)[0])
    X = sum(P @ rng.randn(P.shape[1], m) for P in Qs) * 3 + rng.randn(n, m)
    QZ, RZ, re, _ = cal.projectAndNormalize_ex(Qs, X)
    QZr, RZr, info = ref.projectAndNormalize_ex(Qs, X)
    assert re == info.reorth
    for a, b in zip(RZ, RZr):
        assert np.max(np.abs(a - b)) < 1e-11 * max(1.0, np.max(np.abs(b)))
    assert np.max(np.abs(QZ - QZr)) < 1e-10
    assert np.max(np.abs(QZ.T @ QZ - np.eye(m))) < 1e-13


# ---------------------------------------------------------------- a10 - a14
def _compare_lanczos(out, exp, normA, check_rn=True, t_blocks=None):
    """T is compared within 1e-9 ||A|| on its leading t_blocks x t_blocks
    blocks of s (None: the whole T).  A test limits t_blocks only where the
    ORACLE's own T moves by more than 1e-12 ||A|| under a 1e-15 relative
    perturbation of r ('local' orth after orthogonality is lost: ghost Ritz
    values make later blocks chaotic); the measured spread is in its
    docstring.  No test compares less than the first 2 blocks."""
    assert out.T.shape == exp.T.shape
    assert list(out.reorth) == list(exp.reorth)
    if len(exp.shifts):
        assert np.max(np.abs(out.shifts - exp.shifts)) <= 1e-9 * normA
    s = exp.Bk.shape[1]
    m = exp.T.shape[0] if t_blocks is None else min(max(2, t_blocks) * s, exp.T.shape[0])
    assert np.max(np.abs(out.T[:m, :m] - exp.T[:m, :m])) <= 1e-9 * normA
    # converged Ritz values of the final T
    w = np.sort(np.linalg.eigvals(out.T).real)
    we = np.sort(np.linalg.eigvals(exp.T).real)
    assert abs(w[-1] - we[-1]) <= 1e-10 * normA
    assert abs(w[0] - we[0]) <= 1e-10 * normA
    if check_rn:
        # largest Ritz pair's residual history (the reference's plotted metric)
        a, b = out.ritz_rnorm[:, 0], exp.ritz_rnorm[:, 0]
        big = b > 1e-10
        assert np.all(np.abs(np.log(a[big] / b[big])) < np.log(2.0))
        assert np.all(a[~big] < 1e-9)
        assert np.all(out.orth_err < 1e-6) == np.all(exp.orth_err < 1e-6)


def test_ca_lanczos_config1_monomial(cal, ref):
    A = cal.matrices.diagonal(np.arange(1.0, 1001.0))
    r = np.ones(1000)
    out = cal.ca_lanczos_ex(A, r, 4, 120, "monomial", "local")
    exp = ref.ca_lanczos(A, r, 4, 120, "monomial", "local")
    _compare_lanczos(out, exp, 1000.0)


@pytest.mark.parametrize("N,dim,it,t_blocks", [(32, 2, 80, None), (12, 3, 80, 8)])
def test_ca_lanczos_newton_local(cal, ref, N, dim, it, t_blocks):
    """lap2d 32^2: the whole 80 x 80 T (oracle spread 2e-15 ||A||).  lap3d
    12^3: the leading 8 of 10 blocks (oracle spread per block 5e-15 up to
    block 8, then 2e-11 and 2e-6 ||A||)."""
    A = cal.matrices.laplacian_2d(N) if dim == 2 else cal.matrices.laplacian_3d(N)
    r = ref.matlab_rand(A.shape[0])
    out = cal.ca_lanczos_ex(A, r, 8, it, "newton", "local")
    exp = ref.ca_lanczos(A, r, 8, it, "newton", "local")
    _compare_lanczos(out, exp, 4.0 * dim, t_blocks=t_blocks)


def test_ca_lanczos_newton_full(cal, ref):
    A = cal.matrices.laplacian_2d(24)
    r = ref.matlab_rand(A.shape[0])
    out = cal.ca_lanczos_ex(A, r, 8, 64, "newton", "full")
    exp = ref.ca_lanczos(A, r, 8, 64, "newton", "full")
    _compare_lanczos(out, exp, 8.0)
    assert np.max(out.orth_err) < 1e-12


@pytest.mark.parametrize("N,orth", [(24, "local"), (64, "full"), (40, "local"), (25, "local")])
def test_orth_err_deferred_wide_gram(cal, ref, monkeypatch, N, orth):
    """compute_orth_err (ca_lanczos.m:99-107) of every iteration from one
    block-upper Gram of Q(:,1:sk+1) at the flush (k_gram_wide, lanczos.cpp
    oe_flush; 'local' / 'full' only, Q's columns are final once written)
    against the per-iteration Grams (CAL_OE_DEFER=0) on the same run: the
    same dot products in another summation order.  s = 8, 15 outer
    iterations (121 columns, the bench's shape), 13.8 k / 262 k / 64 k /
    15.6 k rows (the last not a multiple of the kernel's 32-row steps); the
    40^3 case is also run with 14 iterations to a flush with fewer columns
    than the pinned shape."""
    A = cal.matrices.laplacian_3d(N)
    r = ref.matlab_rand(A.shape[0])
    its = [120, 112] if N == 40 else [120]
    for it in its:
        monkeypatch.delenv("CAL_OE_DEFER", raising=False)
        a = cal.ca_lanczos_ex(A, r, 8, it, "newton", orth)
        monkeypatch.setenv("CAL_OE_DEFER", "0")
        b = cal.ca_lanczos_ex(A, r, 8, it, "newton", orth)
        assert np.array_equal(a.T, b.T) and np.array_equal(a.ritz_rnorm, b.ritz_rnorm)
        assert a.orth_err.shape == b.orth_err.shape == (it // 8,)
        assert np.all(b.orth_err > 0)
        assert np.all(np.abs(a.orth_err - b.orth_err) <= 1e-15 + 1e-9 * b.orth_err), (a.orth_err, b.orth_err)
    if orth == "full":
        assert np.max(a.orth_err) < 1e-12


def test_ca_lanczos_bad_args(cal):
    A = cal.matrices.laplacian_2d(8)
    with pytest.raises(ValueError):
        cal.ca_lanczos(A, np.ones(64), 4, 16, "newton", "bogus")
    with pytest.raises(cal.CalError):
        cal.ca_lanczos(A, np.ones(64), 4, 16, "chebyshev", "local")
    with pytest.raises(cal.CalError):  # s > 31: s + 1 exceeds the 32-column TSQR tile
        cal.ca_lanczos(A, np.ones(64), 32, 64, "newton", "local")


@pytest.mark.gpu
def test_orth_coef_device_matches_host(cal, ref):
    """The block-orth s x s algebra on the device (k_orth_coef) reproduces the
    host path bit for bit: projectAndNormalize, normalize, a whole run."""
    rng = np.random.default_rng(7)
    n = 20000
    Qp, _ = np.linalg.qr(rng.standard_normal((n, 9)))
    X = rng.standard_normal((n, 8)) + Qp[:, :8] * 3.0
    ctx = cal.default_context()
    outs = []
    for where in ("device", "host"):
        ctx.set_orth_coef(where)
        outs.append((cal.projectAndNormalize_ex([Qp], X, True), cal.normalize(X[:, :8])))
    ctx.set_orth_coef("device")
    (pa, na), (pb, nb) = outs
    assert np.array_equal(pa[0], pb[0]) and pa[2] == pb[2]
    for a, b in zip(pa[1], pb[1]):
        assert np.array_equal(a, b)
    for a, b in zip(na, nb):
        assert np.array_equal(np.asarray(a), np.asarray(b))
    A = cal.matrices.laplacian_3d(12)
    r = ref.matlab_rand(A.shape[0])
    runs = []
    for where in ("device", "host"):
        c2 = cal.Context(orth_coef=where).set_matrix(A)
        runs.append(cal.ca_lanczos_ex(A, r, 8, 40, "newton", "local", diagnostics=False, ctx=c2))
        c2.close()
    assert np.array_equal(runs[0].T, runs[1].T)
    assert np.array_equal(runs[0].Q, runs[1].Q)
    assert np.array_equal(runs[0].reorth, runs[1].reorth)


@pytest.mark.gpu
def test_orth_coef_device_fallback(cal):
    """A block whose Gram is numerically singular makes the device Cholesky
    fail; the block is redone on the host path (shifted CholQR)."""
    rng = np.random.default_rng(3)
    n = 5000
    B = rng.standard_normal((n, 4))
    X = np.hstack([B, B @ rng.standard_normal((4, 4)) + 1e-12 * rng.standard_normal((n, 4))])
    ctx = cal.default_context()
    res = []
    for where in ("device", "host"):
        ctx.set_orth_coef(where)
        res.append(cal.normalize(X))
    ctx.set_orth_coef("device")
    assert np.array_equal(res[0][0], res[1][0]) and np.array_equal(res[0][1], res[1][1])
    assert res[0][2] == res[1][2]


def test_ca_lanczos_prefetch_invariant(cal, ref):
    """Diagnostics off enables the next step's matrix-powers prefetch (double-
    buffered V); diagnostics never feed back (ca_lanczos.m:228-236), so T and
    Q must be bit-identical to the non-prefetching run."""
    A = cal.matrices.laplacian_2d(40)
    r = ref.matlab_rand(A.shape[0], seed=21)
    ctx = cal.Context().set_matrix(A)
    a = cal.ca_lanczos_ex(A, r, 8, 64, "newton", "local", diagnostics=False, ctx=ctx)
    b = cal.ca_lanczos_ex(A, r, 8, 64, "newton", "local", diagnostics=True, ctx=ctx)
    ctx.close()
    assert np.array_equal(a.T, b.T) and np.array_equal(a.Q, b.Q)
    assert np.array_equal(a.reorth, b.reorth)


@pytest.mark.parametrize("orth", ["periodic", "selective"])
def test_ca_lanczos_periodic_selective(cal, ref, orth):
    """the periodic (omega recurrence + full reorthogonalisation)
    and selective (converged Ritz vectors locked into the projection)
    variants on the reference's own test input (test_convergence_diagonal_
    matrices.m:9-21: diag(linspace(1,100,500)), r = ones, newton), s = 8,
    240 iterations.  Bars: the same break decisions and locked-vector counts
    as the oracle, normest within 1e-10 relative, T within 1e-8 ||A||,
    the extreme Ritz values within 1e-10 ||A||, orthogonality kept."""
    import scipy.sparse as sp
    a = ref.matlab_linspace(1.0, 100.0, 500)
    A = sp.csr_matrix(sp.diags(a))
    r = np.ones(500)
    exp = ref.ca_lanczos(A, r, 8, 240, "newton", orth, diagnostics=True)
    out = cal.ca_lanczos_ex(A, r, 8, 240, "newton", orth, diagnostics=True)
    normA = 100.0
    assert abs(out.info["norm_A"] - exp.norm_A) <= 1e-10 * exp.norm_A
    assert out.info["n_orth_breaks"] == sum(exp.breaks)
    if orth == "selective":
        assert out.info["n_ritz_locked"] == exp.nritz[-1]
    assert list(out.reorth) == list(exp.reorth)
    assert np.max(np.abs(out.T - exp.T)) <= 1e-8 * normA
    w, we = np.sort(np.linalg.eigvals(out.T).real), np.sort(np.linalg.eigvals(exp.T).real)
    assert abs(w[-1] - we[-1]) <= 1e-10 * normA and abs(w[0] - we[0]) <= 1e-10 * normA
    assert np.max(out.orth_err) < 1e-6 and np.max(exp.orth_err) < 1e-6


def test_ca_lanczos_full_s4(cal, ref):
    """'full' orthogonalisation at s = 4 on the restart test's matrix
    (diag(linspace(1,1e4,5000)), r = ones, 60 steps): projection widths 5 ..
    57, i.e. the row-apply shapes (9, 4) and (17, 4) and the wide Grams.  T
    against the oracle (_compare_lanczos), orthogonality at rounding level."""
    import scipy.sparse as sp
    a = ref.matlab_linspace(1.0, 1.0e4, 5000)
    A = sp.csr_matrix(sp.diags(a))
    r = np.ones(5000)
    out = cal.ca_lanczos_ex(A, r, 4, 60, "newton", "full")
    exp = ref.ca_lanczos(A, r, 4, 60, "newton", "full")
    # the prologue's Ritz values are symmetric about the spectrum's centre, so
    # the Leja order has exact ties that rounding breaks either way: the same
    # shifts, possibly in another order (hence another basis; T is basis-free)
    assert np.allclose(np.sort(out.shifts), np.sort(exp.shifts), rtol=0, atol=1e-9 * 1.0e4)
    assert list(out.reorth) == list(exp.reorth)
    assert np.max(np.abs(out.T - exp.T)) <= 1e-9 * 1.0e4
    assert np.max(out.orth_err) < 1e-12


@pytest.mark.parametrize("s", [2, 3, 5, 6])
def test_ca_lanczos_full_block_sizes(cal, ref, s):
    """'full' orthogonalisation at s = 2, 3, 5, 6 (lap2d 24^2, 8 blocks): every
    (projection columns, outputs) shape the device block orthogonalisation
    reaches on the way from 1 to 9 projection columns.  Shifts as a set (Leja
    ties on the symmetric spectrum), flags, T to 1e-9 ||A||, orthogonality."""
    A = cal.matrices.laplacian_2d(24)
    r = ref.matlab_rand(A.shape[0])
    out = cal.ca_lanczos_ex(A, r, s, 8 * s, "newton", "full")
    exp = ref.ca_lanczos(A, r, s, 8 * s, "newton", "full")
    assert np.allclose(np.sort(out.shifts), np.sort(exp.shifts), rtol=0, atol=1e-9 * 8.0)
    assert list(out.reorth) == list(exp.reorth)
    assert np.max(np.abs(out.T - exp.T)) <= 1e-9 * 8.0
    assert np.max(out.orth_err) < 1e-12


def test_restarted_ca_lanczos(cal, ref):
    """the explicit restart driver on the reference's own input
    (test_restart_diagonal_matrices.m:8-28: diag(linspace(1,1e4,5000)),
    r = ones, max_lanczos 60, 10 wanted, s = 4, newton, 'full', tol 1e-8).
    Known answer: the 10 largest diagonal entries; the oracle's eigenvalues;
    the converged vectors orthonormal eigenvectors.  The restart count is
    ill-conditioned here (ten wanted eigenvalues 2 apart at tol 1e-8): over
    98 start vectors ones .* (1 + 1e-15 randn) the oracle takes 90..122
    restarts (median 95; tests/golden/restart_spread_diag5000.json, made by
    make_restart_spread.py), and its own count for r = ones moves with the
    BLAS thread count (93 / 94).  So the count is held as a distribution:
    the device's median over the first 12 of those start vectors lies within
    the oracle's 10..90 % range, and every device count (r = ones included)
    within [80, 170] (the device, like the oracle, has rare short and long
    runs: 82..125 over 32 seeds with either Gram kernel)."""
    import json
    import os
    import scipy.sparse as sp
    a = ref.matlab_linspace(1.0, 1.0e4, 5000)
    A = sp.csr_matrix(sp.diags(a))
    r = np.ones(5000)
    exp = ref.restarted_ca_lanczos(A, r, 60, 10, 4, "newton", "full", 1.0e-8)
    out = cal.restarted_ca_lanczos(A, r, 60, 10, 4, "newton", "full", 1.0e-8)
    assert out["converged"] and exp["converged"]
    assert exp["num_restarts"] in (93, 94)
    assert 80 <= out["num_restarts"] <= 170
    eref = a[::-1][:10]
    assert np.max(np.abs(out["conv_eigs"] - eref)) <= 1e-8 * 1.0e4
    assert np.max(np.abs(out["conv_eigs"] - exp["conv_eigs"])) <= 1e-9 * 1.0e4
    V = out["Q_conv"]
    assert np.max(np.abs(V.T @ V - np.eye(10))) < 1e-8
    res = np.linalg.norm(A @ V - V * out["conv_eigs"], axis=0) / np.abs(out["conv_eigs"])
    assert np.max(res) < 1e-6
    assert np.max(out["orth_err"]) < 1e-10
    spread = np.array(json.load(open(os.path.join(os.path.dirname(__file__), "golden",
                                                  "restart_spread_diag5000.json")))["counts"])
    dev = []
    for seed in range(12):
        rng = np.random.RandomState(seed)
        o = cal.restarted_ca_lanczos(A, np.ones(5000) * (1 + 1e-15 * rng.randn(5000)), 60, 10, 4, "newton", "full",
                                     1.0e-8)
        assert o["converged"]
        assert np.max(np.abs(o["conv_eigs"] - eref)) <= 1e-8 * 1.0e4
        dev.append(o["num_restarts"])
    lo, hi = np.percentile(spread, [10, 90])
    print("restarts: device %d (r = ones), %s (perturbed; median %.1f), oracle %d, oracle 10..90 %%: %.1f..%.1f"
          % (out["num_restarts"], dev, np.median(dev), exp["num_restarts"], lo, hi))
    assert lo <= np.median(dev) <= hi
    assert all(80 <= d <= 170 for d in dev)


def test_restarted_ca_lanczos_local_lap2d(cal, ref):
    """'local' restart on a 2-D Laplacian: the 4 largest eigenvalues (closed form)."""
    A = cal.matrices.laplacian_2d(30)
    r = ref.matlab_rand(900, seed=2)
    exp = ref.restarted_ca_lanczos(A, r, 48, 4, 8, "newton", "local", 1.0e-8)
    out = cal.restarted_ca_lanczos(A, r, 48, 4, 8, "newton", "local", 1.0e-8)
    eref = ref.laplacian_2d_eigs(30)[::-1]
    assert out["converged"] == exp["converged"]
    if out["converged"]:
        assert np.max(np.abs(out["conv_eigs"] - eref[:4])) <= 1e-7 * 8.0
    # 'local' keeps no global orthogonality and lap2d has a double eigenvalue,
    # so the restart count is a chaotic function of rounding: a 1e-15 relative
    # perturbation of r moves the oracle itself between 9 and 10 restarts.
    # Parity is the oracle's spread over ulp-perturbed start vectors.
    rng = np.random.default_rng(0)
    counts = {exp["num_restarts"]}
    for _ in range(5):
        rp = r * (1.0 + 1.0e-15 * rng.standard_normal(r.shape[0]))
        counts.add(ref.restarted_ca_lanczos(A, rp, 48, 4, 8, "newton", "local", 1.0e-8)["num_restarts"])
    assert min(counts) <= out["num_restarts"] <= max(counts), (out["num_restarts"], counts)


# ---- implicit restart (parity unpinned: vs the oracle's IRL,
# analytic spectra and eigsh) ----------------------------------------------

def _irl_check(cal, ref, A, r, ml, nw, s, basis, eref, rel, same_restarts=True):
    exp = ref.impl_restarted_ca_lanczos(A, r, ml, nw, s, basis, "full", 1.0e-8)
    out = cal.impl_restarted_ca_lanczos(A, r, ml, nw, s, basis, "full", 1.0e-8)
    assert out["converged"] and exp["converged"]
    if same_restarts:   # the estimates clear tol by >= 2x either side (oracle)
        assert out["num_restarts"] == exp["num_restarts"]
    scale = abs(eref[0])
    assert np.max(np.abs(out["conv_eigs"] - eref[:nw])) <= rel * scale
    assert np.max(np.abs(out["conv_eigs"] - exp["conv_eigs"])) <= rel * scale
    V = out["Q_conv"]
    assert np.max(np.abs(V.T @ V - np.eye(nw))) < 1e-9
    res = np.linalg.norm(A @ V - V * out["conv_eigs"], axis=0) / np.abs(out["conv_eigs"])
    assert np.max(res) < 1e-7
    assert np.max(out["ritz_est"][-1]) < 1.0e-8 * out["norm_A"]
    return out, exp


def test_impl_restarted_diagonal(cal, ref):
    """diag(linspace(1,1e4,5000)), r = ones (test_restart_diagonal_matrices.m
    input), 60 vectors, 8 wanted, s = 4 Newton: the top 8 diagonal entries,
    the oracle's restart count (14)."""
    import scipy.sparse as sp
    a = ref.matlab_linspace(1.0, 1.0e4, 5000)
    A = sp.csr_matrix(sp.diags(a))
    out, exp = _irl_check(cal, ref, A, np.ones(5000), 60, 8, 4, "newton", a[::-1], 1e-12)
    assert out["num_restarts"] == 14


def test_impl_restarted_many_wanted_copy_path(cal, ref):
    """14 wanted (k = 18 kept vectors): the restart's [V_k | r] has more than
    16 outputs, so it is formed in the work panel and copied back (the in-place
    path takes <= 16, lanczos.cpp); the top 14 diagonal entries and the
    oracle's eigenvalues."""
    import scipy.sparse as sp
    a = ref.matlab_linspace(1.0, 1.0e4, 5000)
    A = sp.csr_matrix(sp.diags(a))
    _irl_check(cal, ref, A, np.ones(5000), 64, 14, 4, "newton", a[::-1], 1e-12, same_restarts=False)


def test_impl_restarted_truncated_monomial(cal, ref):
    """m = 60 with s = 8 (first pass truncated from 64 vectors), monomial basis."""
    import scipy.sparse as sp
    a = ref.matlab_linspace(1.0, 1.0e4, 5000)
    A = sp.csr_matrix(sp.diags(a))
    _irl_check(cal, ref, A, np.ones(5000), 60, 8, 8, "monomial", a[::-1], 1e-10)


def test_impl_restarted_lap2d_multiplicity(cal, ref):
    """lap2d(40) (double eigenvalues): every returned value is an eigenvalue
    of A (closed form), the largest one is found, the Ritz vectors are
    orthonormal eigenvectors.  A single-vector Krylov space sees the second
    copy of a double eigenvalue only through rounding, so neither the
    multiplicities nor the restart count are compared with the oracle's."""
    A = cal.matrices.laplacian_2d(40)
    eref = ref.laplacian_2d_eigs(40)[::-1]
    out = cal.impl_restarted_ca_lanczos(A, ref.matlab_rand(1600), 48, 8, 8, "newton", "full", 1.0e-8)
    assert out["converged"]
    ev = out["conv_eigs"]
    assert np.max(np.min(np.abs(ev[:, None] - eref[None, :]), axis=1)) <= 1e-10 * 8.0
    assert abs(ev[0] - eref[0]) <= 1e-10 * 8.0 and np.all(np.diff(ev) <= 0)
    V = out["Q_conv"]
    assert np.max(np.abs(V.T @ V - np.eye(8))) < 1e-9
    assert np.max(np.linalg.norm(A @ V - V * ev, axis=0)) < 1e-6


def test_impl_restarted_circuit_vs_eigsh(cal, ref):
    """Irregular SPD resistor network (the G3_circuit stand-in of BASELINE
    config 5) against scipy eigsh."""
    from scipy.sparse.linalg import eigsh
    A = cal.matrices.circuit_like(60)
    ev = np.sort(eigsh(A, k=8, which="LA", tol=1e-13)[0])[::-1]
    _irl_check(cal, ref, A, np.ones(A.shape[0]), 64, 8, 8, "newton", ev, 1e-11)


def test_impl_restarted_rejects(cal, ref):
    A = cal.matrices.laplacian_2d(20)
    r = np.ones(400)
    for o in ("local", "periodic", "selective"):
        with pytest.raises(cal.CalError) as ei:
            cal.impl_restarted_ca_lanczos(A, r, 40, 4, 4, "newton", o)
        assert ei.value.status == cal._lib.CAL_ERR_UNSUPPORTED
    with pytest.raises(cal.CalError):
        cal.impl_restarted_ca_lanczos(A, r, 40, 4, 4, "newton", "bogus")
    with pytest.raises(cal.CalError):
        cal.impl_restarted_ca_lanczos(A, r, 12, 8, 4, "newton", "full")


@pytest.mark.parametrize("s,basis", [(1, "newton"), (2, "monomial"), (3, "newton"), (5, "newton"), (6, "monomial"),
                                     (9, "newton"), (12, "newton"), (15, "newton"), (16, "newton"),
                                     (20, "newton"), (24, "newton")])
def test_ca_lanczos_block_sizes(cal, ref, s, basis):
    """Block sizes 1 <= s <= 24 (the ABI takes s <= 31): s + 1 > 9 leaves the
    device-coefficient fast path for the generic sweeps; s + 1 > 16 takes the
    Householder TSQR normalize (32-column tiles); s = 1 is plain Lanczos with
    one-column blocks.  s = 4, 8, 12, 16 with 120 steps is the reference's
    own harness (test_ca_lanczos.m:29-41).  Same bars as the s = 4 / 8 cases;
    T on the whole matrix for s <= 9 (oracle spread <= 6e-13 ||A||), on the
    leading blocks where the oracle's own spread stays <= 3e-12 ||A|| for
    s >= 12 (measured per block: s = 12 up to block 6, then 1e-10, 2e-3;
    s = 15, 16 up to 5, then 5e-8 / 2e-3; s = 20 up to 4... 3e-12 at 4,
    then 0.2; s = 24 up to 2, then 7e-12, 1e-2)."""
    N = 20
    A = cal.matrices.laplacian_2d(N)
    r = ref.matlab_rand(N * N)
    # at most 8 outer iterations: 'local' loses orthogonality on this 400-row
    # problem and by k ~ 10 the reorth test sits on its 0.5 threshold
    it = min(120, 8 * s) if s >= 12 else s * 5
    out = cal.ca_lanczos_ex(A, r, s, it, basis, "local")
    exp = ref.ca_lanczos(A, r, s, it, basis, "local")
    _compare_lanczos(out, exp, 8.0, t_blocks={12: 6, 15: 5, 16: 5, 20: 4, 24: 2}.get(s))


@pytest.mark.parametrize("s,basis", [(2, "monomial"), (4, "monomial"), (4, "newton")])
@pytest.mark.parametrize("start", ["e1", "two"])
def test_ca_lanczos_exhausted_krylov_space(cal, ref, s, basis, start):
    """A start vector inside a 1- or 2-dimensional invariant subspace exhausts
    the Krylov space inside the first block: R of normalize is singular
    (normalize.m:18-35 only flags the rank) and ca_lanczos.m:176-223 then
    divides by it.  The oracle raises on these inputs (MATLAB warns and
    returns Inf/NaN); the HIP path must not hand back an unflagged T: it
    either raises with a negative status or reports the rank deficiency /
    breakdown in info."""
    n = 100
    A = cal.matrices.diagonal(np.arange(1.0, n + 1.0))
    r = np.eye(n)[0] + (np.eye(n)[5] if start == "two" else 0.0)
    with pytest.raises(np.linalg.LinAlgError):
        ref.ca_lanczos(A, r, s, 3 * s, basis, "local", diagnostics=False)
    try:
        out = cal.ca_lanczos_ex(A, r, s, 3 * s, basis, "local", diagnostics=False)
    except cal.CalError as e:
        assert e.status < 0
        return
    assert out.info["n_rank_deficient"] >= 1 or out.info["breakdown"] == 1, (out.info, np.isfinite(out.T).all())


@pytest.mark.parametrize("basis", ["newton", "monomial"])
def test_matrix_powers_split_schedule(cal, ref, monkeypatch, basis):
    """The multi-GPU matrix-powers schedule on one rank (CAL_MPK_FAKE_BAND):
    each power as its interior range, then both boundary pieces in one
    two-range pair-kernel launch.  No exchange is involved, so the powers
    and the whole CA-Lanczos run must keep the unsplit bits."""
    N, s = 30, 8
    A = cal.matrices.laplacian_3d(N)
    n = A.shape[0]
    v = ref.matlab_rand(n, seed=3)
    r = ref.matlab_rand(n)
    lam = np.linspace(0.5, 11.5, s)

    def run():
        ctx = cal.Context().set_matrix(A)
        V = (cal.matrix_powers_newton(A, v, s, lam, 1, ctx=ctx) if basis == "newton"
             else cal.matrix_powers_monomial(A, v / np.linalg.norm(v), s, ctx=ctx))
        out = cal.ca_lanczos_ex(A, r, s, 4 * s, basis, "local", diagnostics=False, ctx=ctx)
        ctx.close()
        return V, out

    V0, o0 = run()
    # the stencil's band, and wider ones (odd: ragged even rounding); a fake
    # band below the matrix's own would read unfinished rows by design
    for band in (N * N, N * N + 1, 3 * N * N + 7):
        monkeypatch.setenv("CAL_MPK_FAKE_BAND", str(band))
        V1, o1 = run()
        assert np.array_equal(V1, V0), band
        assert np.array_equal(o1.T, o0.T) and list(o1.reorth) == list(o0.reorth), band
    monkeypatch.delenv("CAL_MPK_FAKE_BAND")
    if basis == "newton":
        assert np.array_equal(V0, ref.matrix_powers_newton(A, v, s, lam, 1))


def test_matrix_powers_split_schedule_row_kernel(cal, ref, monkeypatch):
    """The split schedule when the pair kernel does not apply (27-point
    stencil: rows of 27 entries, beyond the pair kernel's 8): the two-range
    launch falls back to two row-kernel launches.  Same bits as unsplit."""
    import scipy.sparse as sp
    N, s = 24, 8
    T = sp.diags([np.ones(N - 1), 4.0 * np.ones(N), np.ones(N - 1)], [-1, 0, 1])
    A = sp.kron(sp.kron(T, T), T).tocsr()
    A.sort_indices()
    n = A.shape[0]
    v = ref.matlab_rand(n, seed=4)
    lam = np.linspace(8.5, 200.0, s)

    def run():
        ctx = cal.Context().set_matrix(A)
        assert ctx.spmv_format()[0] == "pattern"
        V = cal.matrix_powers_newton(A, v, s, lam, 1, ctx=ctx)
        ctx.close()
        return V

    V0 = run()
    monkeypatch.setenv("CAL_MPK_FAKE_BAND", str(N * N + N + 1))
    V1 = run()
    monkeypatch.delenv("CAL_MPK_FAKE_BAND")
    assert np.array_equal(V1, V0)
    assert np.array_equal(V0, ref.matrix_powers_newton(A, v, s, lam, 1))


@pytest.mark.parametrize("s,tol_T", [(8, 1e-8), (10, 1e-7)])
def test_ca_lanczos_monomial_full_sweep(cal, ref, s, tol_T):
    """The reference's monomial sweep (test_ca_lanczos_convergence_orthogonality.m:
    54-55: s = 1..10, 'full', 120 steps, A / norm(A,'inf'), r0 = rand) on a
    matrix the image can build, diag(linspace(1,100,500)) / 100.  At s = 10 the
    monomial basis has kappa(V) far beyond u^(-1/2): CholQR2's Cholesky fails
    and the block takes the Householder TSQR.  Bars: 1e-15 perturbations of r
    move the oracle's own T by 3e-11 (s = 8) / 6e-10 (s = 10) and its top ten
    Ritz values by 3e-12 / 5e-11; T within tol_T, top ten Ritz values within
    1e-9, identical reorth flags, orthogonality error < 1e-13."""
    import scipy.sparse as sp
    n = 500
    A = sp.diags(ref.matlab_linspace(1.0, 100.0, n) / 100.0).tocsr()
    r = ref.matlab_rand(n)
    out = cal.ca_lanczos_ex(A, r, s, 120, "monomial", "full", diagnostics=True)
    exp = ref.ca_lanczos(A, r, s, 120, "monomial", "full", diagnostics=True)
    assert list(out.reorth) == list(exp.reorth)
    assert out.T.shape == exp.T.shape
    assert np.max(np.abs(out.T - exp.T)) <= tol_T
    w = np.sort(np.linalg.eigvals(out.T).real)[-10:]
    we = np.sort(np.linalg.eigvals(exp.T).real)[-10:]
    assert np.max(np.abs(w - we)) <= 1e-9
    assert np.max(out.orth_err) < 1e-13


@pytest.mark.parametrize("cond", [1e8, 1e11, 1e14])
def test_project_and_normalize_ill_conditioned(cal, ref, cond):
    """projectAndNormalize (Householder TSQR normalize) on a block whose
    projected part has kappa up to 1e14: R within 20 m kappa u ||Y||, QZ
    orthonormal to 1e-13 (Householder), identical reorth flag.  Orthogonality
    to Qp of the directions with singular values ~ kappa^-1 ||Y|| is lost to
    O(u kappa) in any normalize-after-project scheme, the reference's too: it
    must be within 10x the oracle's own (+ 1e-13)."""
    rng = np.random.RandomState(int(np.log10(cond)))
    n, w, m = 20000, 9, 8
    Qp, _ = np.linalg.qr(rng.randn(n, w))
    Y = _rand_block(n, m, 7, cond)
    Y = Y - Qp @ (Qp.T @ Y)
    X = Y + Qp @ rng.randn(w, m) * 0.3
    QZ, RZ, re, rank = cal.projectAndNormalize_ex([Qp], X)
    QZr, RZr, info = ref.projectAndNormalize_ex([Qp], X)
    assert re == info.reorth
    ny = np.linalg.norm(Y, 2)
    assert np.max(np.abs(RZ[1] - RZr[1])) <= 20 * m * cond * 2.0 ** -53 * ny
    assert np.max(np.abs(RZ[0] - RZr[0])) <= 1e-12 * np.linalg.norm(X, 2)
    assert np.linalg.norm(QZ.T @ QZ - np.eye(m), 2) <= 1e-13
    assert np.max(np.abs(QZ.T @ Qp)) <= 10 * np.max(np.abs(QZr.T @ Qp)) + 1e-13


def test_set_matrix_csc_matlab_layout(cal, ref):
    """The MEX entry for A: MATLAB's CSC arrays (int64 mwIndex jc / ir, pr)
    through cal_set_matrix_csc.  SpMV bit-identical to the CSR entry and to
    the oracle; a whole ca_lanczos run identical bit for bit."""
    import scipy.sparse as sp
    rng = np.random.RandomState(4)
    n = 2000
    B = sp.random(n, n, density=0.003, random_state=rng, format="csr")
    A = (B + B.T + sp.diags(np.full(n, 4.0))).tocsr()
    A.sort_indices()
    c1 = cal.Context().set_matrix_csc(A.tocsc())
    c2 = cal.Context().set_matrix(A)
    v = ref.matlab_rand(n, seed=3) - 0.5
    y1 = c1.spmv(v)
    assert np.array_equal(y1, c2.spmv(v)) and np.array_equal(y1, ref.SpMV(A, v))
    r = ref.matlab_rand(n)
    o1 = cal.ca_lanczos_ex(A, r, 8, 48, "newton", "local", diagnostics=True, ctx=c1)
    o2 = cal.ca_lanczos_ex(A, r, 8, 48, "newton", "local", diagnostics=True, ctx=c2)
    assert np.array_equal(o1.T, o2.T) and np.array_equal(o1.Q, o2.Q)
    assert np.array_equal(o1.ritz_rnorm, o2.ritz_rnorm)
    c1.close()
    c2.close()


def test_set_matrix_csc_nonsymmetric(cal, ref):
    """SpMV.m:8 is a general A*v: a NONSYMMETRIC A through the MATLAB-layout
    CSC entry (cal_set_matrix_csc, what SpMV.mexa64 binds) must give A @ v,
    not A' @ v, bit for bit (CSR rows in ascending column order = MATLAB's
    column-by-column accumulation).  Covers empty rows and columns, a dense
    row and a dense column."""
    import scipy.sparse as sp
    rng = np.random.RandomState(11)
    n = 3000
    B = sp.random(n, n, density=0.002, random_state=rng, format="lil")
    B[5, :] = rng.randn(n)          # a dense row
    B[:, 7] = rng.randn(n, 1)       # a dense column
    B[11, :] = 0.0                  # an empty row
    B[:, 13] = 0.0                  # an empty column
    A = B.tocsr()
    A.eliminate_zeros()
    A.sort_indices()
    assert abs(A - A.T).max() > 0
    c1 = cal.Context().set_matrix_csc(A.tocsc())
    v = ref.matlab_rand(n, seed=5) - 0.5
    y = c1.spmv(v)
    assert np.array_equal(y, ref.SpMV(A, v))
    assert np.max(np.abs(y - A @ v)) <= 1e-12 * np.max(np.abs(A @ v))
    assert np.max(np.abs(y - A.T @ v)) > 1e-3
    c1.close()


def test_normalize_randomize_null_space(cal, ref):
    """normalize(X,'randomizeNullSpace') (normalize.m:28-31,38-51) on a rank-5
    block of 8 columns: same rank; R = S W' and Q(:,1:rank) = Q U match the
    oracle up to the sign of each singular pair; the null-space columns
    (MATLAB rand of a fresh stream, projected, tsqr'd) match to 1e-10; Q
    orthonormal to 1e-13 and Q R = X to 1e-12 ||X||."""
    rng = np.random.RandomState(21)
    n, m, rk = 5000, 8, 5
    X = np.asfortranarray(rng.randn(n, rk) @ rng.randn(rk, m))
    Q, R, rank = cal.normalize(X, "randomizeNullSpace")
    Qr, Rr, rank_r = ref.normalize(X, "randomizeNullSpace")
    assert rank == rank_r == rk
    nx = np.linalg.norm(X, 2)
    assert np.linalg.norm(Q.T @ Q - np.eye(m), 2) <= 1e-13
    assert np.linalg.norm(Q @ R - X, 2) <= 1e-12 * nx
    sg = np.sign(np.sum(Q[:, :rk] * Qr[:, :rk], axis=0))
    assert np.max(np.abs(Q[:, :rk] * sg - Qr[:, :rk])) <= 1e-10
    assert np.max(np.abs(R[:rk] * sg[:, None] - Rr[:rk])) <= 1e-10 * nx
    assert np.max(np.abs(Q[:, rk:] - Qr[:, rk:])) <= 1e-10


def test_project_and_normalize_wide_block_no_reorth_in_span(cal, ref):
    """doreorth = false with 99 % of X inside span(Qp) (w = 40 > 9,
    'cholqr2').  The reference does one projection + normalize
    (projectAndNormalize.m:25-26, no second pass).  The single-sweep wide path
    (R = chol(X'X - C'C) from the algebraic Gram) would cancel here, so it must
    not be taken: the result stays orthonormal to 1e-13 and orthogonal to Qp
    to the level one projection reaches (the oracle's own Qp'QZ, x10)."""
    rng = np.random.RandomState(23)
    n, w, m = 20000, 40, 8
    Qp, _ = np.linalg.qr(rng.randn(n, w))
    X = 0.99 * Qp @ rng.randn(w, m) + 0.01 * rng.randn(n, m) / np.sqrt(n)
    ctx = cal.default_context()
    ctx.set_normalize("cholqr2")
    try:
        QZ, RZ, re, rank = cal.projectAndNormalize_ex([Qp], X, doreorth=False)
    finally:
        ctx.set_normalize("auto")
    QZr, RZr, info = ref.projectAndNormalize_ex([Qp], X, doreorth=False)
    assert re is False or re == 0
    assert np.max(np.abs(QZ.T @ QZ - np.eye(m))) < 1e-13
    assert np.max(np.abs(QZ.T @ Qp)) <= 10 * np.max(np.abs(QZr.T @ Qp)) + 1e-13
    assert np.max(np.abs(RZ[0] - RZr[0])) <= 1e-12 * max(1.0, np.max(np.abs(RZr[0])))


@pytest.mark.parametrize("case", ["spread", "reorth", "ill"])
def test_project_and_normalize_wide_block_cholqr(cal, ref, case):
    """One wide block (w = 40 > 9: the generic sweeps) on the CholQR path.
    'spread': the reorth test does not fire and Y is well conditioned, so the
    single projection + normalize of projectAndNormalize.m:25-26,52-58 runs as
    one Gram and one apply sweep; 'reorth': 90 % of X inside span(Qp), the
    second pass (:63-73); 'ill': X's columns nearly parallel (kappa(Y) ~ 1e6,
    not diagonally dominant): the two-pass CholQR2.  All three against the
    oracle (LAPACK QR + the sign fix)."""
    rng = np.random.RandomState(21)
    n, w, m = 20000, 40, 8
    Qp, _ = np.linalg.qr(rng.randn(n, w))
    if case == "spread":
        X = 0.1 * Qp @ rng.randn(w, m) + rng.randn(n, m) / np.sqrt(n)
    elif case == "reorth":
        X = 0.9 * Qp @ rng.randn(w, m) + 0.1 * rng.randn(n, m) / np.sqrt(n)
    else:
        base = rng.randn(n, 1)
        X = base + 1e-6 * rng.randn(n, m)
    ctx = cal.default_context()
    ctx.set_normalize("cholqr2")
    try:
        QZ, RZ, re, rank = cal.projectAndNormalize_ex([Qp], X)
    finally:
        ctx.set_normalize("auto")
    QZr, RZr, info = ref.projectAndNormalize_ex([Qp], X)
    assert re == info.reorth == (case == "reorth")
    scale = np.max(np.abs(RZr[1]))
    tol_r = 1e-11 if case != "ill" else 1e-6
    assert np.max(np.abs(RZ[0] - RZr[0])) <= 1e-12 * max(1.0, np.max(np.abs(RZr[0])))
    assert np.max(np.abs(RZ[1] - RZr[1])) <= tol_r * scale
    assert np.max(np.abs(QZ.T @ QZ - np.eye(m))) < 1e-13
    assert np.max(np.abs(QZ.T @ Qp)) < 1e-13


def _matlab_extreme(w):
    """min/max of eig(T) as MATLAB takes them: by modulus once any value is
    complex (test_ca_lanczos.m:81-82,87-88 print abs(se - min(eig(T))))."""
    w = np.asarray(w)
    if np.iscomplexobj(w) and np.any(w.imag != 0):
        return w[np.argmin(np.abs(w))], w[np.argmax(np.abs(w))]
    return np.min(w.real), np.max(w.real)


@pytest.mark.parametrize("s", [4, 8, 12, 16])
def test_ca_lanczos_reference_harness(cal, ref, s):
    """The reference's own known-answer harness: test_convergence_diagonal_
    matrices.m:9-21 -> test_ca_lanczos.m:32-41 (N = 500, A = diag(linspace(1,
    100,500)), r = ones, 480 steps, 'periodic', Newton, s = 4, 8, 12, 16).
    The metric the harness prints (test_ca_lanczos.m:79-98): the relative
    error of the smallest and largest eigenvalue of T against the known 1 and
    100 -- below 1e-12 here and within 1e-12 of the oracle's.  Against the
    oracle: the same periodic break count and reorth flags (both stable under
    1e-15 relative perturbations of r in the oracle itself), and T within
    1e-9 ||A|| on the whole 480 x 480 matrix for s = 4, 8 and on the leading
    blocks where the oracle's own spread stays below 1e-12 ||A|| for s = 12
    (27 of 40 blocks) and s = 16 (15 of 30)."""
    import scipy.sparse as sp
    a = ref.matlab_linspace(1.0, 100.0, 500)
    A = sp.csr_matrix(sp.diags(a))
    r = np.ones(500)
    exp = ref.ca_lanczos(A, r, s, 480, "newton", "periodic", diagnostics=False)
    out = cal.ca_lanczos_ex(A, r, s, 480, "newton", "periodic", diagnostics=False)
    assert out.T.shape == exp.T.shape == (480, 480)
    assert out.info["n_orth_breaks"] == sum(exp.breaks)
    assert list(out.reorth) == list(exp.reorth)
    m = {12: 27, 16: 15}.get(s, 480 // s) * s
    assert np.max(np.abs(out.T[:m, :m] - exp.T[:m, :m])) <= 1e-9 * 100.0
    lo, hi = _matlab_extreme(np.linalg.eigvals(out.T))
    elo, ehi = _matlab_extreme(np.linalg.eigvals(exp.T))
    err = (abs(1.0 - lo) / 1.0, abs(100.0 - hi) / 100.0)
    eerr = (abs(1.0 - elo) / 1.0, abs(100.0 - ehi) / 100.0)
    print("s=%d: error in smallest %.3e (oracle %.3e), largest %.3e (oracle %.3e)" % (s, err[0], eerr[0], err[1], eerr[1]))
    assert max(err) < 1e-12 and max(eerr) < 1e-12
    assert abs(err[0] - eerr[0]) < 1e-12 and abs(err[1] - eerr[1]) < 1e-12


def test_ca_lanczos_selective_complex_pair(cal, ref, monkeypatch):
    """'selective' locking of a converged complex-conjugate Ritz pair
    (ca_lanczos.m:317-336: QR(:,nritz) = Q*Vp(:,i) is complex and is
    normalize'd).  No input reachable here produces one, so both sides get the
    same test-only perturbation of eig(T) inside the selective update: the two
    most converged eigenpairs become one conjugate pair 0.5 (w_i + w_j) +-
    1e-3 i with unit vectors (v_i +- i v_j)/sqrt 2 (the oracle through a
    monkeypatched matlab_eig -- the Newton prologue's eig left alone -- the
    device through CAL_TEST_EIG_PAIR).  The device locks the pair as the
    real span Q Re(v), Q Im(v) of the reference's complex columns.  Bars: the
    pair is locked (2 complex members at the last rebuild, as in the oracle),
    the same rebuild count, locked count and reorth flags, T within 1e-8
    ||A||."""
    import math

    import scipy.sparse as sp
    a = ref.matlab_linspace(1.0, 100.0, 500)
    A = sp.csr_matrix(sp.diags(a))
    r = np.ones(500)
    orig, orig_ncb = ref.matlab_eig, ref.newton_change_of_basis
    active = {"on": True}

    def paired(T):
        w, V = orig(T)
        if not active["on"] or np.iscomplexobj(w) or len(w) < 2:
            return w, V
        i, j = np.argsort(np.abs(V[-1, :]), kind="stable")[:2]
        wc, Vc = w.astype(complex), V.astype(complex)
        vi, vj = V[:, i] / np.linalg.norm(V[:, i]), V[:, j] / np.linalg.norm(V[:, j])
        wc[i] = complex(0.5 * (w[i] + w[j]), 1.0e-3)
        wc[j] = np.conj(wc[i])
        Vc[:, i] = (vi + 1j * vj) / math.sqrt(2.0)
        Vc[:, j] = (vi - 1j * vj) / math.sqrt(2.0)
        return wc, Vc

    def ncb(*args, **kw):
        active["on"] = False
        try:
            return orig_ncb(*args, **kw)
        finally:
            active["on"] = True

    monkeypatch.setattr(ref, "matlab_eig", paired)
    monkeypatch.setattr(ref, "newton_change_of_basis", ncb)
    exp = ref.ca_lanczos(A, r, 8, 160, "newton", "selective", diagnostics=False)
    # the device side in a child process on the test build of the library
    # (libcalanczos_testhooks.so, CAL_TEST_HOOKS): the production library
    # carries no result-altering hook
    import json
    import subprocess
    import sys
    import tempfile
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = ("import sys, json, numpy as np, scipy.sparse as sp; sys.path.insert(0, %r)\n"
            "import ca_lanczos_amd as cal\n"
            "from oracle import ca_lanczos_ref as ref\n"
            "A = sp.csr_matrix(sp.diags(ref.matlab_linspace(1.0, 100.0, 500)))\n"
            "out = cal.ca_lanczos_ex(A, np.ones(500), 8, 160, 'newton', 'selective', diagnostics=False)\n"
            "np.save(sys.argv[1], out.T)\n"
            "print(json.dumps({'info': {k: int(out.info[k]) for k in ('n_ritz_complex', 'n_orth_breaks', "
            "'n_ritz_locked')}, 'reorth': [bool(f) for f in out.reorth]}))\n" % root)
    with tempfile.TemporaryDirectory() as td:
        tpath = os.path.join(td, "T.npy")
        env = dict(os.environ, CAL_LIBRARY="testhooks", CAL_TEST_EIG_PAIR="1")
        p = subprocess.run([sys.executable, "-c", code, tpath], env=env, capture_output=True, text=True,
                           timeout=240)
        assert p.returncode == 0, p.stderr[-2000:]
        res = json.loads(p.stdout.strip().splitlines()[-1])
        T = np.load(tpath)
    last = max(i for i, b in enumerate(exp.breaks) if b)
    assert exp.ncomplex[last] == 2
    assert res["info"]["n_ritz_complex"] == 2
    assert res["info"]["n_orth_breaks"] == sum(exp.breaks)
    assert res["info"]["n_ritz_locked"] == exp.nritz[-1]
    assert res["reorth"] == list(exp.reorth)
    assert np.max(np.abs(T - exp.T)) <= 1e-8 * 100.0


def test_production_library_has_no_test_hooks(cal, ref):
    """The same 'selective' run on the production library with
    CAL_TEST_EIG_PAIR set in its environment: the hook is not compiled in,
    so eig(T) is left alone and no complex Ritz pair appears."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = ("import sys, numpy as np, scipy.sparse as sp; sys.path.insert(0, %r)\n"
            "import ca_lanczos_amd as cal\n"
            "from oracle import ca_lanczos_ref as ref\n"
            "assert cal._lib.LIB_PATH.endswith('/libcalanczos.so')\n"
            "A = sp.csr_matrix(sp.diags(ref.matlab_linspace(1.0, 100.0, 500)))\n"
            "out = cal.ca_lanczos_ex(A, np.ones(500), 8, 160, 'newton', 'selective', diagnostics=False)\n"
            "print(int(out.info['n_ritz_complex']))\n" % root)
    env = dict(os.environ, CAL_TEST_EIG_PAIR="1")
    env.pop("CAL_LIBRARY", None)
    p = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-2000:]
    assert p.stdout.strip().splitlines()[-1] == "0"


@pytest.mark.parametrize("fmt", ["auto", "csr"])
def test_impl_restart_normest_async_matches_sync(cal, ref, fmt):
    """The implicit and the explicit restart run normest(A) on its own stream
    beside the Newton prologue and the first CA blocks (lanczos.cpp
    normest_async_*);
    'periodic' CA-Lanczos runs the synchronous normest_dev.  Same kernels in
    the same order: the same norm to the bit, in the matrix's own SpMV format
    and forced to CSR (the rescale in the gathers, mode 3); and the restart
    still matches the oracle's normest-scaled convergence (same restart count
    and eigenvalues as with the synchronous normest's value)."""
    A = cal.matrices.circuit_like(60, seed=3)
    r = ref.matlab_rand(A.shape[0])
    ctx = cal.Context(spmv_format=None if fmt == "auto" else fmt).set_matrix(A)
    p = cal.ca_lanczos_ex(A, r, 4, 40, "newton", "periodic", ctx=ctx)
    irl = cal.impl_restarted_ca_lanczos(A, r, 40, 6, 4, "newton", "full", 1e-8, ctx=ctx)
    irl2 = cal.impl_restarted_ca_lanczos(A, r, 40, 6, 4, "newton", "full", 1e-8, ctx=ctx)
    rst = cal.restarted_ca_lanczos(A, r, 40, 4, 4, "newton", "local", 1e-8, ctx=ctx)  # the explicit restart too
    ctx.close()
    assert rst["norm_A"] == p.info["norm_A"], (rst["norm_A"], p.info["norm_A"])
    assert p.info["norm_A"] > 0 and irl["norm_A"] == p.info["norm_A"], (irl["norm_A"], p.info["norm_A"])
    assert irl2["norm_A"] == irl["norm_A"] and irl2["num_restarts"] == irl["num_restarts"]
    assert np.array_equal(irl2["conv_eigs"], irl["conv_eigs"])
    exp = ref.impl_restarted_ca_lanczos(A, r, 40, 6, 4, "newton", "full", 1.0e-8)
    assert abs(irl["norm_A"] - exp["norm_A"]) <= 1e-12 * exp["norm_A"]
    assert irl["num_restarts"] == exp["num_restarts"]
    assert np.max(np.abs(irl["conv_eigs"] - exp["conv_eigs"])) <= 1e-10 * exp["norm_A"]
