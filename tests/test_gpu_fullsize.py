"""Parity at BASELINE.json's full sizes (configs 2 and 3), through the C ABI.

The small-case parity tests (test_gpu_parity.py) pin every function against
the oracle; these repeat the comparisons the oracle can still afford at the
benchmark sizes, plus size-independent properties where it cannot:

  * config 3 (lap3d_215, n = 9,938,375): SpMV and the Newton matrix powers
    bit-identical to the oracle's sequential CSR SpMV (SpMV.m:8,
    matrix_powers_newton.m:15-54); the CA-Lanczos outer iterations against
    the C/OpenMP restatement (oracle/c, ca_lanczos.m:150-245) to
    1e-9 * ||A|| with identical reorthogonalisation flags over the whole
    15-iteration bench run, extreme Ritz values to 1e-10 * ||A||, the top Ritz
    pair's residual norm recomputed on the host from the device's Q, and the
    size-independent properties (spectrum bounds, last Q block orthonormal);
  * config 3 as named (TSQR normalize): the same 15-iteration comparison
    with the fused Householder TSQR projectAndNormalize on every block;
  * north_star's ~10M-row 5-pt Laplacian (lap2d_3162, n = 9,998,244):
    bit-exact SpMV and the same 15-iteration comparison;
  * config 2 (lap2d_1000, n = 10^6): the whole t = 15 run against the NumPy
    oracle (T to 1e-9 * ||A||, identical flags, extreme Ritz values);
  * config 5 at its full size (the G3_circuit stand-in circuit_1259, n =
    1,585,081, CSR SpMV): the implicitly restarted solve of the bench against
    ARPACK's top 8 (tests/golden/circuit_1259_top8.npz, made by
    tests/golden/make_circuit_eigs.py) to 1e-10 relative, Q_conv orthonormal,
    every residual ||A v - l v|| / |l| below 1e-7.
"""
import math
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

S = 8


def _lap_max(dim, N):
    """Largest eigenvalue of the Dirichlet dim-D Laplacian (stencil 2*dim, -1)."""
    return dim * (2.0 - 2.0 * math.cos(N * math.pi / (N + 1)))


@pytest.fixture(scope="module")
def lap3d(cal):
    return cal.matrices.laplacian_3d(215)


@pytest.fixture(scope="module")
def ctx3d(cal, lap3d):
    ctx = cal.Context().set_matrix(lap3d)
    yield ctx
    ctx.close()


def test_spmv_fullsize_bitexact(ctx3d, lap3d, ref):
    n = lap3d.shape[0]
    v = ref.matlab_rand(n, seed=7)
    assert np.array_equal(ctx3d.spmv(v), ref.SpMV(lap3d, v))
    # A * ones = number of missing neighbours per row (0 inside, 1..3 on the faces)
    y = ctx3d.spmv(np.ones(n))
    assert y.min() == 0.0 and y.max() == 3.0 and np.all(y == np.round(y))


def test_spmv_fullsize_csr_nontemporal_bitexact(cal, lap3d, ref):
    """lap3d_215 in plain CSR (1.03 GB of col / val, larger than the Infinity
    Cache: the kernel's non-temporal loads) and a shifted SpMV, both bit-exact
    against the sequential CSR SpMV (SpMV.m:8, matrix_powers_newton.m:32)."""
    n = lap3d.shape[0]
    ctx = cal.Context(spmv_format="csr").set_matrix(lap3d)
    try:
        assert ctx.spmv_format()[0] == "csr"
        v = ref.matlab_rand(n, seed=9)
        assert np.array_equal(ctx.spmv(v), ref.SpMV(lap3d, v))
        lam = np.array([3.25, 7.5])
        V = cal.matrix_powers_newton(lap3d, v, 2, lam, 0, ctx=ctx)
        assert np.array_equal(V, ref.matrix_powers_newton(lap3d, v, 2, lam, 0))
    finally:
        ctx.close()


def test_matrix_powers_newton_fullsize_bitexact(cal, ctx3d, lap3d, ref):
    n = lap3d.shape[0]
    v = ref.matlab_rand(n, seed=11)
    lam = np.linspace(0.5, 11.5, S)
    V = cal.matrix_powers_newton(lap3d, v, S, lam, 1, ctx=ctx3d)
    Ve = ref.matrix_powers_newton(lap3d, v, S, lam, 1)
    assert V.shape == (n, S + 1)
    assert np.array_equal(V, Ve)


def _run_vs_omp(ctx, A, r, t, nA, lmin, lmax):
    """t outer iterations of ca_lanczos_basic 'local' (s = 8, Newton, the same
    start vector) on the device, diagnostics on, against the C/OpenMP
    restatement (ca_lanczos.m:150-245 with Householder tsqr, tsqr.m:7-12):
    T to 1e-9 ||A||, identical reorth flags, the extreme Ritz values to
    1e-10 ||A||.  The last iteration's residual norm of the largest Ritz pair
    (compute_ritz_rnorm, ca_lanczos.m:88-97) is recomputed on the host --
    x = Q y from the device's Q (streamed in blocks), ||A x - l x|| / ||l x||
    with SciPy's SpMV -- to 1e-8 relative.  Size-independent properties: Ritz
    values inside the analytic spectrum [lmin, lmax], the last Q block
    orthonormal to 1e-13.  Returns the reorth flags."""
    from oracle import omp

    n = A.shape[0]
    ctx.lanczos_begin(r, S, t, "newton", "local")
    for _ in range(t):
        ctx.lanczos_step(True)
    T, rn, _, flags, _ = ctx.lanczos_get()
    Te, fe = omp.ca_lanczos(A, r, S, S * t, "newton")
    assert T.shape == Te.shape == (S * t, S * t)
    assert list(bool(f) for f in flags) == list(fe)
    dT = np.max(np.abs(T - Te))
    assert dT <= 1e-9 * nA, dT
    w = np.sort(np.linalg.eigvals(T).real)
    we = np.sort(np.linalg.eigvals(Te).real)
    assert abs(w[-1] - we[-1]) <= 1e-10 * nA and abs(w[0] - we[0]) <= 1e-10 * nA
    assert w[0] >= lmin * (1 - 1e-9) and w[-1] <= lmax * (1 + 1e-12)
    assert np.max(np.abs(T - T.T)) <= 1e-10 * lmax
    # residual of the largest Ritz pair, recomputed from the device's Q
    ev, V = np.linalg.eig(T)
    i = int(np.argmax(ev.real))
    lam, y = ev[i].real, V[:, i].real
    x = np.zeros(n)
    for c0 in range(0, S * t, S):
        x += ctx.lanczos_get_Q(c0, S) @ y[c0:c0 + S]
    Qb = ctx.lanczos_get_Q(S * (t - 1), S + 1)  # the last block Q(:, s(t-1)+1 : st+1)
    ctx.lanczos_end()
    rn_host = np.linalg.norm(A @ x - lam * x) / np.linalg.norm(lam * x)
    assert abs(rn[t - 1, 0] / rn_host - 1.0) <= 1e-8, (rn[t - 1, 0], rn_host)
    assert np.max(np.abs(Qb.T @ Qb - np.eye(S + 1))) < 1e-13
    print("T max |dT| %.3e (bar %.1e), top Ritz %.15f (omp %.15f), rn %.6e (host %.6e), flags %d/%d"
          % (dT, 1e-9 * nA, w[-1], we[-1], rn[t - 1, 0], rn_host, sum(flags), t))
    return flags


def _lap3d_bounds():
    return 3 * (2.0 - 2.0 * math.cos(math.pi / 216)), _lap_max(3, 215)


def test_ca_lanczos_fullsize_vs_omp(ctx3d, lap3d, ref):
    """BASELINE config 3's workload with the loop's default normalize (the
    fused CholQR2 sweeps): the whole bench run, t = 15, against C/OpenMP."""
    r = ref.matlab_rand(lap3d.shape[0])
    flags = _run_vs_omp(ctx3d, lap3d, r, 15, 12.0, *_lap3d_bounds())
    assert sum(flags) == 15 - 1  # every k > 1 takes the second pass on this input


def test_ca_lanczos_config3_tsqr_fullsize_vs_omp(cal, lap3d, ref):
    """BASELINE config 3 as named: lap3d_215, s = 8 Newton, **TSQR** normalize
    (tsqr.m:7-12 at ca_lanczos.m:178,187), t = 15, against the C/OpenMP
    restatement (whose normalize is Householder TSQR too).  Every block k > 1
    must take the fused TSQR projectAndNormalize (tsqr_fold.hip: 14 runs, 0
    declined), so the 15-step bench run of tsqr_step is pinned end to end."""
    ctx = cal.Context(normalize="tsqr").set_matrix(lap3d)
    try:
        f0 = ctx.tsqr_fold_stats()
        r = ref.matlab_rand(lap3d.shape[0])
        flags = _run_vs_omp(ctx, lap3d, r, 15, 12.0, *_lap3d_bounds())
        f1 = ctx.tsqr_fold_stats()
    finally:
        ctx.close()
    assert sum(flags) == 15 - 1
    assert f1["runs"] - f0["runs"] == 14 and f1["declined"] - f0["declined"] == 0, (f0, f1)
    assert f1["last_est"] < 1e-14


@pytest.fixture(scope="module")
def lap2d_10m(cal):
    return cal.matrices.laplacian_2d(3162)


def test_ca_lanczos_lap2d_3162_vs_omp(cal, lap2d_10m, ref):
    """north_star's literal target, the ~10M-row 5-pt Laplacian (3162^2 =
    9,998,244 rows) at s = 8: SpMV bit-exact against the oracle's sequential
    CSR SpMV (SpMV.m:8), then the whole t = 15 run (default normalize)
    against the C/OpenMP restatement with the same bars as config 3."""
    A = lap2d_10m
    n = A.shape[0]
    assert n == 9998244
    ctx = cal.Context().set_matrix(A)
    try:
        v = ref.matlab_rand(n, seed=7)
        assert np.array_equal(ctx.spmv(v), ref.SpMV(A, v))
        y = ctx.spmv(np.ones(n))  # A * ones: 0 inside, 1 on the edges, 2 at the corners
        assert y.min() == 0.0 and y.max() == 2.0 and np.all(y == np.round(y))
        r = ref.matlab_rand(n)
        lmin = 2 * (2.0 - 2.0 * math.cos(math.pi / 3163))
        _run_vs_omp(ctx, A, r, 15, 8.0, lmin, _lap_max(2, 3162))
    finally:
        ctx.close()


def test_ca_lanczos_config2_vs_oracle(cal, ref):
    """BASELINE config 2 in full: lap2d_1000, s = 8 Newton, t = 15, against
    the NumPy oracle (diagnostics off on both sides)."""
    N = 1000
    A = cal.matrices.laplacian_2d(N)
    r = ref.matlab_rand(N * N)
    it = S * 15
    out = cal.ca_lanczos_ex(A, r, S, it, "newton", "local", diagnostics=False, return_Q=False)
    exp = ref.ca_lanczos(A, r, S, it, "newton", "local", diagnostics=False)
    assert out.T.shape == exp.T.shape
    assert np.max(np.abs(out.shifts - exp.shifts)) < 1e-9 * 8.0
    assert list(out.reorth) == list(exp.reorth)
    assert np.max(np.abs(out.T - exp.T)) <= 1e-9 * 8.0
    w = np.sort(np.linalg.eigvals(out.T).real)
    we = np.sort(np.linalg.eigvals(exp.T).real)
    assert abs(w[-1] - we[-1]) < 1e-10 * 8.0 and abs(w[0] - we[0]) < 1e-10 * 8.0


def test_impl_restarted_config5_fullsize(cal):
    """BASELINE config 5 at n = 1.58 M: impl_restarted_ca_lanczos (m = 64,
    8 wanted, s = 8 Newton, 'full', tol 1e-8; impl_restarted_ca_lanczos.m:
    333-426 with the fixes listed in DESIGN.md §8 f3) on the irregular SPD
    stand-in, r = ones, against the golden ARPACK eigenvalues."""
    gold = np.load(os.path.join(os.path.dirname(__file__), "golden", "circuit_1259_top8.npz"))
    A = cal.matrices.circuit_like(1259)
    assert A.shape[0] == int(gold["n"]) and A.nnz == int(gold["nnz"])
    eref = gold["eigs"]
    out = cal.impl_restarted_ca_lanczos(A, np.ones(A.shape[0]), 64, 8, 8, "newton", "full", 1.0e-8)
    assert out["converged"]
    ev = out["conv_eigs"]
    assert np.all(np.diff(ev) <= 0)
    assert np.max(np.abs(ev - eref) / np.abs(eref)) <= 1e-10, (ev, eref)
    V = out["Q_conv"]
    assert np.max(np.abs(V.T @ V - np.eye(8))) < 1e-9
    res = np.linalg.norm(A @ V - V * ev, axis=0) / np.abs(ev)
    assert np.max(res) < 1e-7
