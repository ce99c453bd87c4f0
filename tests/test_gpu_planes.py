"""The plane-march kernels (k_spmv_planes, k_resid_planes) on
every key mode they take, against the oracle (SpMV.m:6-8,
matrix_powers_newton.m:15-54, compute_ritz_rnorm of ca_lanczos.m:88-97).

Key modes (cal_spmv_plane_info):
  0  uniform slot values (every row with an entry at a slot has the same
     value there, as in the Dirichlet Laplacians): 1-B slot-mask keys;
  1  <= 256 row patterns with slot values that differ between rows (a
     Neumann / graph Laplacian, whose diagonal is the boundary-dependent
     degree): 1-B pattern ids into the LDS value table;
  2  > 256 row patterns (a diagonal that cycles through 100 values): 2-B ids.
Plane geometries: even and odd plane strides P (an odd P makes a plane's
last row pair straddle into the next plane), planes of one and of several
512-row blocks, 2-D (P = N, in-plane reach 1) and 3-D (P = N^2, reach N).

Bars: SpMV and the Newton powers bit-identical to the oracle's sequential
CSR arithmetic; an inf in x reaches exactly the rows that reference it (a
row's absent slots must not pick up x values of the neighbouring rows in
memory: masked, not multiplied by zero); the Ritz residual norms of
random vectors within 1e-12 relative of the oracle's NumPy norms."""
import numpy as np
import pytest
import scipy.sparse as sp

pytestmark = pytest.mark.gpu


def _graph_laplacian(dims):
    """Neumann (graph) Laplacian of a grid: off-diagonals -1 to the grid
    neighbours, diagonal = the degree (3..6 in 3-D: boundary-dependent)."""
    A = None
    n = int(np.prod(dims))
    for d in range(len(dims)):
        e = [sp.identity(m, format="csr") for m in dims]
        m = dims[d]
        e[d] = sp.diags([np.ones(m - 1), np.ones(m - 1)], [-1, 1], format="csr")
        T = e[-1]
        for k in range(len(dims) - 2, -1, -1):
            T = sp.kron(e[k], T, format="csr")
        A = T if A is None else A + T
    deg = np.asarray(A.sum(axis=1)).ravel()
    L = (sp.diags(deg) - A).tocsr()
    L.sort_indices()
    assert L.shape == (n, n)
    return L


def _many_diagonals(cal, N, M):
    """A 2-D Laplacian whose diagonal cycles through M values (exact binary
    fractions): N = 300, M = 100 gives 306 row patterns (> 256: 2-B keys;
    the value table of npat x 5 slots still fits the LDS bound of 2048)."""
    A = cal.matrices.laplacian_2d(N).tolil()
    n = A.shape[0]
    d = 4.0 + (np.arange(n) % M) * 2.0 ** -10
    A.setdiag(d)
    A = A.tocsr()
    A.sort_indices()
    return A


CASES = [
    # (name, builder, expected key mode)
    ("lap3d_20", lambda cal: cal.matrices.laplacian_3d(20), 0),      # P = 400: one block per plane
    ("lap3d_23", lambda cal: cal.matrices.laplacian_3d(23), 0),      # P = 529 odd, 2 blocks per plane
    ("lap3d_33", lambda cal: cal.matrices.laplacian_3d(33), 0),      # P = 1089 odd, 3 blocks per plane
    ("lap2d_300", lambda cal: cal.matrices.laplacian_2d(300), 0),    # 2-D: P = N = 300, reach 1
    ("lap2d_777", lambda cal: cal.matrices.laplacian_2d(777), 0),    # P = 777 odd
    ("graph3d_21", lambda cal: _graph_laplacian((21, 21, 21)), 1),   # degree diagonal, P = 441 odd
    ("graph2d_400", lambda cal: _graph_laplacian((400, 400)), 1),
    ("diag100_2d_300", lambda cal: _many_diagonals(cal, 300, 100), 2),
]


@pytest.fixture(scope="module", params=CASES, ids=[c[0] for c in CASES])
def case(request, cal):
    name, build, km = request.param
    A = build(cal)
    ctx = cal.Context(spmv_format="pattern").set_matrix(A)
    yield name, A, ctx, km
    ctx.close()


def test_plane_march_taken(case):
    name, A, ctx, km = case
    P, H, mode = ctx.spmv_plane_info()
    assert P >= 256 and 0 < H <= 256, (name, P, H)
    assert mode == km, (name, mode)


def test_plane_spmv_bitexact(case, ref):
    name, A, ctx, km = case
    n = A.shape[0]
    rng = np.random.RandomState(11)
    for v in (ref.matlab_rand(n, seed=3) - 0.5, rng.randn(n) * 1e3, np.ones(n)):
        assert np.array_equal(ctx.spmv(v), ref.SpMV(A, v)), name


def test_plane_spmv_inf_does_not_leak(case, ref):
    """inf / nan at positions whose memory neighbours (row +-1, +-N, +-P)
    include rows without an entry for them (grid boundaries): only the rows
    that reference them become non-finite, every other row keeps its bits."""
    name, A, ctx, km = case
    n = A.shape[0]
    P, _, _ = ctx.spmv_plane_info()
    N = int(round(P ** 0.5)) if A.nnz / n > 6 else P
    rng = np.random.RandomState(5)
    for pos in (0, N - 1, N, P - 1, P, n - 1, n // 2 + N - 1, n - P):
        v = rng.randn(n)
        v[pos] = np.inf if pos % 2 else np.nan
        got, exp = ctx.spmv(v), ref.SpMV(A, v)
        assert np.array_equal(np.isnan(got), np.isnan(exp)), (name, pos)
        assert np.array_equal(np.isinf(got), np.isinf(exp)), (name, pos)
        fin = np.isfinite(exp)
        assert np.array_equal(got[fin], exp[fin]), (name, pos)


def test_plane_newton_powers_bitexact(case, cal, ref):
    name, A, ctx, km = case
    n = A.shape[0]
    v = ref.matlab_rand(n)
    lam = np.array([11.5, 0.3, 6.1, 2.2, 9.0, 4.4, 1.1, 7.7])
    for modifiedp in (0, 1):
        assert np.array_equal(cal.matrix_powers_newton(A, v, 8, lam, modifiedp, ctx=ctx),
                              ref.matrix_powers_newton(A, v, 8, lam, modifiedp)), name
    lamc = np.array([7.0, 3 + 0.5j, 3 - 0.5j, 1.0])
    assert np.array_equal(cal.matrix_powers_newton(A, v, 4, lamc, 1, ctx=ctx),
                          ref.matrix_powers_newton(A, v, 4, lamc, 1)), name


def test_plane_ritz_rnorm(case, cal, ref):
    """compute_ritz_rnorm on random Q / Vp / Dp: X = Q Vp on the matrix cores,
    the batched plane-march residual; 1e-12 relative of the oracle's norms
    (the sums run in another order than NumPy's)."""
    name, A, ctx, km = case
    n = A.shape[0]
    rng = np.random.RandomState(2)
    k = 12
    Q = np.linalg.qr(rng.randn(n, k))[0]
    S = rng.randn(k, k)
    d, Vp = np.linalg.eigh(S + S.T)
    d = d * 3.0 + 0.5   # eigenvalues of both signs, none zero
    got = cal.compute_ritz_rnorm(A, Q, Vp, d, ctx=ctx)
    exp = ref.compute_ritz_rnorm(A, Q, Vp, d)
    assert np.all(np.abs(got - exp) <= 1e-12 * exp), (name, np.max(np.abs(got / exp - 1)))


def test_plane_ritz_rnorm_matches_pair_kernel(cal, ref):
    """The plane-march residual and the row-pair residual kernel (the same
    matrix with the plane march off: a two-rank-style slab is not needed, a
    CSR context takes the row kernel) agree to 1e-11 relative on the
    Ritz pairs of a real run (small residuals included)."""
    A = cal.matrices.laplacian_3d(24)
    r = ref.matlab_rand(A.shape[0])
    c1 = cal.Context(spmv_format="pattern").set_matrix(A)
    assert c1.spmv_plane_info()[0] == 576
    out = cal.ca_lanczos_ex(A, r, 8, 64, "newton", "local", diagnostics=False, ctx=c1)
    T = out.T
    d, Vp = np.linalg.eigh((T + T.T) / 2)
    got = cal.compute_ritz_rnorm(A, out.Q, Vp, d, ctx=c1)
    c2 = cal.Context(spmv_format="csr").set_matrix(A)
    exp = cal.compute_ritz_rnorm(A, out.Q, Vp, d, ctx=c2)
    big = exp > 1e-10
    assert np.all(np.abs(got[big] / exp[big] - 1) < 1e-11)
    assert np.all(got[~big] < 1e-9)
    c1.close()
    c2.close()
