"""The library's host-only C++ under AddressSanitizer + UBSan (SURVEY §5,
"Host: -fsanitize=address,undefined").  CPU only.

`make -C ca_lanczos_amd/csrc host-san` compiles dense.cpp (Cholesky,
triangular inverse, Jacobi SVD, tridiagonal QL, Hessenberg QR eig, qrstep),
leja.cpp (the modified Leja ordering and the Newton basis matrix),
host_api.cpp (the calanczos_host.h exports) and tsqr_plan.cpp (the TSQR tree's
level plan and workspace layout) with g++ -fsanitize=address,undefined
-fno-sanitize-recover=all into tests/native/host_check.cpp's driver.  Every
case below runs through it: any out-of-bounds access, use after free, leak or
undefined behaviour aborts the driver and fails the test.  The results are
compared with the product library's own host entry points (the same sources
built by hipcc: bit-identical, no FMA contraction in either build) and with
the oracle."""
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "ca_lanczos_amd", "csrc")
EXE = os.path.join(CSRC, "build", "host_check_san")


@pytest.fixture(scope="module")
def run():
    p = subprocess.run(["make", "-C", CSRC, "host-san"], capture_output=True, text=True)
    assert p.returncode == 0, p.stdout + p.stderr
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:halt_on_error=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")

    def _run(script):
        p = subprocess.run([EXE], input=script, capture_output=True, text=True, env=env, timeout=300)
        assert p.returncode == 0 and "Sanitizer" not in p.stderr and "runtime error" not in p.stderr, p.stderr[-3000:]
        return [ln.split() for ln in p.stdout.splitlines()]

    return _run


def _fmt(*arrays):
    return " ".join("%.17g" % x for a in arrays for x in np.ravel(np.asarray(a, dtype=float), order="F"))


def _f(tok):
    return np.array([float(t) for t in tok])


def test_leja_and_newton_basis(run, cal, ref):
    rng = np.random.RandomState(3)
    cases = [np.sort(rng.uniform(-1, 13, 16)), np.array([1.0, 1.0, 2.0, 5.0, 5.0, 5.0, 7.0, 9.0]),
             np.array([3.0]), np.linspace(0.1, 11.9, 32)]
    script = "".join("leja %d %s %s\n" % (len(x), _fmt(x), _fmt(np.zeros(len(x)))) for x in cases)
    lam = np.array([11.5, 0.3, 6.1, 2.2, 9.0, 4.4, 1.1, 7.7])
    script += "nbm 8 1 %s %s\n" % (_fmt(lam), _fmt(np.zeros(8)))
    lamc = np.array([2 + 1j, 2 - 1j, 5.0, 1.0])
    script += "nbm 4 1 %s %s\n" % (_fmt(lamc.real), _fmt(lamc.imag))
    out = run(script)
    for i, x in enumerate(cases):
        st, yr, yi, idx = out[4 * i: 4 * i + 4]
        if len(np.unique(x)) < len(x):  # repeated shifts: modified_leja.m's error() path, in both
            assert int(st[0]) == -4
            with pytest.raises(Exception):
                ref.leja(x, "m")
            continue
        assert int(st[0]) == 0
        y, ix = cal.leja(x, "nonmodified")
        assert np.array_equal(_f(yr), np.real(y)) and np.array_equal(_f(yi), np.imag(y) if np.iscomplexobj(y) else 0 * _f(yi))
        assert np.array_equal(_f(yr), np.real(ref.leja(x, "m")[0]))
    k = 4 * len(cases)
    B = _f(out[k + 1]).reshape(8, 9).T
    assert np.array_equal(B, ref.newton_basis_matrix(lam, 8, 1))
    Bc = _f(out[k + 3]).reshape(4, 5).T
    assert np.array_equal(Bc, ref.newton_basis_matrix(lamc, 4, 1))


def test_eig_qrstep_tridiag(run, cal):
    from ca_lanczos_amd._lib import lib, ptr
    rng = np.random.RandomState(5)
    mats = [rng.randn(n, n) for n in (1, 2, 7, 40, 121)]
    S = rng.randn(30, 30)
    mats.append(S + S.T)
    g = np.load(os.path.join(ROOT, "tests", "golden", "lap2d_32_s8_newton_local.npz"))
    mats.append(g["T"])
    script = "".join("eig %d %s\n" % (T.shape[0], _fmt(T)) for T in mats)
    m = 20
    d, e = rng.randn(m), rng.rand(m - 1) + 0.1
    H0 = np.diag(d) + np.diag(e, 1) + np.diag(e, -1)
    script += "qrstep %d %.17g %s %s\n" % (m, 0.37, _fmt(H0), _fmt(np.eye(m)))
    a, b = rng.randn(16), rng.rand(15)
    script += "tridiag 16 %s %s\n" % (_fmt(a), _fmt(b))
    out = run(script)
    for i, T in enumerate(mats):
        n = T.shape[0]
        st, wr, wi, V = out[4 * i: 4 * i + 4]
        assert int(st[0]) == 0
        Tf = np.asfortranarray(T)
        wr2, wi2, V2 = np.zeros(n), np.zeros(n), np.zeros((n, n), order="F")
        assert lib.cal_eig(n, ptr(Tf), n, ptr(wr2), ptr(wi2), ptr(V2)) == 0
        assert np.array_equal(_f(wr), wr2) and np.array_equal(_f(wi), wi2)
        assert np.array_equal(_f(V).reshape(n, n).T, V2)
        w = _f(wr) + 1j * _f(wi)
        assert np.max(np.abs(np.sort_complex(w) - np.sort_complex(np.linalg.eigvals(T)))) < 1e-10 * max(1, n)
    k = 4 * len(mats)
    H = np.asfortranarray(H0.copy())
    W = np.asfortranarray(np.eye(m))
    assert lib.cal_qrstep(m, ptr(H), m, ptr(W), m, 0.37) == 0
    assert np.array_equal(_f(out[k + 1]).reshape(m, m).T, H) and np.array_equal(_f(out[k + 2]).reshape(m, m).T, W)
    w = np.zeros(16)
    assert lib.cal_tridiag_eigvals(16, ptr(a), ptr(b), ptr(w)) == 0
    assert np.array_equal(_f(out[k + 4]), w)


def test_eig_values_only_and_batched_qrsteps(run):
    """The implicit restart's host algebra (lanczos.cpp, impl_restarted_ca_lanczos.m:96-107):
    eig_symmetric without vectors gives the same values, bit for bit, as with
    them (the shifts need no vectors), and hess_qrsteps (W's rotations
    batched after all the H steps, eight rows at a time) the same H and W as
    the steps one at a time -- m = 1, 9 (a tail of one row), 60 (the config-5
    m) with the exact shifts of the restart."""
    rng = np.random.RandomState(11)
    script, cases = "", []
    for m in (1, 2, 9, 20, 60):
        d, e = 4 + rng.rand(m), rng.rand(m - 1)
        T = np.diag(d) + np.diag(e, 1) + np.diag(e, -1) + 1e-13 * np.triu(rng.rand(m, m), 2)
        S = 0.5 * (T + T.T)
        w = np.linalg.eigvalsh(S)
        p = max(1, m - 12)
        mu = w[:p]
        H0 = np.tril(np.triu(T, -1))
        script += "eigsym %d %s\n" % (m, _fmt(S))
        script += "qrsteps %d %d %s %s %s\n" % (m, p, _fmt(mu), _fmt(H0 + np.triu(T, 2)), _fmt(np.eye(m)))
        cases.append((m, S))
    out = run(script)
    for i, (m, S) in enumerate(cases):
        o = out[9 * i: 9 * i + 9]
        w, w2, V = _f(o[1]), _f(o[2]), _f(o[3]).reshape(m, m).T
        assert np.array_equal(w, w2), m
        assert np.max(np.abs(w - np.linalg.eigvalsh(S))) <= 1e-12 * 8, m
        assert np.max(np.abs(V.T @ V - np.eye(m))) <= 1e-12, m
        assert np.array_equal(_f(o[5]), _f(o[7])) and np.array_equal(_f(o[6]), _f(o[8])), m


def test_dense_kernels(run):
    """Cholesky (and its failure on an indefinite Gram), triangular inverse
    and the Jacobi SVD of the s x s block algebra, m = 1..32."""
    rng = np.random.RandomState(9)
    script, cases = "", []
    for m in (1, 3, 8, 9, 16, 32):
        X = rng.randn(4 * m + 3, m)
        G = X.T @ X
        R = np.linalg.cholesky(G).T
        script += "chol %d %s\ntriinv %d %s\nsvd %d %s\n" % (m, _fmt(G), m, _fmt(R), m, _fmt(R))
        cases.append((m, G, R))
    script += "chol 3 %s\n" % _fmt(np.diag([1.0, -1.0, 1.0]))
    out = run(script)
    for i, (m, G, R) in enumerate(cases):
        o = out[8 * i: 8 * i + 8]
        assert int(o[0][0]) == 1
        Rc = _f(o[1]).reshape(m, m).T
        assert np.max(np.abs(Rc.T @ Rc - G)) <= 1e-12 * np.abs(G).max()
        Ri = _f(o[3]).reshape(m, m).T
        assert np.max(np.abs(Ri @ R - np.eye(m))) <= 1e-10
        U, S, V = _f(o[5]).reshape(m, m).T, _f(o[6]), _f(o[7]).reshape(m, m).T
        assert np.max(np.abs(U @ np.diag(S) @ V.T - R)) <= 1e-12 * np.abs(R).max()
        assert np.allclose(S, np.linalg.svd(R, compute_uv=False), rtol=1e-12, atol=1e-14 * S.max())
    assert int(out[-2][0]) == 0


def test_matlab_rand(run, ref):
    out = run("rand 1000 5489\nrand 17 7\nrand 0 1\n")
    assert np.array_equal(_f(out[1]), ref.matlab_rand(1000))
    assert np.array_equal(_f(out[3]), ref.matlab_rand(17, seed=7))


@pytest.mark.parametrize("n,m,P", [(9938375, 8, 1), (9938375, 8, 8), (1242296, 8, 8), (1000, 16, 3), (1, 1, 1),
                                   (513, 32, 2), (4096, 8, 4), (40000, 9, 1), (1585478, 8, 8)])
def test_tsqr_plan_layout(run, n, m, P):
    """The TSQR tree's level plan on the configs' shapes (lap3d_215 on 1 and
    8 ranks, a 27-plane slab, G3_circuit at 8 ranks) and edge cases (one
    row, one ragged tile): every buffer inside the workspace, no two
    overlapping, the stack chain and the S chain consistent, the root one
    tile (the driver checks, status 0), for every rank."""
    from math import ceil
    TR = 4096 // (8 if m <= 8 else (16 if m <= 16 else 32))
    script = "".join("plan %d %d %d 1 %d %d\n" % (n, m, TR, P, me) for me in range(P))
    out = run(script)
    i = 0
    for me in range(P):
        assert int(out[i][0]) == 0, (me, out[i])
        need, nlv, nloc = (int(x) for x in out[i + 1])
        lv = [[int(x) for x in out[i + 2 + k]] for k in range(nlv)]
        assert lv[0][2] == ceil(n / TR) and lv[-1][2] == 1
        assert (nloc < nlv) == (P > 1)
        i += 2 + nlv
