"""CPU restatement of the reference CA-Lanczos hot path (NumPy/SciPy).

TEST INFRASTRUCTURE ONLY.  Nothing in the product (``ca_lanczos_amd``,
``libcalanczos.so``) imports, links or calls this module.  Only ``tests/``,
``__graft_entry__.smoke()`` and the ``cpu_baseline`` leg of ``bench.py`` use it,
and only as the checker / the timed CPU baseline.

What it restates
----------------
Every function below follows one MATLAB file of the reference
(magnusgrandin/ca-lanczos, mounted read-only at /root/reference) line by line;
the docstring of each function cites the file:line it follows.  MATLAB
semantics that change results are emulated explicitly:

* sparse ``A*v`` is a sequential per-row sum in increasing column order
  (MATLAB CSC ``mtimes`` and SciPy ``csr_matvec`` accumulate in the same order
  for a sorted, symmetric matrix);
* ``qr(A,0)`` is LAPACK Householder (``numpy.linalg.qr``), ``eig`` dispatches
  to the symmetric solver only for an exactly symmetric matrix;
* ``sort(...,'descend')`` of a complex vector sorts by modulus, then phase,
  and is stable; ``max`` returns the first maximiser and ignores NaN;
* ``sign(0) == 0``; ``linspace`` uses MATLAB's ``d1 + (i*(d2-d1))/n1`` form;
* ``rand`` in a fresh MATLAB session is MT19937 seeded 5489
  (``numpy.random.RandomState(5489).random_sample``).

Parity status
-------------------------------------
MATLAB / Octave cannot run in this pipeline and the reference holds no golden
vectors, so this restatement is **not bit-pinned against MATLAB itself**
("parity unpinned" at the MATLAB-built-in boundary: ``qr``, ``eig``, ``svd``
are MKL inside MATLAB and OpenBLAS/LAPACK here).  It is pinned against the
analytic known answers of the reference's own synthetic test inputs (diagonal
matrices of ``test_convergence_diagonal_matrices.m`` /
``test_restart_diagonal_matrices.m``, BASELINE config 1, and the closed-form
spectra of the Dirichlet Laplacians) by ``tests/test_oracle.py``.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field

import numpy as np
import scipy.sparse as sp
from scipy.linalg import solve_triangular

VERBOSE = False  # mirror the reference's disp() chatter when True


def _disp(msg: str) -> None:
    if VERBOSE:
        print(msg)


# --------------------------------------------------------------------------
# MATLAB helpers
# --------------------------------------------------------------------------

def matlab_rand(n: int, seed: int = 5489) -> np.ndarray:
    """``rand(n,1)`` of a fresh MATLAB session (MT19937, seed 5489)."""
    return np.random.RandomState(seed).random_sample(n)


def matlab_linspace(d1: float, d2: float, n: int) -> np.ndarray:
    """MATLAB ``linspace(d1,d2,n)``: ``d1 + ((0:n1)*(d2-d1))/n1``, ends exact."""
    n1 = n - 1
    i = np.arange(n, dtype=np.float64)
    y = d1 + (i * (d2 - d1)) / n1
    y[0] = d1
    y[-1] = d2
    return y


def _sort_perm(d: np.ndarray, descend: bool) -> np.ndarray:
    """Permutation of MATLAB ``[~,ix] = sort(d)`` (stable; complex by |.|, angle)."""
    idx = list(range(len(d)))
    if np.iscomplexobj(d):
        keys = [(abs(z), math.atan2(z.imag, z.real)) for z in d]
    else:
        keys = [(float(x),) for x in d]
    if descend:
        # stable descending: negate the key, keep Python's stable sort
        return np.array(sorted(idx, key=lambda i: tuple(-k for k in keys[i])), dtype=np.int64)
    return np.array(sorted(idx, key=lambda i: keys[i]), dtype=np.int64)


def _matlab_max(v: np.ndarray):
    """MATLAB ``[m,i] = max(v)``: first maximiser, NaN ignored (all-NaN -> NaN, 0)."""
    best_i, best = -1, None
    for i, x in enumerate(v):
        if isinstance(x, float) and math.isnan(x):
            continue
        if best is None or x > best:
            best, best_i = x, i
    if best is None:
        return float("nan"), 0
    return best, best_i


def _rdiv_upper(X: np.ndarray, R: np.ndarray) -> np.ndarray:
    """MATLAB ``X / R`` for square upper-triangular ``R`` (triangular solve)."""
    return solve_triangular(R, X.T, trans="T", lower=False).T


def eyeshvec(n: int) -> np.ndarray:
    """``eyeshvec`` (ca_lanczos.m:144-147): last unit vector of length n."""
    v = np.zeros(n)
    v[-1] = 1.0
    return v


def matlab_eig(T: np.ndarray):
    """MATLAB ``[V,D] = eig(T)``: symmetric solver iff T is exactly symmetric."""
    if np.array_equal(T, T.T):
        w, V = np.linalg.eigh(T)
        return w, V
    w, V = np.linalg.eig(T)
    if np.iscomplexobj(w) and np.all(w.imag == 0):
        w = w.real
        V = V.real
    return w, V


# --------------------------------------------------------------------------
# a1-a4: SpMV and matrix powers
# --------------------------------------------------------------------------

def SpMV(A, v):
    """``Av = SpMV(A,v)`` -- SpMV.m:6-8 (``Av = A*v``)."""
    return A @ v


def matrix_powers_monomial(A, q, s):
    """matrix_powers_monomial.m:6-12: V(:,1)=A*q; V(:,i)=A*V(:,i-1). n x s."""
    n = len(q)
    V = np.zeros((n, s))
    V[:, 0] = A @ q
    for i in range(1, s):
        V[:, i] = A @ V[:, i - 1]
    return V


def matrix_powers_newton(A, v, s, lam, modifiedp=0):
    """matrix_powers_newton.m:15-54. Returns the n x (s+1) Newton basis."""
    lam = np.asarray(lam)
    n = len(v)
    cplx = np.iscomplexobj(lam) and modifiedp == 0 and np.any(lam.imag != 0)
    V = np.zeros((n, s + 1), dtype=complex if cplx else float)
    V[:, 0] = v
    if modifiedp == 0:
        for k in range(s):                                     # :26-29
            w = SpMV(A, V[:, k])
            V[:, k + 1] = w - lam[k] * V[:, k]
    else:
        for k in range(s):                                     # :31-47
            w = SpMV(A, V[:, k])
            lk = complex(lam[k])
            if lk.imag > 0:
                V[:, k + 1] = w - lk.real * V[:, k]
            elif lk.imag < 0:
                if k == 0:
                    raise ValueError("k==1, but shift %e has a negative imaginary part" % lk.imag)
                V[:, k + 1] = w - lk.real * V[:, k] + (lk.imag ** 2) * V[:, k - 1]
            else:
                V[:, k + 1] = w - lk.real * V[:, k]
    return V


def matrix_powers(A, q, s, Bk, basis):
    """ca_lanczos.m:110-118: basis dispatch; Newton shifts = diag(Bk)."""
    if basis.lower() == "monomial":
        V = np.zeros((len(q), s + 1))
        V[:, 0] = q
        V[:, 1:] = matrix_powers_monomial(A, q, s)
        return V
    if basis.lower() == "newton":
        return matrix_powers_newton(A, q, s, np.diag(Bk)[:s].copy(), 1)
    raise ValueError("ERROR: Unknown basis type: " + basis)


# --------------------------------------------------------------------------
# a5-a9: block orthogonalisation
# --------------------------------------------------------------------------

def tsqr(A):
    """tsqr.m:7-12: Householder ``qr(A,0)`` then diag(R) made non-negative."""
    Q, R = np.linalg.qr(A, mode="reduced")
    d = np.sign(np.diag(R))
    R = d[:, None] * R
    Q = Q * d[None, :]
    return Q, R


def cholqr(X):
    """cholqr.m:3-8: G = X'X; R = chol(G) (upper); Q = X/R."""
    G = X.T @ X
    R = np.linalg.cholesky(G).T
    Q = _rdiv_upper(X, R)
    return Q, R


def _is_empty(B) -> bool:
    return B is None or (hasattr(B, "size") and B.size == 0)


def _col_norms(X):
    return np.array([np.linalg.norm(X[:, j]) for j in range(X.shape[1])])


def project(Q, X, doreorth=False):
    """project.m:7-58: block MGS across blocks, CGS within; optional inverted-test reorth."""
    if not isinstance(Q, (list, tuple)):
        raise TypeError("Input Q (arg 1) to project() must be cell (block) array.")
    if isinstance(X, (list, tuple)):
        raise TypeError("Input X (arg 2) project() must be a column matrix.")
    if len(Q) == 0:                                             # :21-24
        return X, []
    m = X.shape[1]
    R = [None] * len(Q)
    normBefore = np.zeros(m)
    if doreorth:
        normBefore = _col_norms(X)
    for i, Qi in enumerate(Q):                                  # :32-39
        if not _is_empty(Qi):
            R[i] = Qi.T @ X
            X = X - Qi @ R[i]
        else:
            R[i] = np.zeros((0, m))
    if doreorth:                                                # :40-57
        _disp("project(): reorthogonalize")
        normAfter = _col_norms(X)
        normDiff = 0.5 * normBefore - normAfter
        if _matlab_max(normDiff)[0] < 0:
            for i, Qi in enumerate(Q):
                if not _is_empty(Qi):
                    R2 = Qi.T @ X
                    X = X - Qi @ R2
                    R[i] = R[i] + R2
    return X, R


def normalize(X, opt="None", tol=1.0e-8, rng=None):
    """normalize.m:3-36: tsqr + SVD rank check (rank = first i with s_i <= tol*s_1, minus 1)."""
    ncols = X.shape[1]
    Q, R = tsqr(X)
    U, S, Wt = np.linalg.svd(R)
    abs_tol = tol * S[0]
    rank = ncols
    for i in range(ncols):
        if S[i] <= abs_tol:
            rank = i
            break
    if rank == ncols:
        return Q, R, rank
    if opt.lower() == "randomizenullspace":                    # :28-31 (never on the hot path)
        R = np.diag(S) @ Wt
        Q = Q @ U
        Q = _randomize_null_space(Q, rank, rng)
    return Q, R, rank


def _randomize_null_space(Q, rank, rng):
    """normalize.m:38-51 (randomizeNullSpace)."""
    rng = rng if rng is not None else np.random.RandomState(5489)
    nrows, ncols = Q.shape
    null = list(range(rank, ncols))
    Q = Q.copy()
    Q[:, null] = rng.random_sample(nrows * len(null)).reshape((nrows, len(null)), order="F")  # MATLAB fills by columns
    Q[:, null], _ = project([Q[:, :rank]], Q[:, null])
    Q[:, null], _ = tsqr(Q[:, null])
    return Q


@dataclass
class PNInfo:
    """Extra outputs of projectAndNormalize the reference only disp()s."""
    reorth: bool = False
    rank: int = 0
    norms_before: np.ndarray = field(default_factory=lambda: np.zeros(0))
    norms_after: np.ndarray = field(default_factory=lambda: np.zeros(0))


def projectAndNormalize_ex(Q, X, doreorth=True):
    """projectAndNormalize.m:3-90, also returning the reorth flag (disp 'second')."""
    tol = 0.5                                                   # :10
    ncols = X.shape[1]
    nb = len(Q)
    info = PNInfo()
    normsBeforeFirst = np.zeros(ncols)
    if doreorth:                                                # :17-22
        normsBeforeFirst = np.array([math.sqrt(np.sum(X[:, i] ** 2)) for i in range(ncols)])
    Y, RY = project(Q, X, False)                                # :25
    QY, R_, rank = normalize(Y)                                 # :26
    RY = list(RY) + [R_]                                        # :27
    info.rank = rank
    if doreorth:
        normsAfterFirst = np.array([math.sqrt(np.sum(R_[:, i] ** 2)) for i in range(ncols)])
        with np.errstate(divide="ignore", invalid="ignore"):
            rel = np.abs(normsBeforeFirst - normsAfterFirst) / normsBeforeFirst
        reorth = bool(_matlab_max(rel)[0] > tol)                # :52
        info.norms_before, info.norms_after = normsBeforeFirst, normsAfterFirst
        if not reorth:
            return QY, RY, info
        _disp("second")                                         # :62
        info.reorth = True
        Z, RZ = project(Q, Y, False)                            # :63
        QZ, R_, rank = normalize(Z)                             # :64
        RZ = list(RZ) + [R_]
        for i in range(nb):                                     # :71-73
            RZ[i] = RZ[i] + RY[i]
        info.rank = rank
        if rank < ncols:
            _disp("Rank deficient")
        return QZ, RZ, info
    return QY, RY, info


def projectAndNormalize(Q, X, doreorth=True):
    """``[QZ,RZ] = projectAndNormalize(Q,X,doreorth)`` -- projectAndNormalize.m:3-90."""
    QZ, RZ, _ = projectAndNormalize_ex(Q, X, doreorth)
    return QZ, RZ


# --------------------------------------------------------------------------
# a13: Newton prologue (lanczos 'fro', Leja ordering, change-of-basis matrix)
# --------------------------------------------------------------------------

def lanczos_basic(A, q, maxiter, orth="local", diagnostics=False):
    """lanczos.m:85-134 (the three-term recurrence; 'fro' = one CGS pass, lanczos.m:62-66).

    The reference always computes the Ritz residuals / orthogonality error
    here (lanczos.m:117-126, nargout is 4 from lanczos.m:50-52).  They never
    feed back into T or Q; ``diagnostics=True`` reproduces their cost.
    """
    n = len(q)
    Q = np.zeros((n, maxiter + 1))
    Q[:, 0] = q
    alpha = np.zeros(maxiter)
    beta = np.zeros(maxiter)
    rnorm = np.zeros((maxiter, maxiter))
    ortherr = np.zeros(maxiter)
    for j in range(maxiter):                                    # :102
        r = A @ Q[:, j]                                         # :103
        if j > 0:
            r = r - beta[j - 1] * Q[:, j - 1]                   # :105
        alpha[j] = r @ Q[:, j]                                  # :107
        r = r - alpha[j] * Q[:, j]                              # :108
        beta[j] = math.sqrt(r @ r)                              # :109
        Q[:, j + 1] = r / beta[j]                               # :110
        if orth.lower() == "fro":                               # :112-114 -> :62-66
            Rkk = Q[:, : j + 1].T @ Q[:, j + 1]
            Q[:, j + 1] = Q[:, j + 1] - Q[:, : j + 1] @ Rkk
        if diagnostics:                                         # :117-126
            Tj = np.diag(alpha[: j + 1]) + np.diag(beta[:j], 1) + np.diag(beta[:j], -1)
            Dp, Vp = matlab_eig(Tj)
            rnorm[j, : j + 1] = compute_ritz_rnorm(A, Q[:, : j + 1], Vp, Dp)
            ortherr[j] = np.max(Q[:, : j + 1].T @ Q[:, j + 1])
    T = np.diag(alpha) + np.diag(beta[:-1], 1) + np.diag(beta[:-1], -1)   # :131
    return Q[:, :maxiter], T, rnorm, ortherr


def lanczos(A, r, maxiter, orth="local", diagnostics=False):
    """lanczos.m:18-60 for orth in {local, full}: q = r/norm(r) then lanczos_basic."""
    q = r / np.linalg.norm(r)                                   # :47
    o = orth.lower()
    if o == "local":
        return lanczos_basic(A, q, maxiter, "local", diagnostics)
    if o == "full":
        return lanczos_basic(A, q, maxiter, "fro", diagnostics)
    raise NotImplementedError("lanczos orth=%s is outside the hot path" % orth)


def count_multiplicities(x, n):
    """count_multiplicities.m:5-41 (MATLAB ``unique`` sorts; mults from sorted copy)."""
    x = np.asarray(x)
    perm = _sort_perm(x, False)
    xs = x[perm]
    y, ii = [], []
    for i, v in enumerate(xs):
        if i == 0 or v != xs[i - 1]:
            y.append(v)
            ii.append(i)
    y = np.array(y, dtype=x.dtype)
    num_unique = len(y)
    if num_unique == n:                                         # :18-21
        return y, np.ones(n), num_unique
    mults = np.zeros(num_unique)                                # :32-39
    for k in range(num_unique - 1):
        mults[k] = ii[k + 1] - ii[k]
    mults[num_unique - 1] = n - ii[num_unique - 1]
    return y, mults, num_unique


def _is_conj_pair(a, b) -> bool:
    """modified_leja.m:26-39."""
    a, b = complex(a), complex(b)
    return a.real == b.real and a.imag == -b.imag and a.imag != 0


def _seq_prod(v) -> float:
    p = 1.0
    for t in v:
        p = p * t
    return p


def modified_leja(x, n, mults):
    """modified_leja.m:24-196 (recursion unrolled; capacity rescaling kept op for op)."""
    cplx = np.iscomplexobj(x)
    x = np.array(x, dtype=complex if cplx else float)
    mults = np.asarray(mults, dtype=float)
    if len(x) < n:
        raise IndexError("modified_leja: x has fewer than n entries (non-unique shifts)")
    # modified_leja_start (:41-78)
    if n < 1:
        return np.zeros(0), np.zeros(0, dtype=np.int64)
    if n == 1:
        y, outidx = [x[0]], [0]
    else:
        _, j = _matlab_max([abs(v) for v in x[:n]])
        xj = complex(x[j])
        if xj.imag == 0:
            y, outidx = [x[j]], [j]
        elif j > 0 and _is_conj_pair(x[j - 1], x[j]):
            if complex(x[j - 1]).imag < 0:
                raise ValueError("Complex conjugate pair out of order at indices %d and %d" % (j, j + 1))
            y, outidx = [x[j - 1], x[j]], [j - 1, j]
        elif j < n - 1 and _is_conj_pair(x[j], x[j + 1]):
            if xj.imag < 0:
                x[j] = x[j].real
                x[j + 1] = x[j + 1].real
            y, outidx = [x[j], x[j + 1]], [j, j + 1]
        else:
            raise ValueError("Complex shift, not in a pair, occurs at %s of input"
                             % ("beginning" if j == 0 else "end"))
    y = np.array(y, dtype=x.dtype)
    inidx = [i for i in range(n) if i not in outidx]
    # modified_leja_helper (:80-181)
    capacity = 1.0
    num_points = len(outidx)
    first = True
    while inidx:
        if not first and num_points > 1:                        # :95-117
            old_capacity = capacity
            y_last = y[num_points - 1]
            terms = [abs(y_last - x[o]) ** (mults[o] * (1.0 / num_points))
                     for o in outidx[: num_points - 1]]
            capacity = _seq_prod(terms)
            ratio = capacity / old_capacity
            if cplx:  # MATLAB complex ./ real is componentwise (NumPy uses a reciprocal)
                x = x.real / ratio + 1j * (x.imag / ratio)
                y = y.real / ratio + 1j * (y.imag / ratio)
            else:
                x = x / ratio
                y = y / ratio
        first = False
        zprod = []
        for j in inidx:                                         # :121-128
            zprod.append(_seq_prod([(abs(x[j] - x[o]) / capacity) ** mults[o] for o in outidx]))
        max_zprod, k = _matlab_max(zprod)
        j = inidx[k]
        if max_zprod == 0:
            raise ValueError("Product to maximize is zero; either there are multiple shifts, "
                             "or the product underflowed")
        if max_zprod == math.inf:
            raise ValueError("Product to maximize is Inf; must have overflowed")
        xj = complex(x[j])
        if xj.imag == 0:
            inidx = [i for i in inidx if i != j]
            outidx = outidx + [j]
            y = np.append(y, x[j])
            num_points += 1
        elif j > 0 and _is_conj_pair(x[j - 1], x[j]):
            if complex(x[j - 1]).imag < 0:
                raise ValueError("Complex conjugate pair out of order")
            inidx = [i for i in inidx if i not in (j - 1, j)]
            outidx = outidx + [j - 1, j]
            y = np.append(y, [x[j - 1], x[j]])
            num_points += 2
        elif j < n - 1 and _is_conj_pair(x[j], x[j + 1]):
            if xj.imag < 0:
                raise ValueError("Complex conjugate pair out of order")
            inidx = [i for i in inidx if i not in (j, j + 1)]
            outidx = outidx + [j, j + 1]
            y = np.append(y, [x[j], x[j + 1]])
            num_points += 2
        else:
            raise ValueError("Complex shift, not in a pair")
    y = y * capacity                                            # :192
    return y, np.array(outidx, dtype=np.int64)


def real_leja(x):
    """real_leja.m:18-87: unique/multiplicities, sort by real part, pair fix, modified Leja."""
    x = np.asarray(x).ravel()
    n = len(x)
    y, mults, num_unique = count_multiplicities(x, n)           # :44
    perm = _sort_perm(np.real(y), False)                        # :61 (stable)
    y = y[perm]
    mults = np.asarray(mults)[perm]
    k = 0
    while k < num_unique - 1:                                   # :67-81
        if np.imag(y[k]) != 0:
            if np.real(y[k]) == np.real(y[k + 1]) and np.imag(y[k]) == -np.imag(y[k + 1]):
                re, im = np.real(y[k]), abs(np.imag(y[k]))
                y[k] = re + 1j * im
                y[k + 1] = np.real(y[k]) - 1j * abs(np.imag(y[k]))
                k += 2
            else:
                _disp("Error in real_leja, complex numbers.")
                k += 1  # the reference loops forever here; fail forward instead
        else:
            k += 1
    return modified_leja(y, n, mults)                           # :86


def leja(x, which=None):
    """leja.m:23-31.  Any second argument routes to real_leja (the *modified* ordering)."""
    if which is None:
        raise NotImplementedError("nonmodified_leja is not on the ca_lanczos path")
    return real_leja(x)


def newton_basis_matrix(lam, s, modifiedp=0):
    """newton_basis_matrix.m:13-60: (s+1) x s, diag = shifts, subdiag = 1."""
    lam = np.asarray(lam)
    cplx = np.iscomplexobj(lam) and np.any(lam.imag != 0)
    B = np.zeros((s + 1, s), dtype=complex if (cplx and modifiedp == 0) else float)
    if modifiedp == 0:
        for k in range(s):
            B[k, k] = lam[k]
            B[k + 1, k] = 1.0
        return B
    for k in range(s):
        shift = complex(lam[k])
        if shift.imag > 0:
            if k == s - 1:
                raise ValueError("Complex shift occurs at end of shifts without its conjugate")
            if lam[k] != np.conj(lam[k + 1]):
                raise ValueError("Modified Leja ordering broken at k = %d" % (k + 1))
            B[k, k] = shift.real
        elif shift.imag < 0:
            if k == 0:
                raise ValueError("newton_basis_matrix: imaginary part is negative for k = 1")
            if lam[k - 1] != np.conj(lam[k]):
                raise ValueError("Modified Leja ordering broken at k = %d" % k)
            B[k, k] = shift.real
            B[k - 1, k] = -shift.imag ** 2
        else:
            B[k, k] = shift.real
        B[k + 1, k] = 1.0
    return B


def newton_change_of_basis(A, q, s, orth="full"):
    """ca_lanczos.m:66-72: 2s-step Lanczos ('full'), eig, Leja order, B matrix
    (restarted_ca_lanczos.m:63-68 uses orth 'local')."""
    _, T, _, _ = lanczos(A, q, 2 * s, orth)
    basis_eigs = matlab_eig(T)[0]
    shifts, _ = leja(basis_eigs, "nonmodified")
    Bk = newton_basis_matrix(shifts, s, 1)
    return Bk, shifts, np.asarray(basis_eigs)


# --------------------------------------------------------------------------
# a10-a12, a14: the CA-Lanczos driver
# --------------------------------------------------------------------------

def compute_ritz_rnorm(A, Q, Vp, Dp):
    """ca_lanczos.m:88-97: relative residual of every Ritz pair, sorted descending."""
    d = np.asarray(Dp)
    m = Vp.shape[0]
    out = np.zeros(m)
    ix = _sort_perm(d, True)
    for i in range(m):
        lv = d[ix[i]]
        x = Q @ Vp[:, ix[i]]
        out[i] = np.linalg.norm(A @ x - lv * x) / np.linalg.norm(lv * x)
    return out


def compute_orth_err(Q, s):
    """ca_lanczos.m:99-107: max |Q(:,1:j-s-1)'Q(:,j-s:j)| (or max|Q'Q-I| at k=1)."""
    j = Q.shape[1]
    if j > s + 1:
        return float(np.max(np.abs(Q[:, : j - s - 1].T @ Q[:, j - s - 1 : j])))
    return float(np.max(np.abs(Q.T @ Q - np.eye(s + 1))))


@dataclass
class CALanczosResult:
    T: np.ndarray
    Q: np.ndarray
    ritz_rnorm: np.ndarray
    orth_err: np.ndarray
    Bk: np.ndarray
    shifts: np.ndarray
    reorth: list
    R_blocks: list = field(default_factory=list)
    ritz_values: list = field(default_factory=list)


def _extend_T(T, b, k, s, Bk, Rkk_s, Rk_s):
    """The block update of T at k > 1 (ca_lanczos.m:201-223, repeated in
    ca_lanczos_selective :293-318 and ca_lanczos_periodic :411-436); sets
    b[k-1] and returns the extended T."""
    Rkk = np.hstack([np.zeros((s, 1)), Rkk_s[:s, :]])          # :201
    e1s1 = np.zeros((s + 1, 1))
    e1s1[0, 0] = 1.0
    Rk = np.hstack([e1s1, np.vstack([Rkk_s[s : s + 1, :s], Rk_s])])   # :202
    zk = Rk[:s, s : s + 1]
    rho = Rk[s, s]
    rho_t = Rk[s - 1, s - 1]
    bk = Bk[s, s - 1]
    e1 = np.zeros((s, 1))
    e1[0, 0] = 1.0
    es = eyeshvec(s).reshape(s, 1)
    R11 = Rk[:s, :s]
    Tk = (_rdiv_upper(R11 @ Bk[:s, :], R11)                     # :209-211
          + ((bk / rho_t) * zk) @ es.T
          - _rdiv_upper(((b[k - 2] * e1) @ es.T) @ Rkk[:s, :s], R11))
    b[k - 1] = bk * (rho / rho_t)                               # :214
    m = s * (k - 1)
    T11 = T[:m, :m]                                             # :217-223
    T12 = b[k - 2] * np.outer(eyeshvec(m), np.eye(s, 1)[:, 0])
    T21 = b[k - 2] * np.outer(np.eye(s, 1)[:, 0], eyeshvec(m))
    T31 = np.zeros((1, m))
    T32 = b[k - 1] * es.T
    return np.block([[T11, T12], [T21, Tk], [T31, T32]])


def normest(A, tol=1.0e-6, maxiter=100):
    """MATLAB ``normest(S,tol)`` (built-in, not in the reference; restated from
    its published algorithm): power iteration on S'S from x = sum(abs(S))',
    stopping when |e - e0| <= tol*e.  Used by ca_lanczos.m:258,370."""
    x = np.asarray(abs(A).sum(axis=0)).ravel().astype(float)
    e = float(np.sqrt(x @ x))
    if e == 0.0:
        return 0.0
    x = x / e
    e0 = 0.0
    cnt = 0
    while abs(e - e0) > tol * e:
        e0 = e
        Sx = A @ x
        x = A.T @ Sx
        normx = float(np.sqrt(x @ x))
        e = normx / float(np.sqrt(Sx @ Sx))
        x = x / normx
        cnt += 1
        if cnt > maxiter:
            break
    return e


def update_omega(omega_in, alpha, beta, anorm, s):
    """ca_lanczos.m:464-536: the omega recurrence (Simon's estimate of the
    loss of orthogonality), extended by s rows per outer iteration.  Indices
    are MATLAB's, shifted by one."""
    eps_ = np.finfo(float).eps
    n = len(alpha)
    Tn = eps_ * anorm
    al = lambda i: alpha[i - 1]          # noqa: E731 (1-based accessors)
    be = lambda i: beta[i - 1]           # noqa: E731
    if omega_in is None:
        om = np.zeros((s + 1, s + 1))
        O = lambda i, j: om[i - 1, j - 1]    # noqa: E731
        om[0, 0] = 1.0
        om[0, 1] = 0.0
        om[1, 0] = Tn / be(1)
        om[1, 1] = 1.0
        jr = range(2, s + 1)
    else:
        m = omega_in.shape[0] - 1
        om = np.zeros((n + 1, n + 1))
        om[: m + 1, : m + 1] = omega_in
        O = lambda i, j: om[i - 1, j - 1]    # noqa: E731
        jr = range(m + 1, m + s + 1)
    for j in jr:
        binv = 1.0 / be(j)
        v = be(2) * O(j, 2) + (al(1) - al(j)) * O(j, 1) - be(j) * O(j - 1, 1)
        om[j, 0] = binv * (v + Tn) if v > 0 else binv * (v - Tn)
        for k in range(2, j):
            v = be(k + 1) * O(j, k + 1) + (al(k) - al(j)) * O(j, k) + be(k) * O(j, k - 1) - be(j) * O(j - 1, k)
            om[j, k - 1] = binv * (v + Tn) if v > 0 else binv * (v - Tn)
        om[j, j - 1] = binv * Tn
        om[j, j] = 1.0
    return om


def reset_omega(omega_in, anorm, s):
    """ca_lanczos.m:538-549."""
    Tn = np.finfo(float).eps * anorm
    m = omega_in.shape[0] - s - 1
    om = omega_in.copy()
    for j in range(m + 1, m + s + 1):
        om[j, :j] = Tn
        om[j, j] = 1.0
    return om


def ca_lanczos_periodic(A, q, Bk, t, s, basis, diagnostics=True):
    """ca_lanczos.m:362-462: local block orthogonalisation plus a full
    reorthogonalisation of the newest s+1 columns whenever the omega
    estimate reaches sqrt(eps) (the reorthogonalised columns do not feed
    back into T, as in the reference)."""
    n = len(q)
    rnorm = np.zeros((t, t * s))
    ortherr = np.zeros(t)
    Q = np.zeros((n, t * s + 1))
    Q[:, 0] = q
    b = np.zeros(t + 1)
    T = None
    omega = None
    norm_A = normest(A)                                         # :370
    breaks, reorth, ritz = [], [], []
    k = 0
    while k < t:
        k += 1
        if k > 1:
            q = Q[:, (k - 1) * s]
        V = matrix_powers(A, q, s, Bk, basis)
        if k == 1:
            Qb, Rk, _ = normalize(V[:, : s + 1])
            Q[:, : s + 1] = Qb
            T = _rdiv_upper(Rk @ Bk, Rk[:s, :s])
            b[0] = T[s, s - 1]
            reorth.append(False)
        else:
            Qp = Q[:, (k - 2) * s : (k - 1) * s + 1]
            Q_, Rk_, info = projectAndNormalize_ex([Qp], V[:, 1 : s + 1], True)   # :402
            reorth.append(info.reorth)
            Q[:, (k - 1) * s + 1 : k * s + 1] = Q_[:, :s]
            T = _extend_T(T, b, k, s, Bk, Rk_[0], Rk_[1])
        alpha = np.diag(T, 0)                                   # :439-441
        beta = np.diag(T, -1)
        omega = update_omega(omega, alpha, beta, norm_A, s)
        err = 0.0
        for i in range(1, s + 1):                               # :442-448
            row = omega[(k - 1) * s + i, : (k - 1) * s + i]
            row_err = float(np.max(np.abs(row)))
            if row_err > err:
                err = row_err
        brk = err >= math.sqrt(np.finfo(float).eps)             # :449
        breaks.append(brk)
        if brk:
            cols = slice((k - 1) * s, k * s + 1)
            Q[:, cols], _ = projectAndNormalize([Q[:, : (k - 1) * s]], Q[:, cols], True)   # :451
            omega = reset_omega(omega, norm_A, s)
        if diagnostics:
            w, Vp = matlab_eig(T[: s * k, : s * k])
            ritz.append(w)
            rnorm[k - 1, : s * k] = compute_ritz_rnorm(A, Q[:, : s * k], Vp, w)
            ortherr[k - 1] = compute_orth_err(Q[:, : s * k + 1], s)
    res = CALanczosResult(T=T[: s * k, : s * k], Q=Q[:, : s * k], ritz_rnorm=rnorm[:k], orth_err=ortherr[:k],
                          Bk=Bk, shifts=np.zeros(0), reorth=reorth, ritz_values=ritz)
    res.breaks = breaks
    res.norm_A = norm_A
    return res


def ca_lanczos_selective(A, q, Bk, t, s, basis, diagnostics=True):
    """ca_lanczos.m:248-359: local block orthogonalisation against the
    previous block and the converged Ritz vectors QR; QR is rebuilt (all
    converged Ritz vectors, in eig order, then normalize) whenever the count
    b(k)|Vp(sk,i)| < normest(A) sqrt(eps) grows (:321-340).  A converged
    complex-conjugate pair (|Vp(sk,i)| is the same for both) makes the
    reference's QR(:,i:i+1) = Q [v, conj(v)] complex; its span is the real
    span of Q Re(v), Q Im(v), which is what is locked here (same count, same
    projections in exact arithmetic, real arithmetic throughout)."""
    n = len(q)
    rnorm = np.zeros((t, t * s))
    ortherr = np.zeros(t)
    Q = np.zeros((n, t * s + 1))
    Q[:, 0] = q
    b = np.zeros(t + 1)
    T = None
    QR = np.zeros((n, 0))
    norm_A = normest(A)
    norm_sqrt_eps = norm_A * math.sqrt(np.finfo(float).eps)     # :258
    nritz = 0
    breaks, reorth, ritz, nritz_hist, ncplx_hist = [], [], [], [], []
    k = 0
    while k < t:
        k += 1
        if k > 1:
            q = Q[:, (k - 1) * s]
        V = matrix_powers(A, q, s, Bk, basis)
        if k == 1:
            Qb, Rk, _ = normalize(V[:, : s + 1])
            Q[:, : s + 1] = Qb
            T = _rdiv_upper(Rk @ Bk, Rk[:s, :s])
            b[0] = T[s, s - 1]
            reorth.append(False)
        else:
            Qp = Q[:, (k - 2) * s : (k - 1) * s + 1]
            Q_, Rk_, info = projectAndNormalize_ex([Qp, QR[:, :nritz]], V[:, 1 : s + 1], True)   # :287
            reorth.append(info.reorth)
            Q[:, (k - 1) * s + 1 : k * s + 1] = Q_[:, :s]
            T = _extend_T(T, b, k, s, Bk, Rk_[0], Rk_[2])         # Rk_s = Rk_{3} (:291)
        w, Vp = matlab_eig(T[: s * k, : s * k])                 # :321
        conv = [i for i in range(k * s) if b[k - 1] * abs(Vp[s * k - 1, i]) < norm_sqrt_eps]   # :324-328
        brk = len(conv) > nritz                                 # :329
        breaks.append(brk)
        if brk:
            nritz = len(conv)
            # columns in eig order; the pair (i, i+1), Im w(i) > 0, as (Re v, Im v)
            M = np.zeros((k * s, nritz))
            for q_, i in enumerate(conv):
                v = Vp[:, i]
                if np.iscomplexobj(v) and w[i].imag != 0:
                    v = v.real if w[i].imag > 0 else (-v.imag)  # conj(v) of the pair's first: Im -> second column
                M[:, q_] = np.real(v)
            Y = Q[:, : k * s] @ M                               # :334-336
            QR, _, _ = normalize(Y)                             # :339
        nritz_hist.append(nritz)
        ncplx_hist.append(sum(1 for i in conv if np.iscomplexobj(w) and w[i].imag != 0))
        if diagnostics:
            ritz.append(w)
            rnorm[k - 1, : s * k] = compute_ritz_rnorm(A, Q[:, : s * k], Vp, w)
            ortherr[k - 1] = compute_orth_err(Q[:, : s * k + 1], s)
    res = CALanczosResult(T=T[: s * k, : s * k], Q=Q[:, : s * k], ritz_rnorm=rnorm[:k], orth_err=ortherr[:k],
                          Bk=Bk, shifts=np.zeros(0), reorth=reorth, ritz_values=ritz)
    res.breaks = breaks
    res.nritz = nritz_hist
    res.ncomplex = ncplx_hist  # converged Ritz values with a nonzero imaginary part
    res.norm_A = norm_A
    return res


def ca_lanczos_basic(A, q, Bk, t, s, basis, orth="local", diagnostics=True):
    """ca_lanczos.m:150-245 ('local' and 'fro')."""
    n = len(q)
    rnorm = np.zeros((t, t * s))
    ortherr = np.zeros(t)
    Q = np.zeros((n, t * s + 1))
    Q[:, 0] = q
    b = np.zeros(t + 1)
    T = None
    reorth, Rblocks, ritz = [], [], []
    k = 0
    while k < t:                                                # :166
        k += 1
        if k > 1:
            q = Q[:, (k - 1) * s]                               # :171
        V = matrix_powers(A, q, s, Bk, basis)                   # :174
        if k == 1:
            Qb, Rk, _ = normalize(V[:, : s + 1])                # :178
            Q[:, : s + 1] = Qb
            T = _rdiv_upper(Rk @ Bk, Rk[:s, :s])                # :180
            b[0] = T[s, s - 1]                                  # :182
            reorth.append(False)
            Rblocks.append((Rk.copy(),))
        else:
            Qp = Q[:, (k - 2) * s : (k - 1) * s + 1]
            Q_, Rk_, info = projectAndNormalize_ex([Qp], V[:, 1 : s + 1], True)   # :187/:193
            reorth.append(info.reorth)
            Rkk_s, Rk_s = Rk_[0], Rk_[1]
            Rblocks.append((Rkk_s.copy(), Rk_s.copy()))
            if orth == "local":
                Q[:, (k - 1) * s + 1 : k * s + 1] = Q_[:, :s]  # :188
            else:                                               # 'fro' :196-197
                Q[:, (k - 1) * s + 1 : k * s + 1] = Q_
                Qf, _ = projectAndNormalize([Q[:, : (k - 1) * s + 1]], Q[:, (k - 1) * s + 1 : k * s + 1])
                Q[:, (k - 1) * s + 1 : k * s + 1] = Qf
            T = _extend_T(T, b, k, s, Bk, Rkk_s, Rk_s)             # :201-223
        if diagnostics:                                         # :228-236
            Tk_ = T[: s * k, : s * k]
            w, Vp = matlab_eig(Tk_)
            ritz.append(w)
            rnorm[k - 1, : s * k] = compute_ritz_rnorm(A, Q[:, : s * k], Vp, w)
            ortherr[k - 1] = compute_orth_err(Q[:, : s * k + 1], s)
    T = T[: s * k, : s * k]                                     # :241-244
    return CALanczosResult(T=T, Q=Q[:, : s * k], ritz_rnorm=rnorm[:k], orth_err=ortherr[:k],
                           Bk=Bk, shifts=np.zeros(0), reorth=reorth, R_blocks=Rblocks,
                           ritz_values=ritz)


def ca_lanczos(A, r, s, iter, basis, orth="local", diagnostics=True):
    """``[T,Q,rn,oe] = ca_lanczos(A,r,s,iter,basis,orth)`` -- ca_lanczos.m:24-86.

    Returns a CALanczosResult (T, Q, ritz_rnorm, orth_err plus the Newton
    shifts, the per-iteration reorth flags and the R blocks).
    """
    o = orth.lower() if isinstance(orth, str) else str(orth)
    if o not in ("local", "full", "selective", "periodic"):
        raise ValueError("ca_lanczos.m: Invalid option value for orth: %s" % orth)   # :33-38
    t = int(math.ceil(iter / s))                                # :52
    q = r / math.sqrt(r @ r)                                    # :55
    b = basis.lower()
    if b == "monomial":                                         # :63-65
        Bk = np.eye(s + 1)[:, 1 : s + 1]
        shifts = np.zeros(0)
    elif b == "newton":                                         # :66-72
        Bk, shifts, _ = newton_change_of_basis(A, q, s)
    else:
        raise ValueError("ERROR: Unknown basis type: " + basis)  # :57-59
    if o == "periodic":                                         # :80-83
        res = ca_lanczos_periodic(A, q, Bk, t, s, b, diagnostics)
    elif o == "selective":
        res = ca_lanczos_selective(A, q, Bk, t, s, b, diagnostics)
    else:
        res = ca_lanczos_basic(A, q, Bk, t, s, b, "local" if o == "local" else "fro", diagnostics)
    res.shifts = shifts
    return res


# --------------------------------------------------------------------------
# Synthetic matrices used by BASELINE.json configs (oracle-side generators)
# --------------------------------------------------------------------------

def laplacian_2d(N: int) -> sp.csr_matrix:
    """5-point Dirichlet Laplacian on an N x N grid (stencil 4, -1), CSR, sorted."""
    T = sp.diags([-np.ones(N - 1), 2 * np.ones(N), -np.ones(N - 1)], [-1, 0, 1])
    I = sp.identity(N)
    A = (sp.kron(I, T) + sp.kron(T, I)).tocsr()
    A.eliminate_zeros()  # kron of diags() stores explicit zeros; MATLAB sparse does not
    A.sort_indices()
    return A


def laplacian_3d(N: int) -> sp.csr_matrix:
    """7-point Dirichlet Laplacian on an N^3 grid (stencil 6, -1), CSR, sorted."""
    T = sp.diags([-np.ones(N - 1), 2 * np.ones(N), -np.ones(N - 1)], [-1, 0, 1])
    I = sp.identity(N)
    A = (sp.kron(sp.kron(I, I), T) + sp.kron(sp.kron(I, T), I) + sp.kron(sp.kron(T, I), I)).tocsr()
    A.eliminate_zeros()  # kron of diags() stores explicit zeros; MATLAB sparse does not
    A.sort_indices()
    return A


def laplacian_2d_eigs(N: int) -> np.ndarray:
    c = 2.0 - 2.0 * np.cos(np.arange(1, N + 1) * np.pi / (N + 1))
    return np.sort((c[:, None] + c[None, :]).ravel())


def laplacian_3d_eigs(N: int) -> np.ndarray:
    c = 2.0 - 2.0 * np.cos(np.arange(1, N + 1) * np.pi / (N + 1))
    return np.sort((c[:, None, None] + c[None, :, None] + c[None, None, :]).ravel())


# --------------------------------------------------------------------------
# f2: the explicit restart driver (restarted_ca_lanczos.m)
# --------------------------------------------------------------------------

def _restart_lanczos_basic(A, Q_conv, q, Bk, maxiter, s, basis, orth):
    """restarted_ca_lanczos.m:261-367 (``lanczos_basic`` of that file): CA-
    Lanczos kept orthogonal to the converged vectors Q_conv.  Quirk kept: the
    loop runs maxiter+1 outer iterations (``while k <= maxiter``) and the
    output is trimmed to s*maxiter columns (:364-366)."""
    n = len(q)
    Q = np.zeros((n, (maxiter + 1) * s + 1))
    Q[:, 0] = q
    b = np.zeros(maxiter + 2)
    T = None
    k = 0
    while k <= maxiter:                                         # :277
        k += 1
        if k > 1:
            q = Q[:, (k - 1) * s]
        V = matrix_powers(A, q, s, Bk, basis)
        if k == 1:
            Q_, Rk, _ = normalize(V[:, : s + 1])                # :289
            Qn, _ = projectAndNormalize([Q_conv], Q_, True)     # :291
            Q[:, : s + 1] = Qn
            T = _rdiv_upper(Rk @ Bk, Rk[:s, :s])                # :293
            b[0] = T[s, s - 1]
        else:
            Qp = Q[:, (k - 2) * s : (k - 1) * s + 1]
            if orth == "local":                                 # :300-304
                Q_, Rk_ = projectAndNormalize([Qp, Q_conv], V[:, 1 : s + 1], True)
                Q[:, (k - 1) * s + 1 : k * s + 1] = Q_[:, :s]
                Rkk_s, Rk_s = Rk_[0], Rk_[2]
            else:                                               # 'fro' :305-310
                Q_, Rk_ = projectAndNormalize([Qp], V[:, 1 : s + 1], True)
                Rkk_s, Rk_s = Rk_[0], Rk_[1]
                Qf, _ = projectAndNormalize([Q_conv, Q[:, : (k - 2) * s]], Q_, True)
                Q[:, (k - 1) * s + 1 : k * s + 1] = Qf
            T = _extend_T(T, b, k, s, Bk, Rkk_s, Rk_s)
    return Q[:, : s * (k - 1)], T[: s * (k - 1) + 1, : s * (k - 1)]   # :364-366


def restarted_ca_lanczos(A, r, max_lanczos, n_wanted_eigs=10, s=6, basis="newton", orth="local", tol=1.0e-8,
                         max_restarts=200, diagnostics=True):
    """``[E,V,nres,rnorms,orth_err] = restarted_ca_lanczos(A,r,max_lanczos,
    n_wanted_eigs,s,basis,orth,tol)`` -- restarted_ca_lanczos.m:4-198 with
    restart_strategy 'largest'.  Only 'local' and 'full' exist in the
    reference (its lanczos_periodic / lanczos_selective are not defined).
    Returns (conv_eigs, Q_conv, num_restarts, rnorms, orth_err, converged)."""
    o = orth.lower()
    if o not in ("local", "full"):
        raise NotImplementedError("restarted_ca_lanczos.m defines no lanczos_%s" % o)
    norm_A = normest(A)                                         # :35
    tol = tol * norm_A                                          # :39
    n = len(r)
    q = r / math.sqrt(r @ r)                                    # :56
    if basis.lower() == "monomial":
        Bk = np.eye(s + 1)[:, 1 : s + 1]
    else:
        Bk, _, _ = newton_change_of_basis(A, q, s, "local")     # :63-68
    Qc = np.zeros((n, 0))
    conv_eigs, conv_rnorms = [], []
    rnorms = np.zeros((max_restarts, n_wanted_eigs))
    orth_err = []
    num_restarts, nconv, restart = 0, 0, True
    while restart and num_restarts < max_restarts:              # :81
        num_restarts += 1
        iters = max_lanczos // s                                # :86
        if iters == 0:
            break
        Q_new, T = _restart_lanczos_basic(A, Qc[:, :nconv], q, Bk, iters, s, basis.lower(),
                                          "local" if o == "local" else "fro")
        m = s * iters
        w, Vp = matlab_eig(T[:m, :m])                           # :106
        w = np.real(w)
        Vp = np.real(Vp) / np.linalg.norm(np.real(Vp), axis=0)
        beta = T[m, m - 1]                                      # :107
        ritz_norms = beta * np.abs(Vp[m - 1, :])                # :108-111
        k = 0
        for i in range(m):                                      # :114-126
            if ritz_norms[i] < tol:
                k += 1
                w[[i, k - 1]] = w[[k - 1, i]]
                Vp[:, [i, k - 1]] = Vp[:, [k - 1, i]]
                ritz_norms[[i, k - 1]] = ritz_norms[[k - 1, i]]
        newQ = Q_new @ Vp[:, :k]                                # :129-133
        Qc = np.hstack([Qc[:, :nconv], newQ])
        conv_eigs += list(w[:k])
        conv_rnorms += list(ritz_norms[:k])
        if diagnostics:                                         # :140-159
            if num_restarts > 1:
                rnorms[num_restarts - 1, :nconv] = rnorms[num_restarts - 2, :nconv]
            for i in range(k):
                if nconv + i < n_wanted_eigs:
                    lv, x = conv_eigs[nconv + i], Qc[:, nconv + i]
                    rnorms[num_restarts - 1, nconv + i] = np.linalg.norm(A @ x - lv * x) / np.linalg.norm(lv * x)
            rest = w[k:]
            ix = _sort_perm(rest, True)
            for i in range(n_wanted_eigs - nconv - k):
                lv = rest[ix[i]]
                x = Q_new @ Vp[:, k + ix[i]]
                rnorms[num_restarts - 1, nconv + i + k] = np.linalg.norm(A @ x - lv * x) / np.linalg.norm(lv * x)
            Q_ = np.hstack([Qc[:, :nconv], Q_new])              # :162-165
            orth_err.append(np.linalg.norm(np.eye(Q_.shape[1]) - Q_.T @ Q_, "fro"))
        nconv += k
        restart = len(conv_eigs) < n_wanted_eigs                # check_wanted_eigs :236-253
        if restart:                                             # generateStartVector 'largest' :200-214
            l = k
            for j in range(k, m):
                if w[j] > w[l]:
                    l = j
            q = Q_new @ Vp[:, l]
            q = q / math.sqrt(q @ q)
    ce = np.array(conv_eigs)
    ix = _sort_perm(ce, True)                                   # :180-196
    keep = n_wanted_eigs if not restart else nconv
    ix = ix[:keep]
    return dict(conv_eigs=ce[ix], conv_rnorms=np.array(conv_rnorms)[ix], Q_conv=Qc[:, ix],
                num_restarts=num_restarts, rnorms=rnorms[:num_restarts], orth_err=np.array(orth_err),
                converged=not restart, norm_A=norm_A)


# --------------------------------------------------------------------------
# f3: implicitly restarted CA-Lanczos (impl_restarted_ca_lanczos.m)
# --------------------------------------------------------------------------
# The reference file does not run: ``mu`` is undefined (:103),
# ``num_restarts`` is never assigned (:224), the residual update reuses the
# initial r (:110), it calls the standard Lanczos (:88), its 'local' branch
# reads a third R cell that does not exist (:384), it never locks
# anything (so ``nconv`` stays 0) and it always runs max_restarts.  What
# follows is the implicit restart the file sets out to implement (Sorensen's
# IRL, the algorithm its commented-out code at :180-207 and its ``qrstep``
# :623-678 come from) over the file's own CA ``lanczos_basic`` (:333-426).
# Every fix is stated where it is made.  There is no reference output to pin
# against, so this path is **parity unpinned**: tests check it against the
# analytic spectra and scipy.sparse.linalg.eigsh.

IRL_MAX_RESTARTS = 40                                           # :7


def _qr_full(X):
    """MATLAB ``[Q,R] = qr(X)`` of a square matrix (LAPACK Householder)."""
    Q, R = np.linalg.qr(X, mode="complete")
    return Q, R


def qrstep(V, H, mu, k1, k2):
    """impl_restarted_ca_lanczos.m:623-678 (D. C. Sorensen's ``qrstep``): one
    shifted QR step on H(k1:k2,k1:k2), V <- VQ, H <- Q'HQ; a complex mu applies
    the double shift (H - Re(mu) I)^2 + Im(mu)^2 I.  0-based k1..k2 inclusive."""
    kr = slice(k1, k2 + 1)
    k = k2 - k1 + 1
    eta = float(np.imag(mu))
    if abs(eta) > 0:                                            # :651-655
        xi = float(np.real(mu))
        B = H[kr, kr] - xi * np.eye(k)
        Q, _ = _qr_full(B @ B + eta * eta * np.eye(k))
    else:                                                       # :657-660
        Q, _ = _qr_full(H[kr, kr] - float(np.real(mu)) * np.eye(k))
    H[kr, :] = Q.T @ H[kr, :]                                   # :663-665
    H[:, kr] = H[:, kr] @ Q
    V[:, kr] = V[:, kr] @ Q
    m = H.shape[0]
    for j in range(k1, k2 + 1):                                 # :670-672
        H[j + 2 : m, j] = 0.0
    return V, H


def _block_T(Bk, s, bprev, Rkk_s, Rk_s):
    """Tk and the next beta of one CA block (impl_restarted_ca_lanczos.m:
    398-414 = ca_lanczos.m:200-214) from the block's projection coefficients."""
    Rkk = np.hstack([np.zeros((s, 1)), Rkk_s[:s, :]])
    e1s1 = np.zeros((s + 1, 1))
    e1s1[0, 0] = 1.0
    Rk = np.hstack([e1s1, np.vstack([Rkk_s[s : s + 1, :s], Rk_s])])
    zk = Rk[:s, s : s + 1]
    rho, rho_t = Rk[s, s], Rk[s - 1, s - 1]
    bk = Bk[s, s - 1]
    e1 = np.zeros((s, 1))
    e1[0, 0] = 1.0
    es = eyeshvec(s).reshape(s, 1)
    R11 = Rk[:s, :s]
    Tk = (_rdiv_upper(R11 @ Bk[:s, :], R11)
          + ((bk / rho_t) * zk) @ es.T
          - _rdiv_upper(((bprev * e1) @ es.T) @ Rkk[:s, :s], R11))
    return Tk, bk * (rho / rho_t)


def irl_lanczos_basic(A, Q, T, Bk, maxvecs, prevvecs, s, basis, orth, bprev):
    """``lanczos_basic`` of impl_restarted_ca_lanczos.m:333-426: CA blocks of s
    vectors appended to the factorisation A Q(:,1:p) = Q(:,1:p+1) T(1:p+1,1:p),
    p = prevvecs, in place.  Fixes: the blocks run until at least ``maxvecs``
    vectors exist (the reference's ``while nvecs <= maxvecs-s`` stops short
    when maxvecs is not a multiple of s, and m = k+p never is for k = nw+4);
    the first beta is T(p+1,p) (the reference reads ||Q(:,p+1)|| = 1, :354);
    'local' uses the two R cells its single-block call returns (:384 reads a
    third); projectAndNormalize is called with doreorth = true (the reference
    passes false, :380,:386: with one CGS pass the Newton-basis blocks of
    lap2d(40), s = 8, lose orthogonality ~50x per restart and the compressed
    basis drifts until Q_conv'Q_conv is off by 1.6 after 14 restarts).
    Returns the number of vectors built."""
    nvecs = prevvecs
    while nvecs < maxvecs:
        q = Q[:, nvecs]
        V = matrix_powers(A, q, s, Bk, basis)                   # :369
        if nvecs == 0:                                          # :371-380
            Qn, Rk, _ = normalize(V[:, : s + 1])
            Q[:, : s + 1] = Qn
            Tk = _rdiv_upper(Rk @ Bk, Rk[:s, :s])
            T[: s + 1, :s] = Tk
            bprev = Tk[s, s - 1]
        else:
            prev = Q[:, nvecs - s : nvecs + 1]
            if orth == "local":                                 # :381-386
                blocks = [prev]
            else:                                               # :387-392
                blocks = [Q[:, : nvecs - s], prev]
            Q_, Rk_ = projectAndNormalize(blocks, V[:, 1 : s + 1], True)
            Q[:, nvecs + 1 : nvecs + s + 1] = Q_
            Tk, bnew = _block_T(Bk, s, bprev, Rk_[-2], Rk_[-1])
            T[nvecs : nvecs + s, nvecs : nvecs + s] = Tk        # :417-423
            T[nvecs - 1, nvecs] = bprev
            T[nvecs, nvecs - 1] = bprev
            T[nvecs + s, nvecs + s - 1] = bnew
            bprev = bnew
        nvecs += s
    return nvecs


def irl_sizes(max_lanczos, n_wanted_eigs, s):
    """k (kept), p (shifts per restart), m = k + p (impl_restarted_ca_lanczos.m:
    72-74).  Fix: k >= s so the first extension block has a full previous
    block (the reference only runs with n_wanted a multiple of s, :66-70, where
    k = nw + 4 > s already; that restriction is lifted)."""
    k = max(n_wanted_eigs + 4, s)
    p = s * ((max_lanczos - k) // s)
    return k, p, k + p


def _sym_eig(T):
    """Ritz data of the IRL: the symmetric eigensolver on (T+T')/2 (T is
    symmetric up to rounding; ARPACK's dseupd does the same), ascending,
    orthonormal vectors even inside a multiple eigenvalue."""
    return np.linalg.eigh(0.5 * (T + T.T))


def _wanted_order(w):
    """selectShifts 'largest' (:236-243): Ritz values by modulus, descending.
    Fix: the shifts are the Ritz values themselves, not their moduli."""
    return sorted(range(len(w)), key=lambda i: -abs(w[i]))


def impl_restarted_ca_lanczos(A, r, max_lanczos, n_wanted_eigs=10, s=6, basis="newton", orth="local",
                              tol=1.0e-6, max_restarts=IRL_MAX_RESTARTS):
    """``[conv_eigs,Q_conv,num_restarts] = impl_restarted_ca_lanczos(A,r,
    max_lanczos,n_wanted_eigs,s,basis,orth,tol)`` as the intended IRL:

    1. tol = tol*normest(A) (:37-40); v1 = r/||r|| (:53); Bk from a 2s-step
       Lanczos 'full' + Leja + newton_basis_matrix (:229-234).
    2. First pass: CA-Lanczos to m vectors; later passes extend the kept
       k-vector factorisation to m (:85-94).
    3. p = m-k exact shifts (the m-k smallest-modulus Ritz values of T_m) by
       ``qrstep`` (:99-107); compress: r = V_m Q(:,k+1) H(k+1,k) +
       f_m Q(m,k), V_k = V_m Q(:,1:k), v_{k+1} = r/||r||, T(k+1,k) = ||r|| (the
       Sorensen update the reference's :110-114 garble).
    4. Converged when the n_wanted largest-modulus Ritz pairs of T_k (the
       symmetric solver on (T_k+T_k')/2, as for the shifts) all have
       ||r|| |e_k' y| < tol (:127-143, with the reference's ||Q(:,k+1)|| = 1
       replaced by ||r||).
    Returns a dict: conv_eigs (n_wanted, descending), Q_conv (n x n_wanted),
    num_restarts, converged, ritz_est (per restart, the wanted estimates),
    norm_A, k, m."""
    o = orth.lower()
    if o not in ("local", "full", "periodic", "selective"):     # :24-33
        raise ValueError("lanczos.m: Invalid option value for orth: %s" % orth)
    if o != "full":
        # 'local' fails in the reference (:384 reads Rk_{3} of a 2-cell
        # result) and periodic/selective have no lanczos_basic branch (Q_
        # undefined); without a global reorthogonalisation the compressed
        # basis of an implicit restart is not orthonormal, so only 'full' runs
        raise NotImplementedError("impl_restarted_ca_lanczos: only orth 'full' is defined (:381-392)")
    nw = n_wanted_eigs
    k, p, m = irl_sizes(max_lanczos, nw, s)
    if p < s:
        raise ValueError("impl_restarted_ca_lanczos: max_lanczos too small for n_wanted_eigs+4 plus one block")
    norm_A = normest(A)
    tol = tol * norm_A
    n = len(r)
    ncols = s * (-(-m // s)) + 1
    Q = np.zeros((n, ncols))
    T = np.zeros((ncols, ncols - 1))
    Q[:, 0] = r / math.sqrt(r @ r)
    if basis.lower() == "monomial":
        Bk = np.eye(s + 1)[:, 1 : s + 1]
    else:
        Bk, _, _ = newton_change_of_basis(A, Q[:, 0].copy(), s, "full")
    it, converged, est_hist = 0, False, []
    Y = wanted = None
    while not converged and it < max_restarts:
        it += 1
        if it == 1:
            irl_lanczos_basic(A, Q, T, Bk, m, 0, s, basis.lower(), o, 0.0)
        else:
            irl_lanczos_basic(A, Q, T, Bk, m, k, s, basis.lower(), o, T[k, k - 1])
        beta_m = T[m, m - 1]
        H = T[:m, :m].copy()
        w = _sym_eig(H)[0]
        u = [w[i] for i in _wanted_order(w)]
        Qm = np.eye(m)
        j = m
        while j > k:                                            # :99-107
            Qm, H = qrstep(Qm, H, u[j - 1], 0, m - 1)
            j -= 2 if abs(np.imag(u[j - 1])) > 0 else 1
        rv = Q[:, :m] @ Qm[:, k] * H[k, k - 1] + Q[:, m] * (beta_m * Qm[m - 1, k - 1])
        Q[:, :k] = Q[:, :m] @ Qm[:, :k]
        bk = math.sqrt(rv @ rv)
        Q[:, k] = rv / bk
        T[:, :] = 0.0
        T[:k, :k] = H[:k, :k]
        T[k, k - 1] = bk
        wk, Y = _sym_eig(T[:k, :k])
        wanted = _wanted_order(wk)[:nw]
        est = np.array([bk * abs(Y[k - 1, i]) for i in wanted])
        est_hist.append(est)
        converged = bool(np.all(est < tol))
    ev = wk[wanted]
    ix = _sort_perm(ev, True)
    sel = [wanted[i] for i in ix]
    return dict(conv_eigs=wk[sel], Q_conv=Q[:, :k] @ Y[:, sel], num_restarts=it, converged=converged,
                ritz_est=np.array(est_hist), norm_A=norm_A, k=k, m=m)
