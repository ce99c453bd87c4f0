"""MATLAB-named host mirror of the reference hot path over the C ABI.

Each function keeps the reference's name, argument meaning, defaults and
error behaviour (file:line cited per function) and calls the HIP library; a
sparse ``A`` is uploaded once and kept resident in HBM for every later call
with the same matrix object (the "two tiers" boundary of SURVEY §8b).
"""
from __future__ import annotations

import ctypes
import math
import os
import weakref
from dataclasses import dataclass, field

import numpy as np
import scipy.sparse as sp

from . import _lib
from ._lib import CalError, check, dp, f64, iptr, lib, ptr
from .matrices import to_csr


class Context:
    """A device context (``cal_ctx``): one HIP stream, the resident matrix and
    the device-resident CA-Lanczos state."""

    def __init__(self, device: int | None = None, spmv_format: str | None = None, orth_coef: str | None = None,
                 mpk_depth: int | None = None, normalize: str | None = None):
        if device is None:
            device = int(os.environ.get("LOCAL_RANK", "0"))
        h = ctypes.c_void_p()
        st = lib.cal_create(device, ctypes.byref(h))
        if st != 0:
            raise CalError(st, "cal_create(device=%d) failed: no usable HIP device" % device)
        self.h = h
        self.device = device
        self.n = None
        self._keep = []
        fmt = spmv_format or os.environ.get("CAL_SPMV_FORMAT", "auto")
        check(self.h, lib.cal_set_spmv_format(self.h, fmt.encode()), "spmv format")
        if orth_coef:
            self.set_orth_coef(orth_coef)
        if mpk_depth is not None:
            self.set_mpk_depth(mpk_depth)
        if normalize or os.environ.get("CAL_NORMALIZE"):
            self.set_normalize(normalize or os.environ["CAL_NORMALIZE"])

    def set_normalize(self, kind: str):
        """normalize (tsqr.m) backend: "auto", "tsqr" (Householder TSQR
        everywhere) or "cholqr2" (cal_set_normalize)."""
        check(self.h, lib.cal_set_normalize(self.h, kind.encode()), "normalize backend")
        return self

    def normalize_backend(self):
        v = ctypes.c_int()
        check(self.h, lib.cal_get_normalize(self.h, ctypes.byref(v)))
        return ("auto", "tsqr", "cholqr2")[v.value]

    def set_mpk_depth(self, depth: int):
        """Ghost depth of the distributed CA matrix-powers kernel (next
        set_matrix_slab; 1 = one halo exchange per SpMV)."""
        check(self.h, lib.cal_set_mpk_depth(self.h, int(depth)), "mpk depth")
        return self

    def mpk_info(self):
        """{'depth': active depth (1 = off), 'band_l', 'band_r', 'n_rows' (stored rows)}."""
        d, bl, br, nr = ctypes.c_int(), ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
        check(self.h, lib.cal_mpk_info(self.h, ctypes.byref(d), ctypes.byref(bl), ctypes.byref(br), ctypes.byref(nr)))
        return dict(depth=d.value, band_l=bl.value, band_r=br.value, n_rows=nr.value)

    MPK_SCHEDULES = {-1: "none", 0: "one exchange per SpMV", 1: "one deep exchange",
                     2: "one deep exchange overlapped with the interior powers",
                     3: "split schedule, no exchange (single-rank stand-in band)",
                     4: "one deep exchange on the host-staged comm thread overlapped with the interior powers"}

    def mpk_schedule(self):
        """Schedule the last matrix-powers call took (cal_mpk_schedule)."""
        v = ctypes.c_int()
        check(self.h, lib.cal_mpk_schedule(self.h, ctypes.byref(v)))
        return v.value

    def powers_launches(self):
        """SpMV-class launches of the last matrix-powers call (cal_powers_launches)."""
        v = ctypes.c_int()
        check(self.h, lib.cal_powers_launches(self.h, ctypes.byref(v)))
        return v.value

    def tsqr_fold_stats(self):
        """Fused-TSQR projectAndNormalize counters (cal_tsqr_fold_stats):
        blocks run, blocks declined (explicit-Z path), last estimate."""
        r, d, e = ctypes.c_longlong(), ctypes.c_longlong(), ctypes.c_double()
        check(self.h, lib.cal_tsqr_fold_stats(self.h, ctypes.byref(r), ctypes.byref(d), ctypes.byref(e)))
        return dict(runs=r.value, declined=d.value, last_est=e.value)

    def set_tsqr_fold_tol(self, tol: float):
        """The fused TSQR's loss-of-orthogonality acceptance threshold
        (cal_set_tsqr_fold_tol; default 1e-14, 0 declines every block that
        takes the second projection, a negative value every block)."""
        check(self.h, lib.cal_set_tsqr_fold_tol(self.h, float(tol)), "tsqr fold tol")
        return self

    def set_orth_coef(self, where: str):
        """Run the block-orthogonalisation s x s algebra on the "device"
        (default) or on the "host" (same bits; for testing)."""
        check(self.h, lib.cal_set_orth_coef(self.h, where.encode()), "orth coef")
        return self

    def bench_spmv(self, reps=20, shift=0.0):
        """Mean and min SpMV kernel time (ms) on HBM-resident vectors."""
        a, b = ctypes.c_double(), ctypes.c_double()
        check(self.h, lib.cal_bench_spmv(self.h, reps, shift, ctypes.byref(a), ctypes.byref(b)), "bench_spmv")
        return a.value, b.value

    def spmv(self, v):
        v = f64(v).ravel()
        out = np.empty_like(v)
        check(self.h, lib.cal_spmv(self.h, ptr(v), ptr(out)), "SpMV")
        return out

    def spmv_format(self):
        """('pattern'|'csr', number of row patterns, table entries)."""
        a, b, c = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        check(self.h, lib.cal_spmv_format(self.h, ctypes.byref(a), ctypes.byref(b), ctypes.byref(c)))
        return ("pattern" if a.value else "csr", b.value, c.value)

    def spmv_pair_info(self):
        """(pair patterns, their table entries, pairs on the per-row path);
        zeros when the two-rows-per-lane kernel is not in use."""
        a, b, c = ctypes.c_int(), ctypes.c_int(), ctypes.c_int64()
        check(self.h, lib.cal_spmv_pair_info(self.h, ctypes.byref(a), ctypes.byref(b), ctypes.byref(c)))
        return a.value, b.value, c.value

    def spmv_plane_info(self):
        """(plane stride P, in-plane reach H, key mode) of the plane-march
        kernels; (0, 0, -1) when the matrix does not take them."""
        a, b, c = ctypes.c_int64(), ctypes.c_int(), ctypes.c_int()
        check(self.h, lib.cal_spmv_plane_info(self.h, ctypes.byref(a), ctypes.byref(b), ctypes.byref(c)))
        return a.value, b.value, c.value

    def close(self):
        if self.h:
            lib.cal_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -- matrix ---------------------------------------------------------------
    def set_matrix(self, A):
        A = to_csr(A)
        if A.shape[0] != A.shape[1]:
            raise ValueError("A must be square")
        rowptr = np.ascontiguousarray(A.indptr, dtype=np.int64)
        col = np.ascontiguousarray(A.indices, dtype=np.int32)
        val = np.ascontiguousarray(A.data, dtype=np.float64)
        check(self.h, lib.cal_set_matrix_csr(self.h, A.shape[0], rowptr.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)),
                                             col.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), ptr(val)),
              "set_matrix")
        self.n = A.shape[0]
        return self

    def set_matrix_csc(self, A):
        """MATLAB's sparse storage (mxGetJc / mxGetIr / mxGetPr: CSC with int64
        mwIndex arrays) through cal_set_matrix_csc, the entry a MEX shim uses."""
        A = sp.csc_matrix(A)
        A.sort_indices()
        jc = np.ascontiguousarray(A.indptr, dtype=np.int64)
        ir = np.ascontiguousarray(A.indices, dtype=np.int64)
        pr = np.ascontiguousarray(A.data, dtype=np.float64)
        check(self.h, lib.cal_set_matrix_csc(self.h, A.shape[0], jc.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)),
                                             ir.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)), ptr(pr)),
              "set_matrix_csc")
        self.n = A.shape[0]
        return self

    def set_matrix_slab(self, n_global, row0, A_rows):
        """Distributed: rows [row0, row0+nlocal) of A (global column ids)."""
        A_rows = sp.csr_matrix(A_rows)
        A_rows.sort_indices()
        rowptr = np.ascontiguousarray(A_rows.indptr, dtype=np.int64)
        col = np.ascontiguousarray(A_rows.indices, dtype=np.int64)
        val = np.ascontiguousarray(A_rows.data, dtype=np.float64)
        check(self.h, lib.cal_set_matrix_csr_dist(
            self.h, n_global, row0, A_rows.shape[0], rowptr.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)),
            col.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)), ptr(val)), "set_matrix_slab")
        self.n = A_rows.shape[0]
        return self

    def matrix_info(self):
        v = [ctypes.c_int64() for _ in range(4)]
        check(self.h, lib.cal_matrix_info(self.h, *[ctypes.byref(x) for x in v]))
        return dict(n_local=v[0].value, nnz_local=v[1].value, n_global=v[2].value, nghost=v[3].value)

    # -- timers ---------------------------------------------------------------
    def timer_enable(self, on=True):
        check(self.h, lib.cal_timer_enable(self.h, 1 if on else 0))

    def timer_reset(self):
        check(self.h, lib.cal_timer_reset(self.h))

    def comm_stats(self, reset=False):
        """Communicator counters (cal_comm_stats): ranks, kind, RCCL comm
        count, all-reduces and their doubles, halo exchanges and their
        doubles, SpMV rows computed."""
        v = (ctypes.c_int64 * 8)()
        check(self.h, lib.cal_comm_stats(self.h, v, 8, 1 if reset else 0))
        keys = ("nranks", "kind", "rccl_count", "allreduce_calls", "allreduce_doubles", "halo_calls",
                "halo_doubles", "spmv_rows")
        return dict(zip(keys, [int(x) for x in v]))

    def timer_bytes(self, kind="spmv"):
        """Algorithmic HBM bytes of the timed launches of `kind`."""
        b = ctypes.c_double()
        check(self.h, lib.cal_timer_bytes(self.h, kind.encode(), ctypes.byref(b)))
        return b.value

    def timer_read(self, kind="spmv"):
        cnt = ctypes.c_int64()
        tot = ctypes.c_double()
        check(self.h, lib.cal_timer_read(self.h, kind.encode(), ctypes.byref(cnt), ctypes.byref(tot)))
        return cnt.value, tot.value

    def synchronize(self):
        check(self.h, lib.cal_synchronize(self.h))

    # -- communicators ----------------------------------------------------------
    def comm_init_rccl(self, nranks, rank, uid: bytes):
        buf = ctypes.create_string_buffer(uid, 128)
        check(self.h, lib.cal_comm_init_rccl(self.h, nranks, rank, buf), "comm_init_rccl")

    def comm_init_host(self, nranks, rank, allreduce, exchange):
        """allreduce(np.ndarray) sums in place; exchange(peer, send, recv) fills recv."""
        def _ar(user, buf, count):
            try:
                a = np.ctypeslib.as_array(buf, shape=(count,))
                allreduce(a)
                return 0
            except Exception:  # pragma: no cover - reported as CAL_ERR_COMM
                return -1

        def _ex(user, peer, send, ns, recv, nr):
            try:
                s = np.ctypeslib.as_array(send, shape=(ns,)) if ns > 0 else np.zeros(0)
                r = np.ctypeslib.as_array(recv, shape=(nr,)) if nr > 0 else np.zeros(0)
                exchange(peer, s, r)
                return 0
            except Exception:  # pragma: no cover
                return -1

        cb = (_lib.ALLREDUCE_FN(_ar), _lib.EXCHANGE_FN(_ex))
        self._keep.append(cb)
        check(self.h, lib.cal_comm_init_host(self.h, nranks, rank, cb[0], cb[1], None), "comm_init_host")

    # -- step-wise CA-Lanczos ---------------------------------------------------
    def lanczos_begin(self, r, s, max_outer, basis="newton", orth="local"):
        r = f64(r)
        check(self.h, lib.cal_lanczos_begin(self.h, ptr(r), s, max_outer, basis.encode(), orth.encode()),
              "lanczos_begin")
        self._lz = dict(s=s, max_outer=max_outer)

    def lanczos_step(self, diagnostics=False):
        return check(self.h, lib.cal_lanczos_step(self.h, 1 if diagnostics else 0), "lanczos_step")

    def lanczos_state(self):
        k, s, re = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        check(self.h, lib.cal_lanczos_state(self.h, ctypes.byref(k), ctypes.byref(s), ctypes.byref(re)))
        return k.value, s.value, re.value

    def lanczos_get(self):
        k, s, _ = self.lanczos_state()
        sk = s * k
        T = np.zeros((sk, sk), order="F")
        rn = np.zeros((k, sk), order="F")
        oe = np.zeros(k)
        fl = np.zeros(k, dtype=np.int32)
        info = _lib.LanczosInfo()
        check(self.h, lib.cal_lanczos_get(self.h, ptr(T), max(sk, 1), ptr(rn), ptr(oe), iptr(fl),
                                          ctypes.byref(info)))
        return T, rn, oe, fl, info

    def lanczos_get_Q(self, col0, ncols):
        Q = np.zeros((self.n, ncols), order="F")
        check(self.h, lib.cal_lanczos_get_Q(self.h, col0, ncols, ptr(Q)))
        return Q

    def lanczos_end(self):
        check(self.h, lib.cal_lanczos_end(self.h))


# ---------------------------------------------------------------------------
# context cache: one resident copy per matrix object (MATLAB passes A by value
# on every call; the device copy is the "persistent state" of SURVEY §8b)
# ---------------------------------------------------------------------------
_default_ctx: Context | None = None
_matrix_ctx: dict = {}


def default_context() -> Context:
    global _default_ctx
    if _default_ctx is None:
        _default_ctx = Context()
    return _default_ctx


def _evict(key, ref) -> None:
    """Close the context of a matrix that died (its weakref's callback):
    the device copy of A and the work buffers go with it."""
    hit = _matrix_ctx.get(key)
    if hit is not None and hit[0] is ref:
        del _matrix_ctx[key]
        hit[1].close()


def context_for(A) -> Context:
    key = id(A)
    hit = _matrix_ctx.get(key)
    if hit is not None and hit[0]() is A:
        return hit[1]
    if hit is not None:  # a dead matrix's id, reused before its callback ran
        _evict(key, hit[0])
    ctx = Context().set_matrix(A)
    try:
        ref = weakref.ref(A, lambda r, key=key: _evict(key, r))
    except TypeError:  # pragma: no cover  (not weak-referenceable: kept for the process)
        ref = lambda: A  # noqa: E731
    _matrix_ctx[key] = (ref, ctx)
    return ctx


# ---------------------------------------------------------------------------
# a1-a4
# ---------------------------------------------------------------------------
def SpMV(A, v):
    """``Av = SpMV(A,v)`` -- SpMV.m:6-8."""
    ctx = context_for(A)
    v = f64(v).ravel()
    out = np.empty_like(v)
    check(ctx.h, lib.cal_spmv(ctx.h, ptr(v), ptr(out)), "SpMV")
    return out


def matrix_powers_monomial(A, q, s, ctx=None):
    """``V = matrix_powers_monomial(A,q,s)`` (n x s) -- matrix_powers_monomial.m:6-12."""
    ctx = ctx or context_for(A)
    q = f64(q).ravel()
    V = np.zeros((len(q), s), order="F")
    check(ctx.h, lib.cal_matrix_powers_monomial(ctx.h, ptr(q), s, ptr(V)), "matrix_powers_monomial")
    return V


def matrix_powers_newton(A, v, s, lam, modifiedp=0, ctx=None):
    """``V = matrix_powers_newton(A,v,s,lambda,modifiedp)`` (n x (s+1)) -- matrix_powers_newton.m:15-54."""
    ctx = ctx or context_for(A)
    v = f64(v).ravel()
    lam = np.asarray(lam)
    lre = f64(np.real(lam)).ravel()
    lim = f64(np.imag(lam)).ravel() if np.iscomplexobj(lam) else None
    V = np.zeros((len(v), s + 1), order="F")
    check(ctx.h, lib.cal_matrix_powers_newton(ctx.h, ptr(v), s, ptr(lre), ptr(lim), int(modifiedp), ptr(V)),
          "matrix_powers_newton")
    return V


# ---------------------------------------------------------------------------
# a5-a9
# ---------------------------------------------------------------------------
def tsqr(A):
    """``[Q,R] = tsqr(A)`` -- tsqr.m:7-12 (R upper, diag(R) >= 0)."""
    ctx = default_context()
    A = f64(A)
    n, m = A.shape
    Q = np.zeros((n, m), order="F")
    R = np.zeros((m, m), order="F")
    check(ctx.h, lib.cal_tsqr(ctx.h, n, m, ptr(A), ptr(Q), ptr(R)), "tsqr")
    return Q, R


def cholqr(X):
    """``[Q,R] = cholqr(X)`` -- cholqr.m:3-8 (one Cholesky-QR pass)."""
    ctx = default_context()
    X = f64(X)
    n, m = X.shape
    Q = np.zeros((n, m), order="F")
    R = np.zeros((m, m), order="F")
    check(ctx.h, lib.cal_cholqr(ctx.h, n, m, ptr(X), ptr(Q), ptr(R)), "cholqr")
    return Q, R


def _blocks(Q):
    if not isinstance(Q, (list, tuple)):
        raise TypeError("Input Q (arg 1) to project() must be cell (block) array.")
    blocks = [f64(b) if (b is not None and np.size(b) > 0) else None for b in Q]
    widths = np.array([0 if b is None else b.shape[1] for b in blocks], dtype=np.int32)
    arr = (dp * max(len(blocks), 1))(*[ptr(b) if b is not None else None for b in blocks])
    return blocks, widths, arr


def project(Q, X, doreorth=False, ctx=None):
    """``[X,R] = project(Q,X,doreorth)`` -- project.m:7-58."""
    if isinstance(X, (list, tuple)):
        raise TypeError("Input X (arg 2) project() must be a column matrix.")
    if len(Q) == 0:
        return np.array(X, dtype=np.float64), []
    ctx = ctx or default_context()
    X = f64(X)
    n, m = X.shape
    blocks, widths, arr = _blocks(Q)
    R = [np.zeros((int(w), m), order="F") for w in widths]
    Rarr = (dp * len(R))(*[ptr(r) for r in R])
    Xout = np.zeros((n, m), order="F")
    check(ctx.h, lib.cal_project(ctx.h, n, len(blocks), arr, iptr(widths), m, ptr(X), 1 if doreorth else 0,
                                 ptr(Xout), Rarr), "project")
    return Xout, R


def normalize(X, opt="None", tol=1.0e-8, ctx=None):
    """``[Q,R,rank] = normalize(X,opt,tol)`` -- normalize.m:3-36; opt
    'randomizeNullSpace' runs normalize.m:28-31,38-51 (the null-space
    columns drawn from a fresh MATLAB rand stream, seed 5489)."""
    ctx = ctx or default_context()
    X = f64(X)
    n, m = X.shape
    Q = np.zeros((n, m), order="F")
    R = np.zeros((m, m), order="F")
    rank = ctypes.c_int()
    check(ctx.h, lib.cal_normalize_opt(ctx.h, n, m, ptr(X), str(opt).encode(), tol, ptr(Q), ptr(R),
                                       ctypes.byref(rank)), "normalize")
    return Q, R, rank.value


def matlab_rand(count, seed=5489):
    """MATLAB ``rand`` of a fresh session (rng(seed,'twister')): cal_matlab_rand."""
    out = np.zeros(int(count))
    check(None, lib.cal_matlab_rand(int(count), int(seed), ptr(out)), "matlab_rand")
    return out


def projectAndNormalize_ex(Q, X, doreorth=True, ctx=None):
    """projectAndNormalize.m:3-90, also returning (reorth flag, rank).  With
    a distributed context, Q / X are this rank's local rows."""
    ctx = ctx or default_context()
    X = f64(X)
    n, m = X.shape
    blocks, widths, arr = _blocks(Q)
    RZ = [np.zeros((int(w), m), order="F") for w in widths] + [np.zeros((m, m), order="F")]
    RZarr = (dp * len(RZ))(*[ptr(r) for r in RZ])
    QZ = np.zeros((n, m), order="F")
    re, rk = ctypes.c_int(), ctypes.c_int()
    check(ctx.h, lib.cal_project_and_normalize(ctx.h, n, len(blocks), arr, iptr(widths), m, ptr(X),
                                               1 if doreorth else 0, ptr(QZ), RZarr, ctypes.byref(re),
                                               ctypes.byref(rk)), "projectAndNormalize")
    return QZ, RZ, bool(re.value), rk.value


def projectAndNormalize(Q, X, doreorth=True):
    """``[QZ,RZ] = projectAndNormalize(Q,X,doreorth)`` -- projectAndNormalize.m:3-90."""
    QZ, RZ, _, _ = projectAndNormalize_ex(Q, X, doreorth)
    return QZ, RZ


# ---------------------------------------------------------------------------
# a13 host routines
# ---------------------------------------------------------------------------
def leja(x, which=None):
    """``[y,idx] = leja(x,'nonmodified')`` -> real_leja -> modified_leja (leja.m:23-31)."""
    if which is None:
        raise NotImplementedError("nonmodified_leja is not on the ca_lanczos path")
    x = np.asarray(x).ravel()
    n = len(x)
    xr = f64(np.real(x))
    xi = f64(np.imag(x)) if np.iscomplexobj(x) else None
    yr, yi = np.zeros(n), np.zeros(n)
    idx = np.zeros(n, dtype=np.int32)
    st = lib.cal_leja(n, ptr(xr), ptr(xi), ptr(yr), ptr(yi), iptr(idx))
    if st != 0:
        raise CalError(st, "leja: modified Leja ordering failed")
    y = yr + 1j * yi if np.any(yi != 0) else yr
    return y, idx.astype(np.int64)


def newton_basis_matrix(lam, s, modifiedp=0):
    """``B_ = newton_basis_matrix(lambda,s,modifiedp)`` -- newton_basis_matrix.m:13-60."""
    lam = np.asarray(lam)
    lr = f64(np.real(lam)).ravel()
    li = f64(np.imag(lam)).ravel() if np.iscomplexobj(lam) else None
    B = np.zeros((s + 1, s), order="F")
    st = lib.cal_newton_basis_matrix(s, ptr(lr), ptr(li), int(modifiedp), ptr(B))
    if st != 0:
        raise CalError(st, "newton_basis_matrix failed")
    return B


def eig(T):
    """``[V,D] = eig(T)`` as used by ca_lanczos.m:229 -> (w complex/real, V)."""
    T = f64(T)
    n = T.shape[0]
    wr, wi = np.zeros(n), np.zeros(n)
    V = np.zeros((n, n), order="F")
    st = lib.cal_eig(n, ptr(T), n, ptr(wr), ptr(wi), ptr(V))
    if st != 0:
        raise CalError(st, "eig did not converge")
    if np.any(wi != 0):
        Vc = V.astype(complex)
        j = 0
        while j < n:
            if wi[j] > 0:
                Vc[:, j] = V[:, j] + 1j * V[:, j + 1]
                Vc[:, j + 1] = V[:, j] - 1j * V[:, j + 1]
                j += 2
            else:
                j += 1
        return wr + 1j * wi, Vc
    return wr, V


# ---------------------------------------------------------------------------
# a14: the driver
# ---------------------------------------------------------------------------
def compute_ritz_rnorm(A, Q, Vp, Dp, ctx=None):
    """``ritz_rnorm = compute_ritz_rnorm(A,Q,Vp,Dp)`` -- ca_lanczos.m:88-97 (real
    Dp: a vector of eigenvalues or the diagonal matrix).  The Ritz vectors
    x = Q*Vp(:,i) are formed on the device; the values are sorted descending
    as the reference does."""
    ctx = ctx or context_for(A)
    Q = np.asfortranarray(f64(Q))
    Vp = np.asfortranarray(f64(Vp))
    d = f64(np.diag(Dp) if np.ndim(Dp) == 2 else Dp).ravel().copy()
    k = Vp.shape[1]
    if Q.shape[1] != k or Vp.shape[0] != k or d.size != k:
        raise ValueError("compute_ritz_rnorm: Q is n x k, Vp k x k, Dp k values")
    rn = np.zeros(k)
    check(ctx.h, lib.cal_compute_ritz_rnorm(ctx.h, ptr(Q), k, ptr(Vp), ptr(d), ptr(rn)), "compute_ritz_rnorm")
    return rn


@dataclass
class CALanczosOutput:
    T: np.ndarray
    Q: np.ndarray | None
    ritz_rnorm: np.ndarray
    orth_err: np.ndarray
    reorth: np.ndarray
    shifts: np.ndarray
    info: dict = field(default_factory=dict)


def ca_lanczos_ex(A, r, s, iter, basis, orth="local", diagnostics=True, return_Q=True, ctx=None):
    """ca_lanczos.m:24-86 with the extra outputs (flags, shifts, timings)."""
    o = orth.lower() if isinstance(orth, str) else str(orth)
    if o not in ("local", "full", "selective", "periodic"):
        raise ValueError("ca_lanczos.m: Invalid option value for orth: %s" % orth)
    ctx = ctx or context_for(A)
    r = f64(r).ravel()
    t = int(math.ceil(iter / s))
    n = len(r)
    T = np.zeros((s * t, s * t), order="F")
    Q = np.zeros((n, s * t), order="F") if return_Q else None
    rn = np.zeros((t, s * t), order="F")
    oe = np.zeros(t)
    fl = np.zeros(t, dtype=np.int32)
    info = _lib.LanczosInfo()
    st = lib.cal_ca_lanczos(ctx.h, ptr(r), s, iter, basis.encode(), orth.encode(), 1 if diagnostics else 0,
                            ptr(T), ptr(Q), ptr(rn), ptr(oe), iptr(fl), ctypes.byref(info))
    check(ctx.h, st, "ca_lanczos")
    k = info.t
    sk = s * k
    shifts = np.array(info.shifts[: 2 * s]) if basis.lower() == "newton" else np.zeros(0)
    if np.any(np.array(info.shifts_im[: 2 * s]) != 0):
        shifts = shifts + 1j * np.array(info.shifts_im[: 2 * s])
    return CALanczosOutput(
        T=np.array(T[:sk, :sk]), Q=None if Q is None else np.array(Q[:, :sk]),
        ritz_rnorm=np.array(rn[:k, :sk]), orth_err=oe[:k].copy(), reorth=fl[:k].copy(), shifts=shifts,
        info=dict(t=k, n_reorth=info.n_reorth, n_rank_deficient=info.n_rank_deficient,
                  breakdown=info.breakdown, prologue_ms=info.prologue_ms, loop_ms=info.loop_ms,
                  diag_ms=info.diag_ms, status=st, n_orth_breaks=info.n_orth_breaks,
                  n_ritz_locked=info.n_ritz_locked, norm_A=info.norm_A,
                  n_ritz_complex=info.n_ritz_complex))


def ca_lanczos(A, r, s, iter, basis, orth="local"):
    """``[T,Q,ritz_rnorm,orth_err] = ca_lanczos(A,r,s,iter,basis,orth)`` -- ca_lanczos.m:24-86."""
    out = ca_lanczos_ex(A, r, s, iter, basis, orth, diagnostics=True, return_Q=True)
    return out.T, out.Q, out.ritz_rnorm, out.orth_err


# ---------------------------------------------------------------------------
# f2: explicit restart
# ---------------------------------------------------------------------------
MAX_RESTARTS = 200  # restarted_ca_lanczos.m:6


def restarted_ca_lanczos(A, r, max_lanczos, n_wanted_eigs=10, s=6, basis="newton", orth="local", tol=1.0e-8,
                         diagnostics=True, ctx=None):
    """``[E,V,nres,rnorms,orth_err] = restarted_ca_lanczos(A,r,max_lanczos,
    n_wanted_eigs,s,basis,orth,tol)`` -- restarted_ca_lanczos.m:4-198.

    Returns a dict: conv_eigs (descending), Q_conv (n x nconv), num_restarts,
    rnorms (num_restarts x n_wanted_eigs), orth_err (num_restarts),
    converged, norm_A."""
    ctx = ctx or context_for(A)
    r = f64(r).ravel()
    n = len(r)
    E = np.zeros(n_wanted_eigs)
    V = np.zeros((n, n_wanted_eigs), order="F")
    rn = np.zeros((MAX_RESTARTS, n_wanted_eigs), order="F")
    oe = np.zeros(MAX_RESTARTS)
    info = _lib.RestartInfo()
    st = lib.cal_restarted_ca_lanczos(ctx.h, ptr(r), int(max_lanczos), int(n_wanted_eigs), int(s), basis.encode(),
                                      orth.encode(), float(tol), 1 if diagnostics else 0, ptr(E), ptr(V), ptr(rn),
                                      ptr(oe), ctypes.byref(info))
    check(ctx.h, st, "restarted_ca_lanczos")
    k, nr = info.nconv, info.num_restarts
    return dict(conv_eigs=E[:k].copy(), Q_conv=V[:, :k].copy(), num_restarts=nr, rnorms=rn[:nr].copy(),
                orth_err=oe[:nr].copy(), converged=bool(info.converged), norm_A=info.norm_A, ms=info.ms)


IMPL_MAX_RESTARTS = 40  # impl_restarted_ca_lanczos.m:7


def impl_restarted_ca_lanczos(A, r, max_lanczos, n_wanted_eigs=10, s=6, basis="newton", orth="full", tol=1.0e-6,
                              ctx=None, return_Q=True):
    """``[conv_eigs,Q_conv,num_restarts] = impl_restarted_ca_lanczos(A,r,
    max_lanczos,n_wanted_eigs,s,basis,orth,tol)`` -- the implicit restart
    impl_restarted_ca_lanczos.m:4-226 sets out to implement (the file itself
    does not run).  Only orth 'full' is defined.

    Returns a dict: conv_eigs (n_wanted_eigs, descending), Q_conv
    (n x n_wanted_eigs; None with return_Q=False: the Ritz vectors are formed
    on the device but not copied to the host), num_restarts, converged,
    ritz_est (num_restarts x n_wanted_eigs), norm_A."""
    ctx = ctx or context_for(A)
    r = f64(r).ravel()
    n = len(r)
    E = np.zeros(n_wanted_eigs)
    V = np.zeros((n, n_wanted_eigs), order="F") if return_Q else None
    est = np.zeros((IMPL_MAX_RESTARTS, n_wanted_eigs), order="F")
    info = _lib.RestartInfo()
    st = lib.cal_impl_restarted_ca_lanczos(ctx.h, ptr(r), int(max_lanczos), int(n_wanted_eigs), int(s),
                                           basis.encode(), orth.encode(), float(tol), ptr(E),
                                           ptr(V) if return_Q else None, ptr(est),
                                           ctypes.byref(info))
    check(ctx.h, st, "impl_restarted_ca_lanczos")
    k, nr = info.nconv, info.num_restarts
    return dict(conv_eigs=E[:k].copy(), Q_conv=V[:, :k].copy() if return_Q else None, num_restarts=nr,
                ritz_est=est[:nr].copy(),
                converged=bool(info.converged), norm_A=info.norm_A, ms=info.ms)
