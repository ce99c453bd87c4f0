"""The C ABI: the library loads without a GPU, exports every symbol the
public headers declare, and its host-only entry points match the oracle.
CPU only (no compute call needs a GPU here)."""
import ctypes
import os
import re

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared_symbols():
    names = set()
    for h in ("calanczos.h", "calanczos_host.h"):
        src = open(os.path.join(ROOT, "include", h)).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        names |= set(re.findall(r"\b(cal_[a-z0-9_]+)\s*\(", src))
    names -= {"cal_allreduce_fn", "cal_exchange_fn"}
    return names


def test_library_exports_every_declared_symbol(cal):
    lib = ctypes.CDLL(cal.LIB_PATH)
    declared = _declared_symbols()
    assert len(declared) >= 35
    missing = [s for s in declared if not hasattr(lib, s)]
    assert not missing, missing


def test_binding_covers_header():
    from ca_lanczos_amd import _lib
    bound = {s[0] for s in _lib.SIGNATURES}
    assert _declared_symbols() <= bound


def test_version_and_no_gpu_behaviour(cal):
    from ca_lanczos_amd._lib import lib
    assert lib.cal_version() >= 1
    n = ctypes.c_int(-1)
    lib.cal_device_count(ctypes.byref(n))
    h = ctypes.c_void_p()
    st = lib.cal_create(0, ctypes.byref(h))
    if n.value == 0:
        assert st != 0 and not h.value  # fails loudly, no CPU fallback
    else:  # pragma: no cover - a GPU is present
        lib.cal_destroy(h)


def test_leja_bitexact_vs_oracle(cal, ref):
    g = np.load(os.path.join(ROOT, "tests", "golden", "leja.npz"))
    for i in range(5):
        y, idx = cal.leja(g["x%d" % i], "nonmodified")
        assert np.array_equal(y, g["y%d" % i]), i
        assert np.array_equal(idx, g["idx%d" % i]), i
    rng = np.random.RandomState(7)
    for _ in range(20):
        x = np.sort(rng.uniform(-1, 13, 16))
        assert np.array_equal(cal.leja(x, "m")[0], ref.leja(x, "m")[0])


def test_newton_basis_matrix_vs_oracle(cal, ref):
    for lam in (np.array([11.5, 0.3, 6.1, 2.2, 9.0, 4.4, 1.1, 7.7]), np.array([2 + 1j, 2 - 1j, 5.0, 1.0])):
        s = len(lam)
        for modifiedp in (1,):
            assert np.array_equal(cal.newton_basis_matrix(lam, s, modifiedp), ref.newton_basis_matrix(lam, s, modifiedp))
    lam = np.arange(1.0, 5.0)
    assert np.array_equal(cal.newton_basis_matrix(lam, 4, 0), ref.newton_basis_matrix(lam, 4, 0))


def test_eig_general_and_symmetric(cal):
    rng = np.random.RandomState(5)
    for n in (1, 2, 7, 40, 121):
        T = rng.randn(n, n)
        w, V = cal.eig(T)
        assert np.max(np.abs(np.sort_complex(w) - np.sort_complex(np.linalg.eigvals(T)))) < 1e-10 * max(1, n)
        assert np.max(np.abs(T @ V - V * w[None, :])) < 1e-10 * max(1, n)
    S = rng.randn(30, 30)
    S = S + S.T
    w, V = cal.eig(S)
    assert np.isrealobj(w) and np.allclose(w, np.linalg.eigvalsh(S)) and np.allclose(V.T @ V, np.eye(30))


def test_eig_on_ca_lanczos_T(cal):
    g = np.load(os.path.join(ROOT, "tests", "golden", "lap2d_32_s8_newton_local.npz"))
    T = g["T"]
    w, V = cal.eig(T)
    assert np.max(np.abs(np.sort_complex(w) - g["ritz"])) < 1e-10
    assert np.max(np.abs(T @ V - V * w[None, :])) < 1e-10


def test_tridiag_eigvals(cal):
    from ca_lanczos_amd._lib import lib, ptr
    rng = np.random.RandomState(2)
    a, b = rng.randn(16), rng.rand(15)
    w = np.zeros(16)
    assert lib.cal_tridiag_eigvals(16, ptr(a), ptr(b), ptr(w)) == 0
    assert np.allclose(w, np.linalg.eigvalsh(np.diag(a) + np.diag(b, 1) + np.diag(b, -1)), atol=1e-13)


def test_qrstep_matches_oracle_up_to_signs(cal, ref):
    """cal_qrstep (Givens) vs the oracle's qrstep (Householder, the
    reference's impl_restarted_ca_lanczos.m:623-678): the same orthogonal
    similarity up to the signs of Q's columns, on a tridiagonal and on an
    upper-Hessenberg H, with a Ritz-value shift and an arbitrary one."""
    from ca_lanczos_amd._lib import lib, ptr
    rng = np.random.RandomState(4)
    m = 20
    d, e = rng.randn(m), rng.rand(m - 1) + 0.1
    tri = np.diag(d) + np.diag(e, 1) + np.diag(e, -1)
    hess = np.triu(rng.randn(m, m), -1)
    for H0 in (tri, hess):
        for mu in (np.linalg.eigvals(H0).real.min(), 0.37):
            Hr, Wr = H0.copy(), np.eye(m)
            Wr, Hr = ref.qrstep(Wr, Hr, mu, 0, m - 1)
            H = np.asfortranarray(H0.copy())
            W = np.asfortranarray(np.eye(m))
            assert lib.cal_qrstep(m, ptr(H), m, ptr(W), m, float(mu)) == 0
            sg = np.sign(np.sum(W * Wr, axis=0))
            assert np.all(np.abs(sg) == 1)
            # an exact shift makes H - mu I singular: the last rotation acts on
            # rounding-level numbers, so that column agrees to ~1e-10 only
            assert np.max(np.abs(W * sg - Wr)) < 1e-9
            assert np.max(np.abs(H * np.outer(sg, sg) - Hr)) < 1e-9 * np.abs(H0).max()
            assert np.max(np.abs(np.tril(H, -2))) == 0.0


def test_matlab_rand_matches_mt19937(cal, ref):
    """cal_matlab_rand (the null-space fill of normalize's randomizeNullSpace)
    is MATLAB's rand of a fresh session: MT19937 genrand_res53, the oracle's
    RandomState(seed).random_sample."""
    for seed in (5489, 7):
        assert np.array_equal(cal.matlab_rand(1000, seed), ref.matlab_rand(1000, seed=seed))



def test_residency_generation_is_process_wide(cal):
    """cal_residency_invalidate (calanczos_host.h; the MEX tier's explicit
    invalidation after an in-place edit of A, mex/calanczos_invalidate_mex.c)
    bumps the one process-wide generation every shim compares.  Host only."""
    from ca_lanczos_amd._lib import lib
    g0 = lib.cal_residency_generation()
    assert lib.cal_residency_invalidate() == g0 + 1
    assert lib.cal_residency_generation() == g0 + 1


HOOK_NAMES = ["CAL_TEST_EIG_PAIR", "CAL_TEST_PROLOGUE_SPLIT", "CAL_TEST_SELFGRAM_OFF", "CAL_TEST_APPLY_GRAM_OFF",
              "CAL_TEST_NO_PASSB_GATE", "cal_test_first_block_R", "CAL_TEST_NORMEST_SYNC",
              "CAL_TEST_NEST_DIRECT", "CAL_TEST_RESTART_COPY",
              # the pre-round-6 spellings of the same switches, and the tuning log
              "CAL_PROLOGUE_FUSED", "CAL_SELFGRAM_OFF", "CAL_APPLY_GRAM_OFF", "CAL_LOG_GRAM_SHAPES"]


def test_production_library_carries_no_test_switches():
    """The A/B switches and result-altering hooks live in the test build
    only (csrc/Makefile HOOKED objects, -DCAL_TEST_HOOKS): the production
    library's image holds none of their names, the test build holds the
    current ones."""
    prod = open(os.path.join(ROOT, "ca_lanczos_amd", "libcalanczos.so"), "rb").read()
    test = open(os.path.join(ROOT, "ca_lanczos_amd", "libcalanczos_testhooks.so"), "rb").read()
    present = [h for h in HOOK_NAMES if h.encode() in prod]
    assert not present, present
    for h in HOOK_NAMES[:9]:
        assert h.encode() in test, h


def test_context_cache_evicts_dead_matrices(cal, monkeypatch):
    """api.context_for keeps one context per live matrix; when the matrix is
    collected its context is closed and dropped.  A
    stand-in Context records set_matrix / close, so no device is needed."""
    import gc

    import scipy.sparse as sp
    from ca_lanczos_amd import api

    closed = []

    class FakeCtx:
        def set_matrix(self, A):
            self.n = A.shape[0]
            return self

        def close(self):
            closed.append(self.n)

    monkeypatch.setattr(api, "Context", FakeCtx)
    monkeypatch.setattr(api, "_matrix_ctx", {})
    A = sp.identity(5, format="csr")
    B = sp.identity(7, format="csr")
    ca, cb = api.context_for(A), api.context_for(B)
    assert api.context_for(A) is ca and api.context_for(B) is cb
    assert len(api._matrix_ctx) == 2
    del A
    gc.collect()
    assert closed == [5] and len(api._matrix_ctx) == 1
    C = sp.identity(9, format="csr")
    assert api.context_for(C) is not cb and len(api._matrix_ctx) == 2
    del B, C, cb
    gc.collect()
    assert sorted(closed) == [5, 7, 9] and not api._matrix_ctx
