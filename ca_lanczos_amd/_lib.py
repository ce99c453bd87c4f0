"""ctypes binding of libcalanczos.so (the C ABI in include/calanczos.h).

The shared library is built in-tree (``python -c '__graft_entry__.build()'``
or ``make -C ca_lanczos_amd/csrc``).  There is no fallback: if the library is
missing, importing this module raises, and any compute call on a machine
without a HIP device fails with the library's own error.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, c_char_p, c_double, c_int, c_int32, c_int64, c_void_p

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# CAL_LIBRARY=testhooks loads the test build (libcalanczos_testhooks.so: the
# same sources with -DCAL_TEST_HOOKS, csrc/Makefile), which alone carries the
# result-altering test hooks; the production library has none compiled in.
# CAL_LIBRARY=variant_X loads libcalanczos_variant_X.so, a kernel-tuning build
# (`make -C ca_lanczos_amd/csrc variant V=X VFLAGS=...`, measurement only).
_which = os.environ.get("CAL_LIBRARY", "")
LIB_PATH = os.path.join(_HERE, "libcalanczos_testhooks.so" if _which == "testhooks"
                        else ("libcalanczos_%s.so" % _which if _which.startswith("variant_") else "libcalanczos.so"))

if not os.path.exists(LIB_PATH):
    raise ImportError(
        "%s not found: build it with `make -C ca_lanczos_amd/csrc` "
        "(or __graft_entry__.build()); there is no CPU fallback" % LIB_PATH)

lib = ctypes.CDLL(LIB_PATH)

CAL_OK = 0
CAL_ERR_ARG = -1
CAL_ERR_HIP = -2
CAL_ERR_NOMATRIX = -3
CAL_ERR_NUMERIC = -4
CAL_ERR_COMM = -5
CAL_ERR_UNSUPPORTED = -6
CAL_WARN_RANK_DEFICIENT = 1
CAL_WARN_BREAKDOWN = 2

dp = POINTER(c_double)
ip = POINTER(c_int)


class LanczosInfo(ctypes.Structure):
    _fields_ = [
        ("t", c_int), ("s", c_int), ("n_reorth", c_int), ("n_rank_deficient", c_int),
        ("breakdown", c_int), ("shifts", c_double * 64), ("shifts_im", c_double * 64),
        ("prologue_ms", c_double), ("loop_ms", c_double), ("diag_ms", c_double),
        ("n_orth_breaks", c_int), ("n_ritz_locked", c_int), ("norm_A", c_double), ("n_ritz_complex", c_int),
    ]


class RestartInfo(ctypes.Structure):
    _fields_ = [
        ("num_restarts", c_int), ("nconv", c_int), ("converged", c_int),
        ("norm_A", c_double), ("max_ritz_norm", c_double), ("ms", c_double),
    ]


ALLREDUCE_FN = ctypes.CFUNCTYPE(c_int, c_void_p, dp, c_int64)
EXCHANGE_FN = ctypes.CFUNCTYPE(c_int, c_void_p, c_int, dp, c_int64, dp, c_int64)

# (name, restype, argtypes) for every symbol of include/calanczos.h and
# include/calanczos_host.h -- tests check the library exports all of them.
SIGNATURES = [
    ("cal_version", c_int, []),
    ("cal_device_count", c_int, [ip]),
    ("cal_create", c_int, [c_int, POINTER(c_void_p)]),
    ("cal_destroy", None, [c_void_p]),
    ("cal_last_error", c_char_p, [c_void_p]),
    ("cal_synchronize", c_int, [c_void_p]),
    ("cal_timer_enable", c_int, [c_void_p, c_int]),
    ("cal_timer_read", c_int, [c_void_p, c_char_p, POINTER(c_int64), dp]),
    ("cal_timer_bytes", c_int, [c_void_p, c_char_p, dp]),
    ("cal_comm_stats", c_int, [c_void_p, POINTER(c_int64), c_int, c_int]),
    ("cal_timer_reset", c_int, [c_void_p]),
    ("cal_set_matrix_csc", c_int, [c_void_p, c_int64, POINTER(c_int64), POINTER(c_int64), dp]),
    ("cal_set_matrix_csr", c_int, [c_void_p, c_int64, POINTER(c_int64), POINTER(c_int32), dp]),
    ("cal_set_matrix_csr_dist", c_int,
     [c_void_p, c_int64, c_int64, c_int64, POINTER(c_int64), POINTER(c_int64), dp]),
    ("cal_matrix_info", c_int,
     [c_void_p, POINTER(c_int64), POINTER(c_int64), POINTER(c_int64), POINTER(c_int64)]),
    ("cal_set_spmv_format", c_int, [c_void_p, c_char_p]),
    ("cal_set_mpk_depth", c_int, [c_void_p, c_int]),
    ("cal_mpk_info", c_int, [c_void_p, ip, POINTER(c_int64), POINTER(c_int64), POINTER(c_int64)]),
    ("cal_mpk_schedule", c_int, [c_void_p, ip]),
    ("cal_powers_launches", c_int, [c_void_p, ip]),
    ("cal_tsqr_fold_stats", c_int, [c_void_p, ctypes.POINTER(ctypes.c_longlong), ctypes.POINTER(ctypes.c_longlong),
                                     ctypes.POINTER(ctypes.c_double)]),
    ("cal_set_tsqr_fold_tol", c_int, [c_void_p, ctypes.c_double]),
    ("cal_residency_generation", ctypes.c_longlong, []),
    ("cal_residency_invalidate", ctypes.c_longlong, []),
    ("cal_set_normalize", c_int, [c_void_p, c_char_p]),
    ("cal_get_normalize", c_int, [c_void_p, ip]),
    ("cal_set_orth_coef", c_int, [c_void_p, c_char_p]),
    ("cal_spmv_pair_info", c_int, [c_void_p, POINTER(c_int), POINTER(c_int), POINTER(c_int64)]),
    ("cal_spmv_plane_info", c_int, [c_void_p, POINTER(c_int64), POINTER(c_int), POINTER(c_int)]),
    ("cal_spmv_format", c_int, [c_void_p, ip, ip, ip]),
    ("cal_bench_spmv", c_int, [c_void_p, c_int, c_double, dp, dp]),
    ("cal_spmv", c_int, [c_void_p, dp, dp]),
    ("cal_matrix_powers_monomial", c_int, [c_void_p, dp, c_int, dp]),
    ("cal_matrix_powers_newton", c_int, [c_void_p, dp, c_int, dp, dp, c_int, dp]),
    ("cal_tsqr", c_int, [c_void_p, c_int64, c_int, dp, dp, dp]),
    ("cal_cholqr", c_int, [c_void_p, c_int64, c_int, dp, dp, dp]),
    ("cal_project", c_int, [c_void_p, c_int64, c_int, POINTER(dp), ip, c_int, dp, c_int, dp, POINTER(dp)]),
    ("cal_normalize", c_int, [c_void_p, c_int64, c_int, dp, c_double, dp, dp, ip]),
    ("cal_normalize_opt", c_int, [c_void_p, c_int64, c_int, dp, c_char_p, c_double, dp, dp, ip]),
    ("cal_project_and_normalize", c_int,
     [c_void_p, c_int64, c_int, POINTER(dp), ip, c_int, dp, c_int, dp, POINTER(dp), ip, ip]),
    ("cal_ca_lanczos", c_int,
     [c_void_p, dp, c_int, c_int, c_char_p, c_char_p, c_int, dp, dp, dp, dp, ip, POINTER(LanczosInfo)]),
    ("cal_compute_ritz_rnorm", c_int, [c_void_p, dp, c_int, dp, dp, dp]),
    ("cal_lanczos_begin", c_int, [c_void_p, dp, c_int, c_int, c_char_p, c_char_p]),
    ("cal_lanczos_step", c_int, [c_void_p, c_int]),
    ("cal_lanczos_state", c_int, [c_void_p, ip, ip, ip]),
    ("cal_lanczos_get", c_int, [c_void_p, dp, c_int, dp, dp, ip, POINTER(LanczosInfo)]),
    ("cal_lanczos_get_Q", c_int, [c_void_p, c_int64, c_int, dp]),
    ("cal_lanczos_end", c_int, [c_void_p]),
    ("cal_restarted_ca_lanczos", c_int,
     [c_void_p, dp, c_int, c_int, c_int, c_char_p, c_char_p, c_double, c_int, dp, dp, dp, dp,
      POINTER(RestartInfo)]),
    ("cal_impl_restarted_ca_lanczos", c_int,
     [c_void_p, dp, c_int, c_int, c_int, c_char_p, c_char_p, c_double, dp, dp, dp, POINTER(RestartInfo)]),
    ("cal_comm_unique_id", c_int, [c_void_p]),
    ("cal_comm_init_rccl", c_int, [c_void_p, c_int, c_int, c_void_p]),
    ("cal_comm_init_host", c_int, [c_void_p, c_int, c_int, ALLREDUCE_FN, EXCHANGE_FN, c_void_p]),
    ("cal_comm_info", c_int, [c_void_p, ip, ip, ip]),
    # calanczos_host.h
    ("cal_leja", c_int, [c_int, dp, dp, dp, dp, ip]),
    ("cal_newton_basis_matrix", c_int, [c_int, dp, dp, c_int, dp]),
    ("cal_eig", c_int, [c_int, dp, c_int, dp, dp, dp]),
    ("cal_matlab_rand", c_int, [c_int64, ctypes.c_uint, dp]),
    ("cal_tridiag_eigvals", c_int, [c_int, dp, dp, dp]),
    ("cal_qrstep", c_int, [c_int, dp, c_int, dp, c_int, c_double]),
]

for _name, _res, _args in SIGNATURES:
    _f = getattr(lib, _name)
    _f.restype = _res
    _f.argtypes = _args


class CalError(RuntimeError):
    def __init__(self, status, msg):
        super().__init__("%s (status %d)" % (msg, status))
        self.status = status


def f64(a) -> np.ndarray:
    """Column-major (MATLAB layout) float64 copy/view of a vector or matrix."""
    return np.asfortranarray(np.asarray(a, dtype=np.float64))


def ptr(a: np.ndarray):
    if a is None:
        return None
    return a.ctypes.data_as(dp)


def iptr(a: np.ndarray):
    return a.ctypes.data_as(ip)


def check(ctx, status, what=""):
    if status < 0:
        msg = lib.cal_last_error(ctx).decode() if ctx else ""
        raise CalError(status, (what + ": " if what else "") + (msg or "error"))
    return status
