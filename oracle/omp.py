"""ctypes binding of oracle/build/libcal_omp.so, the C/OpenMP restatement of
ca_lanczos_basic 'local' (oracle/c/ca_lanczos_omp.c).  TEST INFRASTRUCTURE
ONLY: the CPU baseline of bench.py and a second oracle in the CPU tests."""
from __future__ import annotations

import ctypes
import math
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "build", "libcal_omp.so")
_lib = None


def build():
    subprocess.run(["make", "-C", HERE], check=True, stdout=subprocess.DEVNULL)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        _lib = ctypes.CDLL(LIB)
        _lib.cal_omp_ca_lanczos_local.restype = ctypes.c_int
        _lib.cal_omp_threads.restype = ctypes.c_int
        _lib.cal_omp_set_threads.restype = ctypes.c_int
        _lib.cal_omp_set_threads.argtypes = [ctypes.c_int]
        _lib.cal_omp_loop_seconds.restype = ctypes.c_double
    return _lib


def threads() -> int:
    return int(lib().cal_omp_threads())


def set_threads(n: int) -> None:
    if lib().cal_omp_set_threads(int(n)) != 0:
        raise ValueError("thread count must be >= 1")


def loop_seconds() -> float:
    """Wall time of the last ca_lanczos_local's outer loop (buffers allocated
    and first-touched before it, as the GPU bench's are resident)."""
    return float(lib().cal_omp_loop_seconds())


def ca_lanczos_local(A, q, Bk, s, t, newton=True):
    """T (st x st) and the reorth flags of t outer iterations of
    ca_lanczos_basic 'local' (ca_lanczos.m:150-245) from the normalised q and
    the change-of-basis matrix Bk ((s+1) x s)."""
    A = A.tocsr()
    n = A.shape[0]
    rp = np.ascontiguousarray(A.indptr, dtype=np.int64)
    col = np.ascontiguousarray(A.indices, dtype=np.int32)
    val = np.ascontiguousarray(A.data, dtype=np.float64)
    q = np.ascontiguousarray(q, dtype=np.float64)
    Bk = np.asfortranarray(Bk, dtype=np.float64)
    T = np.zeros((s * t, s * t), order="F")
    flags = np.zeros(t, dtype=np.int32)
    dp = ctypes.POINTER(ctypes.c_double)
    st = lib().cal_omp_ca_lanczos_local(
        ctypes.c_int64(n), rp.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)),
        col.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), val.ctypes.data_as(dp), q.ctypes.data_as(dp),
        Bk.ctypes.data_as(dp), int(s), int(t), 1 if newton else 0, T.ctypes.data_as(dp),
        flags.ctypes.data_as(ctypes.POINTER(ctypes.c_int)))
    if st != 0:
        raise RuntimeError("cal_omp_ca_lanczos_local failed (%d)" % st)
    return T, [bool(f) for f in flags]


def ca_lanczos(A, r, s, iter, basis="newton"):
    """ca_lanczos(A,r,s,iter,basis,'local') with diagnostics off; the Newton
    prologue comes from the NumPy oracle (ca_lanczos.m:66-72)."""
    from . import ca_lanczos_ref as ref
    q = r / math.sqrt(r @ r)
    if basis == "newton":
        Bk, _, _ = ref.newton_change_of_basis(A, q, s)
    else:
        Bk = np.eye(s + 1)[:, 1 : s + 1]
    return ca_lanczos_local(A, q, Bk, s, int(math.ceil(iter / s)), basis == "newton")
