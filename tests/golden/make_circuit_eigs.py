"""Golden fixture for the full-size config-5 test (tests/test_gpu_fullsize.py):
the 8 largest eigenvalues of the G3_circuit stand-in matrices.circuit_like(1259)
(n = 1,585,081; deterministic, seed 0) by SciPy's ARPACK eigsh, tol 1e-14.
Run from the repo root:  python tests/golden/make_circuit_eigs.py"""
import os
import sys
import time

import numpy as np
from scipy.sparse.linalg import eigsh

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import importlib.util  # noqa: E402
spec = importlib.util.spec_from_file_location("matrices", os.path.join(ROOT, "ca_lanczos_amd", "matrices.py"))
matrices = importlib.util.module_from_spec(spec)
spec.loader.exec_module(matrices)

t0 = time.time()
A = matrices.circuit_like(1259)
w = np.sort(eigsh(A, k=8, which="LA", tol=1e-14, ncv=40)[0])[::-1]
out = os.path.join(ROOT, "tests", "golden", "circuit_1259_top8.npz")
np.savez(out, eigs=w, n=A.shape[0], nnz=A.nnz)
print(out, w, "%.1f s" % (time.time() - t0))
