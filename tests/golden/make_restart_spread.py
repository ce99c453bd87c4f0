"""Oracle restart counts of the explicit restart driver on the reference's own
input (test_restart_diagonal_matrices.m:8-28: diag(linspace(1,1e4,5000)),
max_lanczos 60, 10 wanted, s = 4, newton, 'full', tol 1e-8) for start vectors
r = ones .* (1 + 1e-15 randn) (numpy RandomState(seed), seeds 0..97).  The
count is ill-conditioned (ten wanted eigenvalues 2 apart at tol 1e-8): these
ulp-level perturbations spread it over 90..122.  Written with
OMP_NUM_THREADS=1 OPENBLAS_NUM_THREADS=1 (the oracle's own count also moves
with the BLAS thread count).  tests/test_gpu_parity.py holds the device's
counts on the first seeds against this distribution.

    OMP_NUM_THREADS=1 OPENBLAS_NUM_THREADS=1 python tests/golden/make_restart_spread.py [first last]
"""
import json
import os
import sys

import numpy as np
import scipy.sparse as sp

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from oracle import ca_lanczos_ref as ref  # noqa: E402


def start_vector(seed, n=5000):
    rng = np.random.RandomState(seed)
    return np.ones(n) * (1 + 1e-15 * rng.randn(n))


def main():
    first, last = (int(sys.argv[1]), int(sys.argv[2])) if len(sys.argv) > 2 else (0, 98)
    a = ref.matlab_linspace(1.0, 1.0e4, 5000)
    A = sp.csr_matrix(sp.diags(a))
    counts = {}
    for seed in range(first, last):
        out = ref.restarted_ca_lanczos(A, start_vector(seed), 60, 10, 4, "newton", "full", 1.0e-8)
        counts[seed] = int(out["num_restarts"])
        print(seed, counts[seed], flush=True)
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "restart_spread_diag5000.json")
    if first == 0 and last == 98:
        with open(path, "w") as f:
            json.dump({"input": "diag(linspace(1,1e4,5000)), r = ones .* (1 + 1e-15 randn(seed))",
                       "args": [60, 10, 4, "newton", "full", 1e-8],
                       "counts": [counts[s] for s in range(98)]}, f)


if __name__ == "__main__":
    main()
