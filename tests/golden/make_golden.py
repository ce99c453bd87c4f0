"""Generate tests/golden/*.npz from the oracle restatement (oracle/ca_lanczos_ref.py).

The reference (MATLAB) cannot run in this pipeline and ships no golden
vectors, so these fixtures pin the restatement itself
(regression) on the reference's own synthetic inputs; the analytic spectra
pin it against known answers (tests/test_oracle.py).

    python tests/golden/make_golden.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from oracle import ca_lanczos_ref as ref  # noqa: E402

CASES = {
    # BASELINE config 1
    "c1_diag1000_s4_monomial_local": dict(mat=("diag_range", 1000), r="ones", s=4, iter=120,
                                          basis="monomial", orth="local"),
    # test_convergence_diagonal_matrices.m:9-21 inputs (local orth in place of periodic)
    "diag500_linspace_s4_newton_local": dict(mat=("diag_linspace", 1.0, 100.0, 500), r="ones", s=4, iter=120,
                                             basis="newton", orth="local"),
    # test_restart_diagonal_matrices.m:8-14 inputs, one CA-Lanczos pass
    "diag5000_linspace_s4_newton_full": dict(mat=("diag_linspace", 1.0, 1.0e4, 5000), r="ones", s=4, iter=60,
                                             basis="newton", orth="full"),
    # BASELINE config 2/3 shapes at CPU-test size
    "lap2d_32_s8_newton_local": dict(mat=("lap2d", 32), r="rand", s=8, iter=80, basis="newton", orth="local"),
    "lap3d_12_s8_newton_local": dict(mat=("lap3d", 12), r="rand", s=8, iter=80, basis="newton", orth="local"),
    "lap2d_24_s8_newton_full": dict(mat=("lap2d", 24), r="rand", s=8, iter=64, basis="newton", orth="full"),
    # test_convergence_diagonal_matrices.m:9-21 with its own orth ('periodic'), and the
    # 'selective' option of test_convergence_general_matrices.m:18, on the same matrix
    "diag500_linspace_s8_newton_periodic": dict(mat=("diag_linspace", 1.0, 100.0, 500), r="ones", s=8, iter=240,
                                                basis="newton", orth="periodic"),
    "diag500_linspace_s8_newton_selective": dict(mat=("diag_linspace", 1.0, 100.0, 500), r="ones", s=8,
                                                 iter=240, basis="newton", orth="selective"),
}


def build_matrix(spec):
    import scipy.sparse as sp
    kind = spec[0]
    if kind == "diag_range":
        a = np.arange(1.0, spec[1] + 1.0)
        return sp.csr_matrix(sp.diags(a)), np.sort(a)
    if kind == "diag_linspace":
        a = ref.matlab_linspace(spec[1], spec[2], spec[3])
        return sp.csr_matrix(sp.diags(a)), np.sort(a)
    if kind == "lap2d":
        return ref.laplacian_2d(spec[1]), ref.laplacian_2d_eigs(spec[1])
    if kind == "lap3d":
        return ref.laplacian_3d(spec[1]), ref.laplacian_3d_eigs(spec[1])
    raise ValueError(kind)


def start_vector(kind, n):
    return np.ones(n) if kind == "ones" else ref.matlab_rand(n)


def run_case(spec):
    A, exact = build_matrix(spec["mat"])
    r = start_vector(spec["r"], A.shape[0])
    res = ref.ca_lanczos(A, r, spec["s"], spec["iter"], spec["basis"], spec["orth"], diagnostics=True)
    return A, exact, r, res


def main():
    leja_rng = np.random.RandomState(2024)
    for name, spec in CASES.items():
        A, exact, r, res = run_case(spec)
        w = np.linalg.eigvals(res.T)
        np.savez_compressed(
            os.path.join(HERE, name + ".npz"),
            T=res.T, ritz_rnorm=res.ritz_rnorm, orth_err=res.orth_err, reorth=np.array(res.reorth, dtype=np.int8),
            shifts=res.shifts, Bk=res.Bk, ritz=np.sort_complex(w), exact_extremes=np.array([exact[0], exact[-1]]),
            Q_colsums=res.Q.sum(axis=0), Q_first_rows=res.Q[:4, :],
            breaks=np.array(getattr(res, "breaks", []), dtype=np.int8),
            nritz=np.array(getattr(res, "nritz", []), dtype=np.int32),
            norm_A=np.array(getattr(res, "norm_A", 0.0)),
        )
        print("%-36s T %s  reorth %d/%d  largest Ritz %.12f (exact %.12f)  rn[-1,0] %.2e"
              % (name, res.T.shape, sum(res.reorth), len(res.reorth), np.max(w.real), exact[-1],
                 res.ritz_rnorm[-1, 0]))
    # modified Leja ordering fixtures (modified_leja.m): real sets and conjugate pairs
    sets = [np.sort(leja_rng.uniform(-5.0, 20.0, 16)) for _ in range(4)]
    sets.append(np.array([1.0, 2 + 1j, 2 - 1j, 5.0, -1 + 0.5j, -1 - 0.5j, 3.0, 0.25]))
    out = {}
    for i, x in enumerate(sets):
        y, idx = ref.leja(x, "nonmodified")
        out["x%d" % i], out["y%d" % i], out["idx%d" % i] = x, y, idx
    np.savez_compressed(os.path.join(HERE, "leja.npz"), **out)
    print("leja.npz: %d sets" % len(sets))


if __name__ == "__main__":
    main()
