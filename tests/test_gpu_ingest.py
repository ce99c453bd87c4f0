"""SURVEY §8 row f4 on the device: matrices read from files and fed to the
solvers, as the reference's restart suite does (load(...); A = Problem.A;
test_restarted_ca_lanczos_all_matrices.m:25-30).

Each matrix is written to a Matrix Market file (symmetric, lower triangle,
%.17g values) and to a MATLAB v5 .mat holding the SuiteSparse ``Problem``
struct, read back through ``matrices.load_matrix`` (bit-identical to the
matrix written), and run through the HIP path: ca_lanczos ('local', s = 8
Newton) against the oracle, and the implicit restart against the oracle /
the closed-form spectrum.  bench.py --matrix FILE is the same ingestion in
the benchmark (both drivers).
"""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _write_mtx(path, A):
    import scipy.sparse as sp
    L = sp.tril(A).tocoo()
    with open(path, "w") as f:
        f.write("%%%%MatrixMarket matrix coordinate real symmetric\n%% written by tests/test_gpu_ingest.py\n"
                "%d %d %d\n" % (A.shape[0], A.shape[1], L.nnz))
        np.savetxt(f, np.column_stack([L.row + 1, L.col + 1, L.data]), fmt="%d %d %.17g")


def _write_mat(path, A, name):
    import scipy.io
    scipy.io.savemat(path, {"Problem": {"A": A.tocsc(), "name": name, "kind": "test matrix"}}, format="5")


def _ingest(cal, tmp_path, which, fmt):
    A = cal.matrices.laplacian_2d(40) if which == "lap2d_40" else cal.matrices.circuit_like(200)
    p = os.path.join(str(tmp_path), "%s.%s" % (which, fmt))
    if fmt == "mtx":
        _write_mtx(p, A)
    else:
        _write_mat(p, A, which)
    B = cal.matrices.load_matrix(p)
    assert np.array_equal(A.indptr, B.indptr) and np.array_equal(A.indices, B.indices)
    assert np.array_equal(A.data, B.data)
    return B, p


@pytest.mark.parametrize("fmt", ["mtx", "mat"])
@pytest.mark.parametrize("which", ["lap2d_40", "circuit_200"])
def test_ingested_matrix_ca_lanczos_vs_oracle(cal, ref, tmp_path, which, fmt):
    """ca_lanczos(A, r, 8, 64, 'newton', 'local') on the file's matrix: the
    same reorthogonalisation flags and Newton shifts (1e-9 ||A||), the first
    two blocks of T within 1e-9 ||A|| (later 'local' blocks are chaotic in
    the oracle itself once orthogonality is lost), the extreme Ritz values
    within 1e-10 ||A||, the largest pair's residual history within 2x."""
    A, _ = _ingest(cal, tmp_path, which, fmt)
    n = A.shape[0]
    r = ref.matlab_rand(n)
    out = cal.ca_lanczos_ex(A, r, 8, 64, "newton", "local")
    exp = ref.ca_lanczos(A, r, 8, 64, "newton", "local")
    normA = float(abs(A).sum(axis=1).max())
    assert out.T.shape == exp.T.shape
    assert list(out.reorth) == list(exp.reorth)
    assert np.max(np.abs(out.shifts - exp.shifts)) <= 1e-9 * normA
    assert np.max(np.abs(out.T[:16, :16] - exp.T[:16, :16])) <= 1e-9 * normA
    w, we = np.sort(np.linalg.eigvals(out.T).real), np.sort(np.linalg.eigvals(exp.T).real)
    assert abs(w[-1] - we[-1]) <= 1e-10 * normA and abs(w[0] - we[0]) <= 1e-10 * normA
    a, b = out.ritz_rnorm[:, 0], exp.ritz_rnorm[:, 0]
    big = b > 1e-10
    assert np.all(np.abs(np.log(a[big] / b[big])) < np.log(2.0))


@pytest.mark.parametrize("fmt", ["mtx", "mat"])
def test_ingested_circuit_impl_restart_vs_oracle(cal, ref, tmp_path, fmt):
    """impl_restarted_ca_lanczos(A, r, 48, 6, 8, 'newton', 'full', 1e-8) on
    the file's G3_circuit stand-in (n = 40 000): converged, the oracle's
    eigenvalues within 1e-10 |lambda_1|, orthonormal Ritz vectors with
    residuals below 1e-7 |lambda|."""
    A, _ = _ingest(cal, tmp_path, "circuit_200", fmt)
    r = ref.matlab_rand(A.shape[0])
    exp = ref.impl_restarted_ca_lanczos(A, r, 48, 6, 8, "newton", "full", 1.0e-8)
    out = cal.impl_restarted_ca_lanczos(A, r, 48, 6, 8, "newton", "full", 1.0e-8)
    assert out["converged"] and exp["converged"]
    scale = abs(exp["conv_eigs"][0])
    assert np.max(np.abs(out["conv_eigs"] - exp["conv_eigs"])) <= 1e-10 * scale
    V = out["Q_conv"]
    assert np.max(np.abs(V.T @ V - np.eye(6))) < 1e-9
    res = np.linalg.norm(A @ V - V * out["conv_eigs"], axis=0) / np.abs(out["conv_eigs"])
    assert np.max(res) < 1e-7


def test_ingested_lap2d_impl_restart_spectrum(cal, ref, tmp_path):
    """The same on the .mat lap2d(40) (double eigenvalues): every returned
    value is an eigenvalue of A (closed form) and the largest one is found."""
    A, _ = _ingest(cal, tmp_path, "lap2d_40", "mat")
    eref = ref.laplacian_2d_eigs(40)[::-1]
    out = cal.impl_restarted_ca_lanczos(A, ref.matlab_rand(1600), 48, 8, 8, "newton", "full", 1.0e-8)
    assert out["converged"]
    ev = out["conv_eigs"]
    assert np.max(np.min(np.abs(ev[:, None] - eref[None, :]), axis=1)) <= 1e-10 * 8.0
    assert abs(ev[0] - eref[0]) <= 1e-10 * 8.0


def _bench(*args, timeout=300):
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], cwd=ROOT, capture_output=True,
                       text=True, timeout=timeout)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, p.stdout[-2000:]
    return json.loads(lines[0])


def test_bench_matrix_file_both_drivers(cal, tmp_path):
    """bench.py --matrix FILE (the path a SuiteSparse run takes): the IRL
    driver and the CA-Lanczos driver each print one valid line on the
    file's matrix."""
    _, p = _ingest(cal, tmp_path, "circuit_200", "mtx")
    d = _bench("--matrix", p, "--driver", "irl", "--steps", "2", "--warmup", "1", "--no-cpu-baseline")
    assert d["metric"].startswith("impl_restarted_ca_lanczos solves/sec") and d["unit"] == "solves/s"
    assert d["config"]["workload"].startswith("file:circuit_200.mtx, n=40000")
    assert d["converged"] and d["value"] > 0 and d["steps"] == 2
    assert 0 < d["roofline"]["frac"] < 1.5
    d = _bench("--matrix", p, "--steps", "3", "--warmup", "1", "--no-cpu-baseline", "--no-legs")
    assert d["metric"].startswith("CA-Lanczos outer-iters/sec") and d["value"] > 0
    assert d["config"]["workload"].startswith("file:circuit_200.mtx") and d["steps"] == 3
    assert d["data"].startswith("file circuit_200.mtx")
