"""GPU tests on the test build of the library (libcalanczos_testhooks.so,
CAL_LIBRARY=testhooks): A/B switches and NaN-poisoned scratch that the
production library does not carry.  Each case runs in a child process (the
library is chosen at import), which prints one JSON line.

* The first-block rank test (normalize.m:18-35 inside ca_lanczos.m:176) on a
  start vector in a 1-/2-dimensional invariant subspace: every scratch buffer
  is NaN when allocated and the coefficient scratch is NaN before each block,
  so the device CholQR2 path (blockorth.cpp orth_device) reads nothing it did
  not write.  The rank deficiency must be found from a finite R.
* The fused Newton prologue / normest launches against the separate ones
  (lanczos.m:103-110, ca_lanczos.m:258): the same bits.
* The fused update+Gram block-MGS steps (k_apply_gram, the X'X hand-off into
  the normalize) against the unfused ones (restarted_ca_lanczos.m:291-309,
  impl_restarted_ca_lanczos.m:333-426).
"""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PRELUDE = ("import sys, os, json, ctypes, numpy as np, scipy.sparse as sp; sys.path.insert(0, %r)\n"
           "import ca_lanczos_amd as cal\n"
           "from ca_lanczos_amd import _lib\n"
           "assert _lib.LIB_PATH.endswith('/libcalanczos_testhooks.so')\n"
           "from oracle import ca_lanczos_ref as ref\n" % ROOT)


def run_testhooks(body, timeout=240, **env):
    e = dict(os.environ, CAL_LIBRARY="testhooks")
    e.update(env)
    p = subprocess.run([sys.executable, "-c", PRELUDE + body], env=e, capture_output=True, text=True,
                       timeout=timeout)
    assert p.returncode == 0, p.stderr[-3000:]
    return json.loads(p.stdout.strip().splitlines()[-1])


EXHAUSTED = r"""
lib = _lib.lib
lib.cal_test_first_block_R.restype = ctypes.c_int
n = 100
A = cal.matrices.diagonal(np.arange(1.0, n + 1.0))
big = cal.matrices.laplacian_3d(40)
rows = []
for pre in (False, True):
    ctx = cal.Context()
    if pre:  # the context's scratch sized by a 64000-row run first
        ctx.set_matrix(big)
        cal.ca_lanczos_ex(big, ref.matlab_rand(big.shape[0]), 8, 32, "newton", "local", diagnostics=True, ctx=ctx)
    ctx.set_matrix(A)
    for start in ("one", "two"):
        for s, basis in ((2, "monomial"), (4, "monomial"), (4, "newton"), (8, "newton")):
            r = np.eye(n)[0] + (np.eye(n)[5] if start == "two" else 0.0)
            row = dict(pre=pre, start=start, s=s, basis=basis)
            try:
                out = cal.ca_lanczos_ex(A, r, s, 3 * s, basis, "local", diagnostics=False, ctx=ctx)
                row.update(status=0, nrd=int(out.info["n_rank_deficient"]), brk=int(out.info["breakdown"]))
            except cal.CalError as ex:
                row.update(status=int(ex.status), nrd=-1, brk=-1)
            R = np.zeros((s + 1) * (s + 1))
            m = lib.cal_test_first_block_R(ctx.h, R.ctypes.data_as(ctypes.POINTER(ctypes.c_double)), R.size)
            row["m"] = int(m)
            if m == s + 1:
                R = R.reshape(m, m, order="F")
                row["finite"] = bool(np.isfinite(R).all())
                sv = np.linalg.svd(R, compute_uv=False) if row["finite"] else np.full(m, np.nan)
                row["svratio"] = float(sv[-1] / sv[0])
            rows.append(row)
    ctx.close()
print(json.dumps(rows))
"""


def test_exhausted_krylov_first_block_finite_R_poisoned():
    """With the pass-B gate (product): every case's first-block R is finite
    and rank-deficient (smallest / largest singular value <= 1e-8, the
    normalize.m:19-24 test) and the run reports it.  Without the gate
    (CAL_TEST_NO_PASSB_GATE, the code before the fix), a Cholesky failure on
    the device still ran pass B with the unwritten (here NaN) coefficients
    into Q(:,1:s+1) -- the storage of the first block's input column q --
    before the host redid the block from that input: R comes back NaN.
    That is the intermittent unflagged run of round 5 (the scratch then held
    whatever an earlier test had left in the recycled device memory)."""
    rows = run_testhooks(EXHAUSTED)
    print(json.dumps(rows))
    assert len(rows) == 16
    for row in rows:
        if row["m"] < 0:  # raised before the first block (the Newton prologue's 2s steps broke down)
            assert row["status"] < 0, row
            continue
        assert row["m"] == row["s"] + 1, row
        assert row["finite"], row
        assert row["svratio"] <= 1e-8, row
        assert row["status"] < 0 or row["nrd"] >= 1 or row["brk"] == 1, row
    assert sum(r["m"] > 0 for r in rows) >= 8, rows
    ungated = run_testhooks(EXHAUSTED, CAL_TEST_NO_PASSB_GATE="1")
    print(json.dumps(ungated))
    bad = [r for r in ungated if not r.get("finite", True)]
    assert bad, ungated  # the mechanism: the ungated store reaches R
    print("ungated non-finite first-block R:", [(r["pre"], r["start"], r["s"], r["basis"]) for r in bad])


@pytest.mark.parametrize("N,s", [(40, 8), (23, 4), (70, 16)])
def test_newton_prologue_fused_bitexact(N, s):
    """The Newton prologue's recurrence (lanczos.m:103-110) with each update
    and the dot after it in one launch (k_axpy_dot: k_dot's grid and order,
    the partials summed by the last block in k_reduce's order) against the
    separate axpy / dot / reduce launches (CAL_TEST_PROLOGUE_SPLIT): the same
    bits in T, Q's Ritz residual norms and the orthogonality errors; rows not
    a multiple of the 256-thread blocks (23^3, 70^3 = 343000 > one grid
    stride of 1024 blocks)."""
    res = run_testhooks(r"""
A = cal.matrices.laplacian_3d(%d)
r = ref.matlab_rand(A.shape[0])
os.environ.pop("CAL_TEST_PROLOGUE_SPLIT", None)
a = cal.ca_lanczos_ex(A, r, %d, %d, "newton", "full")
os.environ["CAL_TEST_PROLOGUE_SPLIT"] = "1"
b = cal.ca_lanczos_ex(A, r, %d, %d, "newton", "full")
print(json.dumps(dict(T=bool(np.array_equal(a.T, b.T)), rn=bool(np.array_equal(a.ritz_rnorm, b.ritz_rnorm)),
                      oe=bool(np.array_equal(a.orth_err, b.orth_err)), t=int(a.info["t"]))))
""" % (N, s, 4 * s, s, 4 * s))
    assert res == dict(T=True, rn=True, oe=True, t=4), res


@pytest.mark.parametrize("fmt", ["auto", "csr"])
def test_normest_and_irl_fused_bitexact(fmt):
    """normest (MATLAB built-in, ca_lanczos.m:258) with both norms fused
    (k_norms2 + k_nrm_div; on CSR the rescale of x folded into the next
    SpMV's gathers, mode 3) against the separate dot / reduce / div launches
    (CAL_TEST_PROLOGUE_SPLIT): 'periodic' CA-Lanczos (which takes normest(A)
    for its omega recurrence) and a whole implicit-restart solve (normest,
    the Newton prologue, every restart) give the same bits, in the matrix's
    own SpMV format and forced to CSR."""
    res = run_testhooks(r"""
A = cal.matrices.circuit_like(60, seed=3)
r = ref.matlab_rand(A.shape[0])
fmt = %r
outs = []
for split in (False, True):
    if split:
        os.environ["CAL_TEST_PROLOGUE_SPLIT"] = "1"
    ctx = cal.Context(spmv_format=None if fmt == "auto" else fmt).set_matrix(A)
    assert fmt == "auto" or ctx.spmv_format()[0] == "csr"
    p = cal.ca_lanczos_ex(A, r, 4, 40, "newton", "periodic", ctx=ctx)
    irl = cal.impl_restarted_ca_lanczos(A, r, 40, 6, 4, "newton", "full", 1e-8, ctx=ctx)
    ctx.close()
    outs.append((p, irl))
(p0, i0), (p1, i1) = outs
print(json.dumps(dict(na=bool(p0.info["norm_A"] == p1.info["norm_A"] and p0.info["norm_A"] > 0),
                      ina=bool(i0["norm_A"] == i1["norm_A"]), T=bool(np.array_equal(p0.T, p1.T)),
                      nr=bool(i0["num_restarts"] == i1["num_restarts"]),
                      e=bool(np.array_equal(i0["conv_eigs"], i1["conv_eigs"])),
                      q=bool(np.array_equal(i0["Q_conv"], i1["Q_conv"])))))
""" % fmt)
    assert all(res.values()), res


def test_irl_restart_apply_in_place_bitexact():
    """The implicit restart's [V_k | r] = [V_m | v_{m+1}] M formed in place in
    Q's first k + 1 columns (one row-parallel apply: every row read whole
    before it is written) against the work panel and the copy back
    (CAL_TEST_RESTART_COPY): the same restart count, eigenvalues and Ritz
    vectors to the bit, on the circuit stand-in and on lap2d(40)."""
    res = run_testhooks(r"""
C = cal.matrices.circuit_like(60, seed=3)
D = cal.matrices.laplacian_2d(40)
outs = []
for copy in (False, True):
    if copy:
        os.environ["CAL_TEST_RESTART_COPY"] = "1"
    a = cal.impl_restarted_ca_lanczos(C, ref.matlab_rand(C.shape[0]), 40, 6, 4, "newton", "full", 1e-8)
    b = cal.impl_restarted_ca_lanczos(D, ref.matlab_rand(D.shape[0]), 48, 8, 8, "newton", "full", 1e-8)
    outs.append((a, b))
(a0, b0), (a1, b1) = outs
print(json.dumps(dict(nr=[int(a0["num_restarts"]), int(a1["num_restarts"]), int(b0["num_restarts"]), int(b1["num_restarts"])],
                      e=bool(np.array_equal(a0["conv_eigs"], a1["conv_eigs"]) and np.array_equal(b0["conv_eigs"], b1["conv_eigs"])),
                      q=bool(np.array_equal(a0["Q_conv"], a1["Q_conv"]) and np.array_equal(b0["Q_conv"], b1["Q_conv"])),
                      conv=bool(a0["converged"] and b0["converged"]))))
""")
    assert res["nr"][0] == res["nr"][1] and res["nr"][2] == res["nr"][3], res
    assert res["e"] and res["q"] and res["conv"], res


@pytest.mark.parametrize("fmt", ["auto", "csr"])
def test_normest_graph_vs_launches_bitexact(fmt):
    """The asynchronous normest's chunks replayed as captured HIP graphs
    (lanczos.cpp normest_chunk_graph) against the same launches issued one by
    one (CAL_TEST_NEST_DIRECT): the same norm_A, restart count and
    eigenvalues to the bit, over three solves on one context -- a matrix, a
    second one of another size and format, the first again -- so each graph
    is re-captured when the scratch or the matrix changes."""
    res = run_testhooks(r"""
mats = [cal.matrices.circuit_like(60, seed=3), cal.matrices.laplacian_3d(20)]
fmt = %r
outs = []
for direct in (False, True):
    if direct:
        os.environ["CAL_TEST_NEST_DIRECT"] = "1"
    ctx = cal.Context(spmv_format=None if fmt == "auto" else fmt)
    row = []
    for A in mats + mats[:1]:
        ctx.set_matrix(A)
        r = ref.matlab_rand(A.shape[0])
        irl = cal.impl_restarted_ca_lanczos(A, r, 40, 6, 4, "newton", "full", 1e-8, ctx=ctx)
        row.append([float(irl["norm_A"]), int(irl["num_restarts"]), [float(x) for x in irl["conv_eigs"]]])
    ctx.close()
    outs.append(row)
print(json.dumps(dict(same=outs[0] == outs[1], na=[x[0] for x in outs[0]], nr=[x[1] for x in outs[0]])))
""" % fmt)
    assert res["same"], res
    assert res["na"][0] == res["na"][2] and res["na"][0] != res["na"][1], res


@pytest.mark.parametrize("switch", ["CAL_TEST_APPLY_GRAM_OFF", "CAL_TEST_SELFGRAM_OFF"])
def test_project_blocks_fused_vs_unfused(switch):
    """project_blocks_async (blockorth.cpp): the update of block i fused with
    the Gram of block i + 1 (k_apply_gram) and the last update's X'X handed to
    the normalize (p1_blocks) against the separate launches.  The Grams are
    summed in another order, so the bar is the solvers' tolerance: the
    converged eigenvalues within 1e-10 ||A|| on the block-MGS users -- the
    implicit restart ('full', {Q_conv, Q} blocks; its restart count within 2)
    and the explicit restart ('local' against Q_conv).  The explicit
    restart's count is not compared: on lap2d's double eigenvalues it moves
    with the last bits of a Gram (14 / 20 measured, like the oracle's own
    spread under ulp-perturbed start vectors, test_gpu_parity.py)."""
    res = run_testhooks(r"""
A = cal.matrices.circuit_like(60, seed=3)
r = ref.matlab_rand(A.shape[0])
D = cal.matrices.laplacian_2d(30)
rd = ref.matlab_rand(D.shape[0], seed=7)
outs = []
for off in (False, True):
    if off:
        os.environ[%r] = "1"
    irl = cal.impl_restarted_ca_lanczos(A, r, 40, 6, 4, "newton", "full", 1e-8)
    rst = cal.restarted_ca_lanczos(D, rd, 40, 5, 4, "newton", "local", 1e-8)
    outs.append((irl, rst))
(i0, r0), (i1, r1) = outs
na = float(i0["norm_A"])
print(json.dumps(dict(inr=[int(i0["num_restarts"]), int(i1["num_restarts"])],
                      ie=float(np.max(np.abs(np.sort(i0["conv_eigs"]) - np.sort(i1["conv_eigs"])))) / na,
                      rnr=[int(r0["num_restarts"]), int(r1["num_restarts"])],
                      re=float(np.max(np.abs(np.sort(r0["conv_eigs"]) - np.sort(r1["conv_eigs"])))) / 8.0,
                      ien=[len(i0["conv_eigs"]), len(i1["conv_eigs"])],
                      ren=[len(r0["conv_eigs"]), len(r1["conv_eigs"])])))
""" % switch)
    assert abs(res["inr"][0] - res["inr"][1]) <= 2, res
    assert res["ie"] <= 1e-10 and res["re"] <= 1e-10, res
    assert res["ien"] == [6, 6] and res["ren"][0] == res["ren"][1] >= 1, res


@pytest.mark.parametrize("N,its", [(40, 120), (24, 64)])
def test_full_passb_wide_gram_vs_separate(N, its):
    """'full' orthogonalisation (ca_lanczos.m:197): the local block's pass B
    also forms the next projection's Gram [Qp | Q_new | Qold]' Q_new
    (k_passb_wide) instead of the separate wide Gram sweep
    (CAL_TEST_PASSB_WIDE_OFF).  The Gram is summed in another order, so the
    bar is the solver's: T within 1e-9 ||A||, the same reorth flags, and both
    runs orthonormal to 1e-12 (orth_err of every iteration)."""
    res = run_testhooks(r"""
A = cal.matrices.laplacian_3d(%d)
r = ref.matlab_rand(A.shape[0])
a = cal.ca_lanczos_ex(A, r, 8, %d, "newton", "full")
os.environ["CAL_TEST_PASSB_WIDE_OFF"] = "1"
b = cal.ca_lanczos_ex(A, r, 8, %d, "newton", "full")
print(json.dumps(dict(dT=float(np.max(np.abs(a.T - b.T))), fa=[int(f) for f in a.reorth], fb=[int(f) for f in b.reorth],
                      oa=float(np.max(a.orth_err)), ob=float(np.max(b.orth_err)), t=int(a.info["t"]))))
""" % (N, its, its))
    assert res["dT"] <= 1e-9 * 12.0, res
    assert res["fa"] == res["fb"], res
    assert res["oa"] < 1e-12 and res["ob"] < 1e-12, res
