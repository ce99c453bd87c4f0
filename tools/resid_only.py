"""The batched Ritz-residual kernel alone (cal_compute_ritz_rnorm on
lap3d_215, k random vectors): X = Q Vp then the plane-march residuals; the
target of a kernel profile of k_resid_planes.  Not part of the library."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import ca_lanczos_amd as cal  # noqa: E402


def main():
    N = int(os.environ.get("RESID_N", "215"))
    k = int(os.environ.get("RESID_K", "16"))
    reps = int(os.environ.get("RESID_REPS", "3"))
    A = cal.matrices.laplacian_3d(N)
    n = A.shape[0]
    ctx = cal.Context(spmv_format="pattern").set_matrix(A)
    rng = np.random.RandomState(0)
    Q = np.asfortranarray(rng.standard_normal((n, k)))
    d, Vp = np.linalg.eigh(np.diag(np.arange(1.0, k + 1)))
    out = []
    for _ in range(reps):
        t0 = time.perf_counter()
        rn = cal.compute_ritz_rnorm(A, Q, Vp, d, ctx=ctx)
        out.append(time.perf_counter() - t0)
    print("plane_info", ctx.spmv_plane_info(), "rn[0]", rn[0], "call s", [round(x, 3) for x in out])


if __name__ == "__main__":
    main()
