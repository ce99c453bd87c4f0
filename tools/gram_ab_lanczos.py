"""'full' CA-Lanczos on the restart test's matrix (diag(linspace(1,1e4,5000)),
s = 4, 60 steps) and the restart driver: T, orth error and restart count,
saved per process so that CAL_GRAM_AB=0/1 runs can be compared.  Not part of
the library."""
import os
import sys

import numpy as np
import scipy.sparse as sp

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import ca_lanczos_amd as cal  # noqa: E402

a = np.linspace(1.0, 1.0e4, 5000)
A = sp.csr_matrix(sp.diags(a))
r = np.ones(5000)
out = cal.ca_lanczos_ex(A, r, 4, 60, "newton", "full")
res = cal.restarted_ca_lanczos(A, r, 60, 10, 4, "newton", "full", 1.0e-8)
tag = sys.argv[1]
np.savez(f"gpurun_out/gram_ab_{tag}.npz", T=out.T, oe=out.orth_err, rn=out.ritz_rnorm,
         nres=res["num_restarts"], eigs=res["conv_eigs"])
print(tag, "restarts", res["num_restarts"], "max oe", np.max(out.orth_err))
