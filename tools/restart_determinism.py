"""The explicit-restart driver on the restart test's input, repeated in one
process with other runs in between: the restart count and eigenvalues must
not change (determinism check).  Not part of the library."""
import os
import sys

import numpy as np
import scipy.sparse as sp

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import ca_lanczos_amd as cal  # noqa: E402

a = np.linspace(1.0, 1.0e4, 5000)
A = sp.csr_matrix(sp.diags(a))
r = np.ones(5000)
base = None
for rep in range(4):
    res = cal.restarted_ca_lanczos(A, r, 60, 10, 4, "newton", "full", 1.0e-8)
    e = np.array(res["conv_eigs"])
    print("rep", rep, "restarts", res["num_restarts"], "eig[0]", repr(e[0]) if len(e) else None)
    if base is None:
        base = e
    # other work between the repetitions
    if rep == 1:
        cal.ca_lanczos_ex(cal.matrices.laplacian_3d(24), np.ones(24 ** 3), 8, 120, "newton", "local")
    if rep == 2:
        cal.ca_lanczos_ex(A, r, 4, 60, "newton", "full")
