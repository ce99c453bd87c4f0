"""Exact-breakdown behaviour of the HIP path (Krylov space exhausted in block 1)."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import ca_lanczos_amd as cal
A = cal.matrices.diagonal(np.arange(1.0, 101.0))
for name, r in [("e1", np.eye(100)[0]), ("two", np.eye(100)[0] + np.eye(100)[5])]:
    for s, basis in [(2, "monomial"), (4, "monomial"), (4, "newton")]:
        try:
            out = cal.ca_lanczos_ex(A, r, s, 3 * s, basis, "local", diagnostics=False)
            print(name, s, basis, "ok", out.info, "finite=", np.all(np.isfinite(out.T)), out.T.shape, np.sort(np.linalg.eigvals(out.T).real) if out.T.size else None)
        except Exception as e:
            print(name, s, basis, "raised", type(e).__name__, str(e)[:120])
