import sys, hashlib, numpy as np
sys.path.insert(0, '.')
import ca_lanczos_amd as cal
n = 100
A = cal.matrices.diagonal(np.arange(1.0, n + 1.0))
for start in ("e1", "two"):
    for s, basis in [(2, "monomial"), (4, "monomial"), (4, "newton")]:
        r = np.eye(n)[0] + (np.eye(n)[5] if start == "two" else 0.0)
        for rep in range(3):
            try:
                out = cal.ca_lanczos_ex(A, r, s, 3 * s, basis, "local", diagnostics=False)
                print(start, s, basis, rep, out.info["n_rank_deficient"], out.info["breakdown"], hashlib.md5(out.T.tobytes()).hexdigest()[:8], flush=True)
            except cal.CalError as e:
                print(start, s, basis, rep, "err", e.status, flush=True)
