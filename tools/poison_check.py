"""Uninitialised-device-memory probe: fill and free a large device allocation
with a pattern (torch, then empty_cache so hipMalloc can hand the pages back),
then run the exhausted-Krylov inputs of test_ca_lanczos_exhausted_krylov_space
on fresh contexts and print their flags.  A result that changes with the
pattern reads memory it never wrote.  Not part of the library."""
import hashlib
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import ca_lanczos_amd as cal  # noqa: E402

n = 100
for pat in (float("nan"), 1.0e300, 0.5, -3.0):
    x = torch.full((1 << 29,), pat, dtype=torch.float64, device="cuda")  # 4 GB
    torch.cuda.synchronize()
    del x
    torch.cuda.empty_cache()
    for start in ("e1", "two"):
        for s, basis in [(2, "monomial"), (4, "monomial"), (4, "newton")]:
            A = cal.matrices.diagonal(np.arange(1.0, n + 1.0))
            r = np.eye(n)[0] + (np.eye(n)[5] if start == "two" else 0.0)
            try:
                out = cal.ca_lanczos_ex(A, r, s, 3 * s, basis, "local", diagnostics=False)
                print(pat, start, s, basis, "rankdef", out.info["n_rank_deficient"], "breakdown",
                      out.info["breakdown"], hashlib.md5(out.T.tobytes()).hexdigest()[:8], flush=True)
            except cal.CalError as e:
                print(pat, start, s, basis, "err", e.status, flush=True)
