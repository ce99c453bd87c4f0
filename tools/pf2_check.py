"""T of a short ca_lanczos run (lap2d_1000, 12 outer iterations, diagnostics
off) as a SHA-256, for A/B builds or switches that must keep the bits
(CAL_ROWGRAM_PF2_MB).  Not part of the library."""
import hashlib
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import ca_lanczos_amd as cal  # noqa: E402

wl = bench.Workload(os.environ.get("LEG_WORKLOAD", "lap2d_1000"))
ctx = cal.Context()
ctx.set_matrix(wl.full())
r = np.random.RandomState(5489).random_sample(wl.n)
out = cal.ca_lanczos_ex(None, r, 8, 12, "newton", "local", diagnostics=False, return_Q=False, ctx=ctx)
print(hashlib.sha256(np.ascontiguousarray(out.T).tobytes()).hexdigest(), list(out.reorth)[:3])
