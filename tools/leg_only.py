"""One secondary leg of bench.py alone (a profiling target): LEG_WORKLOAD
(lap3d_215), LEG_FORMAT (auto|csr|pattern), LEG_ORTH (local), LEG_NORMALIZE
(auto|tsqr|cholqr2), LEG_STEPS (10), printed as JSON.  Not part of the library."""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import ca_lanczos_amd as cal  # noqa: E402


def main():
    wl = bench.Workload(os.environ.get("LEG_WORKLOAD", "lap3d_215"))
    fmt = os.environ.get("LEG_FORMAT", "auto")
    ctx = cal.Context(spmv_format=None if fmt == "auto" else fmt,
                      normalize=os.environ.get("LEG_NORMALIZE", "auto"))
    ctx.set_matrix(wl.full())
    r = np.random.RandomState(5489).random_sample(wl.n)
    K = int(os.environ.get("LEG_STEPS", "10"))
    out = []
    for _ in range(int(os.environ.get("LEG_REPS", "2"))):
        leg = bench.timed_leg(ctx, r, 8, K, int(os.environ.get("LEG_WARMUP", "2")), "newton", os.environ.get("LEG_ORTH", "local"), None)
        out.append({k: leg[k] for k in ("outer_iters_per_s", "ms_per_step", "kernel_ms_per_step", "kernel_share")})
    print(json.dumps(out))


if __name__ == "__main__":
    main()
