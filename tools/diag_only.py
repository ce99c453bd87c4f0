"""Diagnostics-on run only (bench.py's diagnostics_run, lap3d_215, t = 15),
once as warmup and `--reps` times timed: the target of a kernel profile of
the Ritz-residual / orthogonality-error work.  Not part of the library."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    reps = int(os.environ.get("DIAG_REPS", "2"))
    sys.argv = [sys.argv[0], "--no-cpu-baseline", "--no-legs"] + sys.argv[1:]
    args = bench.parse()
    E = bench.setup(args)
    ctx, r0, r1 = E["ctx"], E["r0"], E["r1"]
    import numpy as np
    r = np.random.RandomState(5489).random_sample(E["wl"].n)[r0:r1]  # as bench.py
    out = [bench.diagnostics_run(ctx, r, args.s, args) for _ in range(reps + 1)]
    print(json.dumps({"outer_iters_per_s": [round(o["outer_iters_per_s"], 1) for o in out],
                      "diag_ms": [o["diag_ms"] for o in out]}))


if __name__ == "__main__":
    main()
