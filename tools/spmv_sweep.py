"""SpMV kernel timing on one workload (HBM-resident vectors), one line per run.

  python tools/spmv_sweep.py [--workload lap3d_215|circuit_1259] [--format pattern|csr] [--reps 50]

Environment knobs read by the library (e.g. CAL_PAT_ROWS) apply per process.
"""
import argparse
import json
import os
import sys

import numpy as np
import scipy.sparse as sp

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--workload", default="lap3d_215")
    p.add_argument("--format", default="pattern")
    p.add_argument("--reps", type=int, default=50)
    p.add_argument("--shift", type=float, default=1.0)
    a = p.parse_args()
    import ca_lanczos_amd as cal
    from ca_lanczos_amd.matrices import laplacian_rows
    kind, N = a.workload.split("_")
    N = int(N)
    ctx = cal.Context(device=0, spmv_format=a.format)
    if kind == "circuit":
        A = cal.matrices.circuit_like(N)
        n, nnz = A.shape[0], A.nnz
        ctx.set_matrix(A)
        del A
    else:
        dim = {"lap2d": 2, "lap3d": 3}[kind]
        n = N ** dim
        rp, col, val = laplacian_rows(dim, N, 0, n)
        nnz = int(rp[-1])
        ctx.set_matrix(sp.csr_matrix((val, col.astype(np.int32), rp), shape=(n, n)))
        del rp, col, val
    ctx.bench_spmv(a.reps, a.shift)  # warm (clocks, caches)
    mean, mn = ctx.bench_spmv(a.reps, a.shift)
    fmt = ctx.spmv_format()[0]
    pairs = ctx.spmv_pair_info()
    b = 18 * n if fmt == "pattern" else 12 * nnz + 20 * n + 4
    print(json.dumps({"workload": a.workload, "format": fmt, "env": {k: v for k, v in os.environ.items() if k.startswith("CAL_")}, "pairs": pairs,
                      "mean_us": mean * 1e3, "min_us": mn * 1e3, "gbps_mean": b / (mean * 1e-3) / 1e9,
                      "csr_equiv_gbps": (12 * nnz + 20 * n + 4) / (mean * 1e-3) / 1e9}), flush=True)


if __name__ == "__main__":
    main()
