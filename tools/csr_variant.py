"""CSR SpMV variant A/B (CAL_SPMV_CSR in the environment): back-to-back
kernel time of k_spmv on lap3d_215 and circuit_1259 in CSR, and a bit-exact
check against SciPy's sequential CSR SpMV.  Not part of the library."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import ca_lanczos_amd as cal  # noqa: E402
from oracle import ca_lanczos_ref as ref  # noqa: E402

out = {"variant": os.environ.get("CAL_SPMV_CSR", "0")}
for name, A in (("circuit_1259", cal.matrices.circuit_like(1259)), ("lap3d_215", cal.matrices.laplacian_3d(215))):
    ctx = cal.Context(spmv_format="csr").set_matrix(A)
    v = ref.matlab_rand(A.shape[0], seed=3)
    exact = bool(np.array_equal(ctx.spmv(v), ref.SpMV(A, v)))
    avg, mn = ctx.bench_spmv(30, 1.0)
    n, nnz = A.shape[0], A.nnz
    b = 12 * nnz + 20 * n + 4
    out[name] = {"avg_us": avg * 1e3, "min_us": mn * 1e3, "gbps": b / (avg * 1e-3) / 1e9, "bitexact": exact}
    ctx.close()
print(json.dumps(out))
