"""Device restart counts of the explicit restart driver on the perturbed start
vectors of tests/golden/make_restart_spread.py (seeds first..last), beside the
oracle's committed counts.  Run on the GPU box: python tools/restart_spread_dev.py 0 32"""
import json
import os
import sys
import time

import numpy as np
import scipy.sparse as sp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import ca_lanczos_amd as cal  # noqa: E402

first, last = int(sys.argv[1]), int(sys.argv[2])
spread = json.load(open(os.path.join(ROOT, "tests/golden/restart_spread_diag5000.json")))["counts"]
a = 1.0 + (np.arange(5000, dtype=np.float64) * (1.0e4 - 1.0)) / 4999  # MATLAB linspace (oracle.matlab_linspace)
a[-1] = 1.0e4
A = sp.csr_matrix(sp.diags(a))
dev = []
for seed in range(first, last):
    rng = np.random.RandomState(seed)
    r = np.ones(5000) * (1 + 1e-15 * rng.randn(5000))
    t = time.time()
    out = cal.restarted_ca_lanczos(A, r, 60, 10, 4, "newton", "full", 1.0e-8)
    dev.append(int(out["num_restarts"]))
    print(seed, dev[-1], spread[seed] if seed < len(spread) else None, round(time.time() - t, 2), flush=True)
d = np.array(dev)
o = np.array(spread[first:last])
print(json.dumps({"dev_median": float(np.median(d)), "dev_min": int(d.min()), "dev_max": int(d.max()),
                  "oracle_median": float(np.median(o)), "oracle_min": int(o.min()), "oracle_max": int(o.max())}))
