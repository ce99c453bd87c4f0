"""Direct check of the wide Gram (k_gram_ab via cal_project's R = Q'X) against
numpy, single- and two-block Q, row counts off the 64-row step.  Not part of
the library."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import ca_lanczos_amd as cal  # noqa: E402

rng = np.random.RandomState(0)
worst = 0.0
for n in (64, 100, 5000, 5003, 100001):
    for wa in (33, 48, 57, 100, 128):
        Q = rng.randn(n, wa)
        X = rng.randn(n, 4)
        G = Q.T @ X
        _, R = cal.project([Q], X)
        e1 = np.max(np.abs(R[0] - G)) / np.max(np.abs(G))
        _, R2 = cal.project([Q[:, :20], Q[:, 20:]], X)
        e2 = max(np.max(np.abs(R2[0] - G[:20])), np.max(np.abs(R2[1] - G[20:]))) / np.max(np.abs(G))
        worst = max(worst, e1, e2)
        print(n, wa, "%.2e %.2e" % (e1, e2))
print("worst", worst)
