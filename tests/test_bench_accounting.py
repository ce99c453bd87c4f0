"""CPU checks of bench.py's algorithmic-byte accounting: the
per-launch SpMV bytes the roofline line divides by the HIP-event time."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def test_spmv_bytes_one_launch_per_power():
    n, nnz, s = 1000, 7000, 8
    b_csr = 12 * nnz + 20 * n + 4
    # pair patterns / plane-march mask keys: 1 B key + 8 B x + 8 B y per row
    assert bench.spmv_launch_bytes("pattern", 5, n, s, s, b_csr) == 17 * n
    # row patterns without pairs: 2-B ids
    assert bench.spmv_launch_bytes("pattern", 0, n, s, s, b_csr) == 18 * n
    # CSR: SURVEY §8d's 12 nnz + 20 n + 4 whatever the launch count
    assert bench.spmv_launch_bytes("csr", 0, n, s, s, b_csr) == b_csr


def test_spmv_bytes_several_powers_per_launch():
    # a launch computing s / lpp powers reads x and the keys once
    n, s = 1000, 8
    assert bench.spmv_launch_bytes("pattern", 5, n, s, 2, 0) == (9 * 2 + 64) * n / 2
    assert bench.spmv_launch_bytes("pattern", 5, n, s, 1, 0) == (9 + 64) * n


def test_launch_boundaries_withholds_distorted_share():
    """Config 2's leg: when the HIP-event timers visibly
    inflate the small launches (the timed SpMV > 1.3x its back-to-back time)
    kernel_share is withheld and kept beside as kernel_share_timed; the
    rocprof busy share and the HIP-graph A/B come from the committed
    summary."""
    leg = {"kernel_share": 1.25, "kernel_avg_launch_us": {"spmv": 11.4},
           "spmv_kernel_back_to_back": {"avg_us": 7.1}}
    out = bench.launch_boundaries(leg)
    assert leg["kernel_share"] is None and out["kernel_share_timed"] == 1.25
    assert out["timer_distortion"]["spmv_back_to_back_us"] == 7.1
    assert len(out["rocprof_busy_share"]) == 2 and out["hip_graph_powers"]["kept"] is False
    leg2 = {"kernel_share": 0.97, "kernel_avg_launch_us": {"spmv": 36.0},
            "spmv_kernel_back_to_back": {"avg_us": 34.0}}
    out2 = bench.launch_boundaries(leg2)
    assert leg2["kernel_share"] == 0.97 and "timer_distortion" not in out2


def test_restart_spread_fixture():
    """tests/golden/restart_spread_diag5000.json (make_restart_spread.py): the
    oracle's restart counts over 98 perturbed start vectors, which the
    explicit-restart parity test holds the device's median against."""
    import json
    import numpy as np
    d = json.load(open(os.path.join(ROOT, "tests", "golden", "restart_spread_diag5000.json")))
    c = np.array(d["counts"])
    assert len(c) == 98 and c.min() >= 80 and c.max() <= 170
    lo, hi = np.percentile(c, [10, 90])
    assert 90 <= lo <= np.median(c) <= hi <= 125
