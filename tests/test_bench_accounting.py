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
