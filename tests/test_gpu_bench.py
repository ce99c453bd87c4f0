"""bench.py's output contract, on a small workload: one JSON line on stdout
with the fields the driver reads, the roofline and CPU-baseline objects, and
the epoch path that keeps long runs inside the basis budget."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(*args, timeout=240):
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], cwd=ROOT, capture_output=True,
                       text=True, timeout=timeout)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, p.stdout[-2000:]  # exactly one line on stdout
    return json.loads(lines[0])


def test_bench_contract_fields():
    d = _bench("--workload", "lap3d_40", "--steps", "3", "--warmup", "1", "--cpu-iters", "2")
    assert d["metric"].startswith("CA-Lanczos outer-iters/sec") and d["unit"] == "outer-iters/s"
    assert d["value"] > 0 and d["ms_per_step"] > 0
    assert abs(d["value"] - 1e3 / d["ms_per_step"]) <= 1e-6 * d["value"]
    assert (d["n_gpus"], d["steps"], d["warmup"]) == (1, 3, 1)
    assert d["higher_is_better"] is True and d["scaling"] == "strong" and d["vs_baseline"] is None
    assert d["dtype"] == "f64" and d["data"].startswith("synthetic")
    assert d["config"]["workload"].startswith("lap3d_40") and d["config"]["s"] == 8
    rf = d["roofline"]
    assert {"bound", "achieved", "peak", "unit", "frac", "traffic"} <= set(rf)
    assert rf["bound"] == "hbm" and rf["unit"] == "GB/s" and rf["peak"] == 8000.0
    assert rf["achieved"] > 0 and abs(rf["frac"] - rf["achieved"] / rf["peak"]) < 1e-9
    cb = d["cpu_baseline"]
    assert {"value", "unit", "cores", "kind", "sample"} <= set(cb)
    assert cb["value"] > 0 and cb["unit"] == "outer-iters/s" and cb["kind"] in ("port", "reference")
    assert d["reorth_passes"].endswith("/3")
    # the legs of the default line: north_star's 5-pt 10M workload and config 5's driver
    l2 = d["lap2d_3162_step"]
    assert l2["outer_iters_per_s"] > 0 and l2["workload"].startswith("lap2d_3162")
    assert 0 < l2["spmv_frac"] < 1.5 and 0 < l2["roofline"]["frac"] < 1.5
    irl = d["irl"]
    assert irl["converged"] and irl["solves_per_s"] > 0 and irl["spmv_format"] == "csr"
    assert 0 < irl["roofline"]["frac"] < 1.5


def test_bench_epochs_keep_the_line_valid():
    """A basis budget of 20 MB holds only a few outer iterations of lap3d_40:
    the run continues in restarted epochs and still prints one valid line."""
    d = _bench("--workload", "lap3d_40", "--steps", "12", "--warmup", "2", "--no-cpu-baseline",
               "--basis-gb", "0.02")
    assert d["value"] > 0 and d["steps"] == 12
    assert d["reorth_passes"].endswith("/12")


def test_bench_two_ranks_one_line():
    """The driver's N > 1 launch (torch.distributed.run, one rank per GPU),
    rehearsed with 2 ranks on one GPU over the host-staged communicator:
    rank 0 prints the only line, the whole-job rate, no CPU baseline."""
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    p = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "bench.py"),
                        "--gpus", "2", "--steps", "3", "--warmup", "1", "--workload", "lap3d_40", "--comm", "host"],
                       cwd=ROOT, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, p.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["value"] > 0 and d["config"]["parallelism"] == "row-slab x2"
    assert d["config"]["comm"] == "host" and "cpu_baseline" not in d


def test_bench_gpus_flag_launches_ranks():
    """`bench.py --gpus 2` with no launcher (the driver's BENCH command shape)
    starts the two ranks itself -- it must not silently measure one GPU.
    Host-staged communicator: both ranks share the test box's GPU.  The TSQR
    leg runs on both ranks (its tree's root all-gathered)."""
    d = _bench("--gpus", "2", "--steps", "3", "--warmup", "1", "--workload", "lap3d_40", "--comm", "host",
               timeout=300)
    assert d["n_gpus"] == 2 and d["value"] > 0 and d["config"]["parallelism"] == "row-slab x2"
    assert d["config"]["comm"] == "host" and "cpu_baseline" not in d
    assert "tsqr_step" in d and d["tsqr_step"]["outer_iters_per_s"] > 0
    assert d["tsqr_step"]["reorth_passes"] == d["reorth_passes"].replace("/3", "/3")


def test_bench_gpus_flag_rccl_line():
    """The driver's SCALE command (`bench.py --gpus N`, RCCL) rehearsed on the
    one-GPU box: CAL_RCCL_HOSTID_PER_RANK=1 gives each rank its own RCCL host
    id (RCCL refuses two ranks on one device of one host), so the ranks talk
    over RCCL's socket transport.  One line, the RCCL communicator counted on
    every rank, all-reduces and the one deep halo exchange per step."""
    env = dict(os.environ, CAL_RCCL_HOSTID_PER_RANK="1")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "3", "--warmup",
                        "1", "--workload", "lap3d_40"], cwd=ROOT, env=env, capture_output=True, text=True,
                       timeout=300)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, p.stdout[-2000:]
    d = json.loads(lines[0])
    print(json.dumps({k: d.get(k) for k in ("value", "ms_per_step", "comm", "config")}))
    assert d["n_gpus"] == 2 and d["value"] > 0 and d["config"]["comm"] == "rccl"
    c = d["comm"]
    assert c["comm_kind"] == "rccl" and c["rccl_comm_count"] == 2
    assert c["allreduces_per_step"] >= 2 and abs(c["halo_exchanges_per_step"] - 1.0) < 1e-9
    assert c["mpk_redundant_rows_per_step"] > 0
    assert "overlapped" in d["config"]["halo"]
    # BASELINE config 5 on the ranks' slabs of the G3_circuit stand-in
    # (skipped only when this box's socket all-reduces exceed IRL_MAX_ALLREDUCE_US; ~0.1 ms measured)
    irl = d["irl"]
    assert "error" not in irl, irl
    if "skipped" not in irl:
        assert irl["n_ranks"] == 2 and irl["converged"] and irl["solves_per_s"] > 0
    else:
        assert c["allreduce_us_per_step"] / c["allreduces_per_step"] > 1000.0, irl


def test_bench_rejects_mismatched_world():
    """--gpus N under a launcher with another WORLD_SIZE exits non-zero."""
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=120)
    assert p.returncode != 0 and p.stdout.strip() == ""


def test_bench_watchdog_hung_rank_exits_with_stage():
    """a rank whose halo exchange never returns (host-staged
    communicator, CAL_BENCH_TEST_HANG_RANK=1) ends the 2-rank run non-zero
    within the stage limit (CAL_BENCH_STAGE_LIMIT=20 s), with the rank and
    stage on stderr and, when rank 0's watchdog fires before the launcher
    tears the job down, an "error" line naming the stage."""
    import time
    env = dict(os.environ, CAL_BENCH_TEST_HANG_RANK="1", CAL_BENCH_STAGE_LIMIT="20")
    t0 = time.monotonic()
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "3", "--warmup",
                        "1", "--workload", "lap3d_40", "--comm", "host", "--no-legs"], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=240)
    el = time.monotonic() - t0
    assert p.returncode != 0
    assert el < 200
    assert "stage '" in p.stderr and "exceeded 20 s" in p.stderr, p.stderr[-2000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.strip()]
    assert len(lines) <= 1
    if lines:
        d = json.loads(lines[0])
        assert d["value"] is None and d["stage"] in p.stderr and "error" in d
