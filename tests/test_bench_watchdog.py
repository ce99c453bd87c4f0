"""bench.py's per-rank stage watchdog (the first 8-GPU SCALE
run is the first RCCL run with more than one rank, so a hang must end with
the rank and stage named, not at the driver's 600-s limit).  CPU only: two
gloo ranks; rank 1 never joins a collective, rank 0 blocks in it, and each
rank's watchdog ends its process with exit code 3 within the stage limit;
rank 0's stdout carries one JSON line with "error" and "stage"."""
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

_CHILD = r"""
import os, sys, time, json
sys.path.insert(0, %(root)r)
import bench
import torch, torch.distributed as dist
rank, world = int(sys.argv[1]), 2
os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=sys.argv[2])
bench._quiet_stdout()
wd = bench.Watchdog(rank, world, poll=0.1)
wd.enter("init_process_group", 60)
dist.init_process_group("gloo", rank=rank, world_size=world)
wd.enter("first_allreduce", 2.0)
if rank == 1:
    time.sleep(3600)          # never reaches the collective
t = torch.zeros(1)
dist.all_reduce(t)            # rank 0 blocks here
print("unreachable")
"""


def test_watchdog_names_the_hung_stage(tmp_path):
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = str(s.getsockname()[1])
    s.close()
    src = tmp_path / "child.py"
    src.write_text(_CHILD % {"root": ROOT})
    t0 = time.monotonic()
    procs = [subprocess.Popen([sys.executable, str(src), str(r), port], stdout=subprocess.PIPE,
                              stderr=subprocess.PIPE, text=True) for r in range(2)]
    outs = [p.communicate(timeout=120) for p in procs]
    el = time.monotonic() - t0
    assert [p.returncode for p in procs] == [3, 3], [o[1][-800:] for o in outs]
    assert el < 60
    for r, (out, err) in enumerate(outs):
        assert "rank %d/2: stage 'first_allreduce' exceeded" % r in err
    lines = [ln for ln in outs[0][0].splitlines() if ln.strip()]
    assert len(lines) == 1 and outs[1][0].strip() == ""
    d = json.loads(lines[0])
    assert d["stage"] == "first_allreduce" and d["rank"] == 0 and d["value"] is None and "error" in d
    assert d["stages_done_s"][0][0] == "init_process_group"


def test_watchdog_stage_limits_cover_every_stage():
    sys.path.insert(0, ROOT)
    import bench
    for st in ("init_process_group", "comm_init", "matrix_setup", "lanczos_begin", "first_outer_step", "warmup",
               "timed", "legs", "finalize"):
        assert 0 < bench.stage_limit(st) < 600


_CHILD_LEGS = r"""
import os, sys, time, json
sys.path.insert(0, %(root)r)
import bench
import torch, torch.distributed as dist
rank, world = int(sys.argv[1]), 2
os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=sys.argv[2])
bench._quiet_stdout()
wd = bench.Watchdog(rank, world, poll=0.1)
wd.enter("init_process_group", 60)
dist.init_process_group("gloo", rank=rank, world_size=world)
wd.enter("timed", 60)
t = torch.ones(1)
dist.all_reduce(t)            # the headline's max over ranks
wd.fallback = {"metric": "m", "value": 123.0, "n_gpus": world}
wd.enter("legs", 2.0)
if rank == 1:
    time.sleep(3600)          # a secondary leg that never returns
dist.all_reduce(t)            # rank 0 blocks in the leg's collective
print("unreachable")
"""


def test_watchdog_keeps_the_headline_when_a_leg_hangs(tmp_path):
    """A secondary leg that hangs after the headline was measured (e.g. a
    multi-rank leg over a slow transport) ends the ranks with exit code 0 and
    rank 0's one line carries the measured value plus "legs_error"."""
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = str(s.getsockname()[1])
    s.close()
    src = tmp_path / "child_legs.py"
    src.write_text(_CHILD_LEGS % {"root": ROOT})
    procs = [subprocess.Popen([sys.executable, str(src), str(r), port], stdout=subprocess.PIPE,
                              stderr=subprocess.PIPE, text=True) for r in range(2)]
    outs = [p.communicate(timeout=120) for p in procs]
    assert [p.returncode for p in procs] == [0, 0], [o[1][-800:] for o in outs]
    lines = [ln for ln in outs[0][0].splitlines() if ln.strip()]
    assert len(lines) == 1 and outs[1][0].strip() == ""
    d = json.loads(lines[0])
    assert d["value"] == 123.0 and "stage 'legs' exceeded" in d["legs_error"]
