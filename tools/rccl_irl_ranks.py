"""One implicit-restart solve of config 5 (circuit_1259) on W ranks over RCCL,
all ranks on the one GPU of the box (NCCL_HOSTID per rank): per-rank setup and
solve times, to tell a slow shared-GPU rehearsal from a hang.
usage: python tools/rccl_irl_ranks.py W [N]"""
import os
import sys
import time

import numpy as np
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def worker(rank, world, port, N, q):
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), NCCL_HOSTID="cal-rank-%d" % rank,
                      NCCL_SOCKET_IFNAME="lo", NCCL_IB_DISABLE="1")
    import faulthandler
    faulthandler.dump_traceback_later(230, exit=True)
    import ctypes
    import torch
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import ca_lanczos_amd as cal
    from ca_lanczos_amd._lib import check, lib
    t0 = time.time()
    uid = bytearray(128)
    if rank == 0:
        buf = ctypes.create_string_buffer(128)
        check(None, lib.cal_comm_unique_id(buf))
        uid = bytearray(buf.raw)
    t = torch.tensor(list(uid), dtype=torch.uint8)
    dist.broadcast(t, 0)
    A = cal.matrices.circuit_like(N)
    n = A.shape[0]
    b = cal.matrices.slab_bounds(n, world, 1)
    r0, r1 = b[rank], b[rank + 1]
    ctx = cal.Context(0)
    ctx.comm_init_rccl(world, rank, bytes(t.tolist()))
    t1 = time.time()
    ctx.set_matrix_slab(n, r0, A[r0:r1])
    t2 = time.time()
    r = np.random.RandomState(5489).random_sample(n)[r0:r1]
    ctx.comm_stats(reset=True)
    out = cal.impl_restarted_ca_lanczos(None, r, 64, 8, 8, "newton", "full", 1.0e-8, ctx=ctx)
    t3 = time.time()
    st = ctx.comm_stats()
    out2 = cal.impl_restarted_ca_lanczos(None, r, 64, 8, 8, "newton", "full", 1.0e-8, ctx=ctx)
    t4 = time.time()
    q.put((rank, dict(setup_s=t1 - t0, matrix_s=t2 - t1, solve1_s=t3 - t2, solve2_s=t4 - t3,
                      restarts=out["num_restarts"], conv=bool(out["converged"]), nghost=ctx.matrix_info()["nghost"],
                      stats=st, same=bool(np.array_equal(out["conv_eigs"], out2["conv_eigs"])))))
    ctx.close()
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    import socket
    W = int(sys.argv[1])
    N = int(sys.argv[2]) if len(sys.argv) > 2 else 1259
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    mpc = mp.get_context("spawn")
    q = mpc.Queue()
    ps = [mpc.Process(target=worker, args=(k, W, port, N, q)) for k in range(W)]
    for p in ps:
        p.start()
    res = sorted([q.get(timeout=240) for _ in range(W)])
    for k, d in res:
        print(k, d, flush=True)
    for p in ps:
        p.join(timeout=60)
