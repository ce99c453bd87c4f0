"""BASELINE config 4 on its own workload: lap3d_215 (n = 9,938,375) in two
z-slabs of 107 / 108 planes, one rank each, sharing the test box's GPU over
the host-staged communicator (the driver's multi-GPU runs replace exactly
its allreduce / exchange / allgather callbacks with RCCL).

Checked per rank against the single-GPU run of the whole matrix:
  * the deep-halo CA matrix powers (one 8-band exchange for s = 8 powers):
    bit-identical to the oracle's SciPy powers on the rank's rows (compared
    through SHA-256 digests of the column-major blocks);
  * t = 4 outer iterations of ca_lanczos 'local' with diagnostics: T within
    1e-9 ||A||, identical reorth flags, Ritz residual norms above 1e-10
    within 1e-8 relative (the slab of 107 planes has an odd row count: the
    pair-pattern residual kernel must not count the first ghost row);
  * the same with the Householder TSQR normalize, whose tree's root is
    all-gathered across the ranks (SURVEY §8e "RCCL TSQR tree").
"""
import hashlib
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
N, S, IT = 215, 8, 32
LAM = np.array([7.5, 0.5, 3.0, 11.0, 1.5, 5.0, 9.0, 2.5])


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _digest(V):
    return hashlib.sha256(np.asfortranarray(V).tobytes()).hexdigest()


def _worker(rank, world, port, out_q):
    import sys
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import scipy.sparse as sp
    import torch
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import ca_lanczos_amd as cal
    from oracle import ca_lanczos_ref as ref

    def allreduce(a):
        t = torch.from_numpy(a)
        dist.all_reduce(t)

    def exchange(peer, send, recv):
        reqs = []
        if send.size:
            reqs.append(dist.isend(torch.from_numpy(np.ascontiguousarray(send)), peer))
        rt = torch.zeros(recv.size, dtype=torch.float64)
        if recv.size:
            reqs.append(dist.irecv(rt, peer))
        for r in reqs:
            r.wait()
        if recv.size:
            recv[:] = rt.numpy()

    n = N ** 3
    b = cal.matrices.slab_bounds(n, world, N * N)
    r0, r1 = b[rank], b[rank + 1]
    rowptr, col, val = cal.matrices.laplacian_rows(3, N, r0, r1)
    Aloc = sp.csr_matrix((val, col, rowptr), shape=(r1 - r0, n))
    ctx = cal.Context(0, mpk_depth=8)
    ctx.comm_init_host(world, rank, allreduce, exchange)
    ctx.set_matrix_slab(n, r0, Aloc)
    del Aloc, rowptr, col, val
    res = {"mpk": ctx.mpk_info(), "rows": (r0, r1)}
    v = ref.matlab_rand(n, seed=7)[r0:r1]
    Vn = cal.matrix_powers_newton(None, v, S, LAM, 1, ctx=ctx)
    res["sched"] = ctx.mpk_schedule()
    res["powers"] = _digest(Vn)
    del Vn
    r = ref.matlab_rand(n)[r0:r1]
    out = cal.ca_lanczos_ex(None, r, S, IT, "newton", "local", diagnostics=True, return_Q=False, ctx=ctx)
    res["local"] = (out.T, out.ritz_rnorm, list(out.reorth))
    ctx.set_normalize("tsqr")
    out = cal.ca_lanczos_ex(None, r, S, IT, "newton", "local", diagnostics=False, return_Q=False, ctx=ctx)
    res["tsqr"] = (out.T, list(out.reorth))
    ctx.close()
    out_q.put((rank, res))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(900)
def test_config4_lap3d_215_two_slabs(cal, ref):
    world = 2
    A = cal.matrices.laplacian_3d(N)
    n = A.shape[0]
    v = ref.matlab_rand(n, seed=7)
    Vref = ref.matrix_powers_newton(A, v, S, LAM, 1)
    b = cal.matrices.slab_bounds(n, world, N * N)
    dig = [_digest(Vref[b[k]:b[k + 1]]) for k in range(world)]
    del Vref
    r = ref.matlab_rand(n)
    c1 = cal.Context(0).set_matrix(A)
    single = cal.ca_lanczos_ex(A, r, S, IT, "newton", "local", diagnostics=True, return_Q=False, ctx=c1)
    c1.close()
    c2 = cal.Context(0, normalize="tsqr").set_matrix(A)
    single_t = cal.ca_lanczos_ex(A, r, S, IT, "newton", "local", diagnostics=False, return_Q=False, ctx=c2)
    c2.close()
    del A
    mpc = mp.get_context("spawn")
    q = mpc.Queue()
    port = _free_port()
    procs = [mpc.Process(target=_worker, args=(k, world, port, q)) for k in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=800) for _ in range(world)], key=lambda t: t[0])
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    nA = 12.0
    for rank, rr in res:
        r0, r1 = rr["rows"]
        assert (r1 - r0) % 2 == (1 if rank == 0 else 0)   # 107 planes: odd slab
        assert rr["mpk"]["depth"] == 8 and rr["mpk"]["band_l"] == N * N
        assert rr["sched"] == 1                            # one deep exchange (host comm: unsplit)
        assert rr["powers"] == dig[rank], rank             # bit-identical powers
        T, rn, flags = rr["local"]
        assert flags == list(single.reorth)
        assert np.max(np.abs(T - single.T)) <= 1e-9 * nA
        big = single.ritz_rnorm > 1e-10
        assert np.all(np.abs(rn[big] / single.ritz_rnorm[big] - 1.0) <= 1e-8)
        Tt, flags_t = rr["tsqr"]
        assert flags_t == list(single_t.reorth)
        assert np.max(np.abs(Tt - single_t.T)) <= 1e-9 * nA
    assert np.array_equal(res[0][1]["local"][0], res[1][1]["local"][0])
    assert np.array_equal(res[0][1]["tsqr"][0], res[1][1]["tsqr"][0])
