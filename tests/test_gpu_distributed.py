"""The library's own distributed path (cal_set_matrix_csr_dist + halo
exchange + allreduced Grams) on the GPU: 2 ranks share the one GPU of the
test box and talk through the host-staged communicator (gloo callbacks);
RCCL replaces exactly these two callbacks on a multi-GPU node."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, case, out_q):
    import sys
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
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

    dim, N, s, it, orth = case
    A = cal.matrices.laplacian_2d(N) if dim == 2 else cal.matrices.laplacian_3d(N)
    n = A.shape[0]
    b = cal.matrices.slab_bounds(n, world, N ** (dim - 1))
    r0, r1 = b[rank], b[rank + 1]
    ctx = cal.Context(0)
    ctx.comm_init_host(world, rank, allreduce, exchange)
    ctx.set_matrix_slab(n, r0, A[r0:r1])
    info = ctx.matrix_info()
    x = ref.matlab_rand(n, seed=5)
    from ca_lanczos_amd._lib import check, lib, ptr
    xl = np.ascontiguousarray(x[r0:r1])
    y = np.zeros(r1 - r0)
    check(ctx.h, lib.cal_spmv(ctx.h, ptr(xl), ptr(y)))
    ok_spmv = np.array_equal(y, (A @ x)[r0:r1])
    out = cal.ca_lanczos_ex(A, ref.matlab_rand(n)[r0:r1], s, it, "newton", orth, diagnostics=True, ctx=ctx)
    out_q.put((rank, ok_spmv, info, out.T, out.ritz_rnorm, out.orth_err, list(out.reorth),
               (out.info.get("n_orth_breaks"), out.info.get("n_ritz_locked"))))
    ctx.close()
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("case", [(2, 32, 8, 48, "local"), (3, 10, 8, 32, "full"), (2, 24, 8, 64, "periodic"),
                                  (2, 24, 8, 64, "selective")])
def test_two_ranks_one_gpu_match_single(cal, ref, case):
    world = 2
    mpc = mp.get_context("spawn")
    q = mpc.Queue()
    port = _free_port()
    procs = [mpc.Process(target=_worker, args=(r, world, port, case, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=300) for _ in range(world)], key=lambda t: t[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    dim, N, s, it, orth = case
    A = cal.matrices.laplacian_2d(N) if dim == 2 else cal.matrices.laplacian_3d(N)
    r = ref.matlab_rand(A.shape[0])
    single = cal.ca_lanczos_ex(A, r, s, it, "newton", orth, diagnostics=True)
    normA = 4.0 * dim
    for rank, ok_spmv, info, T, rn, oe, flags, brk in res:
        assert ok_spmv, rank
        assert info["nghost"] > 0
        assert flags == list(single.reorth)
        assert brk == (single.info.get("n_orth_breaks"), single.info.get("n_ritz_locked"))
        assert np.max(np.abs(T - single.T)) <= 1e-9 * normA
        # every Ritz pair's residual norm above 1e-10: 1e-8 relative (the
        # config-4 bar); the two runs differ only in the Gram summation order
        big = single.ritz_rnorm > 1e-10
        dev = np.abs(rn[big] / single.ritz_rnorm[big] - 1.0)
        print("case %s rank %d: max rel rn deviation %.2e over %d pairs" % (case, rank, dev.max(), dev.size))
        assert np.all(dev <= 1e-8)
    assert np.array_equal(res[0][3], res[1][3])


def test_rccl_single_rank_matches_local(cal, ref):
    """The RCCL communicator itself (ncclCommInitRank, in-place ncclAllReduce
    of the Gram tiles on the context stream, the distributed matrix setup)
    with one rank: bit-identical to the communicator-free run.  Several ranks
    per GPU are refused by RCCL, so this is the RCCL coverage a one-GPU box
    allows; the multi-rank logic is covered above through the host-staged
    communicator, which differs only in the transport."""
    import ctypes
    from ca_lanczos_amd._lib import lib
    A = cal.matrices.laplacian_3d(14)
    n = A.shape[0]
    r = ref.matlab_rand(n, seed=8)
    uid = ctypes.create_string_buffer(128)
    assert lib.cal_comm_unique_id(uid) == 0
    c1 = cal.Context(0)
    c1.comm_init_rccl(1, 0, uid.raw)
    c1.set_matrix_slab(n, 0, A)
    assert c1.matrix_info()["nghost"] == 0
    out1 = cal.ca_lanczos_ex(A, r, 8, 40, "newton", "local", diagnostics=True, ctx=c1)
    c2 = cal.Context(0).set_matrix(A)
    out2 = cal.ca_lanczos_ex(A, r, 8, 40, "newton", "local", diagnostics=True, ctx=c2)
    assert np.array_equal(out1.T, out2.T)
    assert np.array_equal(out1.Q, out2.Q)
    assert np.array_equal(out1.ritz_rnorm, out2.ritz_rnorm)
    c1.close()
    c2.close()


def _mpk_worker(rank, world, port, case, out_q):
    """One rank: the CA matrix-powers kernel (deep ghost zone, one exchange
    per s powers) against the one-exchange-per-SpMV distributed path."""
    import sys
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
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

    dim, N, s, it, orth = case
    A = cal.matrices.laplacian_2d(N) if dim == 2 else cal.matrices.laplacian_3d(N)
    n = A.shape[0]
    b = cal.matrices.slab_bounds(n, world, N ** (dim - 1))
    r0, r1 = b[rank], b[rank + 1]
    res = {}
    # (depth, CAL_MPK_OVERLAP): 1 splits the powers into the interior
    # trapezoid and the boundary pieces after the exchange (the RCCL default)
    for key, depth, ov in (("8", 8, "0"), ("8s", 8, "1"), ("1", 1, "0")):
        os.environ["CAL_MPK_OVERLAP"] = ov
        ctx = cal.Context(0, mpk_depth=depth)
        ctx.comm_init_host(world, rank, allreduce, exchange)
        ctx.set_matrix_slab(n, r0, A[r0:r1])
        v = ref.matlab_rand(n, seed=7)[r0:r1]
        lam = np.array([7.5, 0.5, 3.0, 11.0, 1.5, 5.0, 9.0, 2.5])[:s]
        Vn = cal.matrix_powers_newton(None, v, s, lam, 1, ctx=ctx)
        Vm = cal.matrix_powers_monomial(None, v / np.linalg.norm(v), s, ctx=ctx)
        out = cal.ca_lanczos_ex(A, ref.matlab_rand(n)[r0:r1], s, it, "newton", orth, diagnostics=False, ctx=ctx)
        res[key] = (ctx.mpk_info(), Vn, Vm, out.T, list(out.reorth))
        ctx.close()
    out_q.put((rank, r0, r1, res))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,case", [(2, (3, 12, 8, 40, "local")), (3, (3, 10, 8, 32, "local")),
                                        (3, (2, 30, 6, 36, "full")), (2, (3, 40, 8, 40, "local")),
                                        (3, (2, 61, 6, 36, "local"))])
def test_mpk_deep_ghost_zone(cal, ref, world, case):
    """Distributed matrix powers with one s-deep halo exchange (the stored
    ghost-zone rows are recomputed redundantly) are bit-identical to the
    single-GPU powers on every rank's rows, and the whole CA-Lanczos run is
    bit-identical to the one-exchange-per-SpMV distributed run.  World 3 on
    10 or 30 planes: the 8-plane ghost zone spans two ranks and is clipped at
    the domain ends.  The split schedule (interior trapezoid, then both
    boundary pieces in one two-range launch) gives the same bits; it needs
    more than 2 s planes per slab (lap3d 40 on 2 ranks, lap2d 61 on 3)."""
    mpc = mp.get_context("spawn")
    q = mpc.Queue()
    port = _free_port()
    procs = [mpc.Process(target=_mpk_worker, args=(r, world, port, case, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=300) for _ in range(world)], key=lambda t: t[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    dim, N, s, it, orth = case
    A = cal.matrices.laplacian_2d(N) if dim == 2 else cal.matrices.laplacian_3d(N)
    n = A.shape[0]
    v = ref.matlab_rand(n, seed=7)
    lam = np.array([7.5, 0.5, 3.0, 11.0, 1.5, 5.0, 9.0, 2.5])[:s]
    Vn = ref.matrix_powers_newton(A, v, s, lam, 1)
    for rank, r0, r1, rr in res:
        info8, info1 = rr["8"][0], rr["1"][0]
        assert info8["depth"] == 8 and info1["depth"] == 1
        assert info8["band_l"] == N ** (dim - 1) and info8["n_rows"] > r1 - r0
        assert np.array_equal(rr["8"][1], Vn[r0:r1]), rank            # newton powers, oracle bits
        assert np.array_equal(rr["8"][1], rr["1"][1]) and np.array_equal(rr["8"][2], rr["1"][2])
        assert np.array_equal(rr["8"][3], rr["1"][3]) and rr["8"][4] == rr["1"][4]   # whole run
        for k in range(1, 4):                                          # the split schedule
            assert np.array_equal(rr["8s"][k], rr["8"][k]), (rank, k)
        assert rr["8s"][4] == rr["8"][4]
    assert all(np.array_equal(res[0][3]["8"][3], x[3]["8"][3]) for x in res)


def _restart_worker(rank, world, port, out_q):
    import sys
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
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

    out = {}
    A = cal.matrices.laplacian_2d(40)
    n = A.shape[0]
    b = cal.matrices.slab_bounds(n, world, 40)
    r0, r1 = b[rank], b[rank + 1]
    ctx = cal.Context(0)
    ctx.comm_init_host(world, rank, allreduce, exchange)
    ctx.set_matrix_slab(n, r0, A[r0:r1])
    r = ref.matlab_rand(n, seed=2)[r0:r1]
    out["irl"] = cal.impl_restarted_ca_lanczos(None, r, 48, 8, 8, "newton", "full", 1.0e-8, ctx=ctx)
    out["erl"] = cal.restarted_ca_lanczos(None, r, 48, 4, 8, "newton", "full", 1.0e-8, ctx=ctx)
    ctx.close()
    out_q.put((rank, r0, r1, out))
    dist.barrier()
    dist.destroy_process_group()


def test_restart_drivers_two_ranks(cal, ref):
    """The explicit (f2) and implicit (f3) restart drivers on 2 row slabs:
    same eigenvalues as the closed form, the same restart count on both ranks,
    and the slabs of the Ritz vectors assemble into orthonormal eigenvectors."""
    world = 2
    mpc = mp.get_context("spawn")
    q = mpc.Queue()
    port = _free_port()
    procs = [mpc.Process(target=_restart_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=300) for _ in range(world)], key=lambda t: t[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    A = cal.matrices.laplacian_2d(40)
    eref = ref.laplacian_2d_eigs(40)[::-1]
    for key, nw in (("irl", 8), ("erl", 4)):
        outs = [x[3][key] for x in res]
        assert all(o["converged"] for o in outs)
        assert outs[0]["num_restarts"] == outs[1]["num_restarts"]
        assert np.array_equal(outs[0]["conv_eigs"], outs[1]["conv_eigs"])
        ev = outs[0]["conv_eigs"]
        # every value is an eigenvalue of A and the largest is found; the
        # explicit restart locks converged vectors, so it also resolves the
        # double eigenvalues -- the implicit one sees a second copy only
        # through rounding (a single-vector Krylov space), so not there
        assert np.max(np.min(np.abs(ev[:, None] - eref[None, :]), axis=1)) <= 1e-10 * 8.0
        assert abs(ev[0] - eref[0]) <= 1e-10 * 8.0
        if key == "erl":
            assert np.max(np.abs(ev - eref[:nw])) <= 1e-10 * 8.0
        V = np.vstack([o["Q_conv"] for o in outs])
        assert V.shape == (A.shape[0], nw)
        assert np.max(np.abs(V.T @ V - np.eye(nw))) < 1e-9
        res_n = np.linalg.norm(A @ V - V * outs[0]["conv_eigs"], axis=0)
        assert np.max(res_n) < 1e-6


def _pn_worker(rank, world, port, heights, out_q):
    """Tier-1 projectAndNormalize (TSQR normalize, the fused fold when its
    shape applies) on row panels whose local heights match the resident
    slab on one rank and not on the other."""
    import sys
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import ca_lanczos_amd as cal

    def allreduce(a):
        t = torch.from_numpy(a)
        dist.all_reduce(t)

    def exchange(peer, send, recv):  # the slab's halo setup
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

    try:
        _pn_run(cal, rank, world, heights, out_q, allreduce, exchange)
    except Exception as e:  # reported, so the parent does not wait out its timeout
        out_q.put((rank, "error", repr(e), None, None))
        raise
    dist.barrier()
    dist.destroy_process_group()


def _pn_run(cal, rank, world, heights, out_q, allreduce, exchange):
    A = cal.matrices.laplacian_2d(200)
    n = A.shape[0]
    b = cal.matrices.slab_bounds(n, world, 200)
    r0, r1 = b[rank], b[rank + 1]
    ctx = cal.Context(0)
    ctx.comm_init_host(world, rank, allreduce, exchange)
    ctx.set_matrix_slab(n, r0, A[r0:r1])
    assert heights[0] == r1 - r0 or rank != 0
    rng = np.random.RandomState(7)
    N = sum(heights)
    Qp = np.linalg.qr(rng.randn(N, 9))[0]
    X = rng.randn(N, 8)
    lo = sum(heights[:rank])
    QZ, RZ, re, rk = cal.projectAndNormalize_ex([Qp[lo:lo + heights[rank]]], X[lo:lo + heights[rank]], True,
                                                ctx=ctx)
    out_q.put((rank, QZ, RZ, re, rk))
    ctx.close()


def test_tier1_project_and_normalize_mismatched_heights(cal, ref):
    """the fold's shape vote must be reached by the same branch on
    every rank.  Rank 0's panel has its slab's height (20000 rows), rank 1's
    does not (20037): both ranks vote by one all-reduce (the run used to hang
    when rank 0 took the slab table and rank 1 the vote).  The result equals
    the one-rank call on the stacked panel to 1e-12."""
    world = 2
    heights = (20000, 20037)
    mpc = mp.get_context("spawn")
    q = mpc.Queue()
    port = _free_port()
    procs = [mpc.Process(target=_pn_worker, args=(r, world, port, heights, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=100) for _ in range(world)], key=lambda t: t[0])
    assert not any(isinstance(r[1], str) for r in res), res
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    rng = np.random.RandomState(7)
    N = sum(heights)
    Qp = np.linalg.qr(rng.randn(N, 9))[0]
    X = rng.randn(N, 8)
    QZ1, RZ1, re1, rk1 = cal.projectAndNormalize_ex([Qp], X, True)
    QZ = np.vstack([r[1] for r in res])
    assert res[0][3] == res[1][3] == re1 and res[0][4] == res[1][4] == rk1
    for r in res:
        for a, b in zip(r[2], RZ1):
            assert np.max(np.abs(a - b)) <= 1e-12 * max(1.0, np.max(np.abs(b)))
    assert np.max(np.abs(QZ - QZ1)) <= 1e-12
    assert np.max(np.abs(QZ.T @ QZ - np.eye(8))) < 1e-13
