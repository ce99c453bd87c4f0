"""The RCCL communicator with several ranks (comm.cpp's kind == 1 branches:
ncclAllReduce of the Gram tiles, ncclSend/ncclRecv of the halo and the deep
ghost zone, ncclAllGather of the TSQR roots, the exchange on the
communicator's own stream overlapped with the interior powers).

The test box has one GPU and RCCL refuses two ranks on one device of one
host ("Duplicate GPU detected").  Each rank therefore states its own host id
(NCCL_HOSTID), so RCCL sees P one-GPU hosts and connects them over its socket
transport on the loopback interface.  The transport differs from xGMI; the
library's calls, their order, their buffers, offsets and streams are the ones
an 8-GPU node runs.  Every result is checked against the single-rank run or
the oracle's bits, as the host-staged tests in test_gpu_distributed.py do."""
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


def _rccl_env(rank):
    # one "host" per rank, sockets over loopback; set before RCCL initialises
    os.environ.update(NCCL_HOSTID="cal-rank-%d" % rank, NCCL_SOCKET_IFNAME="lo", NCCL_IB_DISABLE="1",
                      NCCL_DEBUG=os.environ.get("NCCL_DEBUG", "WARN"))


def _matrix(cal, dim, N):
    if dim == 0:
        return cal.matrices.circuit_like(N)
    return cal.matrices.laplacian_2d(N) if dim == 2 else cal.matrices.laplacian_3d(N)


def _worker(rank, world, port, case, out_q):
    import sys
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    _rccl_env(rank)
    import faulthandler
    faulthandler.dump_traceback_later(150, exit=True)  # a hung rank names its call
    try:
        import torch
        import torch.distributed as dist
        dist.init_process_group("gloo", rank=rank, world_size=world)
        import ctypes
        import ca_lanczos_amd as cal
        from ca_lanczos_amd._lib import check, lib, ptr
        from oracle import ca_lanczos_ref as ref

        uid = bytearray(128)
        if rank == 0:
            buf = ctypes.create_string_buffer(128)
            check(None, lib.cal_comm_unique_id(buf))
            uid = bytearray(buf.raw)
        t = torch.tensor(list(uid), dtype=torch.uint8)
        dist.broadcast(t, 0)
        uid = bytes(t.tolist())

        kind, dim, N, s, it, orth, normalize = case
        A = _matrix(cal, dim, N)
        n = A.shape[0]
        b = cal.matrices.slab_bounds(n, world, N ** (dim - 1) if dim else 1)
        r0, r1 = b[rank], b[rank + 1]
        # config 5's topology (dim 0): the irregular stand-in in CSR, compact ghosts
        ctx = cal.Context(0, mpk_depth=8, normalize=normalize, spmv_format="csr" if dim == 0 else None)
        ctx.comm_init_rccl(world, rank, uid)
        ctx.set_matrix_slab(n, r0, A[r0:r1])
        res = dict(r0=r0, r1=r1, info=ctx.matrix_info(), mpk=ctx.mpk_info())
        x = ref.matlab_rand(n, seed=5)
        xl = np.ascontiguousarray(x[r0:r1])
        y = np.zeros(r1 - r0)
        check(ctx.h, lib.cal_spmv(ctx.h, ptr(xl), ptr(y)))
        res["spmv"] = y
        if kind == "lanczos":
            v = ref.matlab_rand(n, seed=7)[r0:r1]
            lam = np.array([7.5, 0.5, 3.0, 11.0, 1.5, 5.0, 9.0, 2.5])[:s]
            res["Vn"] = cal.matrix_powers_newton(None, v, s, lam, 1, ctx=ctx)
            res["schedule"] = ctx.mpk_schedule()
            out = cal.ca_lanczos_ex(A, ref.matlab_rand(n)[r0:r1], s, it, "newton", orth, diagnostics=True, ctx=ctx)
            res.update(T=out.T, rn=out.ritz_rnorm, oe=out.orth_err, flags=list(out.reorth),
                       brk=(out.info.get("n_orth_breaks"), out.info.get("n_ritz_locked")))
            if normalize == "tsqr":
                res["fold"] = ctx.tsqr_fold_stats()
        elif kind == "circuit":  # config 5's driver on the irregular matrix
            r = ref.matlab_rand(n, seed=2)[r0:r1]
            res["irl"] = cal.impl_restarted_ca_lanczos(None, r, 64, 8, 8, "newton", "full", 1.0e-8, ctx=ctx)
        else:  # the implicit restart (config 5's driver)
            r = ref.matlab_rand(n, seed=2)[r0:r1]
            res["irl"] = cal.impl_restarted_ca_lanczos(None, r, 48, 8, 8, "newton", "full", 1.0e-8, ctx=ctx)
            res["erl"] = cal.restarted_ca_lanczos(None, r, 48, 4, 8, "newton", "full", 1.0e-8, ctx=ctx)
        res["stats"] = ctx.comm_stats()
        ctx.close()
        out_q.put((rank, res))
        dist.barrier()
        dist.destroy_process_group()
    except BaseException as e:  # reported, so the parent does not wait out its timeout
        out_q.put((rank, "error: %r" % (e,)))
        raise


def _run(world, case):
    mpc = mp.get_context("spawn")
    q = mpc.Queue()
    port = _free_port()
    procs = [mpc.Process(target=_worker, args=(r, world, port, case, q)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        res = sorted([q.get(timeout=240) for _ in range(world)], key=lambda t: t[0])
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.exitcode is None:
                p.kill()
    errs = [r for r in res if isinstance(r[1], str)]
    assert not errs, errs
    for p in procs:
        assert p.exitcode == 0
    return [r[1] for r in res]


CASES = [
    # world, (kind, dim, N, s, iters, orth, normalize)
    # lap3d 40 in 2 slabs of 20 planes: > 2s planes, so the exchange overlaps
    # the interior powers on the RCCL stream (schedule 2)
    (2, ("lanczos", 3, 40, 8, 40, "local", "auto")),
    # 3 slabs of 3-4 planes: the 8-deep ghost zone spans two ranks, clipped
    # at the domain ends; 'full' orth; TSQR normalize with the all-gathered root
    (3, ("lanczos", 3, 10, 8, 32, "full", "tsqr")),
    # 4 slabs of lap2d 64 rows: the fused TSQR fold's rank-uniform vote
    (4, ("lanczos", 2, 64, 6, 36, "local", "tsqr")),
    # 'periodic' (omega recurrence, normest over the all-reduced dots) and
    # 'selective' (locked Ritz vectors in the projection)
    (2, ("lanczos", 2, 24, 8, 64, "periodic", "auto")),
    (2, ("lanczos", 2, 24, 8, 64, "selective", "auto")),
    (2, ("irl", 2, 40, 8, 0, "full", "auto")),
    # config 5's topology: circuit_like(200) in CSR, ghost columns scattered
    # over the peer's rows (compact layout, gather kernel, one exchange per SpMV)
    (2, ("circuit", 0, 200, 8, 0, "full", "auto")),
    (3, ("circuit", 0, 200, 8, 0, "full", "auto")),
]


@pytest.mark.parametrize("world,case", CASES)
def test_rccl_ranks_match_single(cal, ref, world, case):
    res = _run(world, case)
    kind, dim, N, s, it, orth, normalize = case
    A = _matrix(cal, dim, N)
    n = A.shape[0]
    normA = 4.0 * dim if dim else float(abs(A).sum(axis=1).max())
    x = ref.matlab_rand(n, seed=5)
    y = A @ x
    for rank, rr in enumerate(res):
        st = rr["stats"]
        assert st["nranks"] == world and st["kind"] == 1 and st["rccl_count"] == world, st
        assert st["allreduce_calls"] > 0 and st["halo_calls"] > 0, st
        assert rr["mpk"]["depth"] == (8 if dim else 1)   # compact ghosts: one exchange per SpMV
        assert np.array_equal(rr["spmv"], y[rr["r0"]:rr["r1"]]), rank
    if kind == "lanczos":
        v = ref.matlab_rand(n, seed=7)
        lam = np.array([7.5, 0.5, 3.0, 11.0, 1.5, 5.0, 9.0, 2.5])[:s]
        Vn = ref.matrix_powers_newton(A, v, s, lam, 1)
        ctx1 = cal.Context(0, normalize=normalize).set_matrix(A)
        single = cal.ca_lanczos_ex(A, ref.matlab_rand(n), s, it, "newton", orth, diagnostics=True, ctx=ctx1)
        for rank, rr in enumerate(res):
            print("world %d case %s rank %d: schedule %d, stats %s" % (world, case, rank, rr["schedule"], rr["stats"]))
            assert np.array_equal(rr["Vn"], Vn[rr["r0"]:rr["r1"]]), rank   # the oracle's bits
            assert rr["flags"] == list(single.reorth)
            assert rr["brk"] == (single.info.get("n_orth_breaks"), single.info.get("n_ritz_locked"))
            assert np.max(np.abs(rr["T"] - single.T)) <= 1e-9 * normA
            big = single.ritz_rnorm > 1e-10
            dev = np.abs(rr["rn"][big] / single.ritz_rnorm[big] - 1.0)
            assert np.all(dev <= 1e-8), dev.max()
            assert np.array_equal(rr["T"], res[0]["T"])            # every rank holds the same T
        if world == 2 and dim == 3 and N == 40:
            assert all(rr["schedule"] == 2 for rr in res), [rr["schedule"] for rr in res]
        ctx1.close()
    elif kind == "circuit":
        c1 = cal.Context(0, spmv_format="csr").set_matrix(A)
        irl1 = cal.impl_restarted_ca_lanczos(A, ref.matlab_rand(n, seed=2), 64, 8, 8, "newton", "full", 1.0e-8,
                                             ctx=c1)
        c1.close()
        outs = [rr["irl"] for rr in res]
        print("circuit_%d x%d over RCCL: restarts %s (single %d)" % (N, world, [o["num_restarts"] for o in outs],
                                                                     irl1["num_restarts"]))
        assert irl1["converged"] and all(o["converged"] for o in outs)
        assert all(o["num_restarts"] == outs[0]["num_restarts"] for o in outs)
        assert abs(outs[0]["num_restarts"] - irl1["num_restarts"]) <= 1
        assert all(np.array_equal(o["conv_eigs"], outs[0]["conv_eigs"]) for o in outs)
        ev = outs[0]["conv_eigs"]
        assert np.max(np.abs(ev - irl1["conv_eigs"]) / np.abs(irl1["conv_eigs"])) <= 1e-10
        V = np.vstack([o["Q_conv"] for o in outs])
        assert np.max(np.abs(V.T @ V - np.eye(V.shape[1]))) < 1e-9
    else:
        eref = ref.laplacian_2d_eigs(N)[::-1]
        for key, nw in (("irl", 8), ("erl", 4)):   # the implicit (f3) and explicit (f2) restarts
            outs = [rr[key] for rr in res]
            assert all(o["converged"] for o in outs)
            assert outs[0]["num_restarts"] == outs[1]["num_restarts"]
            assert np.array_equal(outs[0]["conv_eigs"], outs[1]["conv_eigs"])
            ev = outs[0]["conv_eigs"]
            assert np.max(np.min(np.abs(ev[:, None] - eref[None, :]), axis=1)) <= 1e-10 * normA
            if key == "erl":
                assert np.max(np.abs(ev - eref[:nw])) <= 1e-10 * normA
            V = np.vstack([o["Q_conv"] for o in outs])
            assert V.shape == (n, nw)
            assert np.max(np.abs(V.T @ V - np.eye(nw))) < 1e-9


def _config4_worker(rank, world, port, case, out_q):
    """Config 4 at its own size over RCCL: lap3d_215 in z-slabs, the deep
    ghost zone of the real band (215^2 rows) exchanged on the RCCL stream
    while the interior powers run."""
    import sys
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    _rccl_env(rank)
    import faulthandler
    faulthandler.dump_traceback_later(280, exit=True)
    try:
        import hashlib
        import torch
        import torch.distributed as dist
        dist.init_process_group("gloo", rank=rank, world_size=world)
        import ctypes
        import scipy.sparse as sp
        import ca_lanczos_amd as cal
        from ca_lanczos_amd._lib import check, lib
        from oracle import ca_lanczos_ref as ref

        uid = bytearray(128)
        if rank == 0:
            buf = ctypes.create_string_buffer(128)
            check(None, lib.cal_comm_unique_id(buf))
            uid = bytearray(buf.raw)
        t = torch.tensor(list(uid), dtype=torch.uint8)
        dist.broadcast(t, 0)
        N, s, it = case
        n = N ** 3
        b = cal.matrices.slab_bounds(n, world, N * N)
        r0, r1 = b[rank], b[rank + 1]
        rowptr, col, val = cal.matrices.laplacian_rows(3, N, r0, r1)
        ctx = cal.Context(0, mpk_depth=8)
        ctx.comm_init_rccl(world, rank, bytes(t.tolist()))
        ctx.set_matrix_slab(n, r0, sp.csr_matrix((val, col, rowptr), shape=(r1 - r0, n)))
        del rowptr, col, val
        lam = np.array([7.5, 0.5, 3.0, 11.0, 1.5, 5.0, 9.0, 2.5])[:s]
        Vn = cal.matrix_powers_newton(None, ref.matlab_rand(n, seed=7)[r0:r1], s, lam, 1, ctx=ctx)
        res = dict(r0=r0, r1=r1, sched=ctx.mpk_schedule(),
                   powers=hashlib.sha256(np.asfortranarray(Vn).tobytes()).hexdigest())
        del Vn
        out = cal.ca_lanczos_ex(None, ref.matlab_rand(n)[r0:r1], s, it, "newton", "local", diagnostics=True,
                                return_Q=False, ctx=ctx)
        res.update(T=out.T, rn=out.ritz_rnorm, flags=list(out.reorth), stats=ctx.comm_stats())
        ctx.close()
        out_q.put((rank, res))
        dist.barrier()
        dist.destroy_process_group()
    except BaseException as e:
        out_q.put((rank, "error: %r" % (e,)))
        raise


@pytest.fixture(scope="module")
def config4_single_gpu(cal, ref):
    """The single-GPU Newton powers and 4-iteration run of lap3d_215."""
    N, s, it = 215, 8, 4
    A = cal.matrices.laplacian_3d(N)
    n = A.shape[0]
    c1 = cal.Context(0).set_matrix(A)
    lam = np.array([7.5, 0.5, 3.0, 11.0, 1.5, 5.0, 9.0, 2.5])[:s]
    Vn = cal.matrix_powers_newton(None, ref.matlab_rand(n, seed=7), s, lam, 1, ctx=c1)
    single = cal.ca_lanczos_ex(None, ref.matlab_rand(n), s, it, "newton", "local", diagnostics=True,
                               return_Q=False, ctx=c1)
    c1.close()
    return (N, s, it), Vn, single


@pytest.mark.timeout(600)
@pytest.mark.parametrize("world", [2, 4, 8])
def test_rccl_config4_lap3d_215(cal, ref, config4_single_gpu, world):
    """Config 4 at full size (n = 9,938,375) on 2, 4 and 8 ranks over RCCL (8: the driver's SCALE topology):
    each rank's Newton powers bit-identical to the single-GPU powers of its
    rows, the overlapped schedule taken, and 4 outer iterations with
    diagnostics against the single-GPU run (T within 1e-9 ||A||, identical
    flags, Ritz residuals above 1e-10 within 1e-8 relative)."""
    import hashlib
    case, Vn, single = config4_single_gpu
    mpc = mp.get_context("spawn")
    q = mpc.Queue()
    port = _free_port()
    procs = [mpc.Process(target=_config4_worker, args=(r, world, port, case, q)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        res = sorted([q.get(timeout=400) for _ in range(world)], key=lambda t: t[0])
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.exitcode is None:
                p.kill()
    errs = [r for r in res if isinstance(r[1], str)]
    assert not errs, errs
    for rank, rr in res:
        print("config 4 over RCCL, rank %d rows [%d, %d): schedule %d, stats %s" % (rank, rr["r0"], rr["r1"],
                                                                                   rr["sched"], rr["stats"]))
        assert rr["stats"]["kind"] == 1 and rr["stats"]["rccl_count"] == world
        assert rr["sched"] == 2, rr["sched"]                       # exchange overlapped on the RCCL stream
        assert rr["powers"] == hashlib.sha256(np.asfortranarray(Vn[rr["r0"]:rr["r1"]]).tobytes()).hexdigest()
        assert rr["flags"] == list(single.reorth)
        assert np.max(np.abs(rr["T"] - single.T)) <= 1e-9 * 12.0
        big = single.ritz_rnorm > 1e-10
        assert np.all(np.abs(rr["rn"][big] / single.ritz_rnorm[big] - 1.0) <= 1e-8)
    assert all(np.array_equal(res[0][1]["T"], rr["T"]) for _, rr in res)
