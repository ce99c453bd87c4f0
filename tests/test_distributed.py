"""N > 1 path on CPU: world_size-2/3 gloo runs of the row-slab restatement
(oracle/dist_ref.py, the decomposition the HIP library implements) against
the single-process oracle; halo plans checked for consistency."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

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
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle import ca_lanczos_ref as ref
    from oracle import dist_ref as dr
    dim, N, s, it, basis = case
    A = ref.laplacian_2d(N) if dim == 2 else ref.laplacian_3d(N)
    n = A.shape[0]
    bounds = dr.slab_bounds(n, world, N ** (dim - 1))
    slab = dr.Slab(A, bounds, rank)
    # halo correctness: distributed SpMV == global SpMV on this slab
    x = ref.matlab_rand(n, seed=11)
    y = slab.spmv(x[slab.r0:slab.r1])
    ok_spmv = np.array_equal(y, (A @ x)[slab.r0:slab.r1])
    r = ref.matlab_rand(n)
    T = dr.ca_lanczos_dist(slab, r[slab.r0:slab.r1], s, it, basis)
    out_q.put((rank, ok_spmv, T, len(slab.peers), len(slab.ghost)))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,case", [(2, (2, 16, 8, 40, "newton")), (3, (3, 8, 4, 32, "newton")),
                                        (2, (2, 12, 4, 24, "monomial"))])
def test_row_slab_ca_lanczos_matches_single_process(ref, world, case):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, case, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    dim, N, s, it, basis = case
    A = ref.laplacian_2d(N) if dim == 2 else ref.laplacian_3d(N)
    exp = ref.ca_lanczos(A, ref.matlab_rand(A.shape[0]), s, it, basis, "local", diagnostics=False)
    normA = 4.0 * dim
    for rank, ok_spmv, T, npeers, nghost in res:
        assert ok_spmv, "halo exchange / local CSR wrong on rank %d" % rank
        assert npeers >= 1 and nghost > 0
        assert T.shape == exp.T.shape
        w, we = np.sort(np.linalg.eigvals(T).real), np.sort(np.linalg.eigvals(exp.T).real)
        assert abs(w[-1] - we[-1]) <= 1e-9 * normA and abs(w[0] - we[0]) <= 1e-9 * normA
        m = min(2 * s, T.shape[0])
        assert np.max(np.abs(T[:m, :m] - exp.T[:m, :m])) <= 1e-9 * normA
    # every rank holds the same (replicated) T
    for _, _, T, _, _ in res[1:]:
        assert np.array_equal(T, res[0][2])


def _mpk_worker(rank, world, port, case, out_q):
    import sys
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle import ca_lanczos_ref as ref
    from oracle import dist_ref as dr
    dim, N, s, D = case
    A = ref.laplacian_2d(N) if dim == 2 else ref.laplacian_3d(N)
    n = A.shape[0]
    bounds = dr.slab_bounds(n, world, N ** (dim - 1))
    r0, r1 = bounds[rank], bounds[rank + 1]
    m = dr.MPKSlab(A[r0:r1], bounds, rank, D)
    q = ref.matlab_rand(n, seed=3)
    lam = np.linspace(0.5, 4.0 * dim - 0.5, s)
    # every rank takes part in the exchanges, so the split runs on all or none
    import torch
    ok = torch.tensor([1.0 if m.split_ok(s) else 0.0])
    dist.all_reduce(ok, op=dist.ReduceOp.MIN)
    split = (m.powers_split(q[r0:r1], s, lam), m.powers_split(q[r0:r1], s)) if ok.item() > 0 else None
    out_q.put((rank, r0, r1, m.bl, m.elo, m.ehi, m.powers(q[r0:r1], s, lam), m.powers(q[r0:r1], s), split))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,case", [(2, (3, 9, 8, 8)), (3, (3, 8, 6, 8)), (4, (2, 24, 8, 8)),
                                        (3, (2, 20, 4, 6)), (2, (2, 40, 8, 8)), (3, (2, 61, 6, 8)),
                                        (4, (2, 90, 8, 8))])
def test_mpk_deep_ghost_zone_restatement(ref, world, case):
    """The CA matrix-powers scheme of comm.cpp / runtime.cpp (ghost rows
    fetched from owners, one s-band exchange, shrinking ranges) on gloo:
    the powers equal the global Newton / monomial powers bit for bit on
    every slab, including ghost zones that span several ranks (3-4 ranks on
    8-9 planes with an 8-plane zone) and clip at the domain ends.  Slabs of
    more than 2s planes also run the overlapped schedule (interior powers
    before the exchange, from a NaN ghost zone): same bits, no NaN."""
    ctx = mp.get_context("spawn")
    qq = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_mpk_worker, args=(r, world, port, case, qq)) for r in range(world)]
    for p in procs:
        p.start()
    res = [qq.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    dim, N, s, D = case
    A = ref.laplacian_2d(N) if dim == 2 else ref.laplacian_3d(N)
    q = ref.matlab_rand(A.shape[0], seed=3)
    lam = np.linspace(0.5, 4.0 * dim - 0.5, s)
    Vn = ref.matrix_powers_newton(A, q, s, lam, 1)
    Vm = np.hstack([q[:, None], ref.matrix_powers_monomial(A, q, s)])
    nsplit = 0
    for rank, r0, r1, bl, elo, ehi, Pn, Pm, split in res:
        assert bl == N ** (dim - 1)
        assert elo == max(0, r0 - (D - 1) * bl) and ehi == min(A.shape[0], r1 + (D - 1) * bl)
        assert np.array_equal(Pn, Vn[r0:r1]), rank
        assert np.array_equal(Pm, Vm[r0:r1]), rank
        if split is not None:
            nsplit += 1
            assert np.array_equal(split[0], Pn) and np.array_equal(split[1], Pm), rank
    if min(x[2] - x[1] for x in res) > 2 * s * N ** (dim - 1):  # every slab thick enough
        assert nsplit == world
