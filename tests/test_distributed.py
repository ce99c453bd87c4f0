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
