"""CA-Lanczos outer-iterations/s + SpMV HBM GB/s on MI355X (BASELINE.json).

A "step" is one CA-Lanczos outer iteration (ca_lanczos.m:166-237): s = 8
fused SpMV+Newton-shift launches, the block orthogonalisation against the
previous block (projectAndNormalize), and the host T extension; diagnostics
(Ritz residuals) off, as SURVEY §8d prescribes.  Inputs (A, r, Q, V) are
resident in HBM before the timed region.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--workload lap3d_215]

N > 1 runs one rank per GPU (torch.distributed.run): contiguous z-slabs of
the same matrix, RCCL halo exchange per SpMV and RCCL allreduce of the Gram
blocks (strong scaling, whole-job outer-iters/s).
"""
from __future__ import annotations

import argparse
import ctypes
import json
import math
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X spec (MI355X_MICROARCH.md: 8.0 TB/s)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=int(os.environ.get("WORLD_SIZE", "1")))
    p.add_argument("--steps", type=int, default=15)
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--workload", default="lap3d_215")
    p.add_argument("--s", type=int, default=8)
    p.add_argument("--basis", default="newton")
    p.add_argument("--orth", default="local")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-iters", type=int, default=2, help="outer iterations of the CPU sample")
    p.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "spmv_traffic.json"))
    p.add_argument("--comm", default="rccl", choices=["rccl", "host"],
                   help="N > 1 transport: RCCL (default) or host-staged gloo callbacks (rehearsal of the "
                        "distributed bench with several ranks on one GPU)")
    return p.parse_args()


def workload_dims(name):
    kind, N = name.split("_")
    dim = {"lap2d": 2, "lap3d": 3}[kind]
    return dim, int(N)


def build_rows(dim, N, r0, r1):
    from ca_lanczos_amd.matrices import laplacian_rows
    return laplacian_rows(dim, N, r0, r1)


def cpu_baseline(dim, N, s, iters):
    """The oracle restatement (NumPy/SciPy) timed on this host: Newton
    prologue excluded, `iters` outer iterations of ca_lanczos_basic with
    diagnostics off, on the same matrix and start vector."""
    import scipy.sparse as sp
    from oracle import ca_lanczos_ref as ref
    try:
        from threadpoolctl import threadpool_info
        blas_threads = max([d.get("num_threads", 1) for d in threadpool_info()] or [1])
    except Exception:  # pragma: no cover
        blas_threads = 1
    n = N ** dim
    rowptr, col, val = build_rows(dim, N, 0, n)
    A = sp.csr_matrix((val, col.astype(np.int32), rowptr), shape=(n, n))
    r = ref.matlab_rand(n)
    q = r / math.sqrt(r @ r)
    Bk, _, _ = ref.newton_change_of_basis(A, q, s)
    t0 = time.perf_counter()
    ref.ca_lanczos_basic(A, q, Bk, iters, s, "newton", "local", diagnostics=False)
    dt = time.perf_counter() - t0
    return {"value": iters / dt, "unit": "outer-iters/s", "cores": int(blas_threads), "kind": "port",
            "sample": "oracle/ca_lanczos_ref.py ca_lanczos_basic, %d outer iterations (k=1..%d, s=%d, "
                      "Newton, 'local', diagnostics off) on the same %s matrix; SciPy CSR SpMV is "
                      "single-threaded, LAPACK QR uses %d threads; %.1f s"
                      % (iters, iters, s, "x".join([str(N)] * dim), blas_threads, dt)}


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dim, N = workload_dims(args.workload)
    n = N ** dim
    s = args.s
    plane = N ** (dim - 1)

    import ca_lanczos_amd as cal
    from ca_lanczos_amd.matrices import slab_bounds

    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("gloo", init_method="env://")

    ndev = ctypes.c_int(0)
    cal._lib.lib.cal_device_count(ctypes.byref(ndev))
    ctx = cal.Context(device=local % max(ndev.value, 1))
    bounds = slab_bounds(n, world, plane)
    r0, r1 = bounds[rank], bounds[rank + 1]
    rowptr, col, val = build_rows(dim, N, r0, r1)
    nnz_local = int(rowptr[-1])
    r_full = np.random.RandomState(5489).random_sample(n)  # MATLAB rand(n,1), fresh session
    if world > 1 and args.comm == "host":
        import torch

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
            for q in reqs:
                q.wait()
            if recv.size:
                recv[:] = rt.numpy()

        ctx.comm_init_host(world, rank, allreduce, exchange)
    elif world > 1:
        import torch
        uid = bytearray(128)
        if rank == 0:
            buf = ctypes.create_string_buffer(128)
            cal._lib.check(None, cal._lib.lib.cal_comm_unique_id(buf))
            uid = bytearray(buf.raw)
        t = torch.tensor(list(uid), dtype=torch.uint8)
        dist.broadcast(t, 0)
        ctx.comm_init_rccl(world, rank, bytes(t.tolist()))
    if world > 1:
        import scipy.sparse as sp
        Aloc = sp.csr_matrix((val, col, rowptr), shape=(r1 - r0, n))
        ctx.set_matrix_slab(n, r0, Aloc)
    else:
        import scipy.sparse as sp
        ctx.set_matrix(sp.csr_matrix((val, col.astype(np.int32), rowptr), shape=(n, n)))
    del rowptr, col, val
    nnz_total = nnz_local
    if dist is not None:
        import torch
        tt = torch.tensor([float(nnz_local)], dtype=torch.float64)
        dist.all_reduce(tt)
        nnz_total = int(tt.item())

    K, W = args.steps, args.warmup
    # K timed steps run without per-kernel events (an event pair around each
    # launch adds ~6 us per kernel boundary); KT more steps then run with the
    # HIP-event kernel timers for the per-kernel figures and the roofline.
    KT = max(1, min(K, 5))
    ctx.lanczos_begin(r_full[r0:r1], s, W + K + KT, args.basis, args.orth)
    for _ in range(W):
        ctx.lanczos_step(False)
    ctx.synchronize()
    if dist is not None:
        dist.barrier()
    ctx.synchronize()
    t0 = time.perf_counter()
    for _ in range(K):
        ctx.lanczos_step(False)
    ctx.synchronize()
    t1 = time.perf_counter()
    if dist is not None:
        dist.barrier()
    elapsed = t1 - t0
    ctx.timer_enable(True)
    ctx.timer_reset()
    for _ in range(KT):
        ctx.lanczos_step(False)
    ctx.synchronize()
    spmv_cnt, spmv_ms = ctx.timer_read("spmv")
    gram_cnt, gram_ms = ctx.timer_read("gram")
    apply_cnt, apply_ms = ctx.timer_read("apply")
    ctx.timer_enable(False)
    T, _, _, flags, info = ctx.lanczos_get()
    if dist is not None:
        import torch
        tt = torch.tensor([elapsed, spmv_ms / max(spmv_cnt, 1)], dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed, spmv_avg_ms = float(tt[0]), float(tt[1])
    else:
        spmv_avg_ms = spmv_ms / max(spmv_cnt, 1)

    fmt, npat, nent = ctx.spmv_format()
    npairpat, npent, nsplit = ctx.spmv_pair_info()
    apply_avg_ms = apply_ms / max(apply_cnt, 1)
    gram_avg_ms = gram_ms / max(gram_cnt, 1)
    csr_spmv = None
    host_rt_ms = None
    if world == 1 and rank == 0:
        # the same SpMV in plain CSR (12 B/nonzero), device-resident, for reference
        ctx2 = cal.Context(device=local, spmv_format="csr")
        import scipy.sparse as sp
        rp2, col2, val2 = build_rows(dim, N, 0, n)
        ctx2.set_matrix(sp.csr_matrix((val2, col2.astype(np.int32), rp2), shape=(n, n)))
        del rp2, col2, val2
        csr_spmv = ctx2.bench_spmv(20, 1.0)
        ctx2.close()
        # tier-1 host-pointer SpMV (MATLAB-boundary semantics: PCIe in and out)
        v = np.ones(n)
        ctx.spmv(v)
        t_h = time.perf_counter()
        for _ in range(3):
            ctx.spmv(v)
        host_rt_ms = (time.perf_counter() - t_h) / 3 * 1e3
        del v
    if rank != 0:
        dist.barrier()
        return

    n_loc = r1 - r0
    # per-launch algorithmic bytes:
    #   SpMV CSR: 12 nnz + 20 n + 4; row-pattern: 2 n (ids) + 8 n (x) + 8 n (y);
    #   apply (pass B, chained): (w + m) * 8 read + m * 8 written per row (w = s+1, m = s)
    #   Gram sweeps (P1 and pass A): (w + m) * 8 read per row
    b_csr = 12 * nnz_local + 20 * n_loc + 4
    #   pair patterns: 1 B of id per row (one 2-B id per row pair)
    b_spmv_launch = (17 if npairpat else 18) * n_loc if fmt == "pattern" else b_csr
    b_apply = (2 * s + 1 + s) * 8 * n_loc
    b_gram = (2 * s + 1) * 8 * n_loc
    spmv_gbps = b_spmv_launch / (spmv_avg_ms * 1e-3) / 1e9
    per_step = {"spmv": spmv_ms / KT, "gram": gram_ms / KT, "apply": apply_ms / KT}
    dominant = max(per_step, key=per_step.get)
    dom = {"spmv": (b_spmv_launch, spmv_avg_ms, ("k_spmv_pair (row-pattern SpMV, two rows per lane, + Newton shift)"
                                                 if npairpat else "k_spmv_pat_lds (row-pattern SpMV + Newton shift)")
                    if fmt == "pattern" else "k_spmv (CSR-stream SpMV + Newton shift)"),
           "gram": (b_gram, gram_avg_ms, "k_rowapply Gram sweeps ([Qp|X]'X and pass A, MFMA tile Gram, no store)"),
           "apply": (b_apply, apply_avg_ms, "k_rowapply<17,8,chained> (block orthogonalisation pass B)")}[dominant]
    achieved = dom[0] / (dom[1] * 1e-3) / 1e9
    traffic = None
    if os.path.exists(args.traffic_json):
        try:
            tj = json.load(open(args.traffic_json))
            if tj.get("workload") == args.workload and tj.get("n_gpus", 1) == world:
                traffic = tj.get("classes", {}).get(dominant)
        except Exception:
            traffic = None
    n_reorth = int(np.sum(flags[W:W + K]))
    b_outer = s * (12 * nnz_total + 20 * n + 4) + 8 * n * (5 * s + 2)
    line = {
        "metric": "CA-Lanczos outer-iters/sec (n~10M, s=8)",
        "value": K / elapsed,
        "unit": "outer-iters/s",
        "n_gpus": world,
        "steps": K,
        "warmup": W,
        "ms_per_step": 1e3 * elapsed / K,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (7-pt Dirichlet Laplacian, r = MATLAB rand(n,1) seed 5489)" if dim == 3 else
                "synthetic (5-pt Dirichlet Laplacian, r = MATLAB rand(n,1) seed 5489)",
        "config": {"workload": "%s: %s %dx..., n=%d, nnz=%d" % (args.workload, "7-pt 3-D" if dim == 3 else "5-pt 2-D",
                                                                N, n, nnz_total),
                   "s": s, "basis": args.basis, "orth": args.orth, "parallelism": "row-slab x%d" % world,
                   "comm": (args.comm if world > 1 else "none")},
        "spmv_format": ("%s (%d row patterns, %d entries; %d pair patterns, %d entries, %d split pairs)"
                        % (fmt, npat, nent, npairpat, npent, nsplit)) if fmt == "pattern" else fmt,
        "spmv_gbps": spmv_gbps,
        "spmv_avg_us": spmv_avg_ms * 1e3,
        "spmv_csr_equiv_gbps": b_csr / (spmv_avg_ms * 1e-3) / 1e9,
        "reorth_passes": "%d/%d" % (n_reorth, K),
        "csr_outer_algorithmic_GB": b_outer / 1e9,
        "kernel_ms_per_step": per_step,
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                     "kernel": dom[2], "bytes_per_launch": dom[0], "avg_launch_us": dom[1] * 1e3},
    }
    if csr_spmv is not None:
        line["spmv_csr_kernel"] = {"avg_us": csr_spmv[0] * 1e3, "min_us": csr_spmv[1] * 1e3,
                                   "gbps": b_csr / (csr_spmv[0] * 1e-3) / 1e9, "bytes_per_launch": b_csr}
    if host_rt_ms is not None:
        line["spmv_host_roundtrip_ms"] = host_rt_ms
    if world == 1 and not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline(dim, N, s, args.cpu_iters)
    print(json.dumps(line), flush=True)
    if dist is not None:
        dist.barrier()


if __name__ == "__main__":
    main()
