"""Row-slab distributed restatement of the CA-Lanczos outer loop (NumPy +
torch.distributed/gloo).  TEST INFRASTRUCTURE ONLY.

It follows the same decomposition the HIP library implements
(ca_lanczos_amd/csrc/comm.cpp, blockorth.cpp, lanczos.cpp) so the N > 1
data flow can be exercised on CPU with world_size >= 2:

* rows are split in contiguous slabs (``slab_bounds``); ghost columns are
  numbered after the local rows, grouped by owning rank, ascending global id;
* one halo exchange (pairwise send/recv) before every SpMV;
* every Gram block is a local partial sum + one sum-allreduce;
* block orthogonalisation = [Qp|X]'X Gram -> CholQR pass A with the
  fused Grams -> pass B (second CGS sweep + CholQR2), as in blockorth.cpp;
* all s x s algebra is replicated on every rank.

The result must equal the single-process oracle (ca_lanczos_ref) to rounding.
"""
from __future__ import annotations

import math

import numpy as np
import scipy.sparse as sp
import torch
import torch.distributed as dist

from . import ca_lanczos_ref as ref


def slab_bounds(n, nranks, plane=1):
    nplanes = n // plane
    return [(plane * (nplanes * r // nranks)) for r in range(nranks)] + [n]


class Slab:
    """Local rows [r0, r1) of A with the halo plan of comm.cpp."""

    def __init__(self, A: sp.csr_matrix, bounds, rank):
        self.rank, self.nranks = rank, len(bounds) - 1
        self.r0, self.r1 = bounds[rank], bounds[rank + 1]
        self.n_local = self.r1 - self.r0
        rows = A[self.r0:self.r1].tocsr()
        cols = rows.indices.astype(np.int64)
        ghost = np.unique(cols[(cols < self.r0) | (cols >= self.r1)])
        owner = np.searchsorted(bounds, ghost, side="right") - 1
        self.ghost, self.owner = ghost, owner
        gmap = {g: self.n_local + i for i, g in enumerate(ghost)}
        loc = np.array([c - self.r0 if self.r0 <= c < self.r1 else gmap[c] for c in cols], dtype=np.int64)
        self.A = sp.csr_matrix((rows.data, loc, rows.indptr), shape=(self.n_local, self.n_local + len(ghost)))
        # who needs what: exchange the wanted global ids with each owner
        cnt = torch.zeros(self.nranks * self.nranks, dtype=torch.float64)
        for q in range(self.nranks):
            cnt[rank * self.nranks + q] = float(np.sum(owner == q))
        dist.all_reduce(cnt)
        cnt = cnt.numpy().reshape(self.nranks, self.nranks)
        self.peers, self.send_idx, self.recv_slices = [], [], []
        off = 0
        for q in range(self.nranks):
            if q == rank:
                continue
            nrecv, nsend = int(cnt[rank, q]), int(cnt[q, rank])
            if nrecv == 0 and nsend == 0:
                continue
            want = torch.from_numpy(ghost[owner == q].astype(np.float64))
            theirs = torch.zeros(nsend, dtype=torch.float64)
            self._exchange(q, want, theirs)
            self.peers.append(q)
            self.send_idx.append(theirs.numpy().astype(np.int64) - self.r0)
            self.recv_slices.append(slice(off, off + nrecv))
            off += nrecv

    @staticmethod
    def _exchange(peer, send, recv):
        reqs = []
        if send.numel():
            reqs.append(dist.isend(send, peer))
        if recv.numel():
            reqs.append(dist.irecv(recv, peer))
        for r in reqs:
            r.wait()

    def halo(self, x_local):
        ghost = np.zeros(len(self.ghost))
        for q, idx, sl in zip(self.peers, self.send_idx, self.recv_slices):
            recv = torch.zeros(sl.stop - sl.start, dtype=torch.float64)
            self._exchange(q, torch.from_numpy(np.ascontiguousarray(x_local[idx])), recv)
            ghost[sl] = recv.numpy()
        return np.concatenate([x_local, ghost])

    def spmv(self, x_local):
        return self.A @ self.halo(x_local)


def allreduce(a):
    t = torch.from_numpy(np.ascontiguousarray(a, dtype=np.float64))
    dist.all_reduce(t)
    return t.numpy()


def _chol(G):
    return np.linalg.cholesky(G).T


def two_pass(Qp, X, C, GZ):
    """blockorth.cpp two_pass: returns Q (local rows), R, Ctot."""
    m = X.shape[1]
    Ra = _chol(GZ)
    Rai = np.linalg.inv(Ra)
    Q1 = (X - Qp @ C) @ Rai if Qp is not None else X @ Rai
    G1 = allreduce(Q1.T @ Q1)
    C3 = allreduce(Qp.T @ Q1) if Qp is not None else None
    Gp = G1 - (C3.T @ C3 if C3 is not None else 0.0)
    Rb = _chol(Gp)
    Q = (Q1 - Qp @ C3) @ np.linalg.inv(Rb) if Qp is not None else Q1 @ np.linalg.inv(Rb)
    R = np.triu(Rb @ Ra)
    Ctot = C3 @ Ra if C3 is not None else None
    return Q, R, Ctot


def ca_lanczos_dist(slab: Slab, r_local, s, iter, basis="newton"):
    """'local' orthogonalisation, diagnostics off; returns T (replicated)."""
    t = int(math.ceil(iter / s))
    rr = allreduce(np.array([r_local @ r_local]))[0]
    q = r_local / math.sqrt(rr)
    if basis == "newton":
        # Newton prologue (lanczos 'fro', 2s steps) with allreduced dots
        nq = math.sqrt(allreduce(np.array([q @ q]))[0])
        Qs = [q / nq]
        alpha, beta = [], []
        for j in range(2 * s):
            w = slab.spmv(Qs[j])
            if j > 0:
                w = w - beta[j - 1] * Qs[j - 1]
            alpha.append(allreduce(np.array([w @ Qs[j]]))[0])
            w = w - alpha[j] * Qs[j]
            beta.append(math.sqrt(allreduce(np.array([w @ w]))[0]))
            qn = w / beta[j]
            Qm = np.stack(Qs, axis=1)
            qn = qn - Qm @ allreduce(Qm.T @ qn)
            Qs.append(qn)
        T0 = np.diag(alpha) + np.diag(beta[:-1], 1) + np.diag(beta[:-1], -1)
        shifts, _ = ref.leja(np.linalg.eigvalsh(T0), "nonmodified")
        Bk = ref.newton_basis_matrix(shifts, s, 1)
    else:
        Bk = np.eye(s + 1)[:, 1:]
    Q = np.zeros((slab.n_local, s * t + 1))
    Q[:, 0] = q
    b = []
    T = np.zeros((s * t + 1, s * t))
    for k in range(1, t + 1):
        qk = Q[:, (k - 1) * s]
        V = np.zeros((slab.n_local, s + 1))
        V[:, 0] = qk
        for i in range(s):
            V[:, i + 1] = slab.spmv(V[:, i]) - (Bk[i, i] if basis == "newton" else 0.0) * V[:, i]
        if k == 1:
            G = allreduce(V.T @ V)
            Qb, Rk, _ = two_pass(None, V, None, G)
            Q[:, : s + 1] = Qb
            T[: s + 1, :s] = ref._rdiv_upper(Rk @ Bk, Rk[:s, :s])
            b.append(T[s, s - 1])
            continue
        Qp = Q[:, (k - 2) * s : (k - 1) * s + 1]
        X = V[:, 1:]
        G1 = allreduce(np.hstack([Qp, X]).T @ X)
        C = G1[: s + 1]
        GZ = G1[s + 1 :] - C.T @ C
        Qn, Rs, Ctot = two_pass(Qp, X, C, GZ)
        Q[:, (k - 1) * s + 1 : k * s + 1] = Qn
        Rkk_s = C + Ctot
        Rk = np.zeros((s + 1, s + 1))
        Rk[0, 0] = 1.0
        Rk[0, 1:] = Rkk_s[s, :s]
        Rk[1:, 1:] = Rs
        R11 = Rk[:s, :s]
        Rkk11 = np.hstack([np.zeros((s, 1)), Rkk_s[:s, : s - 1]])
        rho, rho_t, bk = Rk[s, s], Rk[s - 1, s - 1], Bk[s, s - 1]
        es = np.zeros((s, 1))
        es[-1] = 1.0
        e1 = np.zeros((s, 1))
        e1[0] = 1.0
        Tk = (ref._rdiv_upper(R11 @ Bk[:s, :], R11) + ((bk / rho_t) * Rk[:s, s:s + 1]) @ es.T
              - ref._rdiv_upper(((b[k - 2] * e1) @ es.T) @ Rkk11, R11))
        b.append(bk * (rho / rho_t))
        m0 = s * (k - 1)
        T[m0:m0 + s, m0:m0 + s] = Tk
        T[m0 - 1, m0] = b[k - 2]
        T[m0, m0 - 1] = b[k - 2]
        T[m0 + s, m0 + s - 1] = b[k - 1]
    return T[: s * t, : s * t]
