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


# --------------------------------------------------------------------------
# CA matrix powers with an s-deep ghost zone (comm.cpp cal_set_matrix_csr_dist
# + halo_exchange_deep, runtime.cpp powers_dev): every slab stores the rows of
# its (D-1)-band ghost zone, fetched once from their owners; the s powers of
# an outer iteration need one exchange of q's s-band ghost zone.
# --------------------------------------------------------------------------

class MPKSlab:
    """Rows [r0, r1) plus the ghost-zone rows [elo, ehi) of depth D."""

    def __init__(self, A_rows: sp.csr_matrix, bounds, rank, depth):
        self.rank, self.nranks, self.bounds = rank, len(bounds) - 1, bounds
        self.r0, self.r1 = bounds[rank], bounds[rank + 1]
        self.n = bounds[-1]
        self.D = depth
        rows = A_rows.tocsr()  # only this slab's rows (global columns)
        # global band (all-reduced max of row - col and col - row)
        ri = np.repeat(np.arange(self.r0, self.r1), np.diff(rows.indptr))
        d = rows.indices.astype(np.int64) - ri
        bb = torch.zeros(2 * self.nranks, dtype=torch.float64)
        bb[2 * rank] = float(max(0, -d.min())) if d.size else 0.0
        bb[2 * rank + 1] = float(max(0, d.max())) if d.size else 0.0
        dist.all_reduce(bb)
        self.bl = int(bb[0::2].max())
        self.br = int(bb[1::2].max())
        self.elo, self.ehi = self._ext(rank)
        # fetch the ghost-zone rows from their owners (counts, then rows)
        got = {}
        for q in range(self.nranks):
            if q == rank:
                continue
            nlo, nhi = max(bounds[q], self.elo), min(bounds[q + 1], self.ehi)
            qlo, qhi = self._ext(q)
            glo, ghi = max(self.r0, qlo), min(self.r1, qhi)
            get, give = nhi > nlo, ghi > glo
            if not (get or give):
                continue
            s1 = torch.tensor([float(rows.indptr[ghi - self.r0] - rows.indptr[glo - self.r0])] if give else [],
                              dtype=torch.float64)
            r1 = torch.zeros(1 if get else 0, dtype=torch.float64)
            Slab._exchange(q, s1, r1)
            if give:
                sub = rows[glo - self.r0:ghi - self.r0]
                s2 = torch.from_numpy(np.concatenate([np.diff(sub.indptr).astype(np.float64),
                                                      sub.indices.astype(np.float64), sub.data]))
            else:
                s2 = torch.zeros(0, dtype=torch.float64)
            r2 = torch.zeros((nhi - nlo) + 2 * int(r1[0]) if get else 0, dtype=torch.float64)
            Slab._exchange(q, s2, r2)
            if get:
                nr, nz = nhi - nlo, int(r1[0])
                lens = r2[:nr].numpy().astype(np.int64)
                ip = np.concatenate([[0], np.cumsum(lens)])
                got[(nlo, nhi)] = sp.csr_matrix((r2[nr + nz:].numpy(), r2[nr:nr + nz].numpy().astype(np.int64), ip),
                                                shape=(nr, self.n))
        pieces = [got[k] for k in sorted(got) if k[0] < self.r0] + [rows] + \
                 [got[k] for k in sorted(got) if k[0] >= self.r1]
        ext = sp.vstack(pieces).tocsr()
        assert ext.shape[0] == self.ehi - self.elo
        # window: global rows [wlo, whi) of every vector
        self.wlo = max(0, self.r0 - self.D * self.bl)
        self.whi = min(self.n, self.r1 + self.D * self.br)
        self.ext = sp.csr_matrix((ext.data, ext.indices - self.wlo, ext.indptr),
                                 shape=(ext.shape[0], self.whi - self.wlo))

    def _ext(self, q):
        b = self.bounds
        return max(0, b[q] - (self.D - 1) * self.bl), min(self.n, b[q + 1] + (self.D - 1) * self.br)

    def deep_halo(self, x_local, d):
        """Window vector with q's d-band ghost zone received (halo_exchange_deep)."""
        w = np.zeros(self.whi - self.wlo)
        w[self.r0 - self.wlo:self.r1 - self.wlo] = x_local
        b = self.bounds
        for q in range(self.nranks):
            if q == self.rank:
                continue
            if q < self.rank:
                rlo, rhi = max(b[q], self.r0 - d * self.bl), min(b[q + 1], self.r0)
                slo, shi = self.r0, min(self.r1, b[q + 1] + d * self.br)
            else:
                rlo, rhi = max(b[q], self.r1), min(b[q + 1], self.r1 + d * self.br)
                slo, shi = max(self.r0, b[q] - d * self.bl), self.r1
            rc, sc = max(0, rhi - rlo), max(0, shi - slo)
            if rc == 0 and sc == 0:
                continue
            recv = torch.zeros(rc, dtype=torch.float64)
            send = torch.from_numpy(np.ascontiguousarray(x_local[slo - self.r0:slo - self.r0 + sc]))
            Slab._exchange(q, send, recv)
            w[rlo - self.wlo:rlo - self.wlo + rc] = recv.numpy()
        return w

    def powers(self, q_local, s, shifts=None):
        """V (local rows x (s+1)) = [q, (A - l_1)q, ...] from one deep exchange:
        power j on rows [r0 - (s-j) bl, r1 + (s-j) br) of the stored ghost zone."""
        assert s <= self.D
        x = self.deep_halo(q_local, s)
        V = [x]
        for j in range(1, s + 1):
            lo = max(self.elo, self.r0 - (s - j) * self.bl)
            hi = min(self.ehi, self.r1 + (s - j) * self.br)
            y = np.zeros_like(x)
            sub = self.ext[lo - self.elo:hi - self.elo]
            y[lo - self.wlo:hi - self.wlo] = sub @ x
            if shifts is not None:
                y[lo - self.wlo:hi - self.wlo] -= shifts[j - 1] * x[lo - self.wlo:hi - self.wlo]
            V.append(y)
            x = y
        return np.stack([v[self.r0 - self.wlo:self.r1 - self.wlo] for v in V], axis=1)

    def split_ok(self, s):
        """Every power keeps a non-empty interior (more than 2s bands per slab)."""
        lo = self.r0 + s * self.bl if self.elo < self.r0 else self.r0
        hi = self.r1 - s * self.br if self.ehi > self.r1 else self.r1
        return lo < hi

    def powers_split(self, q_local, s, shifts=None):
        """The overlapped schedule of runtime.cpp powers_dev: every power's
        interior [r0 + j bl, r1 - j br) is computed before the exchange, from
        a window whose ghost zone is still NaN, then each power's two
        boundary pieces after it.  A NaN in the result would mean the
        interior read a ghost row it does not own yet."""
        assert s <= self.D and self.split_ok(s)
        wl = self.whi - self.wlo
        V = [np.full(wl, np.nan) for _ in range(s + 1)]
        V[0][self.r0 - self.wlo:self.r1 - self.wlo] = q_local
        dep_lo, dep_hi = self.elo < self.r0, self.ehi > self.r1

        def glo(j):
            return max(self.elo, self.r0 - (s - j) * self.bl)

        def ghi(j):
            return min(self.ehi, self.r1 + (s - j) * self.br)

        def ilo(j):
            return self.r0 + j * self.bl if dep_lo else glo(j)

        def ihi(j):
            return self.r1 - j * self.br if dep_hi else ghi(j)

        def run(j, lo, hi):
            if hi <= lo:
                return
            x = V[j - 1]
            y = self.ext[lo - self.elo:hi - self.elo] @ x
            if shifts is not None:
                y = y - shifts[j - 1] * x[lo - self.wlo:hi - self.wlo]
            V[j][lo - self.wlo:hi - self.wlo] = y

        for j in range(1, s + 1):  # interior trapezoid, exchange in flight
            run(j, ilo(j), ihi(j))
        V[0][:] = np.where(np.isnan(V[0]), self.deep_halo(q_local, s), V[0])
        for j in range(1, s + 1):  # boundary pieces after the exchange
            if dep_lo:
                run(j, glo(j), ilo(j))
            if dep_hi:
                run(j, ihi(j), ghi(j))
        return np.stack([v[self.r0 - self.wlo:self.r1 - self.wlo] for v in V], axis=1)
