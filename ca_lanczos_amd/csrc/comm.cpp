// comm.cpp -- RCCL / host-staged communicators, halo plan, distributed matrix.
#include "comm.hpp"

#include <algorithm>
#include <cstring>
#include <map>

namespace cal {

static int nccl_fail(cal_ctx* c, ncclResult_t r, const char* what) {
    return set_error(c, CAL_ERR_COMM, std::string("RCCL error '") + ncclGetErrorString(r) + "' in " + what);
}

#define CAL_NCCL(ctx, expr)                                        \
    do {                                                           \
        ncclResult_t _r = (expr);                                  \
        if (_r != ncclSuccess) return nccl_fail((ctx), _r, #expr); \
    } while (0)

static int ensure_stage(cal_ctx* c, size_t doubles) {
    Comm* m = c->comm;
    if (doubles <= m->stage_cap) return 0;
    if (m->h_stage) CAL_HIP(c, hipHostFree(m->h_stage));
    m->h_stage = nullptr;
    const size_t n = std::max(doubles, (size_t)65536);
    CAL_HIP(c, hipHostMalloc((void**)&m->h_stage, n * sizeof(double), hipHostMallocDefault));
    m->stage_cap = n;
    return 0;
}

void comm_destroy(cal_ctx* c) {
    if (!c->comm) return;
    Comm* m = c->comm;
    if (m->stream) hipStreamSynchronize(m->stream);
    if (m->nccl) ncclCommDestroy(m->nccl);
    if (m->h_stage) hipHostFree(m->h_stage);
    if (m->ev_q) hipEventDestroy(m->ev_q);
    if (m->ev_halo) hipEventDestroy(m->ev_halo);
    if (m->stream) hipStreamDestroy(m->stream);
    delete c->comm;
    c->comm = nullptr;
}

int allreduce_sum(cal_ctx* c, double* d_buf, int64_t count) {
    Comm* m = c->comm;
    if (!m || m->nranks <= 1 || count <= 0) return 0;
    m->n_allreduce++;
    m->d_allreduce += count;
    if (m->kind == 1) {
        const int t = timer_begin(c, 4);
        CAL_NCCL(c, ncclAllReduce(d_buf, d_buf, (size_t)count, ncclDouble, ncclSum, m->nccl, c->stream));
        timer_end(c, t);
        return 0;
    }
    CAL_TRY(ensure_stage(c, count));
    CAL_HIP(c, hipMemcpyAsync(m->h_stage, d_buf, count * sizeof(double), hipMemcpyDeviceToHost, c->stream));
    CAL_HIP(c, hipStreamSynchronize(c->stream));
    if (m->ar(m->user, m->h_stage, count) != 0) return set_error(c, CAL_ERR_COMM, "allreduce callback failed");
    CAL_HIP(c, hipMemcpyAsync(d_buf, m->h_stage, count * sizeof(double), hipMemcpyHostToDevice, c->stream));
    return 0;
}

int allgather(cal_ctx* c, const double* d_send, double* d_recv, int64_t count) {
    Comm* m = c->comm;
    if (!m || m->nranks <= 1) {
        if (count > 0 && d_recv != d_send)
            CAL_HIP(c, hipMemcpyAsync(d_recv, d_send, count * sizeof(double), hipMemcpyDeviceToDevice, c->stream));
        return 0;
    }
    if (count <= 0) return 0;
    if (m->kind == 1) {
        CAL_NCCL(c, ncclAllGather(d_send, d_recv, (size_t)count, ncclDouble, m->nccl, c->stream));
        return 0;
    }
    // host-staged: every rank contributes its block into zeros, then a sum
    // (x + 0 == x: the gather is exact)
    const int64_t tot = count * m->nranks;
    CAL_HIP(c, hipMemsetAsync(d_recv, 0, tot * sizeof(double), c->stream));
    CAL_HIP(c, hipMemcpyAsync(d_recv + count * m->rank, d_send, count * sizeof(double), hipMemcpyDeviceToDevice,
                              c->stream));
    return allreduce_sum(c, d_recv, tot);
}

int halo_exchange(cal_ctx* c, double* x) {
    Comm* m = c->comm;
    DevMatrix& A = c->A;
    if (!m || m->nranks <= 1 || A.peers.empty()) return 0;
    CAL_HIP(c, launch_gather(A.send_buf, x, A.send_idx, A.send_total, c->stream));
    m->n_halo++;
    m->d_halo += A.send_total + A.nghost;
    // each peer's halo lands contiguously at x + recv_off[p] (origin-relative;
    // negative for the left neighbour in the window layout)
    if (m->kind == 1) {
        const int t = timer_begin(c, 5);
        CAL_NCCL(c, ncclGroupStart());
        for (size_t p = 0; p < A.peers.size(); ++p) {
            if (A.send_cnt[p] > 0)
                CAL_NCCL(c, ncclSend(A.send_buf + A.send_off[p], (size_t)A.send_cnt[p], ncclDouble, A.peers[p], m->nccl,
                                     c->stream));
            if (A.recv_cnt[p] > 0)
                CAL_NCCL(c, ncclRecv(x + A.recv_off[p], (size_t)A.recv_cnt[p], ncclDouble, A.peers[p], m->nccl,
                                     c->stream));
        }
        CAL_NCCL(c, ncclGroupEnd());
        timer_end(c, t);
        return 0;
    }
    const size_t need = (size_t)A.send_total + (size_t)A.nghost;
    CAL_TRY(ensure_stage(c, need));
    double* hs = m->h_stage;
    double* hr = m->h_stage + A.send_total;
    CAL_HIP(c, hipMemcpyAsync(hs, A.send_buf, A.send_total * sizeof(double), hipMemcpyDeviceToHost, c->stream));
    CAL_HIP(c, hipStreamSynchronize(c->stream));
    int64_t packed = 0;
    for (size_t p = 0; p < A.peers.size(); ++p) {
        if (m->ex(m->user, A.peers[p], hs + A.send_off[p], A.send_cnt[p], hr + packed, A.recv_cnt[p]) != 0)
            return set_error(c, CAL_ERR_COMM, "exchange callback failed");
        if (A.recv_cnt[p] > 0)
            CAL_HIP(c, hipMemcpyAsync(x + A.recv_off[p], hr + packed, A.recv_cnt[p] * sizeof(double),
                                      hipMemcpyHostToDevice, c->stream));
        packed += A.recv_cnt[p];
    }
    CAL_HIP(c, hipStreamSynchronize(c->stream));  // hr is reused by the next exchange
    return 0;
}

// The d-deep ghost zone of x for the CA matrix powers (window layout): from
// each rank q < me the rows [max(st[q], row0 - d bl), min(st[q+1], row0)),
// from each q > me [max(st[q], row1), min(st[q+1], row1 + d br)); every piece
// is a contiguous run of the column on both sides, so RCCL sends and
// receives in place (no pack kernel).  Peers ascending on every rank.
int halo_exchange_deep(cal_ctx* c, double* x, int d, hipStream_t hs_st) {
    Comm* m = c->comm;
    DevMatrix& A = c->A;
    if (!m || m->nranks <= 1) return 0;
    const std::vector<int64_t>& st = A.slabs;
    const int64_t row0 = A.row0, row1 = A.row0 + A.n_local;
    const int64_t dl = (int64_t)d * A.band_l, dr = (int64_t)d * A.band_r;
    struct Piece {
        int peer;
        int64_t s_off, s_cnt, r_off, r_cnt;  // relative to the local origin
    };
    std::vector<Piece> pieces;
    int64_t stot = 0, rtot = 0;
    for (int q = 0; q < m->nranks; ++q) {
        if (q == m->rank) continue;
        int64_t rlo, rhi, slo, shi;
        if (q < m->rank) {
            rlo = std::max(st[q], row0 - dl);
            rhi = std::min(st[q + 1], row0);
            slo = row0;
            shi = std::min(row1, st[q + 1] + dr);
        } else {
            rlo = std::max(st[q], row1);
            rhi = std::min(st[q + 1], row1 + dr);
            slo = std::max(row0, st[q] - dl);
            shi = row1;
        }
        const int64_t rc = std::max<int64_t>(0, rhi - rlo), sc = std::max<int64_t>(0, shi - slo);
        if (rc == 0 && sc == 0) continue;
        pieces.push_back({q, slo - row0, sc, rlo - row0, rc});
        stot += sc;
        rtot += rc;
    }
    if (pieces.empty()) return 0;
    m->n_halo++;
    m->d_halo += stot + rtot;
    if (m->kind == 1) {
        const int t = timer_begin_on(c, 5, hs_st);
        CAL_NCCL(c, ncclGroupStart());
        for (const Piece& p : pieces) {
            if (p.s_cnt > 0) CAL_NCCL(c, ncclSend(x + p.s_off, (size_t)p.s_cnt, ncclDouble, p.peer, m->nccl, hs_st));
            if (p.r_cnt > 0) CAL_NCCL(c, ncclRecv(x + p.r_off, (size_t)p.r_cnt, ncclDouble, p.peer, m->nccl, hs_st));
        }
        CAL_NCCL(c, ncclGroupEnd());
        timer_end_on(c, t, hs_st);
        return 0;
    }
    // host-staged: the copies run on hs_st (the compute stream, or the
    // communicator's stream when the exchange overlaps the interior powers;
    // then this runs on the comm thread, runtime.cpp powers_dev)
    CAL_TRY(ensure_stage(c, (size_t)(stot + rtot)));
    double* hs = m->h_stage;
    double* hr = m->h_stage + stot;
    int64_t so = 0;
    for (const Piece& p : pieces) {
        if (p.s_cnt > 0)
            CAL_HIP(c, hipMemcpyAsync(hs + so, x + p.s_off, p.s_cnt * sizeof(double), hipMemcpyDeviceToHost, hs_st));
        so += p.s_cnt;
    }
    CAL_HIP(c, hipStreamSynchronize(hs_st));
    so = 0;
    int64_t ro = 0;
    for (const Piece& p : pieces) {
        if (m->ex(m->user, p.peer, hs + so, p.s_cnt, hr + ro, p.r_cnt) != 0)
            return set_error(c, CAL_ERR_COMM, "exchange callback failed");
        if (p.r_cnt > 0)
            CAL_HIP(c, hipMemcpyAsync(x + p.r_off, hr + ro, p.r_cnt * sizeof(double), hipMemcpyHostToDevice, hs_st));
        so += p.s_cnt;
        ro += p.r_cnt;
    }
    CAL_HIP(c, hipStreamSynchronize(hs_st));
    return 0;
}

int comm_allreduce_host(cal_ctx* c, std::vector<double>& buf) {
    Comm* m = c->comm;
    if (!m || m->nranks <= 1 || buf.empty()) return 0;
    if (m->kind == 2) {
        if (m->ar(m->user, buf.data(), (int64_t)buf.size()) != 0)
            return set_error(c, CAL_ERR_COMM, "allreduce callback failed");
        return 0;
    }
    double* d = nullptr;
    CAL_HIP(c, hipMalloc((void**)&d, buf.size() * sizeof(double)));
    CAL_HIP(c, hipMemcpy(d, buf.data(), buf.size() * sizeof(double), hipMemcpyHostToDevice));
    int s = allreduce_sum(c, d, (int64_t)buf.size());
    if (s == 0) {
        hipStreamSynchronize(c->stream);
        hipMemcpy(buf.data(), d, buf.size() * sizeof(double), hipMemcpyDeviceToHost);
    }
    hipFree(d);
    return s;
}

int comm_exchange_host(cal_ctx* c, int peer, const std::vector<double>& send, std::vector<double>& recv) {
    Comm* m = c->comm;
    if (m->kind == 2) {
        if (m->ex(m->user, peer, send.data(), (int64_t)send.size(), recv.data(), (int64_t)recv.size()) != 0)
            return set_error(c, CAL_ERR_COMM, "exchange callback failed");
        return 0;
    }
    double *ds = nullptr, *dr = nullptr;
    CAL_HIP(c, hipMalloc((void**)&ds, std::max<size_t>(send.size(), 1) * sizeof(double)));
    CAL_HIP(c, hipMalloc((void**)&dr, std::max<size_t>(recv.size(), 1) * sizeof(double)));
    if (!send.empty()) CAL_HIP(c, hipMemcpy(ds, send.data(), send.size() * sizeof(double), hipMemcpyHostToDevice));
    CAL_NCCL(c, ncclGroupStart());
    if (!send.empty()) CAL_NCCL(c, ncclSend(ds, send.size(), ncclDouble, peer, m->nccl, c->stream));
    if (!recv.empty()) CAL_NCCL(c, ncclRecv(dr, recv.size(), ncclDouble, peer, m->nccl, c->stream));
    CAL_NCCL(c, ncclGroupEnd());
    CAL_HIP(c, hipStreamSynchronize(c->stream));
    if (!recv.empty()) CAL_HIP(c, hipMemcpy(recv.data(), dr, recv.size() * sizeof(double), hipMemcpyDeviceToHost));
    hipFree(ds);
    hipFree(dr);
    return 0;
}

}  // namespace cal

using namespace cal;

extern "C" {

int cal_comm_unique_id(void* id128) {
    if (!id128) return CAL_ERR_ARG;
    ncclUniqueId id;
    if (ncclGetUniqueId(&id) != ncclSuccess) return CAL_ERR_COMM;
    memcpy(id128, &id, sizeof(id));
    return 0;
}

// the halo stream (high priority: the exchange's copies / RCCL kernels are
// dispatched between the interior matrix-powers blocks) and its two events
static int comm_make_halo_stream(cal_ctx* c, Comm* m) {
    int lo = 0, hi = 0;
    hipDeviceGetStreamPriorityRange(&lo, &hi);
    if (hipStreamCreateWithPriority(&m->stream, hipStreamNonBlocking, hi) != hipSuccess ||
        hipEventCreateWithFlags(&m->ev_q, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&m->ev_halo, hipEventDisableTiming) != hipSuccess) {
        c->comm = m;
        comm_destroy(c);
        return set_error(c, CAL_ERR_HIP, "halo stream / events");
    }
    return 0;
}

int cal_comm_init_rccl(cal_ctx* c, int nranks, int rank, const void* id128) {
    if (!c || nranks < 1 || rank < 0 || rank >= nranks || !id128) return set_error(c, CAL_ERR_ARG, "bad comm args");
    hipSetDevice(c->device);
    comm_destroy(c);
    Comm* m = new Comm();
    m->nranks = nranks;
    m->rank = rank;
    m->kind = 1;
    ncclUniqueId id;
    memcpy(&id, id128, sizeof(id));
    ncclResult_t r = ncclCommInitRank(&m->nccl, nranks, id, rank);
    if (r != ncclSuccess) {
        delete m;
        return nccl_fail(c, r, "ncclCommInitRank");
    }
    CAL_TRY(comm_make_halo_stream(c, m));
    c->comm = m;
    return 0;
}

int cal_comm_stats(cal_ctx* c, int64_t* stats, int nstats, int reset) {
    if (!c || (nstats > 0 && !stats)) return CAL_ERR_ARG;
    Comm* m = c->comm;
    int64_t v[8] = {m ? m->nranks : 1, m ? m->kind : 0, -1, m ? m->n_allreduce : 0, m ? m->d_allreduce : 0,
                    m ? m->n_halo : 0, m ? m->d_halo : 0, c->stat_spmv_rows};
    if (m && m->kind == 1 && m->nccl) {
        int cnt = 0;
        if (ncclCommCount(m->nccl, &cnt) == ncclSuccess) v[2] = cnt;
    }
    for (int i = 0; i < nstats && i < 8; ++i) stats[i] = v[i];
    if (reset) {
        if (m) m->n_allreduce = m->d_allreduce = m->n_halo = m->d_halo = 0;
        c->stat_spmv_rows = 0;
    }
    return 0;
}

int cal_comm_init_host(cal_ctx* c, int nranks, int rank, cal_allreduce_fn allreduce, cal_exchange_fn exchange,
                       void* user) {
    if (!c || nranks < 1 || rank < 0 || rank >= nranks || !allreduce || !exchange)
        return set_error(c, CAL_ERR_ARG, "bad comm args");
    hipSetDevice(c->device);
    comm_destroy(c);
    Comm* m = new Comm();
    m->nranks = nranks;
    m->rank = rank;
    m->kind = 2;
    m->ar = allreduce;
    m->ex = exchange;
    m->user = user;
    // the same stream / event pair as RCCL: the split matrix-powers schedule
    // runs the host-staged exchange on it from a comm thread (powers_dev)
    CAL_TRY(comm_make_halo_stream(c, m));
    c->comm = m;
    return 0;
}

int cal_comm_info(cal_ctx* c, int* nranks, int* rank, int* kind) {
    if (!c) return CAL_ERR_ARG;
    if (nranks) *nranks = c->comm ? c->comm->nranks : 1;
    if (rank) *rank = c->comm ? c->comm->rank : 0;
    if (kind) *kind = c->comm ? c->comm->kind : 0;
    return 0;
}

// Row slab [row0, row0+nlocal) with global column indices.  Ghost columns are
// numbered n_local.. grouped by owning rank (ascending), ascending global id
// inside a group, so each peer's halo lands contiguously after the local rows.
int cal_set_matrix_csr_dist(cal_ctx* c, int64_t n_global, int64_t row0, int64_t nlocal, const int64_t* rowptr,
                            const int64_t* colind_global, const double* val) {
    if (!c || nlocal < 0 || row0 < 0 || row0 + nlocal > n_global || !rowptr)
        return set_error(c, CAL_ERR_ARG, "cal_set_matrix_csr_dist: bad arguments");
    hipSetDevice(c->device);
    const int nranks = c->comm ? c->comm->nranks : 1;
    const int rank = c->comm ? c->comm->rank : 0;
    // slab starts of every rank
    std::vector<double> starts(nranks + 1, 0.0);
    starts[rank] = (double)row0;
    if (rank == nranks - 1) starts[nranks] = (double)(row0 + nlocal);
    CAL_TRY(comm_allreduce_host(c, starts));
    std::vector<int64_t> st(nranks + 1);
    for (int i = 0; i <= nranks; ++i) st[i] = (int64_t)starts[i];
    if (st[nranks] != n_global) return set_error(c, CAL_ERR_ARG, "slabs do not cover the matrix");
    auto owner = [&](int64_t j) {
        return (int)(std::upper_bound(st.begin(), st.end() - 1, j) - st.begin()) - 1;
    };
    const int64_t nnz = rowptr[nlocal] - rowptr[0];
    if (nnz >= ((int64_t)1 << 31) || nlocal >= ((int64_t)1 << 31))
        return set_error(c, CAL_ERR_UNSUPPORTED, "n and nnz must be < 2^31 per rank");
    // collect ghosts
    std::map<int64_t, int64_t> ghost;  // global -> (owner-ordered) index, filled below
    for (int64_t p = 0; p < nnz; ++p) {
        const int64_t j = colind_global[p];
        if (j < 0 || j >= n_global) return set_error(c, CAL_ERR_ARG, "column index out of range");
        if (j < row0 || j >= row0 + nlocal) ghost[j] = 0;
    }
    // std::map iterates in ascending global id == grouped by owner ascending
    std::vector<std::vector<int64_t>> need(nranks);
    int64_t gi = 0;
    for (auto& kv : ghost) {
        kv.second = gi++;
        need[owner(kv.first)].push_back(kv.first);
    }
    const int64_t nghost = gi;
    // Window layout when every peer's halo is a dense run of global ids (row
    // slabs of a stencil matrix): the vector buffer holds global rows
    // [row0 - lext, row0 + nlocal + rext) contiguously, so col - row stays
    // invariant across the slab boundary (row-pattern SpMV keeps working).
    // Otherwise the compact layout [local | ghosts grouped by peer].
    bool window = nghost > 0;
    int64_t lext = 0, rext = 0;
    for (int q = 0; q < nranks && window; ++q) {
        if (need[q].empty()) continue;
        const int64_t lo = need[q].front(), hi = need[q].back();
        window = (hi - lo + 1) == (int64_t)need[q].size();
        if (lo < row0) lext = std::max(lext, row0 - lo);
        if (hi >= row0 + nlocal) rext = std::max(rext, hi - (row0 + nlocal) + 1);
    }
    if (window && lext + rext > 2 * nghost + 1024) window = false;
    if (!window) {
        lext = 0;
        rext = nghost;
    }
    std::vector<int> rp(nlocal + 1), col(nnz);
    for (int64_t i = 0; i <= nlocal; ++i) rp[i] = (int)(rowptr[i] - rowptr[0]);
    for (int64_t p = 0; p < nnz; ++p) {
        const int64_t j = colind_global[p];
        const bool local = j >= row0 && j < row0 + nlocal;
        col[p] = (local || window) ? (int)(j - row0) : (int)(nlocal + ghost[j]);
    }
    // ---- CA matrix-powers ghost zone -----------------------
    // Agreed by all ranks: the global band (bl, br) and whether every slab
    // has the window layout; the kernel runs when they do, depth D > 1 and
    // the row-pattern format is not excluded.
    const int D = c->mpk_depth_req;
    int64_t bl = 0, br = 0;
    bool all_window = window;
    {
        int64_t lbl = 0, lbr = 0;
        for (int64_t i = 0; i < nlocal; ++i)
            for (int64_t p = rowptr[i] - rowptr[0]; p < rowptr[i + 1] - rowptr[0]; ++p) {
                const int64_t d = colind_global[p] - (row0 + i);
                lbl = std::max(lbl, -d);
                lbr = std::max(lbr, d);
            }
        std::vector<double> bb((size_t)3 * nranks, 0.0);
        bb[(size_t)3 * rank] = (double)lbl;
        bb[(size_t)3 * rank + 1] = (double)lbr;
        bb[(size_t)3 * rank + 2] = window ? 0.0 : 1.0;
        CAL_TRY(comm_allreduce_host(c, bb));
        for (int q = 0; q < nranks; ++q) {
            bl = std::max(bl, (int64_t)bb[(size_t)3 * q]);
            br = std::max(br, (int64_t)bb[(size_t)3 * q + 1]);
            if (bb[(size_t)3 * q + 2] != 0.0) all_window = false;
        }
    }
    const bool mpk = all_window && nranks > 1 && D > 1 && c->spmv_format != 1 && (bl > 0 || br > 0);
    auto ext_of = [&](int q, int64_t* lo, int64_t* hi) {
        *lo = std::max<int64_t>(0, st[q] - (int64_t)(D - 1) * bl);
        *hi = std::min<int64_t>(n_global, st[q + 1] + (int64_t)(D - 1) * br);
    };
    std::vector<int> xrp, xcol;
    std::vector<double> xval;
    int64_t elo = row0, ehi = row0 + nlocal, ext_off = 0;
    int dummy = 0;
    if (mpk) {
        ext_of(rank, &elo, &ehi);
        // rows of the ghost zone, fetched from their owners (ascending peers,
        // counts then rows: lengths, global columns, values)
        std::map<int64_t, std::pair<std::vector<int64_t>, std::vector<double>>> ghost_rows;
        for (int q = 0; q < nranks; ++q) {
            if (q == rank) continue;
            const int64_t nlo = std::max(st[q], elo), nhi = std::min(st[q + 1], ehi);
            int64_t qlo, qhi;
            ext_of(q, &qlo, &qhi);
            const int64_t glo = std::max(row0, qlo), ghi = std::min(row0 + nlocal, qhi);
            const bool get = nhi > nlo, give = ghi > glo;
            if (!get && !give) continue;
            std::vector<double> s1, r1(get ? 1 : 0);
            if (give) s1.push_back((double)(rowptr[ghi - row0] - rowptr[glo - row0]));
            CAL_TRY(comm_exchange_host(c, q, s1, r1));
            std::vector<double> s2, r2;
            if (give) {
                const int64_t p0 = rowptr[glo - row0] - rowptr[0], p1 = rowptr[ghi - row0] - rowptr[0];
                for (int64_t i = glo; i < ghi; ++i) s2.push_back((double)(rowptr[i - row0 + 1] - rowptr[i - row0]));
                for (int64_t p = p0; p < p1; ++p) s2.push_back((double)colind_global[p]);
                for (int64_t p = p0; p < p1; ++p) s2.push_back(val[rowptr[0] + p]);
            }
            if (get) r2.resize((size_t)(nhi - nlo) + 2 * (size_t)r1[0]);
            CAL_TRY(comm_exchange_host(c, q, s2, r2));
            if (get) {
                const int64_t nr = nhi - nlo, nz = (int64_t)r1[0];
                int64_t pc = nr, pv = nr + nz;
                for (int64_t i = 0; i < nr; ++i) {
                    const int64_t len = (int64_t)r2[(size_t)i];
                    auto& row = ghost_rows[nlo + i];
                    for (int64_t e = 0; e < len; ++e) {
                        row.first.push_back((int64_t)r2[(size_t)(pc++)]);
                        row.second.push_back(r2[(size_t)(pv++)]);
                    }
                }
            }
        }
        // stored rows: [dummy] [elo, row0) [local] [row1, ehi); ext_off even
        dummy = ((row0 - elo) & 1) ? 1 : 0;
        ext_off = (row0 - elo) + dummy;
        const int64_t n_rows = dummy + (ehi - elo);
        xrp.assign(1, 0);
        if (dummy) xrp.push_back(0);
        auto push_ghost = [&](int64_t g) -> bool {
            auto it = ghost_rows.find(g);
            if (it == ghost_rows.end()) return false;
            for (size_t e = 0; e < it->second.first.size(); ++e) {
                xcol.push_back((int)(it->second.first[e] - row0));
                xval.push_back(it->second.second[e]);
            }
            xrp.push_back((int)xcol.size());
            return true;
        };
        bool okrows = true;
        for (int64_t g = elo; g < row0 && okrows; ++g) okrows = push_ghost(g);
        for (int64_t i = 0; i < nlocal && okrows; ++i) {
            for (int64_t p = rowptr[i] - rowptr[0]; p < rowptr[i + 1] - rowptr[0]; ++p) {
                xcol.push_back((int)(colind_global[p] - row0));
                xval.push_back(val[rowptr[0] + p]);
            }
            xrp.push_back((int)xcol.size());
        }
        for (int64_t g = row0 + nlocal; g < ehi && okrows; ++g) okrows = push_ghost(g);
        if (!okrows || (int64_t)xrp.size() != n_rows + 1 || xcol.size() >= ((size_t)1 << 31))
            return set_error(c, CAL_ERR_COMM, "mpk: ghost-zone rows incomplete");
        // vector window: D bands each side (deep exchange) + the edge rows'
        // reads one band beyond the stored rows
        const int64_t lw = std::max(lext, (int64_t)D * bl + 2), rw = std::max(rext, (int64_t)D * br + 2);
        CAL_TRY(upload_matrix(c, n_rows, ext_off, nlocal, n_global, row0, nghost, lw, rw, xrp, xcol, xval.data()));
        if (!c->A.use_pat) {  // no row-pattern format: plain slab, one exchange per SpMV
            CAL_TRY(upload_matrix(c, nlocal, 0, nlocal, n_global, row0, nghost, lext, rext, rp, col,
                                  val + rowptr[0]));
        } else {
            DevMatrix& A = c->A;
            A.mpk = true;
            A.mpk_depth = D;
            A.ext_lo = elo;
            A.ext_hi = ehi;
            A.ext_dummy = dummy;
        }
    } else {
        CAL_TRY(upload_matrix(c, nlocal, 0, nlocal, n_global, row0, nghost, lext, rext, rp, col, val + rowptr[0]));
    }
    c->A.band_l = bl;
    c->A.band_r = br;
    c->A.slabs = st;
    // counts matrix: cnt[p*nranks+q] = #entries rank p needs from rank q
    std::vector<double> cnt((size_t)nranks * nranks, 0.0);
    for (int q = 0; q < nranks; ++q) cnt[(size_t)rank * nranks + q] = (double)need[q].size();
    CAL_TRY(comm_allreduce_host(c, cnt));
    DevMatrix& A = c->A;
    int64_t roff = 0, soff = 0;
    std::vector<int> send_idx;
    for (int q = 0; q < nranks; ++q) {
        if (q == rank) continue;
        const int64_t nrecv = (int64_t)cnt[(size_t)rank * nranks + q];
        const int64_t nsend = (int64_t)cnt[(size_t)q * nranks + rank];
        if (nrecv == 0 && nsend == 0) continue;
        // tell q which of its rows we need; learn which of ours q needs
        std::vector<double> want(need[q].begin(), need[q].end()), theirs(nsend);
        CAL_TRY(comm_exchange_host(c, q, want, theirs));
        A.peers.push_back(q);
        A.recv_off.push_back(window ? (nrecv ? need[q].front() - row0 : 0) : nlocal + roff);
        A.recv_cnt.push_back(nrecv);
        A.send_off.push_back(soff);
        A.send_cnt.push_back(nsend);
        for (double g : theirs) send_idx.push_back((int)((int64_t)g - row0));
        roff += nrecv;
        soff += nsend;
    }
    A.send_total = soff;
    if (soff > 0) {
        CAL_HIP(c, hipMalloc((void**)&A.send_idx, soff * sizeof(int)));
        CAL_HIP(c, hipMalloc((void**)&A.send_buf, soff * sizeof(double)));
        CAL_HIP(c, hipMemcpy(A.send_idx, send_idx.data(), soff * sizeof(int), hipMemcpyHostToDevice));
    }
    return 0;
}

}  // extern "C"
