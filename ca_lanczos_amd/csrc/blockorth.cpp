// blockorth.cpp -- tall-skinny block orthogonalisation on the device.
//
// Reference semantics (projectAndNormalize.m:3-90, project.m:7-58,
// normalize.m:3-36, tsqr.m:7-12) re-designed for HBM traffic:
//  * the projected block Y = X - Qp*(Qp'X) (and the second-pass Z) is never
//    written to HBM: every pass re-forms it on the fly inside k_apply from
//    [Qp | X] with a small coefficient matrix;
//  * in the CA-Lanczos loop tsqr's Householder QR is CholQR2 (two
//    Cholesky-QR passes fused with the second projection), which gives the
//    same unique positive-diagonal R up to rounding and O(eps) orthogonality
//    while kappa(Y) < ~1e7; a failed Cholesky falls back to the device
//    Householder TSQR (tsqr.hip / tsqr_tree.cpp, pn_tsqr below), which the
//    host-pointer calls and normalize = "tsqr" use throughout;
//  * a wide projection whose reorth test does not fire is one projection and
//    one normalize, as in the reference: one Gram and one apply sweep;
//  * the reorthogonalisation test of projectAndNormalize.m:52 is evaluated
//    on norms taken from the same Gram (before: diag X'X; after: diag of
//    X'X - C'C = ||Y_i||^2), so the pass count follows the reference.
#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <cmath>
#include <vector>

#include "cal_internal.hpp"
#include "comm.hpp"
#include "dense.hpp"

namespace cal {

static Panel panel_slice(const Panel& P, int c0, int nc) {
    Panel out = panel();
    int base = 0;
    for (int s = 0; s < P.nseg; ++s) {
        const int lo = std::max(c0, base), hi = std::min(c0 + nc, base + P.ncol[s]);
        if (hi > lo) panel_add(out, P.ptr[s] + (int64_t)(lo - base) * P.ld[s], P.ld[s], hi - lo);
        base += P.ncol[s];
    }
    return out;
}

static PanelOut panel_out_slice(const PanelOut& P, int c0, int nc) {
    PanelOut out{};
    int base = 0;
    for (int s = 0; s < P.nseg; ++s) {
        const int lo = std::max(c0, base), hi = std::min(c0 + nc, base + P.ncol[s]);
        if (hi > lo) {
            out.ptr[out.nseg] = P.ptr[s] + (int64_t)(lo - base) * P.ld[s];
            out.ld[out.nseg] = P.ld[s];
            out.ncol[out.nseg] = hi - lo;
            out.nseg++;
            out.total += hi - lo;
        }
        base += P.ncol[s];
    }
    return out;
}

static Panel panel_concat(const Panel& a, const Panel& b) {
    Panel out = a;
    for (int s = 0; s < b.nseg; ++s) panel_add(out, b.ptr[s], b.ld[s], b.ncol[s]);
    return out;
}

static Panel as_panel(const PanelOut& p) {
    Panel out = panel();
    for (int s = 0; s < p.nseg; ++s) panel_add(out, p.ptr[s], p.ld[s], p.ncol[s]);
    return out;
}

static int stage_small(cal_ctx* c, const double* M, size_t count) {
    CAL_TRY(ensure_small(c, count));
    if (c->small_pending) {
        CAL_HIP(c, hipStreamSynchronize(c->stream));
        c->small_pending = false;
    }
    std::copy(M, M + count, c->h_small);
    CAL_HIP(c, hipMemcpyAsync(c->d_small, c->h_small, count * sizeof(double), hipMemcpyHostToDevice, c->stream));
    c->small_pending = true;
    return 0;
}

static int gram_host16(cal_ctx* c, int64_t n, const Panel& A, const Panel& B, double* out);

// out (wa x wb) = A'B, B in chunks of <= 16 columns (the MFMA Gram's B tile)
int gram_host(cal_ctx* c, int64_t n, const Panel& A, const Panel& B, double* out) {
    const int wa = A.total, wb = B.total;
    if (wb <= 16) return gram_host16(c, n, A, B, out);
    for (int j0 = 0; j0 < wb; j0 += 16) {
        const int nb = std::min(16, wb - j0);
        std::vector<double> t((size_t)wa * nb);
        CAL_TRY(gram_host16(c, n, A, panel_slice(B, j0, nb), t.data()));
        for (int j = 0; j < nb; ++j)
            for (int i = 0; i < wa; ++i) out[i + (size_t)(j0 + j) * wa] = t[i + (size_t)j * wa];
    }
    return 0;
}

static int gram_host16(cal_ctx* c, int64_t n, const Panel& A, const Panel& B, double* out) {
    const int wa = A.total, wb = B.total;
    if (wb > 16 || wb < 1 || wa < 1) return set_error(c, CAL_ERR_ARG, "gram: panel widths out of range");
    if (A.nseg > kMaxSeg || B.nseg > kMaxSeg) return set_error(c, CAL_ERR_ARG, "gram: too many segments");
    struct Chunk {
        int c0, nc, ldc;
        int64_t off;
    };
    std::vector<Chunk> ch;
    int64_t off = 0;
    for (int c0 = 0; c0 < wa; c0 += 128) {
        const int nc = std::min(128, wa - c0);
        const GramPlan pl = gram_plan(nc, wb, n);
        ch.push_back({c0, nc, 16 * pl.nta, off});
        off += pl.entries;
    }
    CAL_TRY(ensure_red(c, off));
    for (auto& k : ch) {
        const Panel As = panel_slice(A, k.c0, k.nc);
        const GramPlan pl = gram_plan(k.nc, wb, n);
        CAL_TRY(ensure_partial(c, (size_t)pl.blocks * pl.entries));
        const int t = timer_begin(c, 1, 8.0 * n * (k.nc + wb));
        CAL_HIP(c, launch_gram(As, B, n, pl, c->d_partial, c->stream));
        timer_end(c, t);
        CAL_HIP_OTHER(c, launch_reduce(c->d_partial, pl.blocks, pl.entries, c->d_red + k.off, c->stream));
    }
    CAL_TRY(allreduce_sum(c, c->d_red, off));
    CAL_HIP_OTHER(c, hipMemcpyAsync(c->h_red, c->d_red, off * sizeof(double), hipMemcpyDeviceToHost, c->stream));
    CAL_HIP(c, hipStreamSynchronize(c->stream));
    c->small_pending = false;
    for (auto& k : ch)
        for (int j = 0; j < wb; ++j)
            for (int i = 0; i < k.nc; ++i) out[(k.c0 + i) + (size_t)j * wa] = c->h_red[k.off + (size_t)j * k.ldc + i];
    return 0;
}

// Y = P * M with M (wp x wy, column-major) already on the device; store only.
int apply_dev(cal_ctx* c, int64_t n, const Panel& P, const double* dM, int wy, const PanelOut& Y) {
    const int wp = P.total;
    const int wpp = (wp + 3) & ~3;
    int max_nty = 8192 / (wpp * 16);
    if (wp < 1 || wy < 1 || max_nty < 1) return set_error(c, CAL_ERR_ARG, "apply: panel shape out of range");
    max_nty = max_nty >= 8 ? 8 : (max_nty >= 4 ? 4 : (max_nty >= 2 ? 2 : 1));
    const int cw_max = std::max(16 * max_nty, apply_rows_max_wy(wp));  // store only
    for (int y0 = 0; y0 < wy; y0 += cw_max) {
        const int cw = std::min(cw_max, wy - y0);
        const ApplyPlan pl = apply_plan(wp, cw, n, false, 0);
        const int t = timer_begin(c, 2, 8.0 * n * (wp + cw));
        CAL_HIP(c, launch_apply(P, dM + (size_t)y0 * wp, wp, cw, panel_out_slice(Y, y0, cw), true, 0, n, pl,
                                c->d_partial, c->stream));
        timer_end(c, t);
    }
    return 0;
}

int apply_host(cal_ctx* c, int64_t n, const Panel& P, const double* M, int wy, const PanelOut* Y, double* gram,
               int wq, double* gramp) {
    const int wp = P.total;
    if (wp < 1 || wy < 1) return set_error(c, CAL_ERR_ARG, "apply: empty panel");
    if ((gram || gramp) && wy > 16) return set_error(c, CAL_ERR_ARG, "apply: fused Gram needs <= 16 columns");
    if (wq > 16) return set_error(c, CAL_ERR_ARG, "apply: fused Psub Gram needs <= 16 columns");
    const int wpp = (wp + 3) & ~3;
    int max_nty = 8192 / (wpp * 16);
    if (max_nty < 1) return set_error(c, CAL_ERR_UNSUPPORTED, "apply: panel wider than 512 columns");
    max_nty = max_nty >= 8 ? 8 : (max_nty >= 4 ? 4 : (max_nty >= 2 ? 2 : 1));
    const bool want = gram || gramp;
    // store-only chunks as wide as the row-parallel apply takes
    const int cw_max = (!want && Y) ? std::max(16 * max_nty, apply_rows_max_wy(wp)) : 16 * max_nty;
    CAL_TRY(stage_small(c, M, (size_t)wp * wy));
    ApplyPlan last{};
    for (int y0 = 0; y0 < wy; y0 += cw_max) {
        const int cw = std::min(cw_max, wy - y0);
        const ApplyPlan pl = apply_plan(wp, cw, n, gram != nullptr, gramp ? wq : 0);
        PanelOut Ys{};
        if (Y) Ys = panel_out_slice(*Y, y0, cw);
        if (want) CAL_TRY(ensure_partial(c, (size_t)pl.blocks * pl.entries));
        const int t = timer_begin(c, 2, 8.0 * n * (wp + (Y ? cw : 0)));
        CAL_HIP(c, launch_apply(P, c->d_small + (size_t)y0 * wp, wp, cw, Ys, Y != nullptr, gramp ? wq : 0, n, pl,
                                c->d_partial, c->stream));
        timer_end(c, t);
        last = pl;
    }
    if (!want) return 0;
    CAL_TRY(ensure_red(c, last.entries));
    CAL_HIP_OTHER(c, launch_reduce(c->d_partial, last.blocks, last.entries, c->d_red, c->stream));
    CAL_TRY(allreduce_sum(c, c->d_red, last.entries));
    CAL_HIP_OTHER(c, hipMemcpyAsync(c->h_red, c->d_red, last.entries * sizeof(double), hipMemcpyDeviceToHost, c->stream));
    CAL_HIP(c, hipStreamSynchronize(c->stream));
    c->small_pending = false;
    int base = 0;
    if (gram) {
        for (int j = 0; j < wy; ++j)
            for (int i = 0; i < wy; ++i) gram[i + (size_t)j * wy] = c->h_red[j * 16 + i];
        base = 256;
    }
    if (gramp)
        for (int j = 0; j < wy; ++j)
            for (int i = 0; i < wq; ++i) gramp[i + (size_t)j * wq] = c->h_red[base + j * 16 + i];
    return 0;
}

// ---- hot-shape paths (s <= 8) ---------------------------------------------
static int fetch_tile(cal_ctx* c, int blocks, double* G16, double* e16) {
    const int64_t nent = 272;
    CAL_TRY(ensure_red(c, nent));
    CAL_HIP_OTHER(c, launch_reduce(c->d_partial, blocks, nent, c->d_red, c->stream));
    CAL_TRY(allreduce_sum(c, c->d_red, nent));
    CAL_HIP_OTHER(c, hipMemcpyAsync(c->h_red, c->d_red, nent * sizeof(double), hipMemcpyDeviceToHost, c->stream));
    CAL_HIP(c, hipStreamSynchronize(c->stream));
    c->small_pending = false;
    std::copy(c->h_red, c->h_red + 256, G16);
    std::copy(c->h_red + 256, c->h_red + 272, e16);
    return 0;
}

// G16 = T'T (T <= 16 columns), e16 = E'T (E one column or null).
static int tilegram_host(cal_ctx* c, int64_t n, const Panel& T, const double* E, double* G16, double* e16) {
    // row-parallel loader (lane <-> row, LDS transpose, one MFMA tile)
    ColList cl{};
    const int nt = T.total;
    for (int cc = 0; cc < 16; ++cc) cl.p[cc] = panel_slice(T, cc < nt ? cc : nt - 1, 1).ptr[0];
    cl.p[16] = E ? E : cl.p[0];
    int64_t blocks = (n + 255) / 256;
    blocks = std::max<int64_t>(1, std::min<int64_t>(blocks, kRowGramBlocks));
    CAL_TRY(ensure_partial(c, (size_t)blocks * 272));
    const int t = timer_begin(c, 1, 8.0 * n * (nt + (E ? 1 : 0)));
    CAL_HIP(c, launch_rowgram(cl, nt, E != nullptr, n, (int)blocks, c->d_partial, c->stream));
    timer_end(c, t);
    return fetch_tile(c, (int)blocks, G16, e16);
}

static bool rowapply_ok(int wp, int m, bool gram, int wq) {
    const int WP = rowapply_wpmax(wp), MO = rowapply_mout(m);
    if (!WP || !MO) return false;
    if (WP == 17 && MO == 16 && gram) return false;
    if (gram && ((wq < 8 ? wq : 8) + m > 16 || wq > 9)) return false;
    return true;
}

// Y = P*M (M wp x m col-major) with the row kernel.  kind (see
// launch_rowapply): 0 store, 1 store + tile Gram of [Qp(0:nq) | Y] (Qp =
// first wq columns of P), 2 the Gram without storing Y, 3 chained: store
// [P(0:wq) | Y] * M2 (M2 (wq+m) x m col-major) with Y = P*M recomputed.
static int rowapply_host(cal_ctx* c, int64_t n, const Panel& P, const double* M, int m, const PanelOut& Y, int kind,
                         int wq, double* G16, double* e16, const double* M2 = nullptr) {
    const bool gram = kind == 1 || kind == 2;
    const int wp = P.total;
    const int WP = rowapply_wpmax(wp), MO = rowapply_mout(m);
    std::vector<double> Mp((size_t)WP * MO * (kind == 3 ? 2 : 1) + (kind == 3 ? (size_t)MO * MO : 0), 0.0);
    for (int cc = 0; cc < wp; ++cc)
        for (int j = 0; j < m; ++j) Mp[(size_t)cc * MO + j] = M[cc + (size_t)j * wp];
    if (kind == 3) {
        double* M2p = Mp.data() + (size_t)WP * MO;
        double* M2y = M2p + (size_t)WP * MO;
        for (int j = 0; j < m; ++j) {
            for (int cc = 0; cc < wq; ++cc) M2p[(size_t)cc * MO + j] = M2[cc + (size_t)j * (wq + m)];
            for (int i = 0; i < m; ++i) M2y[(size_t)i * MO + j] = M2[wq + i + (size_t)j * (wq + m)];
        }
    }
    CAL_TRY(stage_small(c, Mp.data(), Mp.size()));
    ColList cl{};
    OutList ol{};
    for (int cc = 0; cc < 17; ++cc) cl.p[cc] = panel_slice(P, cc < wp ? cc : wp - 1, 1).ptr[0];
    for (int j = 0; j < 16; ++j) {
        const PanelOut s1 = panel_out_slice(Y, j < m ? j : 0, 1);
        ol.p[j] = s1.ptr[0];
    }
    int64_t blocks = (n + 255) / 256;  // without the Gram: one row per thread
    if (gram) blocks = std::min<int64_t>(blocks, kRowGramBlocks);
    blocks = std::max<int64_t>(1, blocks);
    if (gram) CAL_TRY(ensure_partial(c, (size_t)blocks * 272));
    // bytes: P read; Y stored except by the Gram-only sweep (kind 2)
    const int t = timer_begin(c, kind == 2 ? 1 : 2, 8.0 * n * (wp + (kind == 2 ? 0 : m)));  // Gram-only sweeps count as "gram"
    CAL_HIP(c, launch_rowapply(cl, c->d_small, wp, m, ol, kind, wq, n, (int)blocks, c->d_partial, c->stream));
    timer_end(c, t);
    if (!gram) return 0;
    return fetch_tile(c, (int)blocks, G16, e16);
}

// ---- small helpers ------------------------------------------------------
static double nan_max(const std::vector<double>& v) {
    double m = NAN;
    for (double x : v)
        if (!std::isnan(x) && (std::isnan(m) || x > m)) m = x;
    return m;
}

static int rank_from_R(int m, const double* R, double tol) {
    std::vector<double> sv(m);
    dense::singular_values(m, R, m, sv.data());
    const double abs_tol = tol * sv[0];
    for (int i = 0; i < m; ++i)
        if (!(sv[i] > abs_tol)) return i;  // normalize.m:19-24 (a non-finite R counts as deficient)
    return m;
}

// Cholesky of G with the shifted-CholQR fallback (Fukaya et al.): returns
// false only if even the shifted matrix is not positive definite.
static bool chol_or_shift(int m, const double* G, int64_t n_glob, double* R, bool* shifted) {
    if (dense::chol_upper(m, G, m, R, m)) return true;
    double tr = 0.0;
    for (int i = 0; i < m; ++i) tr += std::fabs(G[i + (size_t)i * m]);
    const double u = std::ldexp(1.0, -53);
    const double sigma = 11.0 * ((double)m * (double)n_glob + (double)m * (m + 1)) * u * tr;
    std::vector<double> Gs(G, G + (size_t)m * m);
    for (int i = 0; i < m; ++i) Gs[i + (size_t)i * m] += sigma;
    *shifted = true;
    return dense::chol_upper(m, Gs.data(), m, R, m);
}

static int64_t global_rows(cal_ctx* c, int64_t n) { return c->has_A ? std::max(c->A.n_global, n) : n; }

// Two-pass orthonormalisation of the block Z = W*Mz (never stored) against the
// orthonormal block Qp (the first w columns of W; w may be 0):
//   pass A: Q1 = Z Ra^-1, Ra = chol(Z'Z); fused Grams Q1'Q1, Qp'Q1;
//   pass B: Q  = (Q1 - Qp C3) Rb^-1, Rb = chol(Q1'Q1 - C3'C3),
// i.e. CholQR2 inside the block and a second classical Gram-Schmidt pass
// against Qp in the same two sweeps.  Then X = Qp*(RY + Ctot) + Q*R with
// Ctot = C3*Ra and R = Rb*Ra.  On the row kernel Q1 is never stored: pass A
// only accumulates its Grams and pass B recomputes it in registers (kind 3).
// A shifted first Cholesky takes the stored path with one more pass B.
static int two_pass(cal_ctx* c, int64_t n, const Panel& Qp, const Panel& W, const std::vector<double>& Mz, int m,
                    const double* GZ, const PanelOut& Qout, double* R, std::vector<double>& Ctot, bool* shifted) {
    const int w = Qp.total, wp = W.total;
    const int64_t ng = global_rows(c, n);
    std::vector<double> Ra((size_t)m * m), Rai((size_t)m * m), G1((size_t)m * m), C3((size_t)std::max(w, 1) * m, 0.0);
    bool sh = false;
    if (!chol_or_shift(m, GZ, ng, Ra.data(), &sh))
        return set_error(c, CAL_ERR_NUMERIC, "block orthogonalisation: Gram matrix is not positive definite");
    dense::tri_inv_upper(m, Ra.data(), m, Rai.data(), m);
    std::vector<double> M1((size_t)wp * m);
    dense::matmul(wp, m, m, Mz.data(), wp, Rai.data(), m, M1.data(), wp);
    const Panel Q1 = as_panel(Qout);
    const Panel P2 = panel_concat(Qp, Q1);
    const bool fast = rowapply_ok(wp, m, true, w) && rowapply_ok(w + m, m, true, w);
    auto unpack = [&](const double* G16, const double* e16, std::vector<double>& G, std::vector<double>& Cq) {
        const int nq = w < 8 ? w : 8;
        for (int j = 0; j < m; ++j) {
            for (int i = 0; i < m; ++i) G[i + (size_t)j * m] = G16[(nq + i) + (nq + j) * 16];
            for (int i = 0; i < nq; ++i) Cq[i + (size_t)j * w] = G16[i + (nq + j) * 16];
            if (w == 9) Cq[8 + (size_t)j * w] = e16[nq + j];
        }
    };
    // fused Grams of the freshly written block: Q1'Q1 and Qp'Q1
    auto grams = [&](const Panel& P, const std::vector<double>& M, std::vector<double>& G,
                     std::vector<double>& Cq, bool store_only) -> int {
        if (fast) {
            double G16[256], e16[16];
            CAL_TRY(rowapply_host(c, n, P, M.data(), m, Qout, store_only ? 0 : 1, w, G16, e16));
            if (!store_only) unpack(G16, e16, G, Cq);
            return 0;
        }
        if (store_only) return apply_host(c, n, P, M.data(), m, &Qout, nullptr, 0, nullptr);
        if (w == 0) return apply_host(c, n, P, M.data(), m, &Qout, G.data(), 0, nullptr);
        if (w <= 16) return apply_host(c, n, P, M.data(), m, &Qout, G.data(), w, Cq.data());
        CAL_TRY(apply_host(c, n, P, M.data(), m, &Qout, nullptr, 0, nullptr));
        std::vector<double> GG((size_t)(w + m) * m);
        CAL_TRY(gram_host(c, n, P2, Q1, GG.data()));
        for (int j = 0; j < m; ++j) {
            for (int i = 0; i < w; ++i) Cq[i + (size_t)j * w] = GG[i + (size_t)j * (w + m)];
            for (int i = 0; i < m; ++i) G[i + (size_t)j * m] = GG[w + i + (size_t)j * (w + m)];
        }
        return 0;
    };
    // pass-B coefficients from the Grams of Q1: Rb, M2 = [-C3 Rb^-1 ; Rb^-1],
    // Ctot += C3 Racc, Racc = Rb Racc.
    std::vector<double> Racc = Ra, M2((size_t)(w + m) * m);
    Ctot.assign((size_t)w * m, 0.0);
    auto coeffs_b = [&](bool* sh2) -> int {
        std::vector<double> Gp = G1, Rb((size_t)m * m), Rbi((size_t)m * m);
        for (int j = 0; j < m; ++j)
            for (int i = 0; i < m; ++i) {
                double s = 0.0;
                for (int k = 0; k < w; ++k) s += C3[k + (size_t)i * w] * C3[k + (size_t)j * w];
                Gp[i + (size_t)j * m] -= s;
            }
        if (!chol_or_shift(m, Gp.data(), ng, Rb.data(), sh2))
            return set_error(c, CAL_ERR_NUMERIC, "block orthogonalisation: second Cholesky failed");
        dense::tri_inv_upper(m, Rb.data(), m, Rbi.data(), m);
        std::fill(M2.begin(), M2.end(), 0.0);
        for (int j = 0; j < m; ++j) {
            for (int i = 0; i < w; ++i) {
                double s = 0.0;
                for (int k = 0; k <= j; ++k) s += C3[i + (size_t)k * w] * Rbi[k + (size_t)j * m];
                M2[i + (size_t)j * (w + m)] = -s;
            }
            for (int i = 0; i < m; ++i) M2[w + i + (size_t)j * (w + m)] = Rbi[i + (size_t)j * m];
        }
        for (int j = 0; j < m; ++j)
            for (int i = 0; i < w; ++i) {
                double s = 0.0;
                for (int k = 0; k <= j; ++k) s += C3[i + (size_t)k * w] * Racc[k + (size_t)j * m];
                Ctot[i + (size_t)j * w] += s;
            }
        std::vector<double> Rn((size_t)m * m, 0.0);
        dense::matmul(m, m, m, Rb.data(), m, Racc.data(), m, Rn.data(), m);
        for (int j = 0; j < m; ++j)
            for (int i = j + 1; i < m; ++i) Rn[i + (size_t)j * m] = 0.0;
        Racc = Rn;
        return 0;
    };
    if (fast && !sh) {
        double G16[256], e16[16];
        CAL_TRY(rowapply_host(c, n, W, M1.data(), m, Qout, 2, w, G16, e16));  // pass A, Grams only
        unpack(G16, e16, G1, C3);
        bool sh2 = false;
        CAL_TRY(coeffs_b(&sh2));
        CAL_TRY(rowapply_host(c, n, W, M1.data(), m, Qout, 3, w, nullptr, nullptr, M2.data()));  // pass B
        std::copy(Racc.begin(), Racc.end(), R);
        *shifted = *shifted || sh2;
        return 0;
    }
    CAL_TRY(grams(W, M1, G1, C3, false));  // pass A, Q1 stored
    const int passes = sh ? 2 : 1;
    for (int p = 0; p < passes; ++p) {  // pass B
        bool sh2 = false;
        CAL_TRY(coeffs_b(&sh2));
        sh = sh || sh2;
        const bool more = p + 1 < passes;
        CAL_TRY(grams(P2, M2, G1, C3, !more));
    }
    std::copy(Racc.begin(), Racc.end(), R);
    *shifted = *shifted || sh;
    return 0;
}

// ---- device-coefficient path ----------------------------------------------
// The same three sweeps as two_pass (P1 Gram, pass A Grams, chained pass B)
// with the s x s algebra in k_orth_coef, so the whole block is enqueued
// without a host round trip and the host waits once, for R and RY.  Bits are
// identical to the host path.  Returns 1 (nothing usable written to the
// outputs) when a Cholesky failed: the caller then redoes the block on the
// host path, whose fallbacks (direct Y'Y, shifted CholQR) handle it.
static bool orth_device_ok(cal_ctx* c, const Panel& Qp, const Panel& X) {
    const int w = Qp.total, m = X.total, nq = w < 8 ? w : 8;
    return c->orth_coef_device && m >= 1 && w <= 9 && nq + m <= 16 && Qp.nseg + X.nseg <= kMaxSeg &&
           rowapply_ok(w + m, m, true, w);
}

// Spin on the published sequence word.  No HIP call in the fast path: a
// stream query would enqueue a marker behind the prefetched matrix powers and
// stall the next dispatch.  After 2 s without the word, synchronise the stream
// (a faulted kernel reports here) and look once more.
static int wait_published(cal_ctx* c, const unsigned long long* h_seq, unsigned long long seq) {
    const auto t0 = std::chrono::steady_clock::now();
    for (uint64_t spin = 1;; ++spin) {
        if (__atomic_load_n(h_seq, __ATOMIC_ACQUIRE) == seq) return 0;
        if ((spin & 4095) == 0 && std::chrono::steady_clock::now() - t0 > std::chrono::seconds(2)) {
            CAL_HIP(c, hipStreamSynchronize(c->stream));
            if (__atomic_load_n(h_seq, __ATOMIC_ACQUIRE) == seq) return 0;
            return set_error(c, CAL_ERR_HIP, "block orthogonalisation: result never published");
        }
        __builtin_ia32_pause();
    }
}

// p1_blocks > 0 (Qp empty): P1's partials (X'X, the rowgram tile layout) were
// already written to d_partial by that many blocks of the kernel that formed X
// (k_apply_stage<..., 2>, the last block-MGS step): P1 is not launched.
static int orth_device(cal_ctx* c, int64_t n, const Panel& Qp, const Panel& X, bool doreorth, const PanelOut& Qout,
                       double* Rq, double* R, bool* reorth, int p1_blocks = 0) {
    const int w = Qp.total, m = X.total, nq = w < 8 ? w : 8, wp = w + m;
    const int WP = rowapply_wpmax(wp), MO = rowapply_mout(m);
    const Panel W = panel_concat(Qp, X);
    CAL_TRY(ensure_red(c, 4096));
    double* d_tile = c->d_red;
    double* d_st = c->d_red + 1024;
    double* d_mbuf = c->d_red + 2048;
    double* d_out = c->d_red + 3072;
#ifdef CAL_TEST_HOOKS
    // the test build poisons this block's coefficient scratch: whatever the
    // sweeps read that the coefficient steps did not write is NaN
    CAL_HIP(c, hipMemsetAsync(c->d_red, 0xFF, 4096 * sizeof(double), c->stream));
#endif
    // pass B stores only if neither Cholesky failed (out flags [512], [513]):
    // on a failure the host redoes the block from X, and X may share storage
    // with Qout (ca_lanczos.m:176, q = Q(:,1) in the first block)
    const double* gate = test_switch("CAL_TEST_NO_PASSB_GATE") ? nullptr : d_out + 512;
    // sweeps the Infinity Cache holds (17 columns in <= 160 MB: config 2's
    // n = 1e6) run on half the grid: lap2d_1000 6050-6225 -> 6216-6334
    // outer-it/s, while lap3d_215 loses 0.8 % with 512 blocks and the IRL
    // (n = 1.58 M) is unchanged (same-box A/B, profiles/r05/rg/)
    const int64_t rg_cap = (int64_t)n * 8 * 17 <= ((int64_t)160 << 20) ? kRowGramBlocks / 2 : kRowGramBlocks;
    int64_t blocks = std::max<int64_t>(1, std::min<int64_t>((n + 255) / 256, rg_cap));
    CAL_TRY(ensure_partial(c, (size_t)blocks * 272));
    // P1: [Qp(0:nq) | X]' X (+ Qp column 8 as the extra column)
    ColList ct{};
    if (p1_blocks > 0 && w == 0) {
        // formed with X
    } else {
        p1_blocks = 0;
        const Panel T = panel_concat(panel_slice(W, 0, nq), X);
        const int nt = T.total;
        for (int cc = 0; cc < 16; ++cc) ct.p[cc] = panel_slice(T, cc < nt ? cc : nt - 1, 1).ptr[0];
        ct.p[16] = w == 9 ? panel_slice(Qp, 8, 1).ptr[0] : ct.p[0];
        const int t = timer_begin(c, 1, 8.0 * n * (nt + (w == 9 ? 1 : 0)));
        CAL_HIP(c, launch_rowgram(ct, nt, w == 9, n, (int)blocks, c->d_partial, c->stream));
        timer_end(c, t);
    }
    CAL_TRY(ensure_pub(c));
    const unsigned long long seq = ++c->pub_seq;
    double* h_out = c->h_pub;
    unsigned long long* h_seq = reinterpret_cast<unsigned long long*>(c->h_pub + 516);
    unsigned long long* d_seq = reinterpret_cast<unsigned long long*>(c->d_pub + 516);
    // reduce the Gram partials, all-reduce the tile over the ranks, then the
    // s x s algebra; phase 1 publishes R / RY / flags to h_out
    auto coef = [&](int phase, int dore) -> int {
        const int np = phase == 0 && p1_blocks > 0 ? p1_blocks : (int)blocks;
        CAL_HIP_OTHER(c, launch_reduce(c->d_partial, np, 272, d_tile, c->stream));
        CAL_TRY(allreduce_sum(c, d_tile, 272));
        CAL_HIP_OTHER(c, launch_orth_coef(phase, d_tile, d_st, d_mbuf, d_out, w, m, WP, MO, dore,
                                    phase == 1 ? c->d_pub : nullptr, d_seq, seq, c->stream));
        return 0;
    };
    CAL_TRY(coef(0, doreorth ? 1 : 0));
    ColList cw{};
    OutList ol{};
    for (int cc = 0; cc < 17; ++cc) cw.p[cc] = panel_slice(W, cc < wp ? cc : wp - 1, 1).ptr[0];
    for (int j = 0; j < 16; ++j) ol.p[j] = panel_out_slice(Qout, j < m ? j : 0, 1).ptr[0];
    // pass A: Grams of Q1 = W M1, nothing stored
    {
        const int t = timer_begin(c, 1, 8.0 * n * wp);
        CAL_HIP(c, launch_rowapply(cw, d_mbuf, wp, m, ol, 2, w, n, (int)blocks, c->d_partial, c->stream));
        timer_end(c, t);
    }
    CAL_TRY(coef(1, 0));
    // pass B: Q = [Qp | W M1] M2, one store -- with the 'full' projection's
    // Gram [Qp | Q | Qold]' Q when the caller asked for it (k_passb_wide)
    const bool pbw = c->pbw.want && w == 9 && m == 8 && WP == 17 && MO == 8 &&
                     passb_wide_tiles(c->pbw.qold.total) <= kPassbWideMaxTiles && Qp.nseg == 1 &&
                     c->pbw.qold.nseg <= 1;
    c->pbw.want = false;
    c->pbw.ready = false;
    if (pbw) {
        const int ntw = passb_wide_tiles(c->pbw.qold.total);
        const size_t ent = (size_t)128 * ntw;
        const int pblocks = (int)std::max<int64_t>(1, std::min<int64_t>((n + 255) / 256, kRowGramBlocks));
        CAL_TRY(ensure_partial(c, (size_t)pblocks * ent));
        if (ent > c->pbw.cap) {  // (1536 doubles at most: sized for the widest at once)
            if (c->pbw.d) CAL_HIP(c, hipFree(c->pbw.d));
            if (c->pbw.h) CAL_HIP(c, hipHostFree(c->pbw.h));
            c->pbw.d = c->pbw.h = nullptr;
            c->pbw.cap = 0;
            const size_t cap = (size_t)128 * kPassbWideMaxTiles;
            CAL_HIP(c, scratch_malloc((void**)&c->pbw.d, cap * sizeof(double)));
            CAL_HIP(c, hipHostMalloc((void**)&c->pbw.h, cap * sizeof(double), hipHostMallocDefault));
            c->pbw.cap = cap;
        }
        if (!c->pbw.ev) CAL_HIP(c, hipEventCreateWithFlags(&c->pbw.ev, hipEventDisableTiming));
        // bytes: pass B's, plus the Qold columns the Gram reads
        const int t = timer_begin(c, 2, 8.0 * n * (wp + m + c->pbw.qold.total));
        CAL_HIP(c, launch_passb_wide(cw, d_mbuf, ol, c->pbw.qold, n, pblocks, c->d_partial, gate, c->stream));
        timer_end(c, t);
        CAL_HIP_OTHER(c, launch_reduce(c->d_partial, pblocks, (int64_t)ent, c->pbw.d, c->stream));
        CAL_TRY(allreduce_sum(c, c->pbw.d, (int64_t)ent));  // the slabs' Grams (every rank takes this branch)
        CAL_HIP_OTHER(c, hipMemcpyAsync(c->pbw.h, c->pbw.d, ent * sizeof(double), hipMemcpyDeviceToHost, c->stream));
        CAL_HIP(c, hipEventRecord(c->pbw.ev, c->stream));
        c->pbw.ntw = ntw;
    } else {
        const int t = timer_begin(c, 2, 8.0 * n * (wp + m));
        CAL_HIP(c, launch_rowapply(cw, d_mbuf, wp, m, ol, 3, w, n, (int)((n + 255) / 256), c->d_partial, c->stream,
                                   gate));
        timer_end(c, t);
    }
    if (c->pre_wait) {  // e.g. the next step's matrix powers (lanczos_step)
        auto hook = std::move(c->pre_wait);
        c->pre_wait = nullptr;
        CAL_TRY(hook());
    }
    // R, RY and the flags arrive in h_out when the phase-1 algebra ends (before
    // pass B): poll the sequence word; if the stream drains without it, the
    // kernels failed -- report the stream's error
    CAL_TRY(wait_published(c, h_seq, seq));
    if (h_out[512] != 0.0 || h_out[513] != 0.0) return 1;  // (pass B and its Gram skipped: pbw stays not ready)
    c->pbw.ready = pbw;
    std::copy(h_out, h_out + (size_t)m * m, R);
    std::copy(h_out + 256, h_out + 256 + (size_t)w * m, Rq);
    *reorth = h_out[514] != 0.0;
    return 0;
}

int normalize_dev(cal_ctx* c, int64_t n, const Panel& X, const PanelOut& Qout, double* R, double tol, int* rank,
                  bool* shifted, int p1_blocks) {
    const int m = X.total;
    if (use_tsqr(c, m, c->tier1)) {  // tsqr.m: Householder TSQR
        CAL_TRY(tsqr_dev(c, n, X, nullptr, m, Qout, R));
        if (shifted) *shifted = false;
        if (rank) *rank = rank_from_R(m, R, tol);
        return 0;
    }
    auto via_tsqr = [&]() -> int {
        CAL_TRY(tsqr_dev(c, n, X, nullptr, m, Qout, R));
        if (shifted) *shifted = false;
        if (rank) *rank = rank_from_R(m, R, tol);
        return 0;
    };
    if (m > 16 && tsqr_ok(m)) return via_tsqr();  // the CholQR kernels take <= 16 columns
    if (m < 1 || m > 16) return set_error(c, CAL_ERR_ARG, "normalize: 1..32 columns supported");
    if (orth_device_ok(c, panel(), X)) {
        bool ro = false;
        const int st = orth_device(c, n, panel(), X, false, Qout, nullptr, R, &ro, p1_blocks);
        CAL_TRY(st);
        if (st == 0) {
            if (shifted) *shifted = false;
            if (rank) *rank = rank_from_R(m, R, tol);
            return 0;
        }
        c->orth_redone = true;
        // the device Cholesky failed (kappa(X) > ~1e8): Householder TSQR gives
        // the reference's R for any kappa ("cholqr2" keeps shifted CholQR3)
        if (c->normalize_kind != 2) return via_tsqr();
    }
    std::vector<double> G((size_t)m * m), Mz((size_t)m * m, 0.0), Ctot;
    if (X.nseg <= kMaxSeg) {
        double G16[256], e16[16];
        CAL_TRY(tilegram_host(c, n, X, nullptr, G16, e16));
        for (int j = 0; j < m; ++j)
            for (int i = 0; i < m; ++i) G[i + (size_t)j * m] = G16[i + j * 16];
    } else {
        CAL_TRY(gram_host(c, n, X, X, G.data()));
    }
    if (c->normalize_kind != 2) {
        std::vector<double> Rc((size_t)m * m);
        if (!dense::chol_upper(m, G.data(), m, Rc.data(), m)) return via_tsqr();
    }
    for (int i = 0; i < m; ++i) Mz[i + (size_t)i * m] = 1.0;
    bool sh = false;
    CAL_TRY(two_pass(c, n, panel(), X, Mz, m, G.data(), Qout, R, Ctot, &sh));
    if (shifted) *shifted = sh;
    if (rank) *rank = rank_from_R(m, R, tol);
    return 0;
}

// n x m device block for the TSQR paths (materialised Y / Z when the tile
// kernel cannot form them on the fly)
static int ensure_zbuf(cal_ctx* c, int64_t n, int m, double** p, int64_t* ld) {
    *ld = ((std::max<int64_t>(n, 1) + 63) / 64) * 64;
    const size_t need = (size_t)(*ld) * m;
    if (need > c->zbuf_cap) {
        if (c->d_zbuf) CAL_HIP(c, hipFree(c->d_zbuf));
        c->d_zbuf = nullptr;
        CAL_HIP(c, scratch_malloc((void**)&c->d_zbuf, need * sizeof(double)));
        c->zbuf_cap = need;
    }
    *p = c->d_zbuf;
    return 0;
}

// ---- projectAndNormalize with the fused TSQR (tsqr_fold.hip) ---------------
// One CA block (m <= 8 columns against w <= 9) with no host round trip:
// P1 Gram (C = Qp'X) -> k_fold_up (Y formed, tile QR, Qp'Y on the matrix
// cores) -> the tree up -> the Gram reduced -> [several ranks: root
// all-gather + the global levels] -> k_fold_coef1 (reorth flag, R, RY, S, K;
// published) -> k_fold_down (each tile's S from the root's, Q = Q_Y S - Qp K).  The
// host waits once, for the published R.  Returns 2 when the shape does not
// apply, 1 when the fold declined after running (||W|| too large, or a
// non-finite value): the caller then takes the explicit-Z path.
// The fold/no-fold decision must be the same on every rank: the two paths
// issue different collectives.  So is the way it is reached: the branch is
// chosen by rank-uniform facts only (every rank is in the same entry point,
// so c->tier1 agrees, and every rank holds the same slab table).  Inside the
// device-resident loop (not tier 1) a panel is always the resident slab's
// local rows: the shape is checked for every rank's slab from the table, with
// no collective.  A tier-1 panel can have any local height: the ranks' votes
// are agreed by one all-reduce, which every rank issues.
static int fold_shape_all_ranks(cal_ctx* c, int64_t n, int m, int w, bool* ok) {
    const int P = c->comm ? c->comm->nranks : 1;
    *ok = fold_shape_ok(n, m, w);
    if (P == 1) return 0;
    const std::vector<int64_t>& st = c->A.slabs;
    if (!c->tier1 && c->has_A && (int)st.size() == P + 1) {
        // by construction n == n_local here on every rank (a loop panel)
        if (n != c->A.n_local) return set_error(c, CAL_ERR_ARG, "fold: a loop panel that is not the resident slab");
        for (int q = 0; q < P; ++q) *ok = *ok && fold_shape_ok(st[q + 1] - st[q], m, w);
        return 0;
    }
    CAL_TRY(ensure_partial(c, 1));
    const double vote = *ok ? 0.0 : 1.0;
    double sum = 0.0;
    CAL_HIP(c, hipMemcpyAsync(c->d_partial, &vote, sizeof(double), hipMemcpyHostToDevice, c->stream));
    CAL_TRY(allreduce_sum(c, c->d_partial, 1));
    CAL_HIP(c, hipMemcpyAsync(&sum, c->d_partial, sizeof(double), hipMemcpyDeviceToHost, c->stream));
    CAL_HIP(c, hipStreamSynchronize(c->stream));
    *ok = sum == 0.0;
    return 0;
}

static int pn_tsqr_fold(cal_ctx* c, int64_t n, const Panel& Qp, const Panel& X, bool doreorth, const PanelOut& Qout,
                        double* Rq, double* R, PNResult* res) {
    const int w = Qp.total, m = X.total, nq = w < 8 ? w : 8;
    const int P = c->comm ? c->comm->nranks : 1;
    if (m < 1 || m > 8 || w < 1 || w > 9 || Qp.nseg + X.nseg > kMaxSeg || Qout.total != m ||
        Qout.nseg > kMaxSeg || (int64_t)P * m > 512)
        return 2;
    bool shape_ok = false;
    CAL_TRY(fold_shape_all_ranks(c, n, m, w, &shape_ok));
    if (!shape_ok) return 2;
    const int me = c->comm ? c->comm->rank : 0;
    const int64_t n0 = fold_tiles(n), nblk = fold_blocks(n);
    const std::vector<int> nu = fold_levels(n);
    const int nlev = (int)nu.size();
    const int64_t mm = (int64_t)m * m;
    // workspace (doubles): level-0 tiles, the upper levels, scalars
    const size_t t0 = fold_l0_tile_doubles(), tu = fold_tile_doubles();
    size_t off = 0;
    auto take = [&](size_t cnt) {
        const size_t o = off;
        off += (cnt + 7) & ~size_t(7);
        return o;
    };
    const size_t oV0 = take(n0 * t0), otb0 = take(n0 * 16), oR0 = take(n0 * 64);
    size_t oVu[3], oRu[3], oMu[3];
    for (int L = 0; L < nlev; ++L) {
        oVu[L] = take((size_t)nu[L] * tu);
        oRu[L] = take((size_t)nu[L] * 64);
        oMu[L] = take((size_t)nu[L] * 64);
    }
    const size_t oRrm = take(64), oSb = take(64), oSm = take(64), oK = take(72);
    const size_t oOut = take(520), oT1 = take(272), oT2 = take(272);
    const size_t oG = take((size_t)P * mm), oGup = take(mm), oGdn = take((size_t)P * mm);
    if (off > c->fold_cap) {
        if (c->d_fold) CAL_HIP(c, hipFree(c->d_fold));
        c->d_fold = nullptr;
        CAL_HIP(c, scratch_malloc((void**)&c->d_fold, off * sizeof(double)));
        c->fold_cap = off;
    }
    double* const F = c->d_fold;
    double* const d_out = F + oOut;
    FoldArgs fa;
    fa.n = n;
    fa.m = m;
    fa.w = w;
    fa.nblk = (int)nblk;
    fa.n0 = (int)n0;
    fa.nlev = nlev;
    fa.C = F + oT1;
    fa.flags = d_out + 512;
    fa.K = F + oK;
    fa.tol = c->fold_tol;
    fa.V0 = F + oV0;
    fa.tb0 = F + otb0;
    fa.R0 = F + oR0;
    for (int L = 0; L < nlev; ++L) {
        fa.nu[L] = nu[L];
        fa.Vu[L] = F + oVu[L];
        fa.Ru[L] = F + oRu[L];
        fa.Mu[L] = F + oMu[L];
    }
    fa.Rroot_m = F + oRrm;
    const Panel W = panel_concat(Qp, X);
    // P1: [Qp(0:nq) | X]' X (+ Qp column 8), the CholQR2 path's row Gram
    int64_t gblocks = std::max<int64_t>(1, std::min<int64_t>((n + 255) / 256, kRowGramBlocks));
    CAL_TRY(ensure_partial(c, std::max<size_t>((size_t)gblocks * 272, (size_t)nblk * 272)));
    fa.partial = c->d_partial;
    {
        ColList ct{};
        const Panel T = panel_concat(panel_slice(W, 0, nq), X);
        const int nt = T.total;
        for (int cc = 0; cc < 16; ++cc) ct.p[cc] = panel_slice(T, cc < nt ? cc : nt - 1, 1).ptr[0];
        ct.p[16] = w == 9 ? panel_slice(Qp, 8, 1).ptr[0] : ct.p[0];
        const int t = timer_begin(c, 1, 8.0 * n * (nt + (w == 9 ? 1 : 0)));
        CAL_HIP(c, launch_rowgram(ct, nt, w == 9, n, (int)gblocks, c->d_partial, c->stream));
        timer_end(c, t);
    }
    CAL_HIP_OTHER(c, launch_reduce(c->d_partial, (int)gblocks, 272, F + oT1, c->stream));
    CAL_TRY(allreduce_sum(c, F + oT1, 272));
    // up: Y, the tile QRs and the tree to the local root, Qp'Y
    ColList cu{};
    const double* x0 = panel_slice(X, 0, 1).ptr[0];
    for (int k = 0; k < 9; ++k) cu.p[k] = k < w ? panel_slice(Qp, k, 1).ptr[0] : x0;
    for (int j = 0; j < 8; ++j) cu.p[9 + j] = j < m ? panel_slice(X, j, 1).ptr[0] : x0;
    {
        // [Qp | X] read, the factored tiles (m columns) stored
        const int t = timer_begin(c, 1, 8.0 * n * (w + 2 * m));
        CAL_HIP(c, launch_fold_up(cu, fa, c->stream));
        timer_end(c, t);
    }
    // one rank: the root level and the algebra merged (k_fold_root)
    const bool merged = P == 1;
    // (the C2 reduction on a side stream beside the tree levels, and the
    // publish beside the way down, measured 656-661 -> 626-633 outer-it/s:
    // the cross-stream waits cost more than the two short kernels.)  The
    // reduction rides on 72 extra blocks of the level-1 launch.
    const int tree_top = merged ? nlev - 1 : nlev;
    if (tree_top >= 1) fa.red_out = F + oT2;
    {
        const int t = timer_begin(c, 3);
        CAL_HIP(c, launch_fold_tree(fa, c->stream, tree_top));
        timer_end(c, t);
    }
    if (!fa.red_out) CAL_HIP(c, launch_fold_reduce(c->d_partial, (int)nblk, F + oT2, c->stream));
    CAL_TRY(allreduce_sum(c, F + oT2, 72));
    CAL_TRY(ensure_pub(c));
    const unsigned long long seq = ++c->pub_seq;
    double* h_out = c->h_pub;
    unsigned long long* h_seq = reinterpret_cast<unsigned long long*>(c->h_pub + 516);
    unsigned long long* d_seq = reinterpret_cast<unsigned long long*>(c->d_pub + 516);
    const double nglob = (double)global_rows(c, n) * (P > 1 && !c->has_A ? P : 1);
    if (merged) {
        const int t = timer_begin(c, 3);
        CAL_HIP(c, launch_fold_root(fa, F + oT1, F + oT2, d_out, F + oSb, F + oSm, F + oK, w, doreorth ? 1 : 0,
                                    nglob, c->d_pub, d_seq, seq, c->stream));
        timer_end(c, t);
        fa.Stop = F + oSb;
        fa.lds = 8;
    } else {
        // the root over the ranks: all-gather the local roots, factor the stack
        // (the tree kernel's stack level, redundantly on every rank)
        const double* Rtop = fa.Ru[nlev - 1];  // the root level's one R
        int ldr = 8;
        TsqrLevelArgs ga;
        TsqrCols gcols{};
        TsqrQ gq{};
        if (P > 1) {
            CAL_TRY(allgather(c, fa.Rroot_m, F + oG, mm));
            ga.rows = (int64_t)P * m;
            ga.m = m;
            ga.wp = m;
            ga.in = F + oG;
            ga.out = F + oGup;
            const int t = timer_begin(c, 3);
            CAL_HIP(c, launch_tsqr(false, 0, ga, gcols, gq, c->stream));
            timer_end(c, t);
            Rtop = F + oGup;
            ldr = m;
        }
        CAL_HIP(c, launch_fold_coef1(F + oT1, F + oT2, Rtop, ldr, d_out, F + oSb, F + oSm, F + oK, w, m,
                                     doreorth ? 1 : 0, nglob, c->fold_tol, c->d_pub, d_seq, seq, c->stream));
        // down: [the global levels to this rank's root S,] then k_fold_down
        fa.Stop = F + oSb;
        fa.lds = 8;
        if (P > 1) {
            ga.S = F + oSm;
            ga.out = F + oGdn;
            const int t = timer_begin(c, 3);
            CAL_HIP(c, launch_tsqr(true, 0, ga, gcols, gq, c->stream));
            timer_end(c, t);
            fa.Stop = F + oGdn + (size_t)me * mm;
            fa.lds = m;
        }
    }
    OutList qo{};
    for (int j = 0; j < 16; ++j) qo.p[j] = panel_out_slice(Qout, j < m ? j : 0, 1).ptr[0];
    {
        // the tiles and Qp read, Q stored
        const int t = timer_begin(c, 2, 8.0 * n * (w + 2 * m));
        CAL_HIP(c, launch_fold_down(cu, qo, fa, c->stream));
        timer_end(c, t);
    }
    if (c->pre_wait) {  // e.g. the next step's matrix powers (lanczos_step)
        auto hook = std::move(c->pre_wait);
        c->pre_wait = nullptr;
        CAL_TRY(hook());
    }
    CAL_TRY(wait_published(c, h_seq, seq));
    c->fold_runs++;
    c->fold_last_est = h_out[515];
    if (h_out[513] != 0.0) {
        c->fold_declined++;
        return 1;
    }
    std::copy(h_out, h_out + (size_t)mm, R);
    std::copy(h_out + 256, h_out + 256 + (size_t)w * m, Rq);
    const bool reorth = h_out[514] != 0.0;
    if (res) {
        res->reorth = reorth;
        res->rank = rank_from_R(m, R, 1.0e-8);
        res->chol_shifted = false;
    }
    return 0;
}

// projectAndNormalize.m:3-90 against one block with the Householder TSQR
// normalize (tsqr.m): C = Qp'X and X'X from one Gram sweep; the reorth test
// of :45-52 on the algebraic norms ||Y_i||^2 = diag(X'X - C'C); on reorth the
// second projection C2 = Qp'Y (:63, Y = X - Qp C formed on the fly) and
// RZ = C + C2 (:71-73); then TSQR of Z = X - Qp RZ, formed per row inside the
// tile kernel (or materialised first for shapes it does not instantiate).
static int pn_tsqr(cal_ctx* c, int64_t n, const Panel& Qp, const Panel& X, bool doreorth, const PanelOut& Qout,
                   double* Rq, double* R, PNResult* res) {
    const int w = Qp.total, m = X.total, wp = w + m;
    if (!tsqr_ok(m)) return set_error(c, CAL_ERR_UNSUPPORTED, "projectAndNormalize (tsqr): at most 32 columns");
    if (w > 0) {
        const int st = pn_tsqr_fold(c, n, Qp, X, doreorth, Qout, Rq, R, res);
        CAL_TRY(st);
        if (st == 0) return 0;
        if (st == 1) c->orth_redone = true;  // declined after running: the explicit-Z path below
    }
    const Panel W = panel_concat(Qp, X);
    std::vector<double> G1((size_t)wp * m);
    const int nq = w < 8 ? w : 8;
    // [Qp | X]'X: the row-parallel tile Gram of the CholQR2 path when the
    // shapes fit one 16-column tile (+ Qp's ninth column), else k_gram
    const bool tile = w <= 9 && nq + m <= 16 && Qp.nseg + X.nseg <= kMaxSeg;
    if (tile) {
        Panel Tl = panel_slice(W, 0, nq);
        Tl = panel_concat(Tl, X);
        const double* E = w == 9 ? panel_slice(Qp, 8, 1).ptr[0] : nullptr;
        double G16[256], e16[16];
        CAL_TRY(tilegram_host(c, n, Tl, E, G16, e16));
        for (int j = 0; j < m; ++j) {
            for (int i = 0; i < nq; ++i) G1[i + (size_t)j * wp] = G16[i + (nq + j) * 16];
            if (w == 9) G1[8 + (size_t)j * wp] = e16[nq + j];
            for (int i = 0; i < m; ++i) G1[w + i + (size_t)j * wp] = G16[(nq + i) + (nq + j) * 16];
        }
    } else {
        CAL_TRY(gram_host(c, n, W, X, G1.data()));
    }
    std::vector<double> C((size_t)std::max(w, 1) * m, 0.0), before(m);
    double mx = NAN;
    for (int j = 0; j < m; ++j) {
        for (int i = 0; i < w; ++i) C[i + (size_t)j * w] = G1[i + (size_t)j * wp];
        double cc = 0.0;
        for (int k = 0; k < w; ++k) cc += C[k + (size_t)j * w] * C[k + (size_t)j * w];
        const double xx = G1[w + j + (size_t)j * wp];
        before[j] = std::sqrt(xx);
        const double after = std::sqrt(std::max(xx - cc, 0.0));
        const double rel = std::fabs(before[j] - after) / before[j];
        if (!std::isnan(rel) && (std::isnan(mx) || rel > mx)) mx = rel;
    }
    const bool reorth = w > 0 && doreorth && mx > 0.5;
    auto coef = [&](const std::vector<double>& Ct) {
        std::vector<double> M((size_t)wp * m, 0.0);
        for (int j = 0; j < m; ++j) {
            for (int i = 0; i < w; ++i) M[i + (size_t)j * wp] = -Ct[i + (size_t)j * w];
            M[w + j + (size_t)j * wp] = 1.0;
        }
        return M;
    };
    std::vector<double> Ct = C, C2;
    if (reorth) {  // C2 = Qp'Y, Y = W [-C; I]
        std::vector<double> M = coef(C);
        C2.assign((size_t)w * m, 0.0);
        if (rowapply_ok(wp, m, true, w) && W.nseg <= kMaxSeg) {
            // the Gram-only row sweep (pass A's kernel): Qp'Y with Y in registers
            double G16[256], e16[16];
            CAL_TRY(rowapply_host(c, n, W, M.data(), m, Qout, 2, w, G16, e16));
            for (int j = 0; j < m; ++j) {
                for (int i = 0; i < nq; ++i) C2[i + (size_t)j * w] = G16[i + (nq + j) * 16];
                if (w == 9) C2[8 + (size_t)j * w] = e16[nq + j];
            }
        } else if (w <= 16 && m <= 16) {
            CAL_TRY(apply_host(c, n, W, M.data(), m, nullptr, nullptr, w, C2.data()));
        } else {
            double* dY;
            int64_t ldy;
            CAL_TRY(ensure_zbuf(c, n, m, &dY, &ldy));
            const PanelOut Yo = panel_out(dY, ldy, m);
            CAL_TRY(apply_host(c, n, W, M.data(), m, &Yo, nullptr, 0, nullptr));
            CAL_TRY(gram_host(c, n, Qp, as_panel(Yo), C2.data()));
        }
        for (size_t e = 0; e < C2.size(); ++e) Ct[e] = C[e] + C2[e];
    }
    if (w == 0) {
        CAL_TRY(tsqr_dev(c, n, X, nullptr, m, Qout, R));
    } else {
        // Z = Y - Qp C2 on the rounded Y = X - Qp C, as the reference
        // projects the stored Y again (:63)
        std::vector<double> M = coef(C);
        if (reorth)
            for (int j = 0; j < m; ++j)
                for (int i = 0; i < w; ++i) M.push_back(-C2[i + (size_t)j * w]);
        if (tsqr_form_ok(wp, m) && W.nseg <= kMaxSeg) {
            CAL_TRY(stage_small(c, M.data(), M.size()));
            CAL_TRY(tsqr_dev(c, n, W, c->d_small, m, Qout, R, reorth ? c->d_small + (size_t)wp * m : nullptr,
                             reorth ? w : 0));
        } else {
            double* dZ;
            int64_t ldz;
            CAL_TRY(ensure_zbuf(c, n, m, &dZ, &ldz));
            const PanelOut Zo = panel_out(dZ, ldz, m);
            CAL_TRY(apply_host(c, n, W, M.data(), m, &Zo, nullptr, 0, nullptr));
            if (reorth) {
                Panel W2 = panel_concat(Qp, as_panel(Zo));
                CAL_TRY(apply_host(c, n, W2, coef(C2).data(), m, &Zo, nullptr, 0, nullptr));
            }
            CAL_TRY(tsqr_dev(c, n, as_panel(Zo), nullptr, m, Qout, R));
        }
    }
    for (size_t e = 0; e < (size_t)w * m; ++e) Rq[e] = Ct[e];
    if (res) {
        res->reorth = reorth;
        res->rank = rank_from_R(m, R, 1.0e-8);
        res->chol_shifted = false;
    }
    return 0;
}

int project_and_normalize_dev(cal_ctx* c, int64_t n, const Panel& Qp, const Panel& X, bool doreorth,
                              const PanelOut& Qout, double* Rq, double* R, PNResult* res, const double* G1_pre) {
    const int w = Qp.total, m = X.total;
    if (Qp.nseg + X.nseg > kMaxSeg) return set_error(c, CAL_ERR_ARG, "projectAndNormalize: too many segments");
    if (use_tsqr(c, m, c->tier1) || (m > 16 && tsqr_ok(m))) return pn_tsqr(c, n, Qp, X, doreorth, Qout, Rq, R, res);
    if (m < 1 || m > 16) return set_error(c, CAL_ERR_ARG, "projectAndNormalize: 1..32 columns supported");
    if (orth_device_ok(c, Qp, X)) {
        bool ro = false;
        const int st = orth_device(c, n, Qp, X, doreorth, Qout, Rq, R, &ro);
        CAL_TRY(st);
        if (st == 0) {
            if (res) {
                res->reorth = ro;
                res->rank = rank_from_R(m, R, 1.0e-8);
                res->chol_shifted = false;
            }
            return 0;
        }
        c->orth_redone = true;
        // a device Cholesky failed (kappa > ~1e8): the Householder TSQR path
        if (c->normalize_kind != 2 && tsqr_ok(m)) return pn_tsqr(c, n, Qp, X, doreorth, Qout, Rq, R, res);
    }
    const Panel W = panel_concat(Qp, X);
    const int wp = w + m;
    // pass 1: [Qp | X]' X  -> C = Qp'X (project.m:34), X'X (norms before)
    std::vector<double> C((size_t)w * m), GZ((size_t)m * m);
    const int nq = w < 8 ? w : 8;
    if (w <= 9 && nq + m <= 16) {
        // one full MFMA tile [Qp(0:8) | X] + Qp column 8 as the VALU extra
        Panel Tl = panel_slice(W, 0, nq);
        Tl = panel_concat(Tl, X);
        const double* E = nullptr;
        if (w == 9) E = panel_slice(Qp, 8, 1).ptr[0];
        double G16[256], e16[16];
        CAL_TRY(tilegram_host(c, n, Tl, E, G16, e16));
        for (int j = 0; j < m; ++j) {
            for (int i = 0; i < nq; ++i) C[i + (size_t)j * w] = G16[i + (nq + j) * 16];
            if (w == 9) C[8 + (size_t)j * w] = e16[nq + j];
            for (int i = 0; i < m; ++i) GZ[i + (size_t)j * m] = G16[(nq + i) + (nq + j) * 16];
        }
    } else {
        std::vector<double> G1((size_t)wp * m);
        if (G1_pre) std::copy(G1_pre, G1_pre + (size_t)wp * m, G1.begin());  // formed with X (k_passb_wide)
        else CAL_TRY(gram_host(c, n, W, X, G1.data()));
        for (int j = 0; j < m; ++j) {
            for (int i = 0; i < w; ++i) C[i + (size_t)j * w] = G1[i + (size_t)j * wp];
            for (int i = 0; i < m; ++i) GZ[i + (size_t)j * m] = G1[w + i + (size_t)j * wp];
        }
    }
    std::vector<double> before(m), rel(m);
    for (int i = 0; i < m; ++i) before[i] = std::sqrt(GZ[i + (size_t)i * m]);
    // ||Y||^2 = X'X - C'C for Y = X - Qp C (Qp orthonormal); projectAndNormalize.m:45-48
    for (int j = 0; j < m; ++j)
        for (int i = 0; i < m; ++i) {
            double s = 0.0;
            for (int k = 0; k < w; ++k) s += C[k + (size_t)i * w] * C[k + (size_t)j * w];
            GZ[i + (size_t)j * m] -= s;
        }
    for (int i = 0; i < m; ++i) {
        const double after = std::sqrt(std::max(GZ[i + (size_t)i * m], 0.0));
        rel[i] = std::fabs(before[i] - after) / before[i];
    }
    // projectAndNormalize.m:52 -- the reference's second projection.  Here it
    // is always folded into pass B (a second CGS sweep on the stored block);
    // the flag records the reference's decision.
    const bool reorth = doreorth && (nan_max(rel) > 0.5);
    std::vector<double> Mz((size_t)wp * m, 0.0);
    for (int j = 0; j < m; ++j) {
        for (int i = 0; i < w; ++i) Mz[i + (size_t)j * wp] = -C[i + (size_t)j * w];
        Mz[w + j + (size_t)j * wp] = 1.0;
    }
    std::vector<double> Rtmp((size_t)m * m);
    const bool chol_ok = dense::chol_upper(m, GZ.data(), m, Rtmp.data(), m);
    // A wide projection whose reorth test does not fire (projectAndNormalize.m:
    // 52-58: no second pass; the 'fro' projection of ca_lanczos.m:197 against
    // all of Q, whose block is already orthonormal): one projection and the
    // normalize, as the reference does -- Q = [Qp | X] [-C; I] R^-1 with R =
    // chol(Y'Y) in ONE apply sweep after the Gram sweep, instead of the two-
    // pass CholQR2 (four wide sweeps).  Taken only when Y is so well
    // conditioned that one Cholesky pass is orthonormal to rounding: the
    // column-scaled Gram of Y is diagonally dominant with off-diagonal row
    // sums < 1/2, so kappa(Y) < sqrt(3) and the loss of orthogonality ~ 3u.
    // The 0.5 norm-loss test guards it whatever doreorth says: R = chol(X'X -
    // C'C) from the algebraic Gram cancels when most of X lies in span(Qp)
    // (orthogonality ~ u ||X||^2 / ||Y||^2), and with doreorth = false the
    // reorth flag is always off, so it cannot stand in for that test.
    if (w > 9 && !(nan_max(rel) > 0.5) && chol_ok && c->normalize_kind != 1) {
        bool dominant = true;
        for (int i = 0; i < m && dominant; ++i) {
            double off = 0.0;
            const double gii = GZ[i + (size_t)i * m];
            for (int j = 0; j < m; ++j)
                if (j != i) off += std::fabs(GZ[i + (size_t)j * m]) / std::sqrt(gii * GZ[j + (size_t)j * m]);
            dominant = gii > 0.0 && off < 0.5;
        }
        if (dominant) {
            std::vector<double> Ri((size_t)m * m), M1((size_t)wp * m);
            dense::tri_inv_upper(m, Rtmp.data(), m, Ri.data(), m);
            dense::matmul(wp, m, m, Mz.data(), wp, Ri.data(), m, M1.data(), wp);
            CAL_TRY(apply_host(c, n, W, M1.data(), m, &Qout, nullptr, 0, nullptr));
            std::copy(Rtmp.begin(), Rtmp.end(), R);
            std::copy(C.begin(), C.end(), Rq);
            if (res) {
                res->reorth = false;
                res->rank = rank_from_R(m, R, 1.0e-8);
                res->chol_shifted = false;
            }
            return 0;
        }
    }
    if (!chol_ok) {
        if (c->normalize_kind != 2 && tsqr_ok(m)) return pn_tsqr(c, n, Qp, X, doreorth, Qout, Rq, R, res);
        // the algebraic Gram lost definiteness (heavy cancellation): Y'Y directly
        CAL_TRY(apply_host(c, n, W, Mz.data(), m, nullptr, GZ.data(), 0, nullptr));
    }
    bool sh = false;
    std::vector<double> Ctot;
    CAL_TRY(two_pass(c, n, Qp, W, Mz, m, GZ.data(), Qout, R, Ctot, &sh));
    for (size_t e = 0; e < C.size(); ++e) Rq[e] = C[e] + Ctot[e];
    if (res) {
        res->reorth = reorth;
        res->rank = rank_from_R(m, R, 1.0e-8);
        res->chol_shifted = sh;
    }
    return 0;
}

// project.m:7-58 on the device (block MGS across blocks, CGS within).
int project_blocks(cal_ctx* c, int64_t n, int64_t ld, int nb, const std::vector<double*>& dQ,
                          const int* widths, int m, double* dX, bool doreorth, std::vector<std::vector<double>>& R) {
    Panel X = panel();
    panel_add(X, dX, ld, m);
    PanelOut Xo = panel_out(dX, ld, m);
    auto col_norms = [&](std::vector<double>& nr) -> int {
        std::vector<double> G((size_t)m * m);
        CAL_TRY(gram_host(c, n, X, X, G.data()));
        nr.resize(m);
        for (int i = 0; i < m; ++i) nr[i] = std::sqrt(G[i + (size_t)i * m]);
        return 0;
    };
    std::vector<double> before;
    if (doreorth) CAL_TRY(col_norms(before));
    auto one_pass = [&](bool accumulate) -> int {
        for (int i = 0; i < nb; ++i) {
            const int w = widths[i];
            if (w <= 0) continue;
            Panel Qi = panel();
            panel_add(Qi, dQ[i], ld, w);
            std::vector<double> Ri((size_t)w * m);
            CAL_TRY(gram_host(c, n, Qi, X, Ri.data()));  // R{i} = Q{i}'*X
            Panel W = panel();
            panel_add(W, dQ[i], ld, w);
            panel_add(W, dX, ld, m);
            std::vector<double> M((size_t)(w + m) * m, 0.0);
            for (int j = 0; j < m; ++j) {
                for (int r = 0; r < w; ++r) M[r + (size_t)j * (w + m)] = -Ri[r + (size_t)j * w];
                M[w + j + (size_t)j * (w + m)] = 1.0;
            }
            CAL_TRY(apply_host(c, n, W, M.data(), m, &Xo, nullptr, 0, nullptr));  // X = X - Q{i}*R{i}
            if (accumulate)
                for (size_t e = 0; e < Ri.size(); ++e) R[i][e] += Ri[e];
            else
                R[i] = Ri;
        }
        return 0;
    };
    CAL_TRY(one_pass(false));
    if (doreorth) {  // project.m:40-57 (note the inverted test of the reference)
        std::vector<double> after;
        CAL_TRY(col_norms(after));
        double mx = NAN;
        for (int i = 0; i < m; ++i) {
            const double d = 0.5 * before[i] - after[i];
            if (!std::isnan(d) && (std::isnan(mx) || d > mx)) mx = d;
        }
        if (mx < 0) CAL_TRY(one_pass(true));
    }
    return 0;
}

// projectAndNormalize.m:3-90 against several blocks (the general path:
// project.m block MGS across blocks, then normalize; the second projection
// of :52-73 when a column lost more than half its norm).  X is read from dX
// and not modified; dY is an n x m work block; QZ goes to Qout.
// ---- project.m without host round trips (projectAndNormalize's blocks) ----
// Each block's Gram Q{i}'X is reduced on the device into a region of d_red,
// the coefficient matrix [-R{i}; I] is formed there (k_form_projM) and the
// update X - Q{i} R{i} is enqueued right behind it; R{i} goes to pinned host
// memory with an async copy.  The caller reads the copies after its next host
// wait (normalize_dev polls the block's published R), which the stream orders
// after them.  Same kernels and coefficients as project_blocks: same bits.
namespace {
constexpr size_t kAsyncBase = 8192, kAsyncRegion = 8192;  // doubles; Gram at +0, M at +4096
}

static bool async_ok(int nb, const int* widths, int m) {
    if (m < 1 || m > 16 || nb + 1 > 6) return false;
    for (int i = 0; i < nb; ++i)
        if (widths[i] > 128) return false;
    return true;
}

// Gram A'B (A <= 128 columns, B <= 16) reduced (and all-reduced) into d_dst
// (ld *ldc) and copied to h_dst; nothing waits.
int gram_async(cal_ctx* c, int64_t n, const Panel& A, const Panel& B, double* d_dst, double* h_dst, int* ldc,
               double* part, bool bb) {
    if (B.total > 16 || A.total > 128) return set_error(c, CAL_ERR_ARG, "gram_async: A <= 128, B <= 16 columns");
    if (bb && !gram_bb_ok(A.total, B.total)) return set_error(c, CAL_ERR_ARG, "gram_async: no fused B'B here");
    const GramPlan pl = gram_plan(A.total, B.total, n);
    const int64_t ne = pl.entries + (bb ? 256 : 0);
    if (!part) {
        CAL_TRY(ensure_partial(c, (size_t)pl.blocks * ne));
        part = c->d_partial;
    }
    const int t = timer_begin(c, 1, 8.0 * n * (A.total + B.total));
    if (bb) CAL_HIP(c, launch_gram_bb(A, B, n, pl, part, c->stream));
    else CAL_HIP(c, launch_gram(A, B, n, pl, part, c->stream));
    timer_end(c, t);
    CAL_HIP_OTHER(c, launch_reduce(part, pl.blocks, ne, d_dst, c->stream));
    CAL_TRY(allreduce_sum(c, d_dst, ne));
    CAL_HIP(c, hipMemcpyAsync(h_dst, d_dst, ne * sizeof(double), hipMemcpyDeviceToHost, c->stream));
    *ldc = 16 * pl.nta;
    return 0;
}

// One block-MGS pass of project.m over the nb blocks (doreorth = false);
// region r of d_red / h_red holds block r's Gram; ldc[r] its leading dimension.
// dSrc (optional): the input block when it is not dX; the first projection
// reads it and writes dX (no separate copy of X into the work block).
// bb_first: the first block's Gram also forms X'X (the norms before of
// projectAndNormalize.m:17-22) in the same pass, at region + 16 ldc (ld 16).
// self_blocks (optional): the last step's update also forms X'X for the
// normalize that follows (normalize_dev's p1_blocks; 0 when it did not).
static int project_blocks_async(cal_ctx* c, int64_t n, int64_t ld, int nb, const std::vector<double*>& dQ,
                                const int* widths, int m, double* dX, int region0, std::vector<int>& ldc,
                                const double* dSrc = nullptr, bool bb_first = false, int* self_blocks = nullptr) {
    const bool self_off = test_switch("CAL_TEST_SELFGRAM_OFF");  // A/B (test build)
    if (self_blocks) *self_blocks = 0;
    const PanelOut Xo = panel_out(dX, ld, m);
    const double* cur = dSrc ? dSrc : dX;  // where X currently is
    ldc.assign(nb, 0);
    // the update of block i and the Gram of block i + 1 share one pass over
    // the rows (k_apply_gram) where the shapes allow; the test build's
    // CAL_TEST_APPLY_GRAM_OFF keeps them apart (the fused/unfused parity test)
    const bool fuse = !test_switch("CAL_TEST_APPLY_GRAM_OFF");
    bool first = true, have_R = false;  // have_R: block i's Gram already enqueued (fused step)
    for (int i = 0; i < nb; ++i) {
        const int w = widths[i];
        if (w <= 0) continue;
        const size_t off = kAsyncBase + (size_t)(region0 + i) * kAsyncRegion;
        Panel Qi = panel(), X = panel();
        panel_add(Qi, dQ[i], ld, w);
        panel_add(X, cur, ld, m);
        if (!have_R)
            CAL_TRY(gram_async(c, n, Qi, X, c->d_red + off, c->h_red + off, &ldc[i], nullptr,
                               bb_first && first));  // R{i} = Q{i}'*X
        first = false;
        double* dM = c->d_red + off + 4096;
        CAL_HIP_OTHER(c, launch_form_projM(c->d_red + off, ldc[i], w, m, dM, c->stream));
        Panel W = panel();
        panel_add(W, dQ[i], ld, w);
        panel_add(W, cur, ld, m);
        int nx = i + 1;
        while (nx < nb && widths[nx] <= 0) ++nx;
        have_R = fuse && nx < nb && apply_gram_ok(w + m, m, widths[nx]);
        if (have_R) {
            // X = X - Q{i}*R{i} and R{i+1} = Q{i+1}'*X in one pass
            const size_t offn = kAsyncBase + (size_t)(region0 + nx) * kAsyncRegion;
            Panel Qn = panel();
            panel_add(Qn, dQ[nx], ld, widths[nx]);
            const int blocks = apply_gram_blocks(n);
            CAL_TRY(ensure_partial(c, (size_t)blocks * 256));
            const int t = timer_begin(c, 2, 8.0 * n * (w + 2 * m + widths[nx]));
            CAL_HIP(c, launch_apply_gram(W, dM, w + m, m, Xo, Qn, n, c->d_partial, c->stream));
            timer_end(c, t);
            CAL_HIP_OTHER(c, launch_reduce(c->d_partial, blocks, 256, c->d_red + offn, c->stream));
            CAL_TRY(allreduce_sum(c, c->d_red + offn, 256));
            CAL_HIP_OTHER(c, hipMemcpyAsync(c->h_red + offn, c->d_red + offn, 256 * sizeof(double), hipMemcpyDeviceToHost,
                                      c->stream));
            ldc[nx] = 16;
        } else if (self_blocks && !self_off && nx == nb && apply_selfgram_ok(w + m, m)) {
            // the last step: X = X - Q{i}*R{i} and X'X (the normalize's P1) in one pass
            CAL_TRY(ensure_partial(c, (size_t)std::max<int64_t>(apply_gram_blocks(n), (n + 255) / 256) * 272));
            const int t = timer_begin(c, 2, 8.0 * n * (w + 2 * m));
            CAL_HIP(c, launch_apply_selfgram(W, dM, w + m, m, Xo, n, c->d_partial, self_blocks, c->stream));
            timer_end(c, t);
        } else {
            CAL_TRY(apply_dev(c, n, W, dM, m, Xo));  // X = X - Q{i}*R{i}
        }
        cur = dX;
    }
    if (cur != dX) CAL_HIP(c, copy_cols(c, dX, cur, ld, n, m));  // no block to project against
    return 0;
}

static void read_async_R(cal_ctx* c, int nb, const int* widths, int m, int region0, const std::vector<int>& ldc,
                         std::vector<std::vector<double>>& R) {
    for (int i = 0; i < nb; ++i) {
        const int w = widths[i];
        R[i].assign((size_t)std::max(w, 0) * m, 0.0);
        const double* h = c->h_red + kAsyncBase + (size_t)(region0 + i) * kAsyncRegion;
        for (int j = 0; j < m && w > 0; ++j)
            for (int r = 0; r < w; ++r) R[i][r + (size_t)j * w] = h[r + (size_t)j * ldc[i]];
    }
}

int project_and_normalize_blocks_dev(cal_ctx* c, int64_t n, int64_t ld, int nblocks, const std::vector<double*>& dQ,
                                     const int* widths, int m, const double* dX, bool doreorth, double* dY,
                                     const PanelOut& Qout, std::vector<std::vector<double>>& RZ, double* R,
                                     bool* reorth, int* rank) {
    const bool async = async_ok(nblocks, widths, m);
    std::vector<double> before(m);
    std::vector<std::vector<double>> RY(nblocks);
    for (int i = 0; i < nblocks; ++i) RY[i].assign((size_t)std::max(widths[i], 0) * m, 0.0);
    Panel Yp = panel();
    panel_add(Yp, dY, ld, m);
    bool sh = false;
    int rk = m;
    if (async) {
        // (the regions lie above everything the synchronous paths stage in h_red)
        CAL_TRY(ensure_red(c, kAsyncBase + (size_t)(nblocks + 1) * kAsyncRegion));
        // norms before (:17-22): X'X rides on the first block's Gram (same
        // pass over X) when that Gram is the row-staged kernel, else its own
        int b0 = -1;
        for (int i = 0; i < nblocks && b0 < 0; ++i)
            if (widths[i] > 0) b0 = i;
        const bool fused = b0 >= 0 && gram_bb_ok(widths[b0], m);
        int ldx = 16;
        size_t offx = kAsyncBase + (size_t)nblocks * kAsyncRegion;
        if (!fused) {
            Panel Xp = panel();
            panel_add(Xp, dX, ld, m);
            CAL_TRY(gram_async(c, n, Xp, Xp, c->d_red + offx, c->h_red + offx, &ldx));
        }
        std::vector<int> ldc;
        int p1 = 0;
        CAL_TRY(project_blocks_async(c, n, ld, nblocks, dQ, widths, m, dY, 0, ldc, dX, fused, &p1));  // :25
        if (fused) offx = kAsyncBase + (size_t)b0 * kAsyncRegion + 16 * (size_t)ldc[b0];
        CAL_TRY(normalize_dev(c, n, Yp, Qout, R, 1.0e-8, &rk, &sh, p1));  // :26 (waits)
        for (int i = 0; i < m; ++i) before[i] = std::sqrt(c->h_red[offx + i + (size_t)i * ldx]);
        read_async_R(c, nblocks, widths, m, 0, ldc, RY);
    } else {
        Panel Xp = panel();
        panel_add(Xp, dX, ld, m);
        std::vector<double> G((size_t)m * m);
        CAL_TRY(gram_host(c, n, Xp, Xp, G.data()));
        for (int i = 0; i < m; ++i) before[i] = std::sqrt(G[i + (size_t)i * m]);   // :17-22
        CAL_HIP(c, copy_cols(c, dY, dX, ld, n, m));
        CAL_TRY(project_blocks(c, n, ld, nblocks, dQ, widths, m, dY, false, RY));  // :25
        CAL_TRY(normalize_dev(c, n, Yp, Qout, R, 1.0e-8, &rk, &sh));  // :26
    }
    double mx = NAN;
    for (int i = 0; i < m; ++i) {  // :45-48 (after = ||R(:,i)||)
        double after = 0.0;
        for (int r = 0; r < m; ++r) after += R[r + (size_t)i * m] * R[r + (size_t)i * m];
        after = std::sqrt(after);
        const double rel = std::fabs(before[i] - after) / before[i];
        if (!std::isnan(rel) && (std::isnan(mx) || rel > mx)) mx = rel;
    }
    RZ = RY;
    bool re = false;
    if (doreorth && mx > 0.5) {  // :52-73: project the unnormalised Y again
        re = true;
        std::vector<std::vector<double>> R2(nblocks);
        for (int i = 0; i < nblocks; ++i) R2[i].assign((size_t)std::max(widths[i], 0) * m, 0.0);
        if (async) {
            std::vector<int> ldc;
            int p1 = 0;
            CAL_TRY(project_blocks_async(c, n, ld, nblocks, dQ, widths, m, dY, 0, ldc, nullptr, false, &p1));
            CAL_TRY(normalize_dev(c, n, Yp, Qout, R, 1.0e-8, &rk, &sh, p1));
            read_async_R(c, nblocks, widths, m, 0, ldc, R2);
        } else {
            CAL_TRY(project_blocks(c, n, ld, nblocks, dQ, widths, m, dY, false, R2));
            CAL_TRY(normalize_dev(c, n, Yp, Qout, R, 1.0e-8, &rk, &sh));
        }
        for (int i = 0; i < nblocks; ++i)
            for (size_t e = 0; e < R2[i].size(); ++e) RZ[i][e] = R2[i][e] + RY[i][e];
    }
    if (reorth) *reorth = re;
    if (rank) *rank = rk;
    return 0;
}

// Q factor of an n x m block with m > 16 (the converged Ritz vectors of the
// selective variant, normalize(QR) at ca_lanczos.m:339): CholQR2 with the
// shifted fallback on the generic MFMA Gram/apply kernels.  dW is an n x m
// work block; Q goes to dQ.
int normalize_wide_dev(cal_ctx* c, int64_t n, int64_t ld, const double* dX, int m, double* dQ, double* dW) {
    const int64_t ng = global_rows(c, n);
    auto gram_full = [&](const double* d, std::vector<double>& G) -> int {
        Panel A = panel();
        panel_add(A, d, ld, m);
        G.assign((size_t)m * m, 0.0);
        for (int j0 = 0; j0 < m; j0 += 16) {
            const int nb = std::min(16, m - j0);
            Panel B = panel();
            panel_add(B, d + (size_t)j0 * ld, ld, nb);
            std::vector<double> Gc((size_t)m * nb);
            CAL_TRY(gram_host(c, n, A, B, Gc.data()));
            for (int j = 0; j < nb; ++j)
                for (int i = 0; i < m; ++i) G[i + (size_t)(j0 + j) * m] = Gc[i + (size_t)j * m];
        }
        return 0;
    };
    // CholQR2; a shifted first pass makes it shifted CholQR3 (Fukaya et al.)
    const double* src = dX;
    double* bufs[2] = {dW, dQ};
    int total = 2, which = 0;
    for (int pass = 0; pass < total; ++pass) {
        std::vector<double> G, R((size_t)m * m), Ri((size_t)m * m);
        CAL_TRY(gram_full(src, G));
        bool sh = false;
        if (!chol_or_shift(m, G.data(), ng, R.data(), &sh))
            return set_error(c, CAL_ERR_NUMERIC, "normalize: Gram matrix is not positive definite");
        if (sh && pass == 0) total = 3;
        dense::tri_inv_upper(m, R.data(), m, Ri.data(), m);
        Panel P = panel();
        panel_add(P, src, ld, m);
        double* out = bufs[which];
        if (out == src) out = bufs[which ^= 1];
        PanelOut Y = panel_out(out, ld, m);
        CAL_TRY(apply_host(c, n, P, Ri.data(), m, &Y, nullptr, 0, nullptr));
        src = out;
        which ^= 1;
    }
    if (src != dQ)
        CAL_HIP(c, copy_cols(c, dQ, src, ld, n, m));
    return 0;
}

}  // namespace cal
