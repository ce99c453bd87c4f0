// api.cpp -- tier-1 (host-pointer) entry points of the C ABI: each call
// stages its column-major inputs into HBM, runs the device kernels and copies
// the outputs back (SURVEY §8b "two tiers").  These are what a MEX shim of
// SpMV.m, matrix_powers_*.m, tsqr.m, cholqr.m, project.m, normalize.m and
// projectAndNormalize.m binds; the device-resident tier is lanczos.cpp.
#include <algorithm>
#include <random>
#include <cmath>
#include <string>
#include <vector>

#include "../../include/calanczos_host.h"
#include "cal_internal.hpp"
#include "comm.hpp"
#include "dense.hpp"

using namespace cal;

namespace {

int64_t ld_for(int64_t n) {
    int64_t ld = ((n + 63) / 64) * 64;
    return ld > 0 ? ld : 64;
}

// upload host column-major (n x m, ld n) into device (ld dld)
int upload(cal_ctx* c, double* d, int64_t dld, const double* h, int64_t n, int m) {
    if (m <= 0 || n <= 0) return 0;
    CAL_HIP(c, hipMemcpy2DAsync(d, dld * sizeof(double), h, n * sizeof(double), n * sizeof(double), m,
                                hipMemcpyHostToDevice, c->stream));
    return 0;
}

int download(cal_ctx* c, double* h, const double* d, int64_t dld, int64_t n, int m) {
    if (m <= 0 || n <= 0) return 0;
    CAL_HIP(c, hipMemcpy2DAsync(h, n * sizeof(double), d, dld * sizeof(double), n * sizeof(double), m,
                                hipMemcpyDeviceToHost, c->stream));
    CAL_HIP(c, hipStreamSynchronize(c->stream));
    return 0;
}

// marks a tier-1 call for its duration (normalize backend choice, use_tsqr)
struct Tier1 {
    cal_ctx* c;
    explicit Tier1(cal_ctx* cc) : c(cc) {
        if (c) c->tier1 = true;
    }
    ~Tier1() {
        if (c) c->tier1 = false;
    }
};

int check_ctx(cal_ctx* c, bool need_A) {
    if (!c) return CAL_ERR_ARG;
    hipSetDevice(c->device);
    if (need_A && !c->has_A) return set_error(c, CAL_ERR_NOMATRIX, "no matrix set on the context");
    return 0;
}

}  // namespace

extern "C" {

int cal_spmv(cal_ctx* c, const double* v, double* Av) {
    CAL_TRY(check_ctx(c, true));
    if (!v || !Av) return set_error(c, CAL_ERR_ARG, "SpMV: null vector");
    const int64_t n = c->A.n_local, ld = c->A.ld;
    CAL_TRY(ensure_scratch(c, 2 * ld));
    double* x = vcol(c, c->d_scratch, 0);
    double* y = vcol(c, c->d_scratch, 1);
    CAL_TRY(upload(c, x, ld, v, n, 1));
    CAL_TRY(spmv_dev(c, x, y, 0, 0.0, 0.0, nullptr));
    return download(c, Av, y, ld, n, 1);
}

int cal_bench_spmv(cal_ctx* c, int reps, double shift, double* mean_ms, double* min_ms) {
    CAL_TRY(check_ctx(c, true));
    if (reps < 1) return set_error(c, CAL_ERR_ARG, "bench_spmv: reps >= 1");
    const int64_t n = c->A.n_local, ld = c->A.ld;
    CAL_TRY(ensure_scratch(c, 2 * ld));
    CAL_HIP(c, hipMemsetAsync(c->d_scratch, 0, 2 * ld * sizeof(double), c->stream));
    double* x = vcol(c, c->d_scratch, 0);
    double* y = vcol(c, c->d_scratch, 1);
    std::vector<double> ones(n, 1.0);
    CAL_TRY(upload(c, x, ld, ones.data(), n, 1));
    const bool was = c->timing;
    c->timing = true;
    const size_t first = c->timers.size();
    for (int i = 0; i < reps; ++i) CAL_TRY(spmv_dev(c, x, y, shift != 0.0 ? 1 : 0, shift, 0.0, nullptr));
    CAL_HIP(c, hipStreamSynchronize(c->stream));
    double tot = 0.0, mn = 1e300;
    for (size_t i = first; i < c->timers.size(); ++i) {
        float ms = 0.f;
        CAL_HIP(c, hipEventElapsedTime(&ms, c->timers[i].a, c->timers[i].b));
        tot += ms;
        mn = std::min(mn, (double)ms);
    }
    for (size_t i = first; i < c->timers.size(); ++i) {
        c->event_pool.push_back(c->timers[i].a);
        c->event_pool.push_back(c->timers[i].b);
    }
    c->timers.resize(first);
    c->timing = was;
    if (mean_ms) *mean_ms = tot / reps;
    if (min_ms) *min_ms = mn;
    return 0;
}

int cal_matrix_powers_monomial(cal_ctx* c, const double* q, int s, double* V) {
    CAL_TRY(check_ctx(c, true));
    if (!q || !V || s < 1) return set_error(c, CAL_ERR_ARG, "matrix_powers_monomial: bad arguments");
    const int64_t n = c->A.n_local, ld = c->A.ld;
    CAL_TRY(ensure_scratch(c, (size_t)(s + 1) * ld));
    double* W = vcol(c, c->d_scratch, 0);
    CAL_TRY(upload(c, W, ld, q, n, 1));
    std::vector<double*> Y(s);
    for (int i = 0; i < s; ++i) Y[i] = W + (size_t)(i + 1) * ld;
    CAL_TRY(powers_dev(c, s, W, Y.data(), nullptr, nullptr, nullptr));
    return download(c, V, W + ld, ld, n, s);  // V excludes q (matrix_powers_monomial.m:7)
}

int cal_matrix_powers_newton(cal_ctx* c, const double* v, int s, const double* lre, const double* lim, int modifiedp,
                             double* V) {
    CAL_TRY(check_ctx(c, true));
    if (!v || !V || !lre || s < 1) return set_error(c, CAL_ERR_ARG, "matrix_powers_newton: bad arguments");
    const int64_t n = c->A.n_local, ld = c->A.ld;
    CAL_TRY(ensure_scratch(c, (size_t)(s + 1) * ld));
    double* W = vcol(c, c->d_scratch, 0);
    CAL_TRY(upload(c, W, ld, v, n, 1));
    // V(:,k+1) = A V(:,k) - Re(l_k) V(:,k) [+ Im(l_k)^2 V(:,k-1) when Im(l_k) < 0]
    std::vector<double*> Y(s);
    std::vector<double> sh(s), im2(s, 0.0);
    std::vector<const double*> xp(s, nullptr);
    for (int k = 0; k < s; ++k) {
        const double re = lre[k], im = lim ? lim[k] : 0.0;
        Y[k] = W + (size_t)(k + 1) * ld;
        sh[k] = re;
        if (modifiedp == 0) {
            if (im != 0.0)
                return set_error(c, CAL_ERR_UNSUPPORTED, "complex shifts need modifiedp=1 (real basis)");  // :28
        } else if (im < 0.0) {
            if (k == 0)
                return set_error(c, CAL_ERR_NUMERIC, "k==1, but shift has a negative imaginary part");  // :36-38
            im2[k] = im * im;  // :40-41
            xp[k] = W + (size_t)(k - 1) * ld;
        }  // else :34, :43
    }
    CAL_TRY(powers_dev(c, s, W, Y.data(), sh.data(), im2.data(), xp.data()));
    return download(c, V, W, ld, n, s + 1);
}

int cal_tsqr(cal_ctx* c, int64_t n, int m, const double* A, double* Q, double* R) {
    Tier1 t1(c);
    CAL_TRY(check_ctx(c, false));
    if (!A || !Q || !R || m < 1 || n < m) return set_error(c, CAL_ERR_ARG, "tsqr: need an n x m A with n >= m >= 1");
    if (!tsqr_ok(m)) return set_error(c, CAL_ERR_UNSUPPORTED, "tsqr: at most 32 columns on the device");
    const int64_t ld = ld_for(n);
    CAL_TRY(ensure_scratch(c, (size_t)2 * m * ld));
    double* dX = c->d_scratch;
    double* dQ = c->d_scratch + (size_t)m * ld;
    CAL_TRY(upload(c, dX, ld, A, n, m));
    Panel X = panel();
    panel_add(X, dX, ld, m);
    // Householder TSQR whatever the normalize setting: tsqr.m is qr(A,0)
    CAL_TRY(tsqr_dev(c, n, X, nullptr, m, panel_out(dQ, ld, m), R));
    return download(c, Q, dQ, ld, n, m);
}

int cal_normalize(cal_ctx* c, int64_t n, int m, const double* X, double tol, double* Q, double* R, int* rank) {
    return cal_normalize_opt(c, n, m, X, "None", tol, Q, R, rank);
}

int cal_normalize_opt(cal_ctx* c, int64_t n, int m, const double* X, const char* opt, double tol, double* Q,
                      double* R, int* rank) {
    Tier1 t1(c);
    CAL_TRY(check_ctx(c, false));
    if (!X || !Q || !R || n < 1 || m < 1 || m > 32) return set_error(c, CAL_ERR_ARG, "normalize: need 1 <= m <= 32");
    std::string o = opt ? opt : "None";
    for (auto& ch : o) ch = (char)tolower(ch);
    const bool randomize = o == "randomizenullspace";  // normalize.m:28 strcmpi
    const int64_t ld = ld_for(n);
    CAL_TRY(ensure_scratch(c, (size_t)3 * m * ld));
    double* dX = c->d_scratch;
    double* dQ = c->d_scratch + (size_t)m * ld;
    double* dW = c->d_scratch + (size_t)2 * m * ld;
    CAL_TRY(upload(c, dX, ld, X, n, m));
    Panel P = panel();
    panel_add(P, dX, ld, m);
    int rk = 0;
    bool sh = false;
    CAL_TRY(normalize_dev(c, n, P, panel_out(dQ, ld, m), R, tol > 0 ? tol : 1.0e-8, &rk, &sh));  // :14-24
    if (rank) *rank = rk;
    if (randomize && rk < m) {
        // :29-31: [U,S,W] = svd(R); R = S*W'; Q = Q*U; randomizeNullSpace(Q, rank)
        std::vector<double> U((size_t)m * m), S(m), W((size_t)m * m);
        dense::svd(m, R, m, U.data(), S.data(), W.data());
        for (int j = 0; j < m; ++j)
            for (int i = 0; i < m; ++i) R[i + (size_t)j * m] = S[i] * W[j + (size_t)i * m];
        Panel Qp = panel();
        panel_add(Qp, dQ, ld, m);
        const PanelOut Wo = panel_out(dW, ld, m);
        CAL_TRY(apply_host(c, n, Qp, U.data(), m, &Wo, nullptr, 0, nullptr));
        // :43-50: Q(:,null) = rand(nrows, ncols-rank); project against Q(:,1:rank); tsqr
        const int k = m - rk;
        // MATLAB's rand(nrows, k) fills the GLOBAL column-major matrix: on a
        // row slab [row0, row0 + n) of n_global rows, column j is the stream
        // slice j*n_global + row0 ... + n - 1 (each draw takes two 32-bit words)
        int64_t row0 = 0, nglob = n;
        if (c->comm && c->comm->nranks > 1) {
            if (!c->has_A || c->A.n_local != n)
                return set_error(c, CAL_ERR_ARG,
                                 "normalize 'randomizeNullSpace' on a distributed context needs the matrix's row slabs");
            row0 = c->A.row0;
            nglob = c->A.n_global;
        }
        std::vector<double> h((size_t)n * k);
        {
            std::mt19937 g(5489);
            int64_t pos = 0;
            for (int j = 0; j < k; ++j) {
                const int64_t start = (int64_t)j * nglob + row0;
                g.discard((unsigned long long)(2 * (start - pos)));
                dense::matlab_rand(g, n, h.data() + (size_t)j * n);
                pos = start + n;
            }
        }
        double* dN = dW + (size_t)rk * ld;
        CAL_TRY(upload(c, dN, ld, h.data(), n, k));
        if (rk > 0) {
            std::vector<double*> blocks{dW};
            const int widths[1] = {rk};
            std::vector<std::vector<double>> R_(1);
            CAL_TRY(project_blocks(c, n, ld, 1, blocks, widths, k, dN, false, R_));
        }
        Panel Np = panel();
        panel_add(Np, dN, ld, k);
        std::vector<double> Rn((size_t)k * k);
        if (tsqr_ok(k)) {
            CAL_TRY(tsqr_dev(c, n, Np, nullptr, k, panel_out(dN, ld, k), Rn.data()));
        } else {
            CAL_TRY(normalize_wide_dev(c, n, ld, dN, k, dN, dX));
        }
        CAL_TRY(download(c, Q, dW, ld, n, m));
        return CAL_WARN_RANK_DEFICIENT;
    }
    CAL_TRY(download(c, Q, dQ, ld, n, m));
    return rk < m ? CAL_WARN_RANK_DEFICIENT : 0;
}

int cal_cholqr(cal_ctx* c, int64_t n, int m, const double* X, double* Q, double* R) {
    CAL_TRY(check_ctx(c, false));
    if (!X || !Q || !R || n < 1 || m < 1 || m > 32) return set_error(c, CAL_ERR_ARG, "cholqr: need 1 <= m <= 32");
    const int64_t ld = ld_for(n);
    CAL_TRY(ensure_scratch(c, (size_t)2 * m * ld));
    double* dX = c->d_scratch;
    double* dQ = c->d_scratch + (size_t)m * ld;
    CAL_TRY(upload(c, dX, ld, X, n, m));
    Panel P = panel();
    panel_add(P, dX, ld, m);
    std::vector<double> G((size_t)m * m), Ri((size_t)m * m);
    CAL_TRY(gram_host(c, n, P, P, G.data()));  // cholqr.m:5
    if (!dense::chol_upper(m, G.data(), m, R, m))  // :6
        return set_error(c, CAL_ERR_NUMERIC, "chol: Matrix must be positive definite.");
    dense::tri_inv_upper(m, R, m, Ri.data(), m);
    PanelOut out = panel_out(dQ, ld, m);
    CAL_TRY(apply_host(c, n, P, Ri.data(), m, &out, nullptr, 0, nullptr));  // :8 (Q = X/R)
    return download(c, Q, dQ, ld, n, m);
}

int cal_project(cal_ctx* c, int64_t n, int nblocks, const double* const* Q, const int* widths, int m, const double* X,
                int doreorth, double* Xout, double* const* R) {
    Tier1 t1(c);
    CAL_TRY(check_ctx(c, false));
    if (nblocks < 0 || (nblocks > 0 && (!Q || !widths)) || !X || !Xout || n < 1 || m < 1 || m > 32)
        return set_error(c, CAL_ERR_ARG, "project: bad arguments");
    const int64_t ld = ld_for(n);
    int wtot = 0;
    for (int i = 0; i < nblocks; ++i) {
        if (widths[i] < 0 || widths[i] > 128) return set_error(c, CAL_ERR_ARG, "project: block width out of range");
        wtot += widths[i];
    }
    CAL_TRY(ensure_scratch(c, (size_t)(wtot + m) * ld));
    std::vector<double*> dQ(nblocks);
    double* p = c->d_scratch;
    for (int i = 0; i < nblocks; ++i) {
        dQ[i] = p;
        CAL_TRY(upload(c, p, ld, Q[i], n, widths[i]));
        p += (size_t)widths[i] * ld;
    }
    double* dX = p;
    CAL_TRY(upload(c, dX, ld, X, n, m));
    std::vector<std::vector<double>> Rv(nblocks);
    for (int i = 0; i < nblocks; ++i) Rv[i].assign((size_t)std::max(widths[i], 0) * m, 0.0);
    CAL_TRY(project_blocks(c, n, ld, nblocks, dQ, widths, m, dX, doreorth != 0, Rv));
    for (int i = 0; i < nblocks; ++i)
        if (R && R[i] && widths[i] > 0) std::copy(Rv[i].begin(), Rv[i].end(), R[i]);
    return download(c, Xout, dX, ld, n, m);
}

int cal_project_and_normalize(cal_ctx* c, int64_t n, int nblocks, const double* const* Q, const int* widths, int m,
                              const double* X, int doreorth, double* QZ, double* const* RZ, int* reorth, int* rank) {
    Tier1 t1(c);
    CAL_TRY(check_ctx(c, false));
    if (nblocks < 0 || (nblocks > 0 && (!Q || !widths)) || !X || !QZ || n < 1 || m < 1 || m > 32)
        return set_error(c, CAL_ERR_ARG, "projectAndNormalize: bad arguments");
    const int64_t ld = ld_for(n);
    int wtot = 0, nonempty = 0, only = -1;
    for (int i = 0; i < nblocks; ++i) {
        if (widths[i] < 0 || widths[i] > 128) return set_error(c, CAL_ERR_ARG, "block width out of range");
        wtot += widths[i];
        if (widths[i] > 0) {
            nonempty++;
            only = i;
        }
    }
    CAL_TRY(ensure_scratch(c, (size_t)(wtot + 3 * m) * ld));
    std::vector<double*> dQ(nblocks);
    double* p = c->d_scratch;
    for (int i = 0; i < nblocks; ++i) {
        dQ[i] = p;
        CAL_TRY(upload(c, p, ld, Q[i], n, widths[i]));
        p += (size_t)widths[i] * ld;
    }
    double* dX = p;
    double* dY = p + (size_t)m * ld;
    double* dZ = p + (size_t)2 * m * ld;
    CAL_TRY(upload(c, dX, ld, X, n, m));
    std::vector<double> Rm((size_t)m * m);
    int rk = m, re = 0;
    if (nonempty == 1) {
        // the fused device path used by the CA-Lanczos driver
        Panel Qp = panel(), Xp = panel();
        panel_add(Qp, dQ[only], ld, widths[only]);
        panel_add(Xp, dX, ld, m);
        std::vector<double> Rq((size_t)widths[only] * m);
        PNResult res;
        CAL_TRY(project_and_normalize_dev(c, n, Qp, Xp, doreorth != 0, panel_out(dZ, ld, m), Rq.data(), Rm.data(), &res));
        rk = res.rank;
        re = res.reorth ? 1 : 0;
        for (int i = 0; i < nblocks; ++i)
            if (RZ && RZ[i] && widths[i] > 0) std::copy(Rq.begin(), Rq.end(), RZ[i]);
    } else {
        // general restatement (projectAndNormalize.m:3-90) on device panels
        std::vector<std::vector<double>> RZv;
        bool ro = false;
        CAL_TRY(project_and_normalize_blocks_dev(c, n, ld, nblocks, dQ, widths, m, dX, doreorth != 0, dY,
                                                 panel_out(dZ, ld, m), RZv, Rm.data(), &ro, &rk));
        re = ro ? 1 : 0;
        for (int i = 0; i < nblocks; ++i)
            if (RZ && RZ[i] && widths[i] > 0) std::copy(RZv[i].begin(), RZv[i].end(), RZ[i]);
    }
    if (RZ && RZ[nblocks]) std::copy(Rm.begin(), Rm.end(), RZ[nblocks]);
    if (reorth) *reorth = re;
    if (rank) *rank = rk;
    CAL_TRY(download(c, QZ, dZ, ld, n, m));
    return (re && rk < m) ? CAL_WARN_RANK_DEFICIENT : 0;
}

}  // extern "C"
