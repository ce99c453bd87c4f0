// tsqr.cpp -- the TSQR reduction tree on the device (tsqr.m:7-12).
//
// Levels: level 0 factors the n x m panel tile by tile (tsqr.hip k_tsqr);
// level l+1 factors the stack of level l's tile R factors; the last level has
// one tile (the local root).  With several ranks the local roots are
// all-gathered (RCCL allgather, P m^2 doubles) and the global levels -- the
// same kernel on the gathered stack -- run redundantly on every rank, which
// keeps every rank's R and its S block bit-identical.  Then the tree is
// walked down: each level recomputes its tiles' reflectors, forms their Q
// factors and multiplies them by the parent's S block; level 0 writes Q.
// One host wait per call (for R), after the whole down sweep is enqueued.
#include <algorithm>
#include <cmath>
#include <vector>

#include "cal_internal.hpp"
#include "comm.hpp"
#include "tsqr_plan.hpp"

namespace cal {

bool tsqr_ok(int m) { return m >= 1 && tsqr_mm(m) > 0; }

bool use_tsqr(const cal_ctx* c, int m, bool tier1) {
    if (!tsqr_ok(m)) return false;
    if (c->normalize_kind == 1) return true;
    if (c->normalize_kind == 2) return false;
    return tier1;
}

namespace {

int ensure_tsqr(cal_ctx* c, size_t doubles) {
    if (doubles <= c->tsqr_cap) return 0;
    if (c->d_tsqr) CAL_HIP(c, hipFree(c->d_tsqr));
    c->d_tsqr = nullptr;
    const size_t n = std::max(doubles, (size_t)65536);
    CAL_HIP(c, hipMalloc((void**)&c->d_tsqr, n * sizeof(double)));
    c->tsqr_cap = n;
    return 0;
}

}  // namespace

int tsqr_dev(cal_ctx* c, int64_t n, const Panel& W, const double* dM, int m, const PanelOut& Qout, double* R,
             const double* dM2, int w2) {
    if (!tsqr_ok(m)) return set_error(c, CAL_ERR_UNSUPPORTED, "tsqr: 1..32 columns on the device");
    const int wp = W.total;
    const bool form = dM != nullptr;
    if (form ? !tsqr_form_ok(wp, m) : wp != m) return set_error(c, CAL_ERR_ARG, "tsqr: panel shape");
    if (Qout.total != m) return set_error(c, CAL_ERR_ARG, "tsqr: output shape");
    const int64_t TR = tsqr_tile_rows(m), mm = (int64_t)m * m;
    const int P = c->comm ? c->comm->nranks : 1, me = c->comm ? c->comm->rank : 0;
    // level structure and workspace layout (tsqr_plan.cpp): local levels, then
    // (P > 1) the global levels over the all-gathered local roots
    const TsqrPlan plan = tsqr_plan(n, m, TR, form, P, me);
    const std::vector<TsqrLevelPlan>& lv = plan.lv;
    const size_t nlocal = plan.nlocal;
    CAL_TRY(ensure_tsqr(c, plan.need));
    // level 0's factored tiles (4096 doubles each) and tau / beta, kept by the
    // up pass for the down pass (which then neither re-forms nor re-factors)
    const int MM = tsqr_mm(m);
    const size_t vneed = (size_t)lv[0].tiles * (4096 + 2 * (size_t)MM);
    if (vneed > c->tsqrv_cap) {
        if (c->d_tsqrv) CAL_HIP(c, hipFree(c->d_tsqrv));
        c->d_tsqrv = nullptr;
        CAL_HIP(c, hipMalloc((void**)&c->d_tsqrv, vneed * sizeof(double)));
        c->tsqrv_cap = vneed;
    }
    double* const dV = c->d_tsqrv;
    double* const dTB = c->d_tsqrv + (size_t)lv[0].tiles * 4096;
    double* const ws = c->d_tsqr;
    auto at = [&](int64_t off) -> double* { return off < 0 ? nullptr : ws + off; };

    TsqrCols cols{};
    for (int k = 0; k < kTsqrMaxCols; ++k) {
        const int cc = k < wp ? k : 0;
        int base = 0;
        for (int sg = 0; sg < W.nseg; ++sg) {
            if (cc >= base && cc < base + W.ncol[sg]) cols.p[k] = W.ptr[sg] + (int64_t)(cc - base) * W.ld[sg];
            base += W.ncol[sg];
        }
    }
    TsqrQ qo{};
    for (int j = 0; j < 32; ++j) {
        const int cc = j < m ? j : 0;
        int base = 0;
        for (int sg = 0; sg < Qout.nseg; ++sg) {
            if (cc >= base && cc < base + Qout.ncol[sg]) qo.p[j] = Qout.ptr[sg] + (int64_t)(cc - base) * Qout.ld[sg];
            base += Qout.ncol[sg];
        }
    }
    auto args = [&](size_t l, bool down) {
        const TsqrLevelPlan& L = lv[l];
        TsqrLevelArgs a;
        if (l == 0) {
            a.V = dV;
            a.tb = dTB;
        }
        a.rows = L.rows;
        a.m = m;
        a.wp = wp;
        a.M = dM;
        a.in = at(L.in);
        a.out = at(down ? L.down : L.up);
        a.S = at(L.S);
        a.M2 = dM2;
        a.w2 = w2;
        return a;
    };
    // up the tree
    for (size_t l = 0; l < lv.size(); ++l) {
        if (P > 1 && l == nlocal) CAL_TRY(allgather(c, at(lv[nlocal - 1].up), at(lv[nlocal].in), mm));
        const int t = timer_begin(c, l == 0 ? 1 : 3);
        CAL_HIP(c, launch_tsqr(false, lv[l].src, args(l, false), cols, qo, c->stream));
        timer_end(c, t);
    }
    CAL_TRY(ensure_red(c, mm));
    CAL_HIP(c, hipMemcpyAsync(c->h_red, at(lv.back().up), mm * sizeof(double), hipMemcpyDeviceToHost, c->stream));
    if (!c->orth_event) CAL_HIP(c, hipEventCreateWithFlags(&c->orth_event, hipEventDisableTiming));
    CAL_HIP(c, hipEventRecord(c->orth_event, c->stream));
    // down the tree (queued before the host waits for R)
    for (size_t l = lv.size(); l-- > 0;) {
        const int t = timer_begin(c, l == 0 ? 2 : 3);
        CAL_HIP(c, launch_tsqr(true, l == 0 ? 3 : lv[l].src, args(l, true), cols, qo, c->stream));
        timer_end(c, t);
    }
    if (c->pre_wait) {  // e.g. the next step's matrix powers (lanczos_step)
        auto hook = std::move(c->pre_wait);
        c->pre_wait = nullptr;
        CAL_TRY(hook());
    }
    CAL_HIP(c, hipEventSynchronize(c->orth_event));
    c->small_pending = false;
    // R = diag(sign(diag R)) R (tsqr.m:9-10; sign(0) = 0 zeroes the row)
    for (int j = 0; j < m; ++j)
        for (int i = 0; i < m; ++i) {
            const double rii = c->h_red[i + (size_t)i * m];
            const double d = rii > 0.0 ? 1.0 : (rii < 0.0 ? -1.0 : 0.0);
            R[i + (size_t)j * m] = i > j ? 0.0 : d * c->h_red[i + (size_t)j * m];
        }
    return 0;
}

}  // namespace cal
