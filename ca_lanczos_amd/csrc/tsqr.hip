// tsqr.hip -- Householder TSQR on gfx950 (tsqr.m:7-12: [Q,R] = qr(A,0) with
// the positive-diagonal sign fix).
//
// A tall n x m panel (m <= 32) is cut into tiles of TR = 4096/MM rows (MM =
// 8, 16 or 32 >= m): one wave per tile holds it in registers (64 doubles per
// lane: lane l owns rows l + 64 i) and factors it with LAPACK's reflectors
// (dlarfg: beta = -sign(alpha) ||x||, tau = (beta - alpha) / beta,
// v = x / (alpha - beta)).  Every reflector needs ONE wave-wide reduction of
// the vector [||x_below||^2, x'y_{j+1}, ..., x'y_{m-1}] -- all of it is known
// before the reflector is -- done as a fixed DPP butterfly (quad_perm,
// half/full row mirror, row_bcast 15/31) ending in lane 63, so the result is
// bitwise reproducible.  The tile R factors are stacked (one m x m block per
// tile) and the same kernel factors the stack, level by level, until one tile
// remains: that is the TSQR reduction tree (multi-GPU: each rank's local root
// is all-gathered and the global levels run redundantly on every rank).
//
// Q is formed top-down without storing reflectors: each tile RECOMPUTES its
// factorisation from its (unchanged) input -- the same code on the same bits
// gives the same reflectors -- builds its explicit Q factor in place
// (dorg2r), and multiplies it by the m x m block S its parent handed down
// (the root's S is diag(sign(diag R)), the sign fix of tsqr.m:9-12).  At
// level 0 the product is the output Q; above it, it is the S of the children.
//
// HBM traffic at level 0: the panel is read twice (factor, then recompute +
// form) and Q written once; the stack levels are 1/TR-th of that.
#include "cal_internal.hpp"
#include "tsqr_tile.hpp"

namespace cal {

namespace {

using namespace tsqr_tile;

// SRC: 0 stack (block layout), 1 direct columns, 2 formed Z = P M (WP columns),
// 3 (DOWN, level 0) the factored tile UP stored in a.V / a.tb
template <int MM, int SRC, int WP, bool DOWN>
__global__ __launch_bounds__(256) void k_tsqr(TsqrLevelArgs a, TsqrCols P, TsqrQ Q, int64_t ntiles) {
    constexpr int RPL = 64 / MM, TR = 64 * RPL;
    // formed mode: M (wp x m) at [0, WP*MM), the second projection M2 (w2 x m) after it
    __shared__ double Ms[SRC == 2 ? 2 * WP * MM : 1];
    __shared__ double Ss[DOWN ? 4 * MM * MM : 1];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int m = a.m;
    if (SRC == 2) {
        for (int e = threadIdx.x; e < WP * MM; e += 256) {
            const int k = e / MM, c = e % MM;
            Ms[e] = (k < a.wp && c < m) ? a.M[k + (int64_t)c * a.wp] : 0.0;
            Ms[WP * MM + e] = (a.M2 && k < a.w2 && c < m) ? a.M2[k + (int64_t)c * a.w2] : 0.0;
        }
        __syncthreads();
    }
    const int64_t tile = (int64_t)blockIdx.x * 4 + wave;
    if (tile >= ntiles) return;  // whole waves
    const int64_t base = tile * TR;
    const int64_t mm = (int64_t)m * m;
    double x[RPL][MM];
    double tau[MM], beta[MM];
    double* const vt = a.V ? a.V + tile * (int64_t)(64 * RPL * MM) + lane : nullptr;  // lane-contiguous tile store
    if (SRC == 3) {
#pragma unroll
        for (int i = 0; i < RPL; ++i)
#pragma unroll
            for (int c = 0; c < MM; ++c) x[i][c] = vt[(i * MM + c) * 64];
#pragma unroll
        for (int c = 0; c < MM; ++c) {
            tau[c] = a.tb[tile * (2 * MM) + c];
            beta[c] = a.tb[tile * (2 * MM) + MM + c];
        }
    }
    if (SRC == 2) {
        // formed: Z = P M (+ P(:,0:w2) M2), column k outermost so each M entry
        // is read from LDS once per tile, not once per row (the row-inner
        // order re-read all of M for each of the RPL rows and was bound by
        // the LDS return path); per entry the FMA order over k is unchanged
        int64_t rc[RPL];
        bool in[RPL];
#pragma unroll
        for (int i = 0; i < RPL; ++i) {
            const int64_t r = base + lane + 64 * i;
            in[i] = r < a.rows;
            rc[i] = in[i] ? r : 0;
#pragma unroll
            for (int c = 0; c < MM; ++c) x[i][c] = 0.0;
        }
#pragma unroll
        for (int k = 0; k < WP; ++k) {
            double p[RPL];
#pragma unroll
            for (int i = 0; i < RPL; ++i) p[i] = P.p[k][rc[i]];  // host pads p[k >= wp] (zero rows of M)
#pragma unroll
            for (int c = 0; c < MM; ++c) {
                const double mk = Ms[k * MM + c];
#pragma unroll
                for (int i = 0; i < RPL; ++i) x[i][c] = __builtin_fma(p[i], mk, x[i][c]);
            }
        }
        if (a.M2) {
            // projectAndNormalize.m:63: Z = Y - Qp C2 on the ROUNDED
            // Y = X - Qp C (one combined coefficient would lose C2 below
            // u |C|); Qp = the first w2 panel columns (reloaded: cache hits)
#pragma unroll
            for (int k = 0; k < WP; ++k) {
                if (k < a.w2) {
                    double p[RPL];
#pragma unroll
                    for (int i = 0; i < RPL; ++i) p[i] = P.p[k][rc[i]];
#pragma unroll
                    for (int c = 0; c < MM; ++c) {
                        const double mk = Ms[WP * MM + k * MM + c];
#pragma unroll
                        for (int i = 0; i < RPL; ++i) x[i][c] = __builtin_fma(p[i], mk, x[i][c]);
                    }
                }
            }
        }
#pragma unroll
        for (int i = 0; i < RPL; ++i)
#pragma unroll
            for (int c = 0; c < MM; ++c) x[i][c] = in[i] ? x[i][c] : 0.0;
    }
#pragma unroll
    for (int i = 0; i < (SRC >= 2 ? 0 : RPL); ++i) {
        const int64_t r = base + lane + 64 * i;
        const bool in = r < a.rows;
        const int64_t rc = in ? r : 0;
        if (SRC == 0) {
            const int64_t blk = rc / m, rr = rc - blk * m;
            const double* src = a.in + blk * mm + rr;
#pragma unroll
            for (int c = 0; c < MM; ++c) {
                const double v = src[(int64_t)(c < m ? c : 0) * m];
                x[i][c] = (in && c < m) ? v : 0.0;
            }
        } else {
#pragma unroll
            for (int c = 0; c < MM; ++c) {
                const double v = P.p[c][rc];  // host pads p[c >= m] with a valid column
                x[i][c] = (in && c < m) ? v : 0.0;
            }
        }
    }
    if (SRC != 3) tile_geqr2<MM, RPL>(x, tau, beta, m, lane);
    if (!DOWN && vt) {  // level 0: keep the factored tile for the down pass
#pragma unroll
        for (int i = 0; i < RPL; ++i)
#pragma unroll
            for (int c = 0; c < MM; ++c) vt[(i * MM + c) * 64] = x[i][c];
        if (lane < MM) {
            // lane c writes tau[c], beta[c] (the arrays are wave-uniform)
#pragma unroll
            for (int c = 0; c < MM; ++c)
                if (lane == c) {
                    a.tb[tile * (2 * MM) + c] = tau[c];
                    a.tb[tile * (2 * MM) + MM + c] = beta[c];
                }
        }
    }
    if (!DOWN) {
        // R of this tile -> block `tile` of the next level's stack
        if (lane < m) {
            double* dst = a.out + tile * mm + lane;
#pragma unroll
            for (int c = 0; c < MM; ++c)
                if (c < m) dst[(int64_t)c * m] = c < lane ? 0.0 : x[0][c];
        }
        return;
    }
    double* S = Ss + wave * MM * MM;
    if (a.S) {
        const double* src = a.S + tile * mm;
        for (int e = lane; e < MM * MM; e += 64) {
            const int k = e % MM, c = e / MM;
            S[e] = (k < m && c < m) ? src[k + (int64_t)c * m] : 0.0;
        }
    } else {  // root: S = diag(sign(diag R)) (tsqr.m:9-12; sign(0) = 0); lane k writes row k
#pragma unroll
        for (int c = 0; c < MM; ++c) {
            const double sg = beta[c] > 0.0 ? 1.0 : (beta[c] < 0.0 ? -1.0 : 0.0);
            if (lane < MM) S[lane + c * MM] = (lane == c && c < m) ? sg : 0.0;
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    tile_org2r<MM, RPL>(x, tau, m, lane);
    // O = Q_tile S, half of the tile's rows at a time with each S entry read
    // from LDS once per half (per row it was re-read RPL times); per entry
    // the sum over k is in the same order
    constexpr int H = RPL >= 2 ? RPL / 2 : 1;
#pragma unroll
    for (int i0 = 0; i0 < RPL; i0 += H) {
        double o[H][MM];
#pragma unroll
        for (int h = 0; h < H; ++h)
#pragma unroll
            for (int c = 0; c < MM; ++c) o[h][c] = 0.0;
#pragma unroll
        for (int k = 0; k < MM; ++k) {
            if (k < m) {
#pragma unroll
                for (int c = 0; c < MM; ++c) {
                    const double sk = S[k + c * MM];
#pragma unroll
                    for (int h = 0; h < H; ++h) {
                        const double u = x[i0 + h][k] * sk;
                        o[h][c] = o[h][c] + u;
                    }
                }
            }
        }
#pragma unroll
        for (int h = 0; h < H; ++h) {
        const int i = i0 + h;
        const int64_t r = base + lane + 64 * i;
        if (r < a.rows) {
            if (SRC == 0) {
                const int64_t blk = r / m, rr = r - blk * m;
                double* dst = a.out + blk * mm + rr;
#pragma unroll
                for (int c = 0; c < MM; ++c)
                    if (c < m) dst[(int64_t)c * m] = o[h][c];
            } else {
#pragma unroll
                for (int c = 0; c < MM; ++c)
                    if (c < m) Q.p[c][r] = o[h][c];
            }
        }
        }
    }
}

}  // namespace

int tsqr_mm(int m) { return m <= 8 ? 8 : (m <= 16 ? 16 : (m <= 32 ? 32 : 0)); }
int tsqr_tile_rows(int m) {
    const int mm = tsqr_mm(m);
    return mm ? 4096 / mm : 0;
}
bool tsqr_form_ok(int wp, int m) { return (m <= 8 && wp <= 17) || (m > 8 && m <= 16 && wp <= 33); }

hipError_t launch_tsqr(bool down, int src, const TsqrLevelArgs& a, const TsqrCols& P, const TsqrQ& Q,
                       hipStream_t st) {
    const int MM = tsqr_mm(a.m);
    if (!MM || a.rows <= 0) return hipErrorInvalidValue;
    const int64_t tiles = (a.rows + 4096 / MM - 1) / (4096 / MM);
    const dim3 g((unsigned)((tiles + 3) / 4)), b(256);
#define CAL_TQ(MMV, SRCV, WPV)                                                                             \
    do {                                                                                                   \
        if (down) hipLaunchKernelGGL((k_tsqr<MMV, SRCV, WPV, true>), g, b, 0, st, a, P, Q, tiles);          \
        else hipLaunchKernelGGL((k_tsqr<MMV, SRCV, WPV, false>), g, b, 0, st, a, P, Q, tiles);              \
    } while (0)
    if (src == 3) {
        if (!down || !a.V || !a.tb) return hipErrorInvalidValue;
        if (MM == 8) hipLaunchKernelGGL((k_tsqr<8, 3, 0, true>), g, b, 0, st, a, P, Q, tiles);
        else if (MM == 16) hipLaunchKernelGGL((k_tsqr<16, 3, 0, true>), g, b, 0, st, a, P, Q, tiles);
        else hipLaunchKernelGGL((k_tsqr<32, 3, 0, true>), g, b, 0, st, a, P, Q, tiles);
    } else if (src == 2) {
        if (MM == 8 && a.wp <= 17) CAL_TQ(8, 2, 17);
        else if (MM == 16 && a.wp <= 33) CAL_TQ(16, 2, 33);
        else return hipErrorInvalidValue;
    } else if (src == 1) {
        if (MM == 8) CAL_TQ(8, 1, 0);
        else if (MM == 16) CAL_TQ(16, 1, 0);
        else CAL_TQ(32, 1, 0);
    } else {
        if (MM == 8) CAL_TQ(8, 0, 0);
        else if (MM == 16) CAL_TQ(16, 0, 0);
        else CAL_TQ(32, 0, 0);
    }
#undef CAL_TQ
    return hipGetLastError();
}

}  // namespace cal
