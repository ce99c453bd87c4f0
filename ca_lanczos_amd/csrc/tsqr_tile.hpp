// tsqr_tile.hpp -- the register-tile Householder QR shared by the TSQR
// kernels (tsqr.hip: the generic tree; tsqr_fold.hip: the fused CA-step
// TSQR).  One wave holds a tile of 64 * RPL rows x MM columns (lane l owns
// rows l + 64 i) and applies LAPACK's reflectors (dlarfg conventions); every
// wave-wide reduction is a fixed DPP butterfly, so a tile factored twice from
// the same bits gives the same reflectors.  Device code only.
#pragma once

#include <hip/hip_runtime.h>

namespace cal {
namespace tsqr_tile {

// DPP move of a double (two 32-bit halves); disabled rows yield 0
template <int CTRL, int ROWMASK>
__device__ __forceinline__ double dpp_f64(double v) {
    const long long b = __builtin_bit_cast(long long, v);
    const int lo = __builtin_amdgcn_update_dpp(0, (int)b, CTRL, ROWMASK, 0xF, false);
    const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), CTRL, ROWMASK, 0xF, false);
    return __builtin_bit_cast(double, ((long long)hi << 32) | (long long)(unsigned)lo);
}

__device__ __forceinline__ double readlane_f64(double v, int lane) {
    const long long b = __builtin_bit_cast(long long, v);
    const int lo = __builtin_amdgcn_readlane((int)b, lane);
    const int hi = __builtin_amdgcn_readlane((int)(b >> 32), lane);
    return __builtin_bit_cast(double, ((long long)hi << 32) | (long long)(unsigned)lo);
}

// sum over the 64 lanes, returned wave-uniform; fixed order
__device__ __forceinline__ double wave_allsum(double v) {
    v = v + dpp_f64<0xB1, 0xF>(v);   // quad_perm [1,0,3,2]
    v = v + dpp_f64<0x4E, 0xF>(v);   // quad_perm [2,3,0,1]
    v = v + dpp_f64<0x141, 0xF>(v);  // row_half_mirror
    v = v + dpp_f64<0x140, 0xF>(v);  // row_mirror
    v = v + dpp_f64<0x142, 0xA>(v);  // row_bcast:15 into rows 1, 3
    v = v + dpp_f64<0x143, 0xC>(v);  // row_bcast:31 into rows 2, 3
    return readlane_f64(v, 63);
}

// Householder QR of the register tile a (rows lane + 64 i, m <= MM columns,
// zero outside): R in the upper triangle of rows 0..m-1 (row j = lane j, i = 0;
// R(j,j) also in beta[j]), reflector j below the diagonal of column j, tau[j].
template <int MM, int RPL>
__device__ __forceinline__ void tile_geqr2(double (&a)[RPL][MM], double (&tau)[MM], double (&beta)[MM], int m,
                                           int lane) {
#pragma unroll
    for (int j = 0; j < MM; ++j) {
        tau[j] = 0.0;
        beta[j] = 0.0;
        if (j < m) {
        double d[MM];
#pragma unroll
        for (int c = j; c < MM; ++c) d[c] = 0.0;
#pragma unroll
        for (int i = 0; i < RPL; ++i) {
            const bool below = lane + 64 * i > j;
            const double x = below ? a[i][j] : 0.0;
#pragma unroll
            for (int c = j; c < MM; ++c) {
                const double t = x * a[i][c];
                d[c] = d[c] + t;
            }
        }
#pragma unroll
        for (int c = j; c < MM; ++c)
            if (c < m) d[c] = wave_allsum(d[c]);
        const double alpha = readlane_f64(a[0][j], j);
        double t = 0.0, b = alpha, scal = 0.0;
        if (d[j] != 0.0) {  // dlarfg: xnorm == 0 -> H = I
            const double aa = alpha * alpha;
            const double nrm = sqrt(aa + d[j]);
            b = alpha >= 0.0 ? -nrm : nrm;
            t = (b - alpha) / b;
            scal = 1.0 / (alpha - b);
        }
        tau[j] = t;
        beta[j] = b;
        // tau * w_c, w_c = v'y_c = y_c(j) + scal * x'y_c (v_j = 1), in place of d
#pragma unroll
        for (int c = j + 1; c < MM; ++c) {
            if (c < m) {
                const double u = scal * d[c];
                const double w = readlane_f64(a[0][c], j) + u;
                d[c] = t * w;
            } else {
                d[c] = 0.0;
            }
        }
#pragma unroll
        for (int i = 0; i < RPL; ++i) {
            const int row = lane + 64 * i;
            if (row > j) {
                const double v = scal * a[i][j];
                a[i][j] = v;
#pragma unroll
                for (int c = j + 1; c < MM; ++c) {
                    const double u = d[c] * v;
                    a[i][c] = a[i][c] - u;
                }
            } else if (row == j) {  // the pivot row: y_c(j) - tau w_c
                a[i][j] = b;
#pragma unroll
                for (int c = j + 1; c < MM; ++c) a[i][c] = a[i][c] - d[c];
            }
        }
        }
    }
}

// Explicit Q = H_0 ... H_{m-1} [I; 0] in place over the reflectors (dorg2r).
template <int MM, int RPL>
__device__ __forceinline__ void tile_org2r(double (&a)[RPL][MM], const double (&tau)[MM], int m, int lane) {
#pragma unroll
    for (int jj = 0; jj < MM; ++jj) {
        const int j = MM - 1 - jj;
        if (j < m) {
        const double t = tau[j];
        if (j < m - 1) {
            // w_c = v' q_c over rows >= j (v_j = 1), c = j+1..m-1
            double d[MM];
#pragma unroll
            for (int c = j + 1; c < MM; ++c) d[c] = 0.0;
#pragma unroll
            for (int i = 0; i < RPL; ++i) {
                const int row = lane + 64 * i;
                const double v = row > j ? a[i][j] : (row == j ? 1.0 : 0.0);
#pragma unroll
                for (int c = j + 1; c < MM; ++c) {
                    const double u = v * a[i][c];
                    d[c] = d[c] + u;
                }
            }
#pragma unroll
            for (int c = j + 1; c < MM; ++c) d[c] = c < m ? t * wave_allsum(d[c]) : 0.0;
#pragma unroll
            for (int i = 0; i < RPL; ++i) {
                const int row = lane + 64 * i;
                if (row >= j) {
                    const double v = row > j ? a[i][j] : 1.0;
#pragma unroll
                    for (int c = j + 1; c < MM; ++c) {
                        const double u = d[c] * v;
                        a[i][c] = a[i][c] - u;
                    }
                }
            }
        }
#pragma unroll
        for (int i = 0; i < RPL; ++i) {
            const int row = lane + 64 * i;
            const double v = a[i][j];
            const double mt = -t;
            a[i][j] = row > j ? mt * v : (row == j ? 1.0 - t : 0.0);
        }
        }
    }
}

// ---- block-cooperative variants: one tile spread over the NW waves of a
// block (wave w holds tile rows w * 64 * RPLW + lane + 64 i), for the short
// launches of the tree above level 0 whose wall time is one tile's latency.
// Per reflector: wave partial sums (DPP butterfly), then the NW partials and
// the pivot row through LDS (xlds: 2 * NW * 2 * MM doubles, double-buffered
// by column parity) summed in wave order -- every wave computes the same
// tau / beta / w_c.  Called by all NW waves of the block (barriers inside).
template <int MM, int RPLW, int NW>
__device__ __forceinline__ void tile_geqr2_blk(double (&a)[RPLW][MM], double (&tau)[MM], double (&beta)[MM], int m,
                                               int lane, int wave, double* xlds) {
#pragma unroll
    for (int j = 0; j < MM; ++j) {
        tau[j] = 0.0;
        beta[j] = 0.0;
        if (j < m) {
            double d[MM];
#pragma unroll
            for (int c = j; c < MM; ++c) d[c] = 0.0;
#pragma unroll
            for (int i = 0; i < RPLW; ++i) {
                const bool below = wave * 64 * RPLW + lane + 64 * i > j;
                const double x = below ? a[i][j] : 0.0;
#pragma unroll
                for (int c = j; c < MM; ++c) {
                    const double t = x * a[i][c];
                    d[c] = d[c] + t;
                }
            }
#pragma unroll
            for (int c = j; c < MM; ++c)
                if (c < m) d[c] = wave_allsum(d[c]);
            double pv[MM];  // the pivot row (wave 0, lane j, slot 0)
#pragma unroll
            for (int c = j; c < MM; ++c) pv[c] = readlane_f64(a[0][c], j);
            double* buf = xlds + (j & 1) * (NW * 2 * MM);
            if (lane == 0) {
#pragma unroll
                for (int c = j; c < MM; ++c) {
                    buf[wave * 2 * MM + c] = d[c];
                    if (wave == 0) buf[MM + c] = pv[c];
                }
            }
            __syncthreads();
#pragma unroll
            for (int c = j; c < MM; ++c) {
                double sum = buf[c];
#pragma unroll
                for (int w = 1; w < NW; ++w) sum = sum + buf[w * 2 * MM + c];
                d[c] = sum;
                pv[c] = buf[MM + c];
            }
            const double alpha = pv[j];
            double t = 0.0, b = alpha, scal = 0.0;
            if (d[j] != 0.0) {  // dlarfg: xnorm == 0 -> H = I
                const double aa = alpha * alpha;
                const double nrm = sqrt(aa + d[j]);
                b = alpha >= 0.0 ? -nrm : nrm;
                t = (b - alpha) / b;
                scal = 1.0 / (alpha - b);
            }
            tau[j] = t;
            beta[j] = b;
#pragma unroll
            for (int c = j + 1; c < MM; ++c) {
                if (c < m) {
                    const double u = scal * d[c];
                    const double w = pv[c] + u;
                    d[c] = t * w;
                } else {
                    d[c] = 0.0;
                }
            }
#pragma unroll
            for (int i = 0; i < RPLW; ++i) {
                const int row = wave * 64 * RPLW + lane + 64 * i;
                if (row > j) {
                    const double v = scal * a[i][j];
                    a[i][j] = v;
#pragma unroll
                    for (int c = j + 1; c < MM; ++c) {
                        const double u = d[c] * v;
                        a[i][c] = a[i][c] - u;
                    }
                } else if (row == j) {
                    a[i][j] = b;
#pragma unroll
                    for (int c = j + 1; c < MM; ++c) a[i][c] = a[i][c] - d[c];
                }
            }
        }
    }
}

template <int MM, int RPLW, int NW>
__device__ __forceinline__ void tile_org2r_blk(double (&a)[RPLW][MM], const double (&tau)[MM], int m, int lane,
                                               int wave, double* xlds) {
#pragma unroll
    for (int jj = 0; jj < MM; ++jj) {
        const int j = MM - 1 - jj;
        if (j < m) {
            const double t = tau[j];
            if (j < m - 1) {
                double d[MM];
#pragma unroll
                for (int c = j + 1; c < MM; ++c) d[c] = 0.0;
#pragma unroll
                for (int i = 0; i < RPLW; ++i) {
                    const int row = wave * 64 * RPLW + lane + 64 * i;
                    const double v = row > j ? a[i][j] : (row == j ? 1.0 : 0.0);
#pragma unroll
                    for (int c = j + 1; c < MM; ++c) {
                        const double u = v * a[i][c];
                        d[c] = d[c] + u;
                    }
                }
#pragma unroll
                for (int c = j + 1; c < MM; ++c)
                    if (c < m) d[c] = wave_allsum(d[c]);
                double* buf = xlds + (j & 1) * (NW * 2 * MM);
                if (lane == 0) {
#pragma unroll
                    for (int c = j + 1; c < MM; ++c) buf[wave * 2 * MM + c] = d[c];
                }
                __syncthreads();
#pragma unroll
                for (int c = j + 1; c < MM; ++c) {
                    double sum = buf[c];
#pragma unroll
                    for (int w = 1; w < NW; ++w) sum = sum + buf[w * 2 * MM + c];
                    d[c] = c < m ? t * sum : 0.0;
                }
#pragma unroll
                for (int i = 0; i < RPLW; ++i) {
                    const int row = wave * 64 * RPLW + lane + 64 * i;
                    if (row >= j) {
                        const double v = row > j ? a[i][j] : 1.0;
#pragma unroll
                        for (int c = j + 1; c < MM; ++c) {
                            const double u = d[c] * v;
                            a[i][c] = a[i][c] - u;
                        }
                    }
                }
            }
#pragma unroll
            for (int i = 0; i < RPLW; ++i) {
                const int row = wave * 64 * RPLW + lane + 64 * i;
                const double v = a[i][j];
                const double mt = -t;
                a[i][j] = row > j ? mt * v : (row == j ? 1.0 - t : 0.0);
            }
        }
    }
}

}  // namespace tsqr_tile
}  // namespace cal
