// tsqr_fold.hip -- projectAndNormalize with the Householder TSQR normalize
// (projectAndNormalize.m:3-90, normalize.m:14, tsqr.m:7-12) for one CA block
// (m <= 8 new columns against a previous block Qp of w <= 9 columns), fused
// into few launches with no host round trip:
//
//   P1      [Qp | X]'X on the row Gram sweep (blockorth.cpp): C = Qp'X (read
//           by k_fold_up straight from the reduced tile) and the norms of
//           the reorth test of :45-52 (evaluated in k_fold_coef1).
//   up      k_fold_up: Y = X - Qp C formed per row (project.m:30), the
//           register-tile Householder QR of Y (256-row tiles, one per wave),
//           and -- from the same registers -- the Gram [Qp | Y]'[Qp | Y] on
//           the matrix cores, i.e. the second projection's C2 = Qp'Y (:63).
//   tree    k_fold_tree: the stacked tile R factors, 256 per 2048-row tile,
//           level by level to the local root (one block per tile).
//   coef1   k_fold_coef1: Y = Q_Y R_Y from the tree.  With the second
//           projection Z = Y - Qp C2, Z'Z = Y'Y - C2'C2, so with W = C2 R_Y^-1:
//           R_Z = U R_Y, U = chol(I - W'W), and Q_Z = Q_Y U^-1 - Qp W U^-1.
//           The root's S block becomes diag(sign) U^-1 (tsqr.m:9-12's sign fix
//           folded in) and K = W U^-1 is the down pass's correction.
//           I - W'W is perfectly conditioned when the first projection did
//           its job (||W|| << 1): the explicit-Z path (blockorth.cpp pn_tsqr)
//           is taken instead when ||W||_F > 1/2.  R = R_Z, RY = C + C2
//           (:71-73), the flag, published to pinned host memory.
//   down    k_fold_down: level 0, Q = Q_tile S - Qp K, one store.  Every
//           tile's Q factor is used in its compact-WY form Q = E - V M,
//           M = T V_top' (dlarft's T from V'V and tau): the up pass stores M
//           per upper tile, so a level-0 wave forms its own S block by walking
//           the tree down from the root's S through 8 x 8 products (no
//           launch per level), and its 256 rows as E S - V (M S) (no
//           reflector-by-reflector sweep).
//
// HBM traffic per block (n rows): P1 (w+m)·8n, up (w+m)·8n + m·8n (the
// factored tiles), down m·8n (tiles) + w·8n (Qp, only when the second
// projection runs) + m·8n (Q).  Everything above level 0 is n/64 rows.
#include "cal_internal.hpp"
#include "tsqr_tile.hpp"

#include <vector>

namespace cal {

namespace {

using namespace tsqr_tile;
typedef double fd4 __attribute__((ext_vector_type(4)));
typedef double fd2 __attribute__((ext_vector_type(2)));

constexpr int FM = 8;             // register tile width (m <= 8)
constexpr int L0RPL = 4;          // rows per lane of a level-0 tile
constexpr int FTR0 = 64 * L0RPL;  // 256 rows per level-0 tile
constexpr int FTPB = 4;           // level-0 tiles (waves) per block
constexpr int UW = 4;             // waves of an upper-level block (one tile per block)
constexpr int URPL = 2;           // rows per lane of each wave's share of an upper tile
constexpr int FTR = 64 * URPL * UW;  // 512 rows per upper tile
constexpr int FG = FTR / FM;      // R factors (of the level below) per upper tile: 64
constexpr int FTLD = 17;        // padded LDS row of the Gram transpose
// timing-probe switches (tools/fold_probe.hip; never set in the library)
#ifndef FOLD_PROBE
#define FOLD_PROBE 0
#endif
constexpr int kProbe = FOLD_PROBE;  // bit 1: no Gram, 2: no tile QR, 3: no tile store, 4: tree level 1 only
#ifndef FOLD_UP_WPE
#define FOLD_UP_WPE 4  // k_fold_up waves per SIMD (VGPR budget 512 / WPE)
#endif
#ifndef FOLD_DOWN_WPE
#define FOLD_DOWN_WPE 3  // k_fold_down waves per SIMD (150 VGPRs)
#endif
#ifndef CAL_FOLD_DOWN_NT
#define CAL_FOLD_DOWN_NT 1  // non-temporal Q stores in k_fold_down (tuning switch)
#endif

__device__ __forceinline__ fd4 fmfma(double a, double b, fd4 c) {
    return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ void fwsync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// factored register tile <-> lane-contiguous storage (64 doubles per lane slot)
#ifndef CAL_FOLD_TILE_NT
// bit 0: non-temporal stores of the factored tiles (up), bit 1: their loads
// (down): the tiles (636 MB at n = 9.94 M) outgrow the Infinity Cache before
// the down pass reads them back in the same order (707/708 -> 711/718
// outer-it/s on the TSQR headline, same box, profiles/r05/ab/)
#define CAL_FOLD_TILE_NT 3
#endif
template <int RPL>
__device__ __forceinline__ void fstore_tile(double* V, int lane, const double (&x)[RPL][FM]) {
    double* vt = V + lane;
#pragma unroll
    for (int i = 0; i < RPL; ++i)
#pragma unroll
        for (int c = 0; c < FM; ++c) {
            if (CAL_FOLD_TILE_NT & 1) __builtin_nontemporal_store(x[i][c], &vt[(i * FM + c) * 64]);
            else vt[(i * FM + c) * 64] = x[i][c];
        }
}
template <int RPL>
__device__ __forceinline__ void fload_tile(const double* V, int lane, double (&x)[RPL][FM]) {
    const double* vt = V + lane;
#pragma unroll
    for (int i = 0; i < RPL; ++i)
#pragma unroll
        for (int c = 0; c < FM; ++c)
            x[i][c] = (CAL_FOLD_TILE_NT & 2) ? __builtin_nontemporal_load(&vt[(i * FM + c) * 64]) : vt[(i * FM + c) * 64];
}
__device__ __forceinline__ void fstore_tb(double* tb, int lane, const double (&tau)[FM], const double (&beta)[FM]) {
#pragma unroll
    for (int c = 0; c < FM; ++c)
        if (lane == c) {
            tb[c] = tau[c];
            tb[FM + c] = beta[c];
        }
}
__device__ __forceinline__ void fload_tau(const double* tb, double (&tau)[FM]) {
#pragma unroll
    for (int c = 0; c < FM; ++c) tau[c] = tb[c];
}
// R of a factored tile (row j in lane j, slot 0) -> an 8 x 8 column-major
// block (zeros below the diagonal and outside m x m); lanes 0..7 write
__device__ __forceinline__ void fput_R(double* Rb, int lane, int m, const double (&x0)[FM]) {
    if (lane < FM) {
#pragma unroll
        for (int c = 0; c < FM; ++c) Rb[c * FM + lane] = (lane < m && c >= lane && c < m) ? x0[c] : 0.0;
    }
}
// rows [r0, r0 + 64 RPL) of a stack of R blocks into a register tile: block
// b holds stack rows 8b .. 8b+7 (its 8 x 8 column-major R; rows >= m are
// zero, which leaves the R of the stack unchanged), zero past `rows`
template <int RPL>
__device__ __forceinline__ void fload_stack(const double* Rs, int64_t r0, int64_t rows, int lane,
                                            double (&x)[RPL][FM]) {
#pragma unroll
    for (int i = 0; i < RPL; ++i) {
        const int64_t r = r0 + lane + 64 * i;
        const bool in = r < rows;
        const double* src = Rs + (in ? (r >> 3) * 64 + (r & 7) : 0);
#pragma unroll
        for (int c = 0; c < FM; ++c) {
            const double v = src[c * FM];
            x[i][c] = in ? v : 0.0;
        }
    }
}
// O = Q S for the register rows (S 8 x 8 column-major in LDS, k < m ascending)
__device__ __forceinline__ void fmul_S(const double (&q)[FM], const double* S, int m, double (&o)[FM]) {
#pragma unroll
    for (int c = 0; c < FM; ++c) o[c] = 0.0;
#pragma unroll
    for (int k = 0; k < FM; ++k) {
        if (k < m) {
            // row k of S read right before use (see k_fold_up's C rows)
#pragma unroll
            for (int c = 0; c < FM; ++c) asm volatile("" : "+v"(o[c]));
#pragma unroll
            for (int c = 0; c < FM; ++c) {
                const double u = q[k] * S[k + c * FM];
                o[c] = o[c] + u;
            }
        }
    }
}

// ---- compact WY (dlarft, forward, columnwise) ------------------------------
// V, the reflector matrix of a factored tile: unit diagonal, zero above it,
// the stored reflector entries below (columns >= m zero).  Q = H_0 ... H_{m-1}
// [I; 0] = E - V M with M = T V_top' (m x m), T the upper triangular factor
// of H_0 ... H_{m-1} = I - V T V'.
__device__ __forceinline__ double fv(double x, int64_t row, int c, int m) {
    return c < m ? (row > c ? x : (row == c ? 1.0 : 0.0)) : 0.0;
}
// a factored register tile (rows row0 + 64 i) turned into V in place
template <int RPL>
__device__ __forceinline__ void fv_tile(double (&x)[RPL][FM], int64_t row0, int m) {
#pragma unroll
    for (int i = 0; i < RPL; ++i)
#pragma unroll
        for (int c = 0; c < FM; ++c) x[i][c] = fv(x[i][c], row0 + 64 * i, c, m);
}
// this lane's rows' part of V'V (x holds V, see fv_tile), strictly upper
// entries G(a, b), a < b, numbered e = b (b - 1) / 2 + a; entries E0 .. E0 +
// NE - 1 into g
constexpr int NG = FM * (FM - 1) / 2;
__device__ __forceinline__ constexpr int gram_b(int e) {
    int b = 1;
    for (int q = 2; q < FM; ++q) b = e >= q * (q - 1) / 2 ? q : b;
    return b;
}
template <int RPL, int E0, int NE>
__device__ __forceinline__ void fgram_v(const double (&x)[RPL][FM], double (&g)[NE]) {
#pragma unroll
    for (int e = 0; e < NE; ++e) g[e] = 0.0;
#pragma unroll
    for (int i = 0; i < RPL; ++i) {
#pragma unroll
        for (int e = 0; e < NE; ++e) {
            const int b = gram_b(E0 + e), a = E0 + e - b * (b - 1) / 2;
            g[e] = __builtin_fma(x[i][a], x[i][b], g[e]);
        }
    }
}
// The NE wave sums of g (fixed order) into out[a + 8 b] (LDS).  One DPP step
// folds lane pairs; the even lanes' pair sums go through the wave's LDS
// scratch (32 x NE doubles), where lanes 2e and 2e + 1 each add one half of
// value e's 32 rows and a second DPP step joins the halves: ~150
// instructions for the 28 sums instead of ~560 for 28 butterflies.
template <int E0, int NE>
__device__ __forceinline__ void wave_gram_sums(double (&g)[NE], double* scratch, double* out, int lane) {
#pragma unroll
    for (int e = 0; e < NE; ++e) g[e] = g[e] + dpp_f64<0xB1, 0xF>(g[e]);  // quad_perm [1,0,3,2]
    if ((lane & 1) == 0) {
#pragma unroll
        for (int e = 0; e < NE; ++e) scratch[(lane >> 1) * NE + e] = g[e];
    }
    fwsync();
    const int e = lane >> 1, h = lane & 1;
    double s = 0.0;
    if (e < NE) {
#pragma unroll
        for (int r = 0; r < 16; ++r) s = s + scratch[(16 * h + r) * NE + e];
    }
    const double sw = dpp_f64<0xB1, 0xF>(s);  // the partner lane's half (all lanes active)
    const double lo = h ? sw : s, hi = h ? s : sw;
    if (e < NE && h == 0) {
        const int b = gram_b(E0 + e), a = E0 + e - b * (b - 1) / 2;
        out[a + FM * b] = lo + hi;
    }
    fwsync();
}
// all NG sums in two halves (half the partial registers live at a time)
template <int RPL>
__device__ __forceinline__ void wave_gram(const double (&x)[RPL][FM], double* scratch, double* out, int lane) {
    // (scheduling barriers: the halves' partial products must not overlap)
    __builtin_amdgcn_sched_barrier(0);
    {
        double g[NG / 2];
        fgram_v<RPL, 0, NG / 2>(x, g);
        wave_gram_sums<0, NG / 2>(g, scratch, out, lane);
    }
    __builtin_amdgcn_sched_barrier(0);
    {
        double g[NG - NG / 2];
        fgram_v<RPL, NG / 2, NG - NG / 2>(x, g);
        wave_gram_sums<NG / 2, NG - NG / 2>(g, scratch, out, lane);
    }
    __builtin_amdgcn_sched_barrier(0);
}
// Row r of T, then row r of M = T V_top' (r < m; zero otherwise).  G: V'V
// (entry a + 8 b, a < b), Vt: V's top 8 rows (entry r + 8 c), both in LDS.
// T(r, r) = tau_r, T(r, i) = -tau_i sum_{r <= k < i} T(r, k) G(k, i): a row of
// T depends only on its own earlier entries.
__device__ __forceinline__ void fwy_row(const double* G, const double* Vt, const double (&tau)[FM], int m, int r,
                                        double (&mrow)[FM]) {
    double t[FM];
#pragma unroll
    for (int i = 0; i < FM; ++i) {
        double s = 0.0;
#pragma unroll
        for (int k = 0; k < i; ++k) s = k >= r ? __builtin_fma(t[k], G[k + FM * i], s) : s;
        t[i] = i < m ? (i == r ? tau[i] : (i > r ? -tau[i] * s : 0.0)) : 0.0;
    }
#pragma unroll
    for (int j = 0; j < FM; ++j) {
        double s = 0.0;
#pragma unroll
        for (int k = 0; k <= j; ++k) s = k >= r ? __builtin_fma(t[k], Vt[j + FM * k], s) : s;
        mrow[j] = (j < m && r < m) ? s : 0.0;
    }
}
// M of an upper-level tile spread over the NW waves of a block (rows wave *
// 64 RPLW + lane + 64 i) into Mout (entry r + 8 c); x is turned into V.
// All waves call it.
template <int RPLW, int NW>
__device__ __forceinline__ void fold_wy_blk(double (&x)[RPLW][FM], const double (&tau)[FM], int m, int lane,
                                            int wave, double (*gw)[64], double (*scr)[32 * (NG - NG / 2)], double* Vt,
                                            double* __restrict__ Mout) {
    fv_tile<RPLW>(x, (int64_t)wave * 64 * RPLW + lane, m);
    wave_gram<RPLW>(x, scr[wave], gw[wave], lane);
    if (wave == 0 && lane < FM) {
#pragma unroll
        for (int c = 0; c < FM; ++c) Vt[lane + FM * c] = x[0][c];
    }
    __syncthreads();
    if (wave == 0) {
        double sum = gw[0][lane];
#pragma unroll
        for (int v = 1; v < NW; ++v) sum = sum + gw[v][lane];
        fwsync();
        gw[0][lane] = sum;
        fwsync();
        if (lane < FM) {
            double mrow[FM];
            fwy_row(gw[0], Vt, tau, m, lane, mrow);
#pragma unroll
            for (int j = 0; j < FM; ++j) Mout[lane + FM * j] = mrow[j];
        }
    }
}

}  // namespace

// Level-0 tile formation (256 rows, chunk i = rows base + lane + 64 i):
// Y = X - Qp C (project.m:30; the product first, k ascending) into the
// register tile x; with GRAM also the rows [Qp(0:9) | Y] through the wave's
// LDS rows tlw onto the matrix cores: one v_mfma_f64_16x16x4f64 per 4 rows
// with A = the rows' first 16 columns, B = the 16 columns from column 9 on,
// so acc(i, j) accumulates C2(i, j) = Qp(:,i)'Y(:,j) for i < 9, j < 8 (the
// other outputs are unused; tlw has FTLD + 16 spare doubles for B's tail).
template <bool GRAM>
__device__ __forceinline__ void fform(const ColList P, const double* Cs, double* tlw, int64_t base, int64_t n,
                                      int lane, int m, int w, double (&x)[L0RPL][FM], fd4& acc) {
    const int c16 = lane & 15, g = lane >> 4;
    double p[17];
    auto load = [&](int i) {
        const int64_t r = base + lane + 64 * i;
        const int64_t rr = r < n ? r : n - 1;  // a valid row; masked below
#pragma unroll
        for (int k = 0; k < 17; ++k) p[k] = P.p[k][rr];
    };
    load(0);
#pragma unroll
    for (int i = 0; i < L0RPL; ++i) {
        // keep chunk i's loads and LDS traffic inside its iteration (the
        // scheduler would otherwise hoist every chunk's loads and spill)
        asm volatile("" ::: "memory");
        const bool in = base + lane + 64 * i < n;
        double t[FM];
#pragma unroll
        for (int cc = 0; cc < FM; ++cc) t[cc] = 0.0;
#pragma unroll
        for (int k = 0; k < 9; ++k) {
            // one C row per k, read right before use: the pin takes the
            // accumulators as operands, so row k's FMAs retire before row
            // k+1's broadcasts issue (otherwise all 72 C values are held)
#pragma unroll
            for (int cc = 0; cc < FM; ++cc) asm volatile("" : "+v"(t[cc]));
#pragma unroll
            for (int cc = 0; cc < FM; cc += 2) {
                const fd2 v = *reinterpret_cast<const fd2*>(&Cs[k * FM + cc]);
                t[cc] = __builtin_fma(p[k], v[0], t[cc]);
                t[cc + 1] = __builtin_fma(p[k], v[1], t[cc + 1]);
            }
        }
#pragma unroll
        for (int cc = 0; cc < FM; ++cc) x[i][cc] = (in && cc < m) ? p[9 + cc] - t[cc] : 0.0;
        if (GRAM) {
            double* trow = tlw + lane * FTLD;
#pragma unroll
            for (int cc = 0; cc < 9; ++cc) trow[cc] = (in && cc < w) ? p[cc] : 0.0;
#pragma unroll
            for (int cc = 0; cc < 8; ++cc) trow[9 + cc] = x[i][cc];
        }
        if (i + 1 < L0RPL) load(i + 1);  // the next chunk's loads fly during the Gram
        if (GRAM) {
            fwsync();
            if (!(kProbe & 2)) {
#pragma unroll
                for (int kk = 0; kk < 16; ++kk) {
                    const int row = 4 * kk + g;
                    const double av = tlw[row * FTLD + c16];
                    const double bv = tlw[row * FTLD + 9 + c16];
                    acc = fmfma(av, bv, acc);
                }
            }
            fwsync();
        }
    }
}

// P: column pointers, slots 0..8 the previous block Qp (slots >= w padded
// with a valid column: their coefficients are zero), slots 9..16 X (slots
// >= 9 + m padded).  One 256-row tile per wave, 4 independent waves per
// block (no block-level step: a serial tail would hold the block's slots).
// Registers are kept under 168 (3 waves per SIMD) so that 12 waves per CU
// keep their next chunk's 17 column loads in flight.
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(FOLD_UP_WPE))) void k_fold_up(ColList P, FoldArgs a) {
    __shared__ double Cs[9 * FM];
    __shared__ double tl[FTPB][64 * FTLD + 16];  // per-wave Gram transpose; then the block's partials
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int c16 = lane & 15, g = lane >> 4;
    const int m = a.m, w = a.w;
    const int64_t n = a.n;
    const int b = blockIdx.x;
    {  // C = Qp'X straight from the reduced P1 tile [Qp(0:nq) | X]'[...] (+ Qp column 8)
        const int nq = w < 8 ? w : 8;
        for (int e = tid; e < 9 * FM; e += 256) {
            const int k = e / FM, cc = e % FM;
            Cs[e] = (k < w && cc < m) ? (k < 8 ? a.C[k + (nq + cc) * 16] : a.C[256 + nq + cc]) : 0.0;
        }
    }
    __syncthreads();
    const int64_t ntiles = (n + FTR0 - 1) / FTR0;
    const int64_t tile = (int64_t)b * FTPB + wave;
    fd4 acc = fd4{0.0, 0.0, 0.0, 0.0};
    if (tile < ntiles) {
        const int64_t base = tile * FTR0;
        double x[L0RPL][FM];
        double tau[FM], beta[FM];
        fform<true>(P, Cs, tl[wave], base, n, lane, m, w, x, acc);
        if (!(kProbe & 4)) tile_geqr2<FM, L0RPL>(x, tau, beta, m, lane);
        if (a.V0 && !(kProbe & 8)) {  // stored for the down pass (V0 null: it re-forms the tile)
            fstore_tile<L0RPL>(a.V0 + tile * (64 * L0RPL * FM), lane, x);
            fstore_tb(a.tb0 + tile * (2 * FM), lane, tau, beta);
        }
        fput_R(a.R0 + tile * 64, lane, m, x[0]);
    }
    __syncthreads();  // the transposes are done (tl is reused below)
    // the block's C2 partial: entry i + 9 j (i < 9, j < 8), entry-major
    double* red = &tl[0][0];
    if (wave > 0) {
#pragma unroll
        for (int r = 0; r < 4; ++r) red[((wave - 1) * 64 + lane) * 4 + r] = acc[r];
    }
    __syncthreads();
    if (wave == 0) {
        const int64_t nb = a.nblk;
        double* out = a.partial + b;
#pragma unroll
        for (int r = 0; r < 3; ++r) {
            double v = acc[r];
            v = v + red[(0 * 64 + lane) * 4 + r];
            v = v + red[(1 * 64 + lane) * 4 + r];
            v = v + red[(2 * 64 + lane) * 4 + r];
            const int i = g + 4 * r, j = c16;  // acc[r] of lane l holds D(g + 4r, c16)
            if (i < 9 && j < 8) out[(int64_t)(i + 9 * j) * nb] = v;
        }
    }
}

// The tree above level 0: one 512-row tile (64 R factors of the level below,
// 8 rows each) per block, spread over its 4 waves (128 rows each) with the
// block-cooperative tile QR -- these launches are latency-bound, one tile's
// QR deep: ~18 us for one wave alone, ~8 us over 4 waves (2048-row tiles over
// 8 or 16 waves, one level fewer, measured 2x and 9x slower per level: the
// per-reflector LDS exchange grows with the waves).  Level L = 1 .. nlev, the
// last one the root (one tile): three levels up to 67 M rows.  Each tile
// stores its reflectors and its WY matrix M (the down pass's input).
// Kernel boundaries order the levels (a device-scope release in every block
// of a launch writes each XCD's L2 back: 2.8 ms measured when k_fold_up did).
// With red_out set, level 1 has 72 extra blocks that reduce the up launch's
// C2 partials, one entry each (k_fold_reduce's job, without its launch).
__global__ __launch_bounds__(64 * UW) void k_fold_tree(FoldArgs a, int L) {
    __shared__ double xlds[2 * UW * 2 * FM];
    __shared__ double gw[UW][64], Vt[64];
    __shared__ double scr[UW][32 * (NG - NG / 2)];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, m = a.m;
    const int t = blockIdx.x;
    if (L == 1 && a.red_out && t >= a.nu[0]) {  // the 72 extra blocks: one C2 entry each
        const int e = t - a.nu[0];
        const double* p = a.partial + (int64_t)e * a.nblk;
        double s = 0.0;
        for (int i = tid; i < a.nblk; i += 64 * UW) s = s + p[i];
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) s = s + __shfl_xor(s, o, 64);
        if (lane == 0) xlds[wave] = s;
        __syncthreads();
        if (tid == 0) {
            double v = 0.0;
            for (int k = 0; k < UW; ++k) v = v + xlds[k];
            a.red_out[e] = v;
        }
        return;
    }
    const double* Rin = L == 1 ? a.R0 : a.Ru[L - 2];
    const int nin = L == 1 ? a.n0 : a.nu[L - 2];
    const int64_t rows = (int64_t)((nin - t * FG) < FG ? (nin - t * FG) : FG) * FM;
    double x[URPL][FM], tau[FM], beta[FM];
    fload_stack<URPL>(Rin + (int64_t)t * FG * 64, (int64_t)wave * 64 * URPL, rows, lane, x);
    tile_geqr2_blk<FM, URPL, UW>(x, tau, beta, m, lane, wave, xlds);
    fstore_tile<URPL>(a.Vu[L - 1] + (int64_t)t * (64 * URPL * UW * FM) + (int64_t)wave * URPL * FM * 64, lane, x);
    if (wave == 0) {
        fput_R(a.Ru[L - 1] + (int64_t)t * 64, lane, m, x[0]);
        // the root's R with leading dimension m as well (the stack layout of
        // tsqr.hip, for the all-gather of the local roots over several ranks)
        if (L == a.nlev && lane < m)
            for (int cc = 0; cc < m; ++cc) a.Rroot_m[lane + cc * m] = cc >= lane ? x[0][cc] : 0.0;
    }
    fold_wy_blk<URPL, UW>(x, tau, m, lane, wave, gw, scr, Vt, a.Mu[L - 1] + (int64_t)t * 64);
}

// ---- the s x s algebra --------------------------------------------------
// Phase 1 (after the tree, the Gram tile reduced, and on several ranks the
// global levels): Rtop the root R (ld ldr, raw signs), G the up launch's
// reduced C2 = Qp'Y (9 x 8, ld 9).  Writes S_top (8 x 8, ld 8; and ld m
// to Sm), K (9 x 8, ld 9), out (R, RY, flags) and publishes out.  One wave;
// the 8 x 8 matrices in LDS (column-major, ld 8), entry (r, c) computed by
// lane r + 8c, triangular inverses by one lane per column.
__device__ __forceinline__ void finv_col(const double* T, double* Ti, int j, int m) {
    // column j of T^-1 (T upper, m x m): back substitution, i descending
    double col[FM];
#pragma unroll
    for (int i = FM - 1; i >= 0; --i) {
        double s = (i == j) ? 1.0 : 0.0;
#pragma unroll
        for (int k = i + 1; k < FM; ++k) s = (k <= j) ? s - T[i + k * FM] * col[k] : s;
        col[i] = (i <= j && j < m) ? s / T[i + i * FM] : 0.0;
    }
#pragma unroll
    for (int i = 0; i < FM; ++i) Ti[i + j * FM] = col[i];
}

// The body, one wave (lane 0..63; its LDS hand-offs stay inside the wave).
// Sl: S_top also into this LDS array (the merged root kernel), or null.
__device__ __forceinline__ void fold_coef1_body(const double* T1, const double* G, const double* Rtop, int ldr,
                                                double* __restrict__ out, double* __restrict__ Sbuf,
                                                double* __restrict__ Sm, double* __restrict__ Kbuf, int w, int m,
                                                int doreorth, double nglob, double tol, double* Sl, int lane) {
    __shared__ double Cs[9 * FM], C2s[9 * FM], RT[64], XX[64];
    __shared__ double RY[64], Ri[64], Ws[9 * FM], U[64], Ui[64], D[FM];
    __shared__ int fail, reo;
    const int r = lane & 7, c = lane >> 3, nq = w < 8 ? w : 8;
    const bool in = r < m && c < m;
    // stage every input once (one round of global loads): C = Qp'X and the
    // diagonal X'X from the P1 tile T1, C2 = Qp'Y from the Gram tile G, the
    // root R (ld ldr, raw signs)
    // (every load issued before the first wait: one memory round trip; the
    // addresses are valid for every lane, the selects come after)
    const int e1 = lane + 64 < 9 * FM ? lane + 64 : lane;
    auto t1_at = [&](int e) {
        const int i = e % 9, j = e / 9, jj = nq + (j < FM ? j : 0);
        return T1[i < 8 ? i + jj * 16 : 256 + jj];
    };
    const double ta = t1_at(lane), tb = t1_at(e1), ga = G[lane], gb = G[e1];
    const double rtv = Rtop[(r < m ? r : 0) + (c < m ? c : 0) * ldr];
    const double xxv = T1[(nq + (lane < m ? lane : 0)) * 17];
    __builtin_amdgcn_sched_barrier(0);  // all six loads issue before any use waits
    {
        const int i = lane % 9, j = lane / 9, i1 = e1 % 9, j1 = e1 / 9;
        const bool ok = i < w && j < m, ok1 = i1 < w && j1 < m;
        Cs[lane] = ok ? ta : 0.0;
        C2s[lane] = ok ? ga : 0.0;  // the up launch's reduced Qp'Y (entry i + 9 j)
        Cs[e1] = ok1 ? tb : 0.0;    // (lanes >= 8: e1 = lane, the same value again)
        C2s[e1] = ok1 ? gb : 0.0;
    }
    RT[lane] = in ? rtv : 0.0;
    XX[lane] = lane < m ? xxv : 0.0;
    fwsync();
    // the reorth test of projectAndNormalize.m:17-22,45-52 on the algebraic
    // norms ||Y_j||^2 = X_j'X_j - C_j'C_j: column j on lane j, then the
    // NaN-ignoring max over the columns (order-free)
    {
        double rj = NAN;
        if (lane < m) {
            double cc = 0.0;
            for (int k = 0; k < w; ++k) cc = cc + Cs[k + lane * 9] * Cs[k + lane * 9];
            const double before = sqrt(XX[lane]);
            const double after = sqrt(fmax(XX[lane] - cc, 0.0));
            rj = fabs(before - after) / before;
        }
#pragma unroll
        for (int o = 4; o >= 1; o >>= 1) {
            const double q = __shfl_xor(rj, o, 64);
            rj = isnan(rj) ? q : (isnan(q) ? rj : fmax(rj, q));
        }
        if (lane == 0) {
            reo = (w > 0 && doreorth && rj > 0.5) ? 1 : 0;
            fail = 0;
            out[512] = 0.0;
            out[514] = reo ? 1.0 : 0.0;
        }
    }
    if (lane < FM) {
        const double rii = RT[lane * 9];
        D[lane] = rii > 0.0 ? 1.0 : (rii < 0.0 ? -1.0 : 0.0);  // sign(0) = 0 (tsqr.m:9-10)
    }
    U[lane] = (r == c && r < m) ? 1.0 : 0.0;
    Ui[lane] = U[lane];
    fwsync();
    double xmax = 0.0;
    for (int j = 0; j < m; ++j) xmax = fmax(xmax, sqrt(XX[j]));
    const bool reorth = reo != 0;
    RY[lane] = (in && r <= c) ? D[r] * RT[lane] : 0.0;  // R_Y = D R
    fwsync();
    double est = 0.0;
    if (reorth) {
        if (lane < FM) finv_col(RY, Ri, lane, m);  // R_Y^-1 (Inf / NaN at a zero pivot)
        fwsync();
        // W = C2 R_Y^-1 (w x m)
        for (int e = lane; e < 9 * FM; e += 64) {
            const int i = e % 9, cc = e / 9;
            double v = 0.0;
            for (int k = 0; k <= cc; ++k) v = v + C2s[i + k * 9] * Ri[k + cc * FM];
            Ws[i + cc * 9] = v;
        }
        fwsync();
        // A = I - W'W (entry per lane); ||W||_F^2, ||R_Y^-1||_F^2
        double a = (r == c && r < m) ? 1.0 : 0.0;
        if (in)
            for (int k = 0; k < w; ++k) a = a - Ws[k + r * 9] * Ws[k + c * 9];
        double nw = Ws[lane] * Ws[lane] + (lane < 8 ? Ws[64 + lane] * Ws[64 + lane] : 0.0);
        double nri = Ri[lane] * Ri[lane];
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) {
            nw = nw + __shfl_xor(nw, o, 64);
            nri = nri + __shfl_xor(nri, o, 64);
        }
        // the fold's loss of orthogonality ~ 2 ||W|| ||E||, E = Qp'Q_Y - W
        // (the rounding of C2 and of Y's factorization through R_Y^-1):
        // ||E|| <~ u sqrt(n) max||X_j|| ||R_Y^-1||; decline (explicit Z)
        // unless that is below tol (FoldArgs::tol: kFoldTol unless the context sets another)
        // and ||W||_F <= 1/2
        est = 2.0 * sqrt(nw) * 0x1p-53 * sqrt(nglob) * xmax * sqrt(nri);
        int bad = !(nw <= 0.25) || !(est <= tol);  // also NaN / Inf
        // U = chol(A), upper, in registers: lane (r, c), pivot rows by
        // shuffles (dense::chol_upper's operations and order)
        double uv = 0.0;
        for (int j = 0; j < m && !bad; ++j) {
            const double sj = __shfl(a, j + 8 * j, 64);
            if (!(sj > 0.0) || !isfinite(sj)) {
                bad = 1;
                break;
            }
            const double ujj = sqrt(sj);
            if (r == j) uv = c == j ? ujj : (c > j && c < m ? a / ujj : 0.0);
            const double ujr = __shfl(uv, j + 8 * r, 64), ujc = __shfl(uv, j + 8 * c, 64);
            if (r > j && c >= r) a = a - ujr * ujc;
        }
        if (!bad) U[lane] = (in && r <= c) ? uv : 0.0;
        if (lane == 0) fail = bad;
        fwsync();
        if (!fail && lane < FM) finv_col(U, Ui, lane, m);
        fwsync();
    }
    if (!reorth && !(est <= tol)) {  // est = 0 here: only a negative tol (decline every block)
        if (lane == 0) fail = 1;
        fwsync();
    }
    if (lane == 0) {
        out[513] = fail ? 1.0 : 0.0;
        out[515] = est;
    }
    if (!fail) {
        // S_top = D U^-1, R_Z = U R_Y
        const double sv = D[r] * Ui[lane];
        Sbuf[lane] = sv;
        if (in) Sm[r + c * m] = sv;
        double rz = 0.0;
        for (int k = r; k <= c; ++k) rz = rz + U[r + k * FM] * RY[k + c * FM];
        if (in) out[r + c * m] = r <= c ? rz : 0.0;
        // K = W U^-1 (9 x 8, ld 9)
        for (int e = lane; e < 9 * FM; e += 64) {
            const int i = e % 9, cc = e / 9;
            double kv = 0.0;
            if (reorth)
                for (int k = 0; k <= cc; ++k) kv = kv + Ws[i + k * 9] * Ui[k + cc * FM];
            Kbuf[e] = kv;
        }
        // RY = C + C2 (projectAndNormalize.m:71-73)
        for (int e = lane; e < w * m; e += 64) {
            const int i = e % w, j = e / w;
            out[256 + e] = Cs[i + j * 9] + (reorth ? C2s[i + j * 9] : 0.0);
        }
    }
    if (Sl) Sl[lane] = fail ? 0.0 : D[r] * Ui[lane];
    fwsync();
}

// R, RY and the flags (out) to pinned host memory, then the sequence word
// (system-scope release): the host's wait_published reads them
__device__ __forceinline__ void fold_publish(const double* out, int w, int m, double* __restrict__ hout,
                                             unsigned long long* __restrict__ hseq, unsigned long long seq,
                                             int lane) {
    for (int e = lane; e < m * m; e += 64) hout[e] = out[e];
    for (int e = lane; e < w * m; e += 64) hout[256 + e] = out[256 + e];
    if (lane < 4) hout[512 + lane] = out[512 + lane];
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    fwsync();
    if (lane == 0) {
        __threadfence_system();
        __hip_atomic_store(hseq, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

__global__ __launch_bounds__(64) void k_fold_coef1(const double* __restrict__ T1, const double* __restrict__ G,
                                                  const double* __restrict__ Rtop, int ldr, double* __restrict__ out,
                                                  double* __restrict__ Sbuf, double* __restrict__ Sm,
                                                  double* __restrict__ Kbuf, int w, int m, int doreorth, double nglob,
                                                  double tol, double* __restrict__ hout,
                                                  unsigned long long* __restrict__ hseq, unsigned long long seq) {
    fold_coef1_body(T1, G, Rtop, ldr, out, Sbuf, Sm, Kbuf, w, m, doreorth, nglob, tol, nullptr, threadIdx.x);
    if (hout) fold_publish(out, w, m, hout, hseq, seq, threadIdx.x);
}

// Fixed-order reduction of the up launch's Gram partials (entry-major,
// nparts per entry): one 1024-thread block per entry; same sum on every run.
__global__ __launch_bounds__(1024) void k_fold_reduce(const double* __restrict__ part, int nparts,
                                                     double* __restrict__ outv) {
    __shared__ double ws[16];
    const int64_t e = blockIdx.x;
    const double* p = part + e * nparts;
    double s = 0.0;
    for (int i = threadIdx.x; i < nparts; i += 1024) s = s + p[i];
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) s = s + __shfl_xor(s, o, 64);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (lane == 0) ws[wave] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
        double t = 0.0;
        for (int k = 0; k < 16; ++k) t = t + ws[k];
        outv[e] = t;
    }
}

// One rank: the root level and the s x s algebra in one block (k_fold_tree's
// root tile, then k_fold_coef1 on wave 0): two latency-bound launches in one.
// The root's reflectors and WY matrix are stored like any tile's; the
// publish comes last.
__global__ __launch_bounds__(64 * UW) void k_fold_root(FoldArgs a, const double* __restrict__ T1,
                                                       const double* __restrict__ G, double* __restrict__ out,
                                                       double* __restrict__ Sbuf, double* __restrict__ Sm,
                                                       double* __restrict__ Kbuf, int w, int doreorth, double nglob,
                                                       double* __restrict__ hout,
                                                       unsigned long long* __restrict__ hseq, unsigned long long seq) {
    __shared__ double xlds[2 * UW * 2 * FM];
    __shared__ double Rl[64];
    __shared__ double gw[UW][64], Vt[64];
    __shared__ double scr[UW][32 * (NG - NG / 2)];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, m = a.m;
    const int L = a.nlev;
    const double* Rin = L == 1 ? a.R0 : a.Ru[L - 2];
    const int64_t rows = (int64_t)(L == 1 ? a.n0 : a.nu[L - 2]) * FM;  // one tile (<= FG R blocks)
    double x[URPL][FM], tau[FM], beta[FM];
    fload_stack<URPL>(Rin, (int64_t)wave * 64 * URPL, rows, lane, x);
    tile_geqr2_blk<FM, URPL, UW>(x, tau, beta, m, lane, wave, xlds);
    if (wave == 0) fput_R(Rl, lane, m, x[0]);
    fstore_tile<URPL>(a.Vu[L - 1] + (int64_t)wave * URPL * FM * 64, lane, x);
    // the WY matrix's Gram shares first (every wave), then the s x s algebra
    // and the publish on wave 0 while wave 1 sums the Gram and writes M: the
    // algebra no longer waits for wave 0's Gram share and M is off the
    // critical path (fold_wy_blk's work, split over two waves)
    fv_tile<URPL>(x, (int64_t)wave * 64 * URPL + lane, m);
    wave_gram<URPL>(x, scr[wave], gw[wave], lane);
    if (wave == 0 && lane < FM) {
#pragma unroll
        for (int c = 0; c < FM; ++c) Vt[lane + FM * c] = x[0][c];
    }
    __syncthreads();
    if (wave == 0) {
        fold_coef1_body(T1, G, Rl, FM, out, Sbuf, Sm, Kbuf, w, m, doreorth, nglob, a.tol, nullptr, lane);
        if (hout) fold_publish(out, w, m, hout, hseq, seq, lane);
    } else if (wave == 1) {
        double sum = gw[0][lane];
#pragma unroll
        for (int v = 1; v < UW; ++v) sum = sum + gw[v][lane];
        fwsync();
        gw[0][lane] = sum;
        fwsync();
        if (lane < FM) {
            double mrow[FM];
            fwy_row(gw[0], Vt, tau, m, lane, mrow);
#pragma unroll
            for (int j = 0; j < FM; ++j) a.Mu[L - 1][lane + FM * j] = mrow[j];
        }
    }
}

// Level 0: Q = Q_tile S - Qp K, one store.  Q: output columns (slots >= m
// unused); P as in k_fold_up (Qp in slots 0..8).  Independent waves.  Each
// wave first forms its tile's S block: from the root's S (Stop, ld lds) down
// the levels, S_child = E S - V(rows) (M S) on the 8 stack rows of its
// ancestor at each level (lane r + 8 c holds entry (r, c); 8 x 8 products by
// shuffles), then its own tile's M from V'V, and the rows as
// E S - V (M S) - Qp K.
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(FOLD_DOWN_WPE))) void k_fold_down(ColList P, OutList Q,
                                                                                           FoldArgs a) {
    __shared__ double Ks[9 * FM];
    __shared__ double Vts[FTPB][64], Ms[FTPB][64], Ss[FTPB][64], Ns[FTPB][64];
    const int tid = threadIdx.x, lane = tid & 63, m = a.m, w = a.w;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // uniform: the tile's scalars by scalar loads
    const int64_t n = a.n;
    const int64_t ntiles = (n + FTR0 - 1) / FTR0;
    const int64_t tile = (int64_t)blockIdx.x * FTPB + wave;
    for (int e = tid; e < 9 * FM; e += 256) {
        const int k = e % 9, cc = e / 9;
        Ks[e] = (k < w && cc < m) ? a.K[e] : 0.0;
    }
    const bool corr = a.flags[2] != 0.0;
    // a declined fold (flags[1], written by the coefficient step before this
    // launch) stores nothing: S and K are stale then, and Q may alias X,
    // which the explicit-Z path that follows reads again
    const bool declined = a.flags[1] != 0.0;
    __syncthreads();
    if (tile >= ntiles || declined) return;
    const int r8 = lane & 7, c8 = lane >> 3;
    const int nlev = a.nlev;
    // the ancestors' V rows and M (loads first: they do not depend on S)
    double vv[3], mv[3];
#pragma unroll
    for (int l = 0; l < 3; ++l) {
        vv[l] = 0.0;
        mv[l] = 0.0;
        if (l < nlev) {
            const int64_t tl = tile >> (6 * (l + 1));
            const int row = 8 * (int)((tile >> (6 * l)) & 63) + r8;
            const double* V = a.Vu[l] + tl * (64 * URPL * UW * FM) + (row >> 7) * (URPL * FM * 64) +
                              (((row >> 6) & 1) * FM + c8) * 64 + (row & 63);
            vv[l] = fv(*V, row, c8, m);
            mv[l] = a.Mu[l][tl * 64 + lane];
        }
    }
    double S = (r8 < m && c8 < m) ? a.Stop[r8 + c8 * a.lds] : 0.0;
    double x[L0RPL][FM], tau[FM];
    fload_tile<L0RPL>(a.V0 + tile * (64 * L0RPL * FM), lane, x);
    fload_tau(a.tb0 + tile * (2 * FM), tau);
    // the wave's loads issued before its s x s work: the first two row
    // chunks of Qp for the correction too (in flight during the chain and
    // the Gram)
    const int64_t base = tile * FTR0;
    constexpr int CH = 2;  // row chunks per pass of the row phase
    double q[CH][9];
    auto loadq = [&](int i0) {
#pragma unroll
        for (int ii = 0; ii < CH; ++ii) {
            const int64_t r = base + lane + 64 * (i0 + ii);
            const int64_t rr = r < n ? r : n - 1;
#pragma unroll
            for (int k = 0; k < 9; ++k) q[ii][k] = P.p[k][rr];
        }
    };
    if (corr) loadq(0);
    // the chain through LDS (wave-private arrays, free until the tile's own M)
    double* const Sw = Ss[wave];
    double* const Mw = Ms[wave];
    double* const Vw = Vts[wave];
    double* const Nw0 = Ns[wave];
#pragma unroll
    for (int l = 2; l >= 0; --l) {
        if (l < nlev) {
            Sw[lane] = S;
            Mw[lane] = mv[l];
            Vw[lane] = vv[l];
            fwsync();
            double nv = 0.0;
#pragma unroll
            for (int j = 0; j < FM; ++j) nv = __builtin_fma(Mw[r8 + FM * j], Sw[j + FM * c8], nv);
            Nw0[lane] = nv;
            fwsync();
            double sn = ((tile >> (6 * l)) & 63) == 0 ? S : 0.0;
#pragma unroll
            for (int k = 0; k < FM; ++k) sn = sn - Vw[r8 + FM * k] * Nw0[k + FM * c8];
            fwsync();
            S = sn;
        }
    }
    // level 0: the tile's explicit Q factor (dorg2r in registers; measured
    // 384 us a launch against 422 for E S - V (M S) with M from V'V here:
    // the Gram's reductions cost more than the reflector sweep)
    Ss[wave][lane] = S;
    fwsync();
    tile_org2r<FM, L0RPL>(x, tau, m, lane);
#pragma unroll
    for (int i = 0; i < L0RPL; ++i) {
        asm volatile("" ::: "memory");
        double o[FM];
        fmul_S(x[i], Ss[wave], m, o);
        const int ii = i % CH;
        if (corr) {
            double t[FM];
#pragma unroll
            for (int cc = 0; cc < FM; ++cc) t[cc] = 0.0;
#pragma unroll
            for (int k = 0; k < 9; ++k) {
#pragma unroll
                for (int cc = 0; cc < FM; ++cc) asm volatile("" : "+v"(t[cc]));
#pragma unroll
                for (int cc = 0; cc < FM; ++cc) t[cc] = __builtin_fma(q[ii][k], Ks[k + cc * 9], t[cc]);
            }
#pragma unroll
            for (int cc = 0; cc < FM; ++cc) o[cc] = o[cc] - t[cc];
            if (ii == CH - 1 && i + 1 < L0RPL) loadq(i + 1);
        }
        const int64_t r = base + lane + 64 * i;
        if (r < n) {
            // (non-temporal, as pass B's: Q is read again only after the next
            // step's matrix powers; with the round-5 plane-march SpMV 694-697
            // -> 706-707 outer-it/s on the TSQR headline, same box,
            // profiles/r05/ab/; round 4 had measured no difference)
#pragma unroll
            for (int cc = 0; cc < FM; ++cc)
                if (cc < m) {
                    if (CAL_FOLD_DOWN_NT) __builtin_nontemporal_store(o[cc], &Q.p[cc][r]);
                    else Q.p[cc][r] = o[cc];
                }
        }
    }
}

int fold_tiles(int64_t n) { return (int)((n + FTR0 - 1) / FTR0); }
int fold_blocks(int64_t n) { return (fold_tiles(n) + FTPB - 1) / FTPB; }
// tiles of the upper levels 1, 2, ... (the last one has one tile: the root)
std::vector<int> fold_levels(int64_t n) {
    std::vector<int> nu;
    int64_t cnt = fold_tiles(n);
    do {
        cnt = (cnt + FG - 1) / FG;
        nu.push_back((int)cnt);
    } while (cnt > 1);
    return nu;
}
bool fold_shape_ok(int64_t n, int m, int w) {
    if (n < 1 || m < 1 || m > FM || w < 1 || w > 9) return false;
    return fold_levels(n).size() <= 3;  // up to 64^3 level-0 tiles
}
size_t fold_l0_tile_doubles() { return (size_t)64 * L0RPL * FM; }
size_t fold_tile_doubles() { return (size_t)64 * URPL * UW * FM; }

hipError_t launch_fold_up(const ColList& P, const FoldArgs& a, hipStream_t st) {
    hipLaunchKernelGGL(k_fold_up, dim3(a.nblk), dim3(256), 0, st, P, a);
    return hipGetLastError();
}
hipError_t launch_fold_tree(const FoldArgs& a, hipStream_t st, int upto) {
    for (int L = 1; L <= (upto >= 0 ? upto : a.nlev); ++L)
        hipLaunchKernelGGL(k_fold_tree, dim3(a.nu[L - 1] + (L == 1 && a.red_out ? 72 : 0)), dim3(64 * UW), 0, st, a,
                           L);
    return hipGetLastError();
}
hipError_t launch_fold_reduce(const double* partial, int nparts, double* outv, hipStream_t st) {
    hipLaunchKernelGGL(k_fold_reduce, dim3(72), dim3(1024), 0, st, partial, nparts, outv);
    return hipGetLastError();
}
hipError_t launch_fold_coef1(const double* T1, const double* G, const double* Rtop, int ldr, double* out,
                             double* Sbuf, double* Sm, double* Kbuf, int w, int m, int doreorth, double nglob,
                             double tol, double* hout, unsigned long long* hseq, unsigned long long seq,
                             hipStream_t st) {
    hipLaunchKernelGGL(k_fold_coef1, dim3(1), dim3(64), 0, st, T1, G, Rtop, ldr, out, Sbuf, Sm, Kbuf, w, m, doreorth,
                       nglob, tol, hout, hseq, seq);
    return hipGetLastError();
}
hipError_t launch_fold_root(const FoldArgs& a, const double* T1, const double* G, double* out, double* Sbuf,
                            double* Sm, double* Kbuf, int w, int doreorth, double nglob, double* hout,
                            unsigned long long* hseq, unsigned long long seq, hipStream_t st) {
    hipLaunchKernelGGL(k_fold_root, dim3(1), dim3(64 * UW), 0, st, a, T1, G, out, Sbuf, Sm, Kbuf, w, doreorth, nglob,
                       hout, hseq, seq);
    return hipGetLastError();
}
hipError_t launch_fold_down(const ColList& P, const OutList& Q, const FoldArgs& a, hipStream_t st) {
    hipLaunchKernelGGL(k_fold_down, dim3(a.nblk), dim3(256), 0, st, P, Q, a);
    return hipGetLastError();
}

}  // namespace cal
