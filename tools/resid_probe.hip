// Probe: the memory-access scheme of the Ritz-residual gather (k_resid_pairs)
// on the 7-point stencil of lap3d_215, one column per Ritz vector.  Not part
// of the library.  Per Ritz vector l and row r: y = 6 x[r] - sum of the six
// neighbours - l x[r]; the kernel sums y^2 per vector (block partials).
//   hipcc -O3 -ffp-contract=off --offload-arch=gfx950 tools/resid_probe.hip -o /tmp/resid_probe
// Modes (row pair per lane, 16-B loads):
//   0  seven loads (odd offsets 8-B aligned)            -- k_resid_pairs
//   1  +-1 from the centre by DPP wave shifts            -- k_resid_pairs LANE
//   2  every odd slot as an aligned load + DPP shift     (5 aligned loads)
//   3  LDS windows: the block's three x windows staged with aligned loads
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

constexpr int N = 215;
constexpr int64_t P = (int64_t)N * N;
constexpr int64_t NR = P * N;

__device__ __forceinline__ double2 ld16(const double* p) {
    double2 v;
    __builtin_memcpy(&v, p, 16);
    return v;
}
template <int CTRL>
__device__ __forceinline__ double dshift(double v, double edge) {
    const unsigned long long b = (unsigned long long)__double_as_longlong(v);
    const unsigned long long o = (unsigned long long)__double_as_longlong(edge);
    const unsigned lo = (unsigned)__builtin_amdgcn_update_dpp((int)(unsigned)o, (int)(unsigned)b, CTRL, 0xf, 0xf, false);
    const unsigned hi = (unsigned)__builtin_amdgcn_update_dpp((int)(unsigned)(o >> 32), (int)(unsigned)(b >> 32), CTRL, 0xf, 0xf, false);
    return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}
constexpr int SHL1 = 0x130;  // lane i <- lane i + 1
constexpr int SHR1 = 0x138;  // lane i <- lane i - 1

__device__ __forceinline__ int xcd_remap(int b, int nwg) {
    const int q = nwg >> 3, r = nwg & 7, x = b & 7, i = b >> 3;
    return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + i;
}

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v = v + __shfl_xor(v, off, 64);
    return v;
}

// rows of the two rows of a pair from the 7 slot pairs (slot order -P,-N,-1,0,1,N,P)
__device__ __forceinline__ void pair_y(const double2 (&s)[7], double l, double& y0, double& y1) {
    y0 = 0.0;
    y1 = 0.0;
    const double c[7] = {-1.0, -1.0, -1.0, 6.0, -1.0, -1.0, -1.0};
#pragma unroll
    for (int e = 0; e < 7; ++e) {
        y0 = y0 + c[e] * s[e].x;
        y1 = y1 + c[e] * s[e].y;
    }
    y0 = y0 - l * s[3].x;
    y1 = y1 - l * s[3].y;
}

template <int MODE, int CPB, int PPT>
__global__ __launch_bounds__(256) void k_res(const double* __restrict__ X, int64_t ld, const double* __restrict__ lam,
                                             double* __restrict__ partial) {
    __shared__ double ws[CPB][4];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int64_t npairs = NR / 2;
    const int64_t b0 = (int64_t)xcd_remap(blockIdx.x, gridDim.x) * 256 * PPT;
    double acc[CPB];
#pragma unroll
    for (int q = 0; q < CPB; ++q) acc[q] = 0.0;
    const int64_t off[7] = {-P, -N, -1, 0, 1, N, P};
    for (int j = 0; j < PPT; ++j) {
        const int64_t t = b0 + (int64_t)j * 256 + tid;
        if (b0 + (int64_t)j * 256 >= npairs) break;
        const bool ok = t < npairs;
        const int64_t r = 2 * (ok ? t : npairs - 1);
        const int64_t tw = __builtin_amdgcn_readfirstlane((unsigned)(2 * (b0 + j * 256 + (tid & ~63))));
#pragma unroll
        for (int q = 0; q < CPB; ++q) {
            const double* x = X + (int64_t)(blockIdx.y * CPB + q) * ld;
            double2 s[7];
            if (MODE == 0) {
#pragma unroll
                for (int e = 0; e < 7; ++e) s[e] = ld16(x + r + off[e]);
            } else if (MODE == 1) {
                s[0] = ld16(x + r - P);
                s[1] = ld16(x + r - N);
                s[3] = ld16(x + r);
                s[5] = ld16(x + r + N);
                s[6] = ld16(x + r + P);
                const double xl = x[tw - 1], xr = x[tw + 128];
                s[2] = make_double2(dshift<SHR1>(s[3].y, xl), s[3].x);
                s[4] = make_double2(s[3].y, dshift<SHL1>(s[3].x, xr));
            } else {  // MODE 2: aligned + shifts
                s[3] = ld16(x + r);
                const double2 a0 = ld16(x + r - P - 1), a1 = ld16(x + r - N - 1), a5 = ld16(x + r + N - 1),
                              a6 = ld16(x + r + P - 1);
                // (the tail wave's lanes past the rows: clamp into the column's padding)
                auto cl = [](int64_t i) { return i < NR + P + 4095 ? i : NR + P + 4095; };
                const double e0 = x[cl(tw + 128 - P - 1)], e1 = x[cl(tw + 128 - N - 1)], e5 = x[cl(tw + 128 + N - 1)],
                             e6 = x[cl(tw + 128 + P - 1)];
                s[0] = make_double2(a0.y, dshift<SHL1>(a0.x, e0));
                s[1] = make_double2(a1.y, dshift<SHL1>(a1.x, e1));
                s[5] = make_double2(a5.y, dshift<SHL1>(a5.x, e5));
                s[6] = make_double2(a6.y, dshift<SHL1>(a6.x, e6));
                const double xl = x[tw - 1], xr = x[tw + 128];
                s[2] = make_double2(dshift<SHR1>(s[3].y, xl), s[3].x);
                s[4] = make_double2(s[3].y, dshift<SHL1>(s[3].x, xr));
            }
            double y0, y1;
            pair_y(s, lam[blockIdx.y * CPB + q], y0, y1);
            if (ok) acc[q] = acc[q] + (y0 * y0 + y1 * y1);
        }
    }
#pragma unroll
    for (int q = 0; q < CPB; ++q) {
        const double v = wave_sum(acc[q]);
        if (lane == 0) ws[q][wave] = v;
    }
    __syncthreads();
    if (tid < CPB)
        partial[(int64_t)(blockIdx.y * CPB + tid) * gridDim.x + blockIdx.x] =
            ((ws[tid][0] + ws[tid][1]) + ws[tid][2]) + ws[tid][3];
}

// MODE 3: LDS windows.  Block rows [R, R + B), B = 512 PPT.  Per vector the
// windows w0 = [R - P - 1, R - P + B + 1), w1 = [R - N - 1, R + B + N + 1),
// w2 = [R + P - 1, R + P + B + 1) (even starts: aligned 16-B loads), staged
// into LDS by the whole block, then each thread's row pairs read their slots
// from LDS.  One vector at a time, double-buffered.
template <int PPT>
__global__ __launch_bounds__(256) void k_res_lds(const double* __restrict__ X, int64_t ld, int cpb,
                                                 const double* __restrict__ lam, double* __restrict__ partial) {
    constexpr int B = 512 * PPT;
    constexpr int L0 = B + 2, L1 = B + 2 * N + 2;  // window lengths (rows)
    constexpr int WL = 2 * L0 + L1;                // rows per vector
    constexpr int WLP = (WL + 1) & ~1;
    __shared__ __attribute__((aligned(16))) double win[2][WLP];
    __shared__ double ws[4];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int64_t R = (int64_t)xcd_remap(blockIdx.x, gridDim.x) * B;
    const int64_t st[3] = {R - P - 1, R - N - 1, R + P - 1};
    const int ln[3] = {L0, L1, L0};
    const int base[3] = {0, L0, L0 + L1};
    auto stage = [&](int q, int buf) {
        const double* x = X + (int64_t)(blockIdx.y * cpb + q) * ld;
#pragma unroll
        for (int w = 0; w < 3; ++w)
            for (int i = 2 * tid; i < ln[w]; i += 512) {
                const double2 v = ld16(x + st[w] + i);
                *reinterpret_cast<double2*>(&win[buf][base[w] + i]) = v;
            }
    };
    stage(0, 0);
    for (int q = 0; q < cpb; ++q) {
        __syncthreads();  // window q staged; buffer (q+1)&1 free
        if (q + 1 < cpb) stage(q + 1, (q + 1) & 1);
        const double* w = win[q & 1];
        const double l = lam[blockIdx.y * cpb + q];
        double acc = 0.0;
#pragma unroll
        for (int j = 0; j < PPT; ++j) {
            const int rl = 2 * (j * 256 + tid);  // local row of the pair
            const bool ok = R + rl + 1 < NR + 1 && R + rl < NR;
            double2 s[7];
            s[0] = make_double2(w[rl + 1], w[rl + 2]);                        // x[r - P] (w0 starts at R - P - 1)
            s[1] = make_double2(w[L0 + rl + 1], w[L0 + rl + 2]);              // x[r - N]
            s[2] = make_double2(w[L0 + rl + N], w[L0 + rl + N + 1]);          // x[r - 1]
            s[3] = make_double2(w[L0 + rl + N + 1], w[L0 + rl + N + 2]);      // x[r]
            s[4] = make_double2(w[L0 + rl + N + 2], w[L0 + rl + N + 3]);      // x[r + 1]
            s[5] = make_double2(w[L0 + rl + 2 * N + 1], w[L0 + rl + 2 * N + 2]);  // x[r + N]
            s[6] = make_double2(w[L0 + L1 + rl + 1], w[L0 + L1 + rl + 2]);    // x[r + P]
            double y0, y1;
            pair_y(s, l, y0, y1);
            if (ok) acc = acc + (y0 * y0 + y1 * y1);
        }
        const double v = wave_sum(acc);
        if (lane == 0) ws[wave] = v;
        __syncthreads();
        if (tid == 0)
            partial[(int64_t)(blockIdx.y * cpb + q) * gridDim.x + blockIdx.x] = ((ws[0] + ws[1]) + ws[2]) + ws[3];
    }
}


// MODE 4: row-interleaved X: groups of G vectors stored
// [row][G] (64 B per row for G = 8); 4 lanes per row (G = 8) or 2 (G = 4),
// each lane 16 B = two vectors of one row, so every slot load is 16-B
// aligned and a wave's load is one contiguous run.  One group per block.
template <int G, int RPT>
__global__ __launch_bounds__(256) void k_res_int(const double* __restrict__ Xi, int64_t ldg,
                                                 const double* __restrict__ lam, double* __restrict__ partial) {
    constexpr int LPR = G / 2;             // lanes per row
    constexpr int RPW = 64 / LPR;          // rows per wave
    constexpr int RPB = 4 * RPW;           // rows per block iteration
    __shared__ double ws[4][G];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int c = lane % LPR;              // the lane's vector pair
    const double* xg = Xi + (int64_t)blockIdx.y * ldg;
    const int64_t b0 = (int64_t)xcd_remap(blockIdx.x, gridDim.x) * RPB * RPT;
    const double l0 = lam[blockIdx.y * G + 2 * c], l1 = lam[blockIdx.y * G + 2 * c + 1];
    const int64_t off[7] = {-P, -N, -1, 0, 1, N, P};
    const double cf[7] = {-1.0, -1.0, -1.0, 6.0, -1.0, -1.0, -1.0};
    double a0 = 0.0, a1 = 0.0;
    for (int j = 0; j < RPT; ++j) {
        const int64_t r = b0 + (int64_t)j * RPB + wave * RPW + lane / LPR;
        if (b0 + (int64_t)j * RPB >= NR) break;
        const bool ok = r < NR;
        const int64_t rr = ok ? r : NR - 1;
        double y0 = 0.0, y1 = 0.0;
        double2 xc;
#pragma unroll
        for (int e = 0; e < 7; ++e) {
            const double2 v = ld16(xg + (rr + off[e]) * G + 2 * c);
            if (e == 3) xc = v;
            y0 = y0 + cf[e] * v.x;
            y1 = y1 + cf[e] * v.y;
        }
        y0 = y0 - l0 * xc.x;
        y1 = y1 - l1 * xc.y;
        if (ok) {
            a0 = a0 + y0 * y0;
            a1 = a1 + y1 * y1;
        }
    }
    // lanes with the same c hold the same two vectors: sum over the wave's rows
#pragma unroll
    for (int o = 32; o >= LPR; o >>= 1) {
        a0 = a0 + __shfl_xor(a0, o, 64);
        a1 = a1 + __shfl_xor(a1, o, 64);
    }
    if (lane < LPR) {
        ws[wave][2 * lane] = a0;
        ws[wave][2 * lane + 1] = a1;
    }
    __syncthreads();
    if (tid < G)
        partial[(int64_t)(blockIdx.y * G + tid) * gridDim.x + blockIdx.x] =
            ((ws[0][tid] + ws[1][tid]) + ws[2][tid]) + ws[3][tid];
}

// MODE 5: plane march (one row per lane).  A block owns 256 consecutive rows
// of a plane (rows xy0 .. xy0 + 255 of every plane) and walks Z planes; the
// -P / 0 / +P slots of row r are x[r - P], x[r], x[r + P]: the previous,
// current and next plane's centre values of the same lane, so each x value
// is loaded once as "next" and reused from registers twice.  The +-1 slots
// from loads (DPP = false) or wave shifts of the centre (DPP = true); +-N
// from loads (L1/L2 hits: the same plane).
template <int Z, bool DPP>
__global__ __launch_bounds__(256) void k_res_z(const double* __restrict__ X, int64_t ld, const double* __restrict__ lam,
                                               double* __restrict__ partial) {
    __shared__ double ws[4];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    constexpr int64_t NXY = (P + 255) / 256;      // row blocks per plane
    const int bi = xcd_remap(blockIdx.x, gridDim.x);
    const int64_t xyb = bi % NXY, zb = bi / NXY;
    const int64_t xy = xyb * 256 + tid;
    const bool okxy = xy < P;
    const int64_t z0 = zb * Z;
    const double* x = X + (int64_t)blockIdx.y * ld;
    const double l = lam[blockIdx.y];
    const int64_t xyc = okxy ? xy : P - 1;
    double xp = x[xyc + (z0 - 1) * P], xc = x[xyc + z0 * P];
    double acc = 0.0;
    const int zend = (int)(N - z0 < Z ? N - z0 : Z);  // planes of this block (never past the last one)
#pragma unroll 2
    for (int z = 0; z < zend; ++z) {
        const int64_t r = xyc + (z0 + z) * P;
        const double xn = x[r + P];
        double xm1, xp1;
        if (DPP) {
            const int64_t rw = (int64_t)__builtin_amdgcn_readfirstlane((unsigned)(r & 0xffffffff));  // lane 0's row
            const double el = x[rw - 1], er = x[rw + 64];
            xm1 = dshift<SHR1>(xc, el);
            xp1 = dshift<SHL1>(xc, er);
        } else {
            xm1 = x[r - 1];
            xp1 = x[r + 1];
        }
        const double xmn = x[r - N], xpn = x[r + N];
        double y = 0.0;
        y = y + (-1.0) * xp;
        y = y + (-1.0) * xmn;
        y = y + (-1.0) * xm1;
        y = y + 6.0 * xc;
        y = y + (-1.0) * xp1;
        y = y + (-1.0) * xpn;
        y = y + (-1.0) * xn;
        y = y - l * xc;
        if (okxy) acc = acc + y * y;
        xp = xc;
        xc = xn;
    }
    const double v = wave_sum(acc);
    if (lane == 0) ws[wave] = v;
    __syncthreads();
    if (tid == 0) partial[(int64_t)blockIdx.y * gridDim.x + blockIdx.x] = ((ws[0] + ws[1]) + ws[2]) + ws[3];
}

// MODE 6: plane march over row pairs.  Lane = the pair (xy, xy + 1) of every
// plane z (rows r = xy + z P, r odd on odd planes when P is odd: 8-B aligned
// 16-B loads); the next plane's centre pair x[r + P .. r + P + 1] is loaded
// once and carried as the centre, then as the -P slot; +-1 by wave shifts
// of the centre pair (one scalar load per wave edge); +-N loaded.  The
// plane's last pair straddles into the next plane when P is odd: only its
// first row counts.
template <int Z, int SKIP = 0>
__global__ __launch_bounds__(256) void k_res_zp(const double* __restrict__ X, int64_t ld, const double* __restrict__ lam,
                                                double* __restrict__ partial) {
    __shared__ double ws[4];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    constexpr int64_t NPP = (P + 1) / 2;           // pairs per plane
    constexpr int64_t NXY = (NPP + 255) / 256;     // pair blocks per plane
    const int bi = xcd_remap(blockIdx.x, gridDim.x);
    const int64_t xyb = bi % NXY, zb = bi / NXY;
    const int64_t tp = xyb * 256 + tid;            // pair index within the plane
    const bool okp = tp < NPP;
    const int64_t xy = 2 * (okp ? tp : NPP - 1);
    const bool two = xy + 1 < P;                   // the straddling pair counts one row
    const int64_t z0 = zb * Z;
    const double* x = X + (int64_t)blockIdx.y * ld;
    const double l = lam[blockIdx.y];
    double2 xp = ld16(x + xy + (z0 - 1) * P), xc = ld16(x + xy + z0 * P);
    double acc = 0.0;
    const int zend = (int)(N - z0 < Z ? N - z0 : Z);
    const int64_t xyw = 2 * (xyb * 256 + (tid & ~63));  // lane 0's xy
#pragma unroll 2
    for (int z = 0; z < zend; ++z) {
        const int64_t r = xy + (z0 + z) * P;
        const double2 xn = ld16(x + r + P);
        const int64_t rw = xyw + (z0 + z) * P;
        // timing-only switches: SKIP bit 0 drops the +-N loads, bit 1 the edge loads
        const double el = (SKIP & 2) ? 0.0 : x[rw - 1], er = (SKIP & 2) ? 0.0 : x[rw + 128];
        const double2 xm1 = make_double2(dshift<SHR1>(xc.y, el), xc.x);
        const double2 xp1 = make_double2(xc.y, dshift<SHL1>(xc.x, er));
        const double2 xmn = (SKIP & 1) ? xp : ld16(x + r - N), xpn = (SKIP & 1) ? xn : ld16(x + r + N);
        double y0 = 0.0, y1 = 0.0;
        y0 = y0 + (-1.0) * xp.x;  y1 = y1 + (-1.0) * xp.y;
        y0 = y0 + (-1.0) * xmn.x; y1 = y1 + (-1.0) * xmn.y;
        y0 = y0 + (-1.0) * xm1.x; y1 = y1 + (-1.0) * xm1.y;
        y0 = y0 + 6.0 * xc.x;     y1 = y1 + 6.0 * xc.y;
        y0 = y0 + (-1.0) * xp1.x; y1 = y1 + (-1.0) * xp1.y;
        y0 = y0 + (-1.0) * xpn.x; y1 = y1 + (-1.0) * xpn.y;
        y0 = y0 + (-1.0) * xn.x;  y1 = y1 + (-1.0) * xn.y;
        y0 = y0 - l * xc.x;
        y1 = y1 - l * xc.y;
        if (okp) acc = acc + (y0 * y0 + (two ? y1 * y1 : 0.0));
        xp = xc;
        xc = xn;
    }
    const double v = wave_sum(acc);
    if (lane == 0) ws[wave] = v;
    __syncthreads();
    if (tid == 0) partial[(int64_t)blockIdx.y * gridDim.x + blockIdx.x] = ((ws[0] + ws[1]) + ws[2]) + ws[3];
}

// floor: one streaming 16-B read of x per row pair (sum of squares), same grid shape
__global__ __launch_bounds__(256) void k_read(const double* __restrict__ X, int64_t ld, double* __restrict__ partial) {
    __shared__ double ws[4];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const double* x = X + (int64_t)blockIdx.y * ld;
    double acc = 0.0;
    for (int64_t t = (int64_t)blockIdx.x * 256 + tid; t < NR / 2; t += (int64_t)gridDim.x * 256) {
        const double2 v = ld16(x + 2 * t);
        acc = acc + (v.x * v.x + v.y * v.y);
    }
    const double v = wave_sum(acc);
    if (lane == 0) ws[wave] = v;
    __syncthreads();
    if (tid == 0) partial[(int64_t)blockIdx.y * gridDim.x + blockIdx.x] = ((ws[0] + ws[1]) + ws[2]) + ws[3];
}

// MODE 7: pair plane march with the plane's in-plane neighbours from LDS.
// A block owns the row pairs xy0 .. xy0 + 511 of every plane and walks Z
// planes; per plane it stages the window x[zP + xy0 - H, zP + xy0 + 512 + H)
// (H = N + 1 rows each side: every in-plane slot of its rows) with
// contiguous 16-B loads into one of three LDS buffers, two planes ahead of
// its use; the -P / +P slots are the same lanes' centre pairs of the
// previous / next plane (registers, LDS).  SPMV: also store y (the SpMV).
template <int Z, bool SPMV>
__global__ __launch_bounds__(256) void k_res_zw(const double* __restrict__ X, int64_t ld, const double* __restrict__ lam,
                                                double* __restrict__ partial, double* __restrict__ Y) {
    constexpr int H = N + 1;                   // even
    constexpr int WR = 512 + 2 * H;            // window rows
    constexpr int WP = WR / 2;                 // window pairs
    constexpr int LPT = (WP + 255) / 256;      // staged pairs per thread
    __shared__ __attribute__((aligned(16))) double win[3][WR];
    __shared__ double ws[4];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    constexpr int64_t NXY = (P + 511) / 512;   // 512-row blocks per plane
    const int bi = xcd_remap(blockIdx.x, gridDim.x);
    const int64_t xyb = bi % NXY, zb = bi / NXY;
    const int64_t xy0 = xyb * 512;
    const int64_t z0 = zb * Z;
    const int zend = (int)(N - z0 < Z ? N - z0 : Z);
    const double* x = X + (int64_t)blockIdx.y * ld;
    double* y = SPMV ? Y + (int64_t)blockIdx.y * ld : nullptr;
    const double l = lam[blockIdx.y];
    const int lr = 2 * tid;                    // the lane's pair, rows xy0 + lr, + 1
    const bool okp = xy0 + lr < P;
    const bool two = xy0 + lr + 1 < P;         // the straddling pair (P odd) counts one row
    const int wi = lr + H;
    double2 st[LPT];
    auto load_plane = [&](int64_t z) {         // window of plane z into registers
        const int64_t g = z * P + xy0 - H;
#pragma unroll
        for (int k = 0; k < LPT; ++k) {
            const int pi = tid + 256 * k;
            st[k] = pi < WP ? ld16(x + g + 2 * pi) : make_double2(0.0, 0.0);
        }
    };
    auto store_plane = [&](int b) {
#pragma unroll
        for (int k = 0; k < LPT; ++k) {
            const int pi = tid + 256 * k;
            if (pi < WP) *reinterpret_cast<double2*>(&win[b][2 * pi]) = st[k];
        }
    };
    auto rd = [&](int b, int i) { return make_double2(win[b][i], win[b][i + 1]); };
    // prologue: planes z0, z0 + 1 staged; the -P pair loaded
    double2 xp = ld16(x + (z0 - 1) * P + xy0 + (okp ? lr : 0));
    load_plane(z0);
    store_plane(0);
    if (zend > 1) {
        load_plane(z0 + 1);
        store_plane(1);
    } else {  // the block's last plane is the matrix's last: +P is the zero padding
        load_plane(z0 + 1);
        store_plane(1);
    }
    __syncthreads();
    double acc = 0.0;
    for (int z = 0; z < zend; ++z) {
        const int bc = z % 3, bn = (z + 1) % 3, bs = (z + 2) % 3;
        if (z + 2 <= zend) load_plane(z0 + z + 2);  // two planes ahead (the last one: +P of the last plane)
        const double2 xc = rd(bc, wi), xn = rd(bn, wi);
        const double2 xmn = rd(bc, wi - N), xpn = rd(bc, wi + N);
        const double2 xm1 = rd(bc, wi - 1), xp1 = rd(bc, wi + 1);
        double y0 = 0.0, y1 = 0.0;
        y0 = y0 + (-1.0) * xp.x;  y1 = y1 + (-1.0) * xp.y;
        y0 = y0 + (-1.0) * xmn.x; y1 = y1 + (-1.0) * xmn.y;
        y0 = y0 + (-1.0) * xm1.x; y1 = y1 + (-1.0) * xm1.y;
        y0 = y0 + 6.0 * xc.x;     y1 = y1 + 6.0 * xc.y;
        y0 = y0 + (-1.0) * xp1.x; y1 = y1 + (-1.0) * xp1.y;
        y0 = y0 + (-1.0) * xpn.x; y1 = y1 + (-1.0) * xpn.y;
        y0 = y0 + (-1.0) * xn.x;  y1 = y1 + (-1.0) * xn.y;
        if (SPMV) {
            const int64_t r = (z0 + z) * P + xy0 + lr;
            if (okp) y[r] = y0;
            if (two) y[r + 1] = y1;
        } else {
            y0 = y0 - l * xc.x;
            y1 = y1 - l * xc.y;
            if (okp) acc = acc + (y0 * y0 + (two ? y1 * y1 : 0.0));
        }
        xp = xc;
        if (z + 2 <= zend) store_plane(bs);
        __syncthreads();
    }
    const double v = wave_sum(acc);
    if (lane == 0) ws[wave] = v;
    __syncthreads();
    if (tid == 0) partial[(int64_t)blockIdx.y * gridDim.x + blockIdx.x] = ((ws[0] + ws[1]) + ws[2]) + ws[3];
}

int main(int argc, char** argv) {
    const int nvec = argc > 1 ? atoi(argv[1]) : 32;
    const int64_t pad = P + 4096;  // >= the widest read past a column end (LDS windows: B + 2 rows)
    const int64_t ld = ((NR + 2 * pad) + 63) & ~(int64_t)63;
    double* X;
    CK(hipMalloc(&X, (size_t)ld * nvec * 8));
    CK(hipMemset(X, 0, (size_t)ld * nvec * 8));
    {
        std::vector<double> h(NR);
        for (int v = 0; v < nvec; ++v) {
            uint64_t s = 88172645463325252ull + v;
            for (int64_t i = 0; i < NR; ++i) {
                s ^= s << 13; s ^= s >> 7; s ^= s << 17;
                h[i] = (double)(s >> 11) * 0x1p-53 - 0.5;
            }
            CK(hipMemcpy(X + (size_t)v * ld + pad, h.data(), NR * 8, hipMemcpyHostToDevice));
        }
    }
    const double* X0 = X + pad;  // origin of column 0; column v at X0 + v ld
    std::vector<double> hl(nvec);
    for (int v = 0; v < nvec; ++v) hl[v] = 0.1 * v;
    double* lam;
    CK(hipMalloc(&lam, nvec * 8));
    CK(hipMemcpy(lam, hl.data(), nvec * 8, hipMemcpyHostToDevice));
    const int64_t npairs = NR / 2;
    double* part;
    // partials: one per (vector, block); the finest grid is the interleaved
    // kernel's 64 rows per block
    const size_t part_cap = (size_t)nvec * (size_t)(NR / 64 + 2);
    CK(hipMalloc(&part, part_cap * 8));
    auto check_grid = [&](int nb) {
        if ((size_t)nb * nvec > part_cap) {
            printf("grid %d x %d exceeds the partial buffer\n", nb, nvec);
            exit(2);
        }
    };
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    std::vector<double> ref;
    auto sums = [&](int nb) {
        std::vector<double> hp((size_t)nvec * nb), s(nvec, 0.0);
        CK(hipMemcpy(hp.data(), part, hp.size() * 8, hipMemcpyDeviceToHost));
        for (int v = 0; v < nvec; ++v)
            for (int b = 0; b < nb; ++b) s[v] += hp[(size_t)v * nb + b];
        return s;
    };
    auto report = [&](const char* name, float ms, int nb) {
        std::vector<double> s = sums(nb);
        double md = 0.0;
        if (ref.empty()) ref = s;
        for (int v = 0; v < nvec; ++v) md = fmax(md, fabs(s[v] - ref[v]) / fabs(ref[v]));
        printf("%-22s %8.2f us/vector  (%6.0f GB/s of x)  max rel diff %.2e\n", name, ms * 1e3 / nvec,
               NR * 8.0 / (ms * 1e-3 / nvec) / 1e9, md);
    };
#define RUN(MODE, CPB, PPT)                                                                                   \
    {                                                                                                         \
        const int nb = (int)((npairs + 256 * PPT - 1) / (256 * PPT));                                         \
        check_grid(nb);                                                                                       \
        dim3 g(nb, nvec / CPB);                                                                               \
        for (int rep = 0; rep < 2; ++rep) hipLaunchKernelGGL((k_res<MODE, CPB, PPT>), g, dim3(256), 0, 0, X0, ld, lam, part); \
        CK(hipEventRecord(e0));                                                                               \
        for (int rep = 0; rep < 5; ++rep) hipLaunchKernelGGL((k_res<MODE, CPB, PPT>), g, dim3(256), 0, 0, X0, ld, lam, part); \
        CK(hipEventRecord(e1));                                                                               \
        CK(hipEventSynchronize(e1));                                                                          \
        float ms;                                                                                             \
        CK(hipEventElapsedTime(&ms, e0, e1));                                                                 \
        char nm[64];                                                                                          \
        snprintf(nm, 64, "mode%d cpb%d ppt%d", MODE, CPB, PPT);                                               \
        report(nm, ms / 5, nb);                                                                               \
    }
#define RUNL(PPT, CPB)                                                                                        \
    {                                                                                                         \
        const int nb = (int)((NR + 512 * PPT - 1) / (512 * PPT));                                             \
        check_grid(nb);                                                                                       \
        dim3 g(nb, nvec / CPB);                                                                               \
        for (int rep = 0; rep < 2; ++rep) hipLaunchKernelGGL((k_res_lds<PPT>), g, dim3(256), 0, 0, X0, ld, CPB, lam, part); \
        CK(hipEventRecord(e0));                                                                               \
        for (int rep = 0; rep < 5; ++rep) hipLaunchKernelGGL((k_res_lds<PPT>), g, dim3(256), 0, 0, X0, ld, CPB, lam, part); \
        CK(hipEventRecord(e1));                                                                               \
        CK(hipEventSynchronize(e1));                                                                          \
        float ms;                                                                                             \
        CK(hipEventElapsedTime(&ms, e0, e1));                                                                 \
        char nm[64];                                                                                          \
        snprintf(nm, 64, "lds ppt%d cpb%d", PPT, CPB);                                                        \
        report(nm, ms / 5, nb);                                                                               \
    }
#define RUNI(G, RPT)                                                                                          \
    {                                                                                                         \
        constexpr int RPB = 4 * (64 / (G / 2));                                                               \
        const int nb = (int)((NR + RPB * RPT - 1) / (RPB * RPT));                                             \
        check_grid(nb);                                                                                       \
        dim3 g(nb, nvec / G);                                                                                 \
        const int64_t ldg = (NR + 2 * pad) * G;                                                               \
        double* Xi;                                                                                           \
        CK(hipMalloc(&Xi, (size_t)ldg * (nvec / G) * 8));                                                     \
        CK(hipMemset(Xi, 0, (size_t)ldg * (nvec / G) * 8));                                                   \
        {                                                                                                     \
            std::vector<double> hc(NR), hi((size_t)NR * G);                                                   \
            for (int gq = 0; gq < nvec / G; ++gq) {                                                           \
                for (int v = 0; v < G; ++v) {                                                                 \
                    CK(hipMemcpy(hc.data(), X0 + (size_t)(gq * G + v) * ld, NR * 8, hipMemcpyDeviceToHost)); \
                    for (int64_t i = 0; i < NR; ++i) hi[(size_t)i * G + v] = hc[i];                           \
                }                                                                                             \
                CK(hipMemcpy(Xi + (size_t)gq * ldg + pad * G, hi.data(), (size_t)NR * G * 8, hipMemcpyHostToDevice)); \
            }                                                                                                 \
        }                                                                                                     \
        const double* Xi0 = Xi + pad * G;                                                                     \
        for (int rep = 0; rep < 2; ++rep) hipLaunchKernelGGL((k_res_int<G, RPT>), g, dim3(256), 0, 0, Xi0, ldg, lam, part); \
        CK(hipEventRecord(e0));                                                                               \
        for (int rep = 0; rep < 5; ++rep) hipLaunchKernelGGL((k_res_int<G, RPT>), g, dim3(256), 0, 0, Xi0, ldg, lam, part); \
        CK(hipEventRecord(e1));                                                                               \
        CK(hipEventSynchronize(e1));                                                                          \
        float ms;                                                                                             \
        CK(hipEventElapsedTime(&ms, e0, e1));                                                                 \
        char nm[64];                                                                                          \
        snprintf(nm, 64, "interleaved G%d rpt%d", G, RPT);                                                    \
        report(nm, ms / 5, nb);                                                                               \
        CK(hipFree(Xi));                                                                                      \
    }
#define RUNZ(Z, D)                                                                                            \
    {                                                                                                         \
        constexpr int64_t NXY = (P + 255) / 256;                                                              \
        const int nb = (int)(NXY * ((N + Z - 1) / Z));                                                        \
        check_grid(nb);                                                                                       \
        dim3 g(nb, nvec);                                                                                     \
        for (int rep = 0; rep < 2; ++rep) hipLaunchKernelGGL((k_res_z<Z, D>), g, dim3(256), 0, 0, X0, ld, lam, part); \
        CK(hipEventRecord(e0));                                                                               \
        for (int rep = 0; rep < 5; ++rep) hipLaunchKernelGGL((k_res_z<Z, D>), g, dim3(256), 0, 0, X0, ld, lam, part); \
        CK(hipEventRecord(e1));                                                                               \
        CK(hipEventSynchronize(e1));                                                                          \
        float ms;                                                                                             \
        CK(hipEventElapsedTime(&ms, e0, e1));                                                                 \
        char nm[64];                                                                                          \
        snprintf(nm, 64, "plane march Z%d dpp%d", Z, (int)D);                                                 \
        report(nm, ms / 5, nb);                                                                               \
    }
#define RUNZP(Z) RUNZPS(Z, 0)
#define RUNZPS(Z, SK)                                                                                         \
    {                                                                                                         \
        constexpr int64_t NXY = ((P + 1) / 2 + 255) / 256;                                                    \
        const int nb = (int)(NXY * ((N + Z - 1) / Z));                                                        \
        check_grid(nb);                                                                                       \
        dim3 g(nb, nvec);                                                                                     \
        for (int rep = 0; rep < 2; ++rep) hipLaunchKernelGGL((k_res_zp<Z, SK>), g, dim3(256), 0, 0, X0, ld, lam, part); \
        CK(hipEventRecord(e0));                                                                               \
        for (int rep = 0; rep < 5; ++rep) hipLaunchKernelGGL((k_res_zp<Z, SK>), g, dim3(256), 0, 0, X0, ld, lam, part); \
        CK(hipEventRecord(e1));                                                                               \
        CK(hipEventSynchronize(e1));                                                                          \
        float ms;                                                                                             \
        CK(hipEventElapsedTime(&ms, e0, e1));                                                                 \
        char nm[64];                                                                                          \
        snprintf(nm, 64, "pair plane march Z%d skip%d", Z, SK);                                                          \
        report(nm, ms / 5, nb);                                                                               \
    }
    double* Ybuf;
    CK(hipMalloc(&Ybuf, (size_t)ld * nvec * 8));
    double* Y0 = Ybuf + pad;
#define RUNZW(Z, SP)                                                                                          \
    {                                                                                                         \
        constexpr int64_t NXY = (P + 511) / 512;                                                              \
        const int nb = (int)(NXY * ((N + Z - 1) / Z));                                                        \
        check_grid(nb);                                                                                       \
        dim3 g(nb, nvec);                                                                                     \
        for (int rep = 0; rep < 2; ++rep) hipLaunchKernelGGL((k_res_zw<Z, SP>), g, dim3(256), 0, 0, X0, ld, lam, part, Y0); \
        CK(hipEventRecord(e0));                                                                               \
        for (int rep = 0; rep < 5; ++rep) hipLaunchKernelGGL((k_res_zw<Z, SP>), g, dim3(256), 0, 0, X0, ld, lam, part, Y0); \
        CK(hipEventRecord(e1));                                                                               \
        CK(hipEventSynchronize(e1));                                                                          \
        float ms;                                                                                             \
        CK(hipEventElapsedTime(&ms, e0, e1));                                                                 \
        char nm[64];                                                                                          \
        snprintf(nm, 64, "lds plane march Z%d spmv%d", Z, (int)SP);                                           \
        if (SP) printf("%-22s %8.2f us/vector\n", nm, ms * 1e3 / 5 / nvec);                                 \
        else report(nm, ms / 5, nb);                                                                          \
    }
    RUN(0, 1, 1);
    RUNZW(4, false);
    RUNZW(8, false);
    RUNZW(16, false);
    RUNZW(32, false);
    RUNZW(8, true);
    RUNZW(16, true);
    RUNZP(8);
    RUNZPS(8, 1);
    RUNZPS(8, 2);
    RUNZPS(8, 3);
    for (int nbr : {2048, 4096, 8192}) {
        check_grid(nbr);
        dim3 g(nbr, nvec);
        hipLaunchKernelGGL(k_read, g, dim3(256), 0, 0, X0, ld, part);
        CK(hipEventRecord(e0));
        for (int rep = 0; rep < 5; ++rep) hipLaunchKernelGGL(k_read, g, dim3(256), 0, 0, X0, ld, part);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        printf("streaming read %5d blk %8.2f us/vector  (%6.0f GB/s)\n", nbr, ms * 1e3 / 5 / nvec,
               NR * 8.0 / (ms * 1e-3 / 5 / nvec) / 1e9);
    }
    return 0;
}
