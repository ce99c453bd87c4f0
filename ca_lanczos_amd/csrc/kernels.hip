// kernels.hip -- hand-written gfx950 (CDNA4) kernels of the CA-Lanczos hot path.
//
// Compiled with -ffp-contract=off: every a*b+c below rounds twice, exactly
// like the reference's (and the oracle's) unfused sparse/dense arithmetic, so
// the SpMV and the Newton matrix-powers recurrence are bit-identical to a
// sequential CSR SpMV.  MFMA accumulates inside the matrix core.
//
// Kernels:
//   k_spmv          CSR-stream SpMV: coalesced val/col loads of a row block,
//                   products staged in LDS, sequential per-row sums
//                   (bit-exact), fused Newton shift (matrix_powers_newton.m:31-47).
//   k_spmv_pat_lds, k_spmv_pair
//                   row-pattern SpMV (lossless pattern table, one / two rows
//                   per lane), same arithmetic, same shift epilogue; the pair
//                   kernel also takes two row ranges (the split matrix powers).
//   k_spmv_pair_resid
//                   Ritz residual sums ||A x - l x||^2, ||l x||^2 on the pair
//                   patterns (compute_ritz_rnorm), nothing stored.
//   k_rowapply      the hot block-orthogonalisation sweeps (s <= 8): Gram
//                   tiles through LDS onto v_mfma_f64_16x16x4f64, the
//                   coefficient apply in registers, the chained pass B.
//   k_orth_coef     the s x s algebra between the sweeps; publishes R / RY.
//   k_gram, k_apply tall-skinny C = A^T B / Y = P M (+ Grams) on MFMA tiles
//                   for the generic widths ('full', restarts).
//   k_apply_rows    row-parallel store-only Y = P M (wide panels, up to 64
//                   outputs per launch).
//   k_reduce        fixed-order sum of block partials.
//   k_dot, k_axpy_sub(_dev), k_div(_sqrt), k_gather, k_spmv_resid,
//   k_form_projM, k_abs_rowsum: small vector kernels.
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <type_traits>
#include <utility>

#include "cal_internal.hpp"

namespace cal {

typedef double d4 __attribute__((ext_vector_type(4)));
typedef double d2 __attribute__((ext_vector_type(2)));

constexpr int kSpmvThreads = 256;
constexpr int kSpmvNnz = 2048;  // LDS-staged nonzeros per row block (16 KiB)
// the plane march (k_spmv_planes, k_resid_planes): planes per block of the
// residual kernel (rows of a plane per block: kPlaneBlockRows)
#ifndef CAL_RESID_PLANES
#define CAL_RESID_PLANES 32
#endif
constexpr int kResidPlanes = CAL_RESID_PLANES;

// Column c of a panel.  The segment table is taken by value and read with
// static indices only: binding a reference to a by-value kernel argument
// makes the compiler copy the struct to scratch in every thread (184 B per
// thread, re-read per column).
template <typename T, typename PT>
__device__ __forceinline__ T* seg_col(const PT P, int c) {
    T* res = P.ptr[0];
    int base = 0;
#pragma unroll
    for (int q = 0; q < kMaxSeg; ++q) {
        const int nq = q < P.nseg ? P.ncol[q] : 0;
        if (c >= base && c < base + nq) res = P.ptr[q] + (int64_t)(c - base) * P.ld[q];
        base += nq;
    }
    return res;
}
__device__ __forceinline__ const double* pcol(const Panel P, int c) { return seg_col<const double>(P, c); }
__device__ __forceinline__ double* pcol_out(const PanelOut P, int c) { return seg_col<double>(P, c); }

__device__ __forceinline__ d4 mfma64(double a, double b, d4 c) {
    return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}

// --------------------------------------------------------------------------
// SpMV (SpMV.m:8) with the Newton epilogue (matrix_powers_newton.m:28-43)
// --------------------------------------------------------------------------
template <int MODE>
__device__ __forceinline__ double spmv_epilogue(double sum, const SpmvArgs& a, int r) {
    if (MODE == 0 || MODE == 3) return sum;
    double t = a.shift * a.x[r];
    double y = sum - t;
    if (MODE == 2) {
        double u = a.im2 * a.xprev[r];
        y = y + u;
    }
    return y;
}

// XCD-aware block order: the hardware deals consecutive blocks round-robin
// over the 8 XCDs (each with its own L2); the remap gives each XCD one
// contiguous run of blocks, so the x lines a row block gathers from its
// neighbours' rows are found in that XCD's L2.
__device__ __forceinline__ int xcd_remap(int b, int nwg) {
    const int q = nwg >> 3, r = nwg & 7, x = b & 7, i = b >> 3;
    return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + i;
}

// NT: col / val stream once per SpMV, so they are loaded non-temporally and
// leave the caches to x, whose lines the neighbouring rows gather again.
// V = 2: each thread loads two consecutive nonzeros (one 8-B col pair, one
// 16-B val pair), half the load instructions of V = 1.  Same products, same
// per-row order.
template <bool NT, typename T>
__device__ __forceinline__ T ldnt(const T* p) {
    if constexpr (NT) return __builtin_nontemporal_load(p);
    else return *p;
}

template <int MODE, int NIT, bool NT, int V>
__global__ __launch_bounds__(kSpmvThreads) void k_spmv(SpmvArgs a) {
    __shared__ double prod[kSpmvNnz];
    const int b = a.xcd ? xcd_remap(blockIdx.x, gridDim.x) : (int)blockIdx.x;
    const int tid = threadIdx.x;
    const int r0 = a.blk[b], r1 = a.blk[b + 1];
    const int p0 = a.rowptr[r0], p1 = a.rowptr[r1];
    const int cnt = p1 - p0;
    // MODE 3: normest's S * (x / norm(x)), the division per gathered element
    // (MATLAB's x = x/normx, then S*x: the same quotients and products)
    const double sx = MODE == 3 ? sqrt(*a.xnrm) : 1.0;
    if (cnt <= kSpmvNnz) {
        if (cnt > 0) {
            // all loads first (clamped, never branched around: one vmcnt wait
            // per phase), then the dependent x gathers, then LDS products.
            const int pl = p1 - 1;
            constexpr int NI = (NIT + V - 1) / V;
            int ci[NI][V];
            double v[NI][V], xv[NI][V];
#pragma unroll
            for (int it = 0; it < NI; ++it) {
#pragma unroll
                for (int u = 0; u < V; ++u) {
                    const int p = min(p0 + (it * kSpmvThreads + tid) * V + u, pl);
                    ci[it][u] = ldnt<NT>(a.col + p);
                    v[it][u] = ldnt<NT>(a.val + p);
                }
            }
#pragma unroll
            for (int it = 0; it < NI; ++it)
#pragma unroll
                for (int u = 0; u < V; ++u) {
                    xv[it][u] = a.x[ci[it][u]];
                    if (MODE == 3) xv[it][u] = xv[it][u] / sx;
                }
#pragma unroll
            for (int it = 0; it < NI; ++it)
#pragma unroll
                for (int u = 0; u < V; ++u) {
                    const int q = (it * kSpmvThreads + tid) * V + u;
                    if (q < cnt) prod[q] = v[it][u] * xv[it][u];
                }
        }
        __syncthreads();
        const int r = r0 + tid;
        if (r < r1) {
            const int q0 = a.rowptr[r] - p0, q1 = a.rowptr[r + 1] - p0;
            double sum = 0.0;
            for (int j = q0; j < q1; ++j) sum = sum + prod[j];
            a.y[r] = spmv_epilogue<MODE>(sum, a, r);
        }
    } else {
        // one long row (> kSpmvNnz nonzeros): chunked, still summed in order
        double sum = 0.0;
        for (int c = p0; c < p1; c += kSpmvNnz) {
            const int m = min(kSpmvNnz, p1 - c);
            for (int q = tid; q < m; q += kSpmvThreads) {
                double xq = a.x[a.col[c + q]];
                if (MODE == 3) xq = xq / sx;
                prod[q] = a.val[c + q] * xq;
            }
            __syncthreads();
            if (tid == 0)
                for (int j = 0; j < m; ++j) sum = sum + prod[j];
            __syncthreads();
        }
        if (tid == 0) a.y[r0] = spmv_epilogue<MODE>(sum, a, r0);
    }
}

template <int MODE, bool NT, int V>
static hipError_t launch_spmv_mode2(const SpmvArgs& a, int nit, hipStream_t st) {
    dim3 g(a.nblk), b(kSpmvThreads);
    switch (nit) {
        case 1: hipLaunchKernelGGL((k_spmv<MODE, 1, NT, V>), g, b, 0, st, a); break;
        case 2: hipLaunchKernelGGL((k_spmv<MODE, 2, NT, V>), g, b, 0, st, a); break;
        case 3: hipLaunchKernelGGL((k_spmv<MODE, 3, NT, V>), g, b, 0, st, a); break;
        case 4: hipLaunchKernelGGL((k_spmv<MODE, 4, NT, V>), g, b, 0, st, a); break;
        case 5: hipLaunchKernelGGL((k_spmv<MODE, 5, NT, V>), g, b, 0, st, a); break;
        case 6: hipLaunchKernelGGL((k_spmv<MODE, 6, NT, V>), g, b, 0, st, a); break;
        case 7: hipLaunchKernelGGL((k_spmv<MODE, 7, NT, V>), g, b, 0, st, a); break;
        default: hipLaunchKernelGGL((k_spmv<MODE, 8, NT, V>), g, b, 0, st, a); break;
    }
    return hipGetLastError();
}

// one nonzero per thread and iteration (two: slower on both matrices below).
// col / val stream once per SpMV: when the matrix is larger than the
// Infinity Cache (a.nt, set by spmv_dev) they are loaded non-temporally, so
// the cache keeps x's lines for the neighbouring rows' gathers -- 200 vs
// 208 us on lap3d_215 in CSR (1.03 GB); a matrix that fits (circuit_1259,
// 123 MB) is still there at the next SpMV and keeps plain loads (23.0 us,
// 31.5 non-temporal; profiles/r04/csr_variants)
template <int MODE>
static hipError_t launch_spmv_mode(const SpmvArgs& a, int nit, hipStream_t st) {
    return a.nt ? launch_spmv_mode2<MODE, true, 1>(a, nit, st) : launch_spmv_mode2<MODE, false, 1>(a, nit, st);
}

hipError_t launch_spmv(const SpmvArgs& a0, hipStream_t st) {
    if (a0.nblk <= 0) return hipSuccess;
    SpmvArgs a = a0;
    a.xcd = 1;  // XCD-contiguous row blocks (hardware order measured 1.08x -> 1.35x traffic)
    // a.mode carries the per-matrix iteration count in bits 8..15
    const int nit = (a.mode >> 8) & 0xff;
    switch (a.mode & 0xff) {
        case 0: return launch_spmv_mode<0>(a, nit, st);
        case 1: return launch_spmv_mode<1>(a, nit, st);
        case 2: return launch_spmv_mode<2>(a, nit, st);
        case 3: return a.xnrm ? launch_spmv_mode<3>(a, nit, st) : hipErrorInvalidValue;
        default: return hipErrorInvalidValue;
    }
}

// --------------------------------------------------------------------------
// Row-pattern SpMV (same arithmetic as k_spmv, different storage): thread
// <-> row; the row's pattern id (2 B) selects its (col - row, value) list in
// a small L1/L2-resident table.  HBM traffic per row: 2 B of id + the x
// gathers (contiguous across a wave for a stencil) + 8 B of y.
// XCD-aware remap: the hardware deals blocks round-robin over the 8 XCDs;
// remapping gives each XCD a contiguous run of rows, so the x lines of the
// neighbouring planes (col - row = +-N^2) are re-read from that XCD's L2.
// --------------------------------------------------------------------------
// (xcd_remap: defined above k_spmv)

// fixed-order butterfly sum over the 64 lanes of a wave
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v = v + __shfl_xor(v, off, 64);
    return v;
}

template <int MODE, int MAXLEN>
__global__ __launch_bounds__(256) void k_spmv_pat(PatArgs a) {
    const int lb = xcd_remap(blockIdx.x, gridDim.x);
    const int64_t r = (int64_t)lb * 256 + threadIdx.x;
    if (r >= a.n) return;
    const int pid = a.pat[r];
    const int2 pi = a.pinfo[pid];
    const int last = pi.y > 0 ? pi.y - 1 : 0;
    double v[MAXLEN], xv[MAXLEN];
#pragma unroll
    for (int e = 0; e < MAXLEN; ++e) {  // clamped, unconditional loads
        const int ee = pi.x + (e < pi.y ? e : last);
        v[e] = a.pval[ee];
        xv[e] = a.x[r + a.pdelta[ee]];
    }
    double sum = 0.0;
#pragma unroll
    for (int e = 0; e < MAXLEN; ++e) {  // CSR order, unfused: bit-identical to k_spmv
        const double t = v[e] * xv[e];
        if (e < pi.y) sum = sum + t;
    }
    double y = sum;
    if (MODE != 0) {
        const double t = a.shift * a.x[r];
        y = y - t;
        if (MODE == 2) {
            const double u = a.im2 * a.xprev[r];
            y = y + u;
        }
    }
    a.y[r] = y;
}

// Row-pattern SpMV with the pattern table (npat*8 + nent*12 bytes) staged
// into LDS, so the per-row lookups are LDS broadcasts and the vector-memory
// path only carries the 2-B ids, the x gathers and the y stores.  The grid is
// persistent: each block sweeps a contiguous run of 256-row chunks and the
// XCD remap makes the runs of one XCD contiguous.  The blocks of an XCD move
// in near lockstep, so the +-plane neighbour rows a block gathers are the
// rows another block of the same XCD is reading at the same time (measured:
// 146 MB fetched per SpMV vs 205 MB for an interleaved sweep, same time).
// The ids of the next chunk are loaded before this chunk's gathers and store
// (vmcnt retires in order: an id load issued after the y store would wait
// for that store).
template <int MODE, int MAXLEN>
__global__ __launch_bounds__(256) void k_spmv_pat_lds(PatArgs a, int npat, int nent, int chunks_per_block) {
    extern __shared__ __attribute__((aligned(16))) double lds_tab[];
    int2* s_info = reinterpret_cast<int2*>(lds_tab);
    double* s_val = lds_tab + npat;
    int* s_delta = reinterpret_cast<int*>(s_val + nent);
    for (int i = threadIdx.x; i < npat; i += 256) s_info[i] = a.pinfo[i];
    for (int i = threadIdx.x; i < nent; i += 256) {
        s_val[i] = a.pval[i];
        s_delta[i] = a.pdelta[i];
    }
    __syncthreads();
    const int lb = xcd_remap(blockIdx.x, gridDim.x);
    const int c0 = lb * chunks_per_block;
    const int c1 = min(c0 + chunks_per_block, a.nblk);
    constexpr int nbx = 1;
    auto row_of = [&](int ch) -> int64_t {
        const int64_t r = (int64_t)ch * 256 + threadIdx.x;
        return ch < c1 && r < a.n ? r : -1;
    };
    int64_t rn = row_of(c0);
    int pidn = a.pat[rn >= 0 ? rn : 0];
    for (int ch = c0; ch < c1; ch += nbx) {
        const int64_t rv = rn;
        const int64_t r = rv >= 0 ? rv : 0;  // row 0 exists (a.n > 0): harmless reads
        const int2 pi = s_info[pidn];
        rn = row_of(ch + nbx);
        pidn = a.pat[rn >= 0 ? rn : 0];
        const int last = pi.y > 0 ? pi.y - 1 : 0;
        double xv[MAXLEN];
#pragma unroll
        for (int e = 0; e < MAXLEN; ++e) {
            const int ee = pi.x + (e < pi.y ? e : last);
            xv[e] = a.x[r + s_delta[ee]];
        }
        double sum = 0.0;
#pragma unroll
        for (int e = 0; e < MAXLEN; ++e) {
            const double t = s_val[pi.x + (e < pi.y ? e : 0)] * xv[e];
            const double acc = sum + t;
            sum = e < pi.y ? acc : sum;
        }
        double y = sum;
        if (MODE != 0) {
            const double t = a.shift * a.x[r];
            y = y - t;
            if (MODE == 2) {
                const double u = a.im2 * a.xprev[r];
                y = y + u;
            }
        }
        if (rv >= 0) a.y[r] = y;
    }
}

// Two rows per lane on pair patterns (runtime.cpp build_pair_patterns):
// rows 2t and 2t+1 share one merged table entry list, so every entry is ONE
// 16-B load x[r+o .. r+o+1] serving both rows -- the wave issues half the
// gather instructions and cache-line requests of a row-per-lane kernel, and
// y leaves as one 16-B store.  Entry flags mark which row adds the entry;
// each row adds exactly its own entries in column order (bit-identical to
// CSR).  Pairs marked kPairSplit (rare: domain ends, odd n) take the
// per-row path.  The XCD remap makes each XCD's chunks contiguous, so the
// +-plane neighbour lines stay in its L2.  Requires x, y (and xprev) 16-B
// aligned at the origin (checked at launch).
__device__ __forceinline__ double2 ld16(const double* p) {
    double2 v;
    __builtin_memcpy(&v, p, 16);  // 8-B aligned for odd offsets: still one dwordx4
    return v;
}

// Lane-shared slot loads (PatArgs::pmid = MAXLEN / 2: slots pmid -+ 1 are the
// offsets -+1).  When the 64 lanes of a wave hold 64 consecutive row pairs,
// slot -1 (x[r0 - 1], x[r0]) and slot +1 (x[r0 + 1], x[r0 + 2]) are the
// neighbouring lanes' centre loads x[r0 .. r0 + 1], moved over by one DPP
// wave shift per half, and the wave's two outer rows come from one broadcast
// load each: 5 of the 7 slots of a 7-point stencil are vector loads, and the
// centre also serves the shift term.  The values are the loaded ones, so the
// sums are bit-identical.  Other waves (a launch's tail, a two-range launch's
// gap) load every slot.
template <int CTRL>
__device__ __forceinline__ double dpp_wave_shift(double v, double edge) {
    const unsigned long long b = (unsigned long long)__double_as_longlong(v);
    const unsigned long long o = (unsigned long long)__double_as_longlong(edge);
    const unsigned lo = (unsigned)__builtin_amdgcn_update_dpp((int)(unsigned)o, (int)(unsigned)b, CTRL, 0xf, 0xf, false);
    const unsigned hi =
        (unsigned)__builtin_amdgcn_update_dpp((int)(unsigned)(o >> 32), (int)(unsigned)(b >> 32), CTRL, 0xf, 0xf, false);
    return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}
constexpr int kDppWaveShl1 = 0x130;  // lane i <- lane i + 1 (lane 63 keeps `edge`)
constexpr int kDppWaveShr1 = 0x138;  // lane i <- lane i - 1 (lane 0 keeps `edge`)

// wave-uniform: the lanes' stored pair indices t are consecutive; b0 = lane 0's
template <int MAXLEN>
__device__ __forceinline__ bool pair_lane_run(const PatArgs& a, int64_t t, int64_t& b0) {
    if (!(MAXLEN >= 3 && (MAXLEN & 1)) || a.pmid != MAXLEN / 2) return false;
    const int64_t base = t - (int64_t)(threadIdx.x & 63);
    const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)base);
    const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)((unsigned long long)base >> 32));
    b0 = (int64_t)(((unsigned long long)hi << 32) | lo);
    return __builtin_amdgcn_ballot_w64(base == b0) == ~0ull;
}

template <int MAXLEN>
__device__ __forceinline__ void pair_slot_loads(const PatArgs& a, const double* x, int64_t r0, bool run, int64_t b0,
                                                double2 (&xc)[MAXLEN]) {
    constexpr int Z = MAXLEN / 2;
#pragma unroll
    for (int e = 0; e < MAXLEN; ++e) {
        if (MAXLEN >= 3 && (MAXLEN & 1) && run && (e == Z - 1 || e == Z + 1)) continue;
        int64_t ad = r0 + a.pslot[e];
        ad = ad < a.xlo ? a.xlo : (ad > a.xhi - 2 ? a.xhi - 2 : ad);
        xc[e] = ld16(x + ad);
    }
    if constexpr (MAXLEN >= 3 && (MAXLEN & 1)) {
        if (!run) return;
        int64_t el = 2 * b0 - 1, er = 2 * b0 + 128;  // x[lane 0's r0 - 1], x[lane 63's r0 + 2]
        el = el < a.xlo ? a.xlo : (el > a.xhi - 1 ? a.xhi - 1 : el);
        er = er < a.xlo ? a.xlo : (er > a.xhi - 1 ? a.xhi - 1 : er);
        const double xl = x[el], xr = x[er];
        xc[Z - 1] = make_double2(dpp_wave_shift<kDppWaveShr1>(xc[Z].y, xl), xc[Z].x);
        xc[Z + 1] = make_double2(xc[Z].y, dpp_wave_shift<kDppWaveShl1>(xc[Z].x, xr));
    }
}

// The pair table (a few KB) is staged in LDS per block; the block's id
// load is issued before the staging loads so both share one memory round
// trip.  Split pairs (and the lone last row of an odd n) read the row
// tables from global memory (rare).
template <int MODE, int MAXLEN, bool CANON, int TB = 256>
__global__ __launch_bounds__(TB) void k_spmv_pair(PatArgs a, const uint16_t* __restrict__ ppat,
                                                  const int2* __restrict__ ppinfo, const int* __restrict__ ppoff,
                                                  const double2* __restrict__ ppval) {
    extern __shared__ __attribute__((aligned(16))) double lds_pair[];
    double2* s_pv = reinterpret_cast<double2*>(lds_pair);
    int2* s_pinfo = reinterpret_cast<int2*>(s_pv + a.npent);
    int* s_poff = reinterpret_cast<int*>(s_pinfo + (CANON ? 0 : a.nppat));
    const int tid = threadIdx.x;
    const int64_t npairs = (a.n + 1) >> 1;  // compact pairs (both ranges)
    const int64_t tc = (int64_t)xcd_remap(blockIdx.x, gridDim.x) * TB + tid;
    const int64_t tcl = tc < npairs ? tc : npairs - 1;
    const int64_t t = tcl + (tcl >= a.gap_at ? a.gap : 0);  // stored pair (skips the gap)
    const int id = ppat[t];
    // canonical slots: slot e always loads x[r + pslot[e] .. +1] (clamped to
    // the column; a slot no row of the pair uses is discarded), so the x
    // loads depend on neither the id nor the table and leave first
    double2 xc[CANON ? MAXLEN : 1];
    double2 xs = make_double2(0.0, 0.0), xp = make_double2(0.0, 0.0);  // shift terms
    {
        const int64_t r0 = 2 * t;
        bool mid = false;
        if constexpr (CANON) {
            int64_t b0 = 0;
            const bool run = pair_lane_run<MAXLEN>(a, t, b0);
            pair_slot_loads<MAXLEN>(a, a.x, r0, run, b0, xc);
            mid = MAXLEN >= 3 && (MAXLEN & 1) && a.pmid == MAXLEN / 2;
        }
        const int64_t rc = r0 < a.xhi - 2 ? r0 : a.xhi - 2;
        if constexpr (MODE != 0) {
            if constexpr (CANON) xs = mid ? xc[MAXLEN / 2] : ld16(a.x + rc);  // the centre slot is x[rc]
            else xs = ld16(a.x + rc);
        }
        if (MODE == 2) xp = ld16(a.xprev + rc);
    }
    for (int i = tid; i < a.npent; i += TB) {
        s_pv[i] = ppval[i];
        s_poff[i] = ppoff[i];
    }
    if (!CANON)
        for (int i = tid; i < a.nppat; i += TB) s_pinfo[i] = ppinfo[i];
    __syncthreads();
    if (tc >= npairs) return;
    const int64_t r = 2 * t;
    if (id != kPairSplit) {  // both rows exist (the lone last row is split)
        // canonical tables: every pair pattern has MAXLEN entries in one
        // global slot order -> entry id * MAXLEN + e, no length checks
        const int2 pi = CANON ? make_int2(id * MAXLEN, MAXLEN) : s_pinfo[id];
        const int last = pi.y > 0 ? pi.y - 1 : 0;
        int code[MAXLEN];
        double2 xv[MAXLEN];
#pragma unroll
        for (int e = 0; e < MAXLEN; ++e) {
            code[e] = s_poff[pi.x + (CANON || e < pi.y ? e : last)];
            if (!CANON) xv[e] = ld16(a.x + r + (code[e] >> 2));
        }
        if (CANON)  // loads issued before the id and table arrive (see above)
#pragma unroll
            for (int e = 0; e < MAXLEN; ++e) xv[e] = xc[e];
        double y0 = 0.0, y1 = 0.0;
#pragma unroll
        for (int e = 0; e < MAXLEN; ++e) {
            const double2 v = s_pv[pi.x + (CANON || e < pi.y ? e : last)];
            const double t0 = v.x * xv[e].x, t1 = v.y * xv[e].y;
            double a0 = y0 + t0, a1 = y1 + t1;
            // both sums computed unconditionally (the selects stay v_cndmask;
            // otherwise the compiler branches and splits the 16-B loads)
            asm volatile("" : "+v"(a0), "+v"(a1));
            y0 = ((CANON || e < pi.y) && (code[e] & 1)) ? a0 : y0;
            y1 = ((CANON || e < pi.y) && (code[e] & 2)) ? a1 : y1;
        }
        if (MODE != 0) {
            const double u0 = a.shift * xs.x, u1 = a.shift * xs.y;
            y0 = y0 - u0;
            y1 = y1 - u1;
            if (MODE == 2) {
                const double w0 = a.im2 * xp.x, w1 = a.im2 * xp.y;
                y0 = y0 + w0;
                y1 = y1 + w1;
            }
        }
        double2 o;
        o.x = y0;
        o.y = y1;
        *reinterpret_cast<double2*>(a.y + r) = o;
        return;
    }
    // split pair: each row on its own from the row tables
    for (int k = 0; k < 2 && r + k < a.n + 2 * a.gap; ++k) {
        const int64_t rr = r + k;
        const int2 pi = a.pinfo[a.pat[rr]];
        double sum = 0.0;
        for (int e = 0; e < pi.y; ++e) {
            const double tv = a.pval[pi.x + e] * a.x[rr + a.pdelta[pi.x + e]];
            sum = sum + tv;
        }
        double y = sum;
        if (MODE != 0) {
            const double u = a.shift * a.x[rr];
            y = y - u;
            if (MODE == 2) {
                const double w = a.im2 * a.xprev[rr];
                y = y + w;
            }
        }
        a.y[rr] = y;
    }
}

// Ritz residual partials ||A x - l x||^2 and ||l x||^2 for a real Ritz value
// l (compute_ritz_rnorm, ca_lanczos.m:88-97) on the canonical pair patterns:
// the products and their order are k_spmv_pair's MODE 1 (y = A x - l x),
// nothing is stored, and each block leaves its two sums entry-major in
// partial[e * gridDim.x + block] (e = 0 residual, 1 scale).
template <int MAXLEN>
__global__ __launch_bounds__(256) void k_spmv_pair_resid(PatArgs a, const uint16_t* __restrict__ ppat,
                                                        const int* __restrict__ ppoff,
                                                        const double2* __restrict__ ppval,
                                                        double* __restrict__ partial) {
    extern __shared__ __attribute__((aligned(16))) double lds_pair[];
    double2* s_pv = reinterpret_cast<double2*>(lds_pair);
    int* s_poff = reinterpret_cast<int*>(s_pv + a.npent);
    __shared__ double ws[2][4];
    const int tid = threadIdx.x;
    const int64_t npairs = (a.n + 1) >> 1;
    const int64_t t = (int64_t)xcd_remap(blockIdx.x, gridDim.x) * 256 + tid;
    const int64_t tcl = t < npairs ? t : npairs - 1;
    const int id = ppat[tcl];
    const int64_t r0 = 2 * tcl;
    double2 xc[MAXLEN];
    int64_t b0 = 0;
    const bool run = pair_lane_run<MAXLEN>(a, tcl, b0);
    pair_slot_loads<MAXLEN>(a, a.x, r0, run, b0, xc);
    const bool mid = MAXLEN >= 3 && (MAXLEN & 1) && a.pmid == MAXLEN / 2;
    const double2 xs = mid ? xc[MAXLEN / 2] : ld16(a.x + (r0 < a.xhi - 2 ? r0 : a.xhi - 2));
    for (int i = tid; i < a.npent; i += 256) {
        s_pv[i] = ppval[i];
        s_poff[i] = ppoff[i];
    }
    __syncthreads();
    double num = 0.0, den = 0.0;
    if (t < npairs) {
        if (id != kPairSplit) {
            const int base = id * MAXLEN;
            double y0 = 0.0, y1 = 0.0;
#pragma unroll
            for (int e = 0; e < MAXLEN; ++e) {
                const int code = s_poff[base + e];
                const double2 v = s_pv[base + e];
                const double t0 = v.x * xc[e].x, t1 = v.y * xc[e].y;
                double a0 = y0 + t0, a1 = y1 + t1;
                asm volatile("" : "+v"(a0), "+v"(a1));
                y0 = (code & 1) ? a0 : y0;
                y1 = (code & 2) ? a1 : y1;
            }
            const double u0 = a.shift * xs.x, u1 = a.shift * xs.y;
            y0 = y0 - u0;
            y1 = y1 - u1;
            // an odd local slab's last row pairs with the first stored ghost
            // row (distributed layout, not split): that row belongs to the
            // next rank and must not enter this rank's sums
            const bool two = r0 + 1 < a.n;
            num = y0 * y0 + (two ? y1 * y1 : 0.0);
            den = u0 * u0 + (two ? u1 * u1 : 0.0);
        } else {  // split pair: each row from the row tables
            for (int k = 0; k < 2 && r0 + k < a.n; ++k) {
                const int64_t rr = r0 + k;
                const int2 pi = a.pinfo[a.pat[rr]];
                double sum = 0.0;
                for (int e = 0; e < pi.y; ++e) {
                    const double tv = a.pval[pi.x + e] * a.x[rr + a.pdelta[pi.x + e]];
                    sum = sum + tv;
                }
                const double u = a.shift * a.x[rr];
                const double y = sum - u;
                num = num + y * y;
                den = den + u * u;
            }
        }
    }
    num = wave_sum(num);
    den = wave_sum(den);
    const int lane = tid & 63, wave = tid >> 6;
    if (lane == 0) {
        ws[0][wave] = num;
        ws[1][wave] = den;
    }
    __syncthreads();
    if (tid == 0) {
        partial[blockIdx.x] = ((ws[0][0] + ws[0][1]) + ws[0][2]) + ws[0][3];
        partial[gridDim.x + blockIdx.x] = ((ws[1][0] + ws[1][1]) + ws[1][2]) + ws[1][3];
    }
}

constexpr size_t kPatLdsMax = 64 * 1024;

// the pair kernel needs 16-B aligned columns, rows <= 8 entries and an LDS-sized pair table
bool spmv_pat_pair_path(const PatArgs& a) {
    const bool al16 = (((uintptr_t)a.x | (uintptr_t)a.y | (uintptr_t)(a.mode == 2 ? a.xprev : nullptr)) & 15) == 0;
    const size_t lds2 = (size_t)a.npent * 20 + (size_t)a.nppat * 8 + 16;
    return a.ppat && al16 && a.maxlen <= 8 && lds2 <= kPatLdsMax;
}

// ---- the plane march -------------------------------------------------------
// For matrices in canonical slots -P < ... < +P (pslot[0] = -P, pslot[L-1] =
// +P, P >= 256) whose inner slots reach H <= 256 rows -- the 7-point (P =
// N^2, N < 256) and 5-point (P = N) Laplacians -- on a single slab.  A block
// owns the rows xy0 .. xy0 + 511 of every plane (r = xy + z P) for Z planes;
// lane t owns the row pair xy0 + 2t, + 1.  Per plane the block stages the
// window x[zP + xy0 - H, zP + xy0 + 512 + H) in LDS, split by row parity:
// E[p] = x(g + 2p), O[p] = x(g + 2p + 1) with g = zP + xy0 - H, so that
// every slot of a row pair is read as 8-B values at consecutive addresses
// across the lanes (ds_read_b64, conflict-free; the pair layout's 16-B lane
// stride made every 8-B read 2-way and ds_read2_b64 runs at half rate).
// Each lane loads its own row pair (pair t + H/2 of the window) with one
// 16-B buffer load and keeps it in registers for three planes: as the +P
// slot of plane z - 1, the centre of plane z, the -P slot of plane z + 1;
// lanes t < H also load one halo pair.  Plane z0 + j + 2 is loaded at the
// top of step j and stored at its end, so the loads have a plane's work to
// land.  Rows outside the column read 0 (a negative row's 32-bit byte offset
// is >= 2^31, past the descriptor's range, as is a row at or past ld; ld <
// 2^28).  Each x value leaves HBM about once ((Z + 2) / Z: a block also
// stages its neighbours' first and last plane); the in-plane gathers are LDS
// reads.  When P is odd the plane's last pair straddles into the next plane:
// only its first row belongs to the block.
//
// Every row adds its own entries in slot (= column) order.  Where some row of
// a wave lacks slot e (the host's per-wave OR of the rows' missing slots,
// DevMatrix::wavemask, one uniform dword per plane and block), slot e's x
// values enter each row ANDed with the row's mask bit, i.e. as +0.0 where the
// row has no entry: 0 * (+0.0) adds a zero, which leaves a running sum that
// is never -0.0 unchanged, and a non-finite x outside a row never leaks into
// it (the SpMV's contract, k_spmv_pair).  A slot every row of the wave has is
// added unmasked.  NEG1 (uniform values, -1 at every slot but the middle: the
// Laplacians) adds y - x for those slots: (-1) * x is exact, so y + (-1) * x
// and y - x are the same bits.  So the sums are the bits of k_spmv /
// k_spmv_pair.
// KM = 0: uniform slot values (cval; every row with an entry at slot e has
// the value cval[e], as in the Laplacians): the keys are the rows' slot mask
// bytes.  KM = 1 / 2: the keys are the rows' pattern ids (1 / 2 B) into the
// LDS value / mask tables.
template <int MAXLEN, int KM, bool LN, bool NEG1>
struct PlaneMarch {
    static constexpr int KB = KM == 2 ? 2 : 1;                  // key bytes per row
    typedef unsigned int u4 __attribute__((ext_vector_type(4)));
    static constexpr int L2 = (MAXLEN + 1) & ~1;                // table row stride (16-B reads)
    static constexpr int KD = (kPlaneBlockRows * KB + 6) / 4 + 1;  // key dwords per plane (with the alignment slack)
    static constexpr int KR = (KD + 255) / 256;                 // key dword rounds per thread
    static constexpr int MID = MAXLEN / 2;                      // LN: slots MID - 1, MID, MID + 1 = -1, 0, +1
    // one plane buffer: E (window pairs' even rows) then O (odd rows), each
    // for up to 512 pairs (H <= 256): compile-time strides, so every LDS
    // access is a per-lane address set up once plus an immediate offset
    static constexpr int EO = 512, BUF = 2 * EO;
    // plain scalars and pointers only: a reference to the by-value kernel
    // argument would make every thread copy it to scratch; row indices are
    // 32-bit (planes_ok: ld < 2^28)
    int H, tid, pc, zend, P, n, xy0, z0, nxy, xyb, wsh;
    bool in0, in1, full, halo;
    double* win;      // [3][BUF]
    uint32_t* keys;   // [3][KD]
    double* s_rz;     // npat x L2 slot values (0 where the row has no entry)
    uint8_t* s_rm;    // npat slot masks
    __amdgpu_buffer_rsrc_t rx, rk, rw;
    int ps[MAXLEN];     // slot offsets (compile-time indices only)
    double cv[MAXLEN];  // KM = 0: the slot values
    int ia[MAXLEN], ib[MAXLEN];  // in-plane slots: the lane's window indices of its two values (buffer 0)
    int cof16, hof16;   // the lane's own / halo pair, window byte offsets
    int ph;             // the halo pair's index
    int k4[KR];         // the lane's key dwords (clamped), byte offsets
    double2 st0, st1;   // the prefetched plane's own and halo pair (registers)
    uint32_t kst[KR];
    uint32_t wmv;       // the prefetched plane's wave masks (uniform)

    __device__ static __amdgpu_buffer_rsrc_t rsrc(const void* p, int64_t bytes) {
        const uint64_t pl = (uint64_t)(uintptr_t)p;
        const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)pl);
        const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(pl >> 32));
        return __builtin_amdgcn_make_buffer_rsrc((void*)(uintptr_t)(((uint64_t)hi << 32) | lo), (short)0,
                                                 (int)__builtin_amdgcn_readfirstlane((uint32_t)bytes), 0x00020000);
    }
    __host__ __device__ static size_t lds_bytes(int npat) {
        return (size_t)3 * BUF * 8 + (((size_t)3 * KD * 4 + 15) & ~(size_t)15) +
               (KM == 0 ? 0 : (size_t)npat * L2 * 8 + (size_t)npat) + 16;
    }
    // the fields are passed one by one from the kernel's by-value PatArgs
    __device__ PlaneMarch(int64_t P_, int H_, int64_t n_, int64_t ld_, const double* x, const void* key,
                          const uint32_t* wavemask, const double* rzval, const uint8_t* rzmask, int npat,
                          double* lds, int bi, int Z) {
        H = H_;
        tid = threadIdx.x;
        P = (int)P_;
        n = (int)n_;
        nxy = (P + kPlaneBlockRows - 1) / kPlaneBlockRows;
        const int nz = (n + P - 1) / P;
        xyb = bi % nxy;
        xy0 = xyb * kPlaneBlockRows;
        z0 = (bi / nxy) * Z;
        zend = nz - z0 < Z ? nz - z0 : Z;
        in0 = xy0 + 2 * tid < P;
        in1 = xy0 + 2 * tid + 1 < P;
        full = xy0 + kPlaneBlockRows <= P && (int64_t)(z0 + zend) * P <= n_;
        wsh = 8 * __builtin_amdgcn_readfirstlane(tid >> 6);
        pc = tid + H / 2;
        const int h = tid < H ? tid : H - 1;
        halo = tid < H;
        ph = h < H / 2 ? h : h + 256;
        cof16 = 16 * pc;
        hof16 = 16 * ph;
        win = lds;
        keys = reinterpret_cast<uint32_t*>(win + 3 * BUF);
        s_rz = reinterpret_cast<double*>(keys + ((3 * KD + 3) & ~3));
        s_rm = reinterpret_cast<uint8_t*>(s_rz + npat * L2);
        if (KM != 0) {
            for (int i = tid; i < npat * L2; i += 256) {
                const int q = i / L2, e = i % L2;
                s_rz[i] = e < MAXLEN ? rzval[q * MAXLEN + e] : 0.0;
            }
            for (int i = tid; i < npat; i += 256) s_rm[i] = rzmask[i];
        }
#pragma unroll
        for (int k = 0; k < KR; ++k) k4[k] = 4 * min(tid + 256 * k, KD - 1);
        rx = rsrc(x, ld_ * 8);
        // the key arrays carry >= 4 zero bytes past the rows (upload_matrix), so
        // every aligned dword load that reaches a real row lies inside
        rk = rsrc(key, (KB * n_ + 7) & ~(int64_t)3);
        rw = rsrc(wavemask, (int64_t)(nz + 1) * nxy * 4);
    }
    // after ps[] is set: the in-plane slots' window indices.  Rows 2t + H + o,
    // + 1 are (E, O)[pc + o / 2] for even o, else (O[pc + floor(o / 2)],
    // E[pc + ceil(o / 2)])
    __device__ void slots() {
#pragma unroll
        for (int e = 0; e < MAXLEN; ++e) {
            const int o = ps[e];
            ia[e] = ((o & 1) ? EO : 0) + pc + (o >> 1);
            ib[e] = ((o & 1) ? 0 : EO) + pc + ((o + 1) >> 1);
        }
    }
    // 16 B at byte offset off of the column: off < 0 (as 32 bits >= 2^31) or
    // past ld * 8 reads 0.  A load that straddles the descriptor's end returns
    // 0 as a whole (measured), so planes_ok requires ld >= n + 2: only padding
    // rows can straddle.  No range branches: a branch around a load makes the
    // compiler wait for every outstanding load at the join.
    __device__ double2 ld16(int off) const {
        const u4 w = __builtin_amdgcn_raw_buffer_load_b128(rx, off, 0, 0);
        return make_double2(__builtin_bit_cast(double, ((uint64_t)w.y << 32) | w.x),
                            __builtin_bit_cast(double, ((uint64_t)w.w << 32) | w.z));
    }
    __device__ double2 ld2(int row) const { return ld16(row * 8); }
    // issue plane z's loads into registers: the lane's own pair, its halo pair
    // (lanes past H load lane H - 1's again and do not store it), the keys, the
    // waves' masks.
    __device__ void load(int z) {
        const int g8 = (z * P + xy0 - H) * 8;
        st0 = ld16(g8 + cof16);
        st1 = ld16(g8 + hof16);
        const int al = ((z * P + xy0) * KB) & ~3;
#pragma unroll
        for (int k = 0; k < KR; ++k) kst[k] = __builtin_amdgcn_raw_buffer_load_b32(rk, al + k4[k], 0, 0);
        wmv = __builtin_amdgcn_raw_buffer_load_b32(rw, 0, (z * nxy + xyb) * 4, 0);
    }
    // the prefetched plane into LDS buffer B
    template <int B>
    __device__ void store() {
        double* w = win + B * BUF;
        w[pc] = st0.x;
        w[EO + pc] = st0.y;
        if (halo) {
            w[ph] = st1.x;
            w[EO + ph] = st1.y;
        }
        char* kb = reinterpret_cast<char*>(keys + B * KD);
#pragma unroll
        for (int k = 0; k < KR; ++k) *reinterpret_cast<uint32_t*>(kb + k4[k]) = kst[k];
    }
    __device__ unsigned wave_bits(uint32_t v) const {
        return (__builtin_amdgcn_readfirstlane(v) >> wsh) & 0xffu;
    }
    // One step of the march on plane z0 + j, whose window is buffer B: plane
    // z0 + j + 2 is loaded into registers first, f(j, B, xp, xc, xn, wm)
    // computes plane z0 + j (r[(B + 2) % 3] / r[B] / r[(B + 1) % 3]: the
    // lane's pair of planes j - 1 / j / j + 1, wm the wave's mask), then the
    // prefetched plane goes into buffer (B + 2) % 3 and register set
    // (B + 2) % 3 (plane j - 1's, no longer needed), and the block syncs.
    template <int B, typename F>
    __device__ void step(int j, double2 (&r)[3], unsigned (&w)[3], F&& f) {
        constexpr int BP = (B + 2) % 3, BN = (B + 1) % 3;
        if (j + 2 <= zend) load(z0 + j + 2);
        f(j, std::integral_constant<int, B>{}, r[BP], r[B], r[BN], w[B]);
        // the plane's arithmetic stays ahead of the stores, which wait for
        // the prefetch (the compiler otherwise sinks it below them).  The
        // store is unconditional: in the last step it writes the registers
        // again into the buffer of plane zend - 2, which no step reads any
        // more.
        __builtin_amdgcn_sched_barrier(0);
        asm volatile("" ::: "memory");
        store<BP>();
        r[BP] = st0;
        w[BP] = wave_bits(wmv);
        __syncthreads();
    }
    // The march, unrolled by three so that the buffer of every access and the
    // roles of the three register pairs are compile-time.  xp: the lane's pair
    // of plane z0 - 1, loaded before the march; the pairs are pinned once the
    // prologue's stores have waited for the loads (loads return in order), so
    // the loop's first use does not wait for the prefetch issued at the top of
    // the step.
    template <typename F>
    __device__ void march(const double2& xp, F&& f) {
        double2 r[3];
        unsigned w[3];
        load(z0);
        store<0>();
        r[0] = st0;
        w[0] = wave_bits(wmv);
        load(z0 + 1);
        store<1>();
        r[1] = st0;
        w[1] = wave_bits(wmv);
        r[2] = xp;
        w[2] = 0;
        asm volatile("" : "+v"(r[0].x), "+v"(r[0].y), "+v"(r[1].x), "+v"(r[1].y), "+v"(r[2].x), "+v"(r[2].y));
        __syncthreads();
        for (int j = 0; j < zend; j += 3) {
            step<0>(j, r, w, f);
            if (j + 1 < zend) step<1>(j + 1, r, w, f);
            if (j + 2 < zend) step<2>(j + 2, r, w, f);
        }
    }
    // the lane's two row keys of plane z (buffer B)
    template <int B>
    __device__ void row_keys(int z, unsigned& k0, unsigned& k1) const {
        const int kofs = ((z * P + xy0) * KB) & 3;
        const uint8_t* kp = reinterpret_cast<const uint8_t*>(keys + B * KD) + kofs + 2 * tid * KB;
        if (KB == 1) {
            k0 = kp[0];
            k1 = kp[1];
        } else {
            k0 = *reinterpret_cast<const uint16_t*>(kp);
            k1 = *reinterpret_cast<const uint16_t*>(kp + 2);
        }
    }
    // x with the row's slot-e bit: x, or +0.0 where the row has no entry
    __device__ static double keep(double x, unsigned m, int e) {
        const unsigned k = 0u - ((m >> e) & 1u);
        uint2 v = __builtin_bit_cast(uint2, x);
        v.x &= k;
        v.y &= k;
        return __builtin_bit_cast(double, v);
    }
    // y0 / y1: the slot sums of the lane's two rows of plane z (buffer B),
    // each row's own entries in slot (= column) order.  Z0: the sums start
    // from +0.0 (the stored SpMV: a zero sum is +0.0, as in k_spmv); the
    // residual squares its sums and starts from the first product.
    template <bool Z0, int B>
    __device__ void sums(int z, const double2& xp, const double2& xc, const double2& xn, unsigned wm, double& y0,
                         double& y1) const {
        const double* w = win + B * BUF;
        unsigned k0 = 0, k1 = 0, m0 = 0, m1 = 0;
        if (KM != 0 || wm != 0) {
            row_keys<B>(z, k0, k1);
            m0 = KM == 0 ? k0 : s_rm[k0];
            m1 = KM == 0 ? k1 : s_rm[k1];
        }
        double lo = 0.0, hi = 0.0;
        if (LN) {
            lo = w[EO + pc - 1];  // row 2t + H - 1
            hi = w[pc + 1];       // row 2t + H + 2
        }
#pragma unroll
        for (int e = 0; e < MAXLEN; ++e) {
            double2 v;
            if (e == 0) v = xp;
            else if (e == MAXLEN - 1) v = xn;
            else if (LN && e == MID - 1) v = make_double2(lo, xc.x);
            else if (LN && e == MID) v = xc;
            else if (LN && e == MID + 1) v = make_double2(xc.y, hi);
            else v = make_double2(w[ia[e]], w[ib[e]]);
            if (wm >> e & 1u) {
                v.x = keep(v.x, m0, e);
                v.y = keep(v.y, m1, e);
            }
            if (NEG1 && e != MID) {  // coefficient -1: y + (-1) x == y - x
                if (e == 0 && !Z0) {
                    y0 = -v.x;
                    y1 = -v.y;
                } else if (e == 0) {
                    y0 = 0.0 - v.x;
                    y1 = 0.0 - v.y;
                } else {
                    y0 = y0 - v.x;
                    y1 = y1 - v.y;
                }
                continue;
            }
            const double c0 = KM == 0 ? cv[e] : s_rz[k0 * L2 + e];
            const double c1 = KM == 0 ? cv[e] : s_rz[k1 * L2 + e];
            const double t0 = c0 * v.x, t1 = c1 * v.y;
            if (e == 0 && !Z0) {
                y0 = t0;
                y1 = t1;
            } else if (e == 0) {
                y0 = 0.0 + t0;
                y1 = 0.0 + t1;
            } else {
                y0 = y0 + t0;
                y1 = y1 + t1;
            }
        }
    }
};

#define CAL_PLANE_MARCH(PM, XPTR, Zv)                                                                          \
    PlaneMarch<MAXLEN, KM, LN, NEG1> PM(a.plane_P, a.plane_H, a.n, a.ld, XPTR,                                 \
                                        KM == 0 ? (const void*)a.rowmask                                      \
                                                : (KM == 1 ? (const void*)a.rowkey8 : (const void*)a.pat),    \
                                        a.wavemask, a.rzval, a.rzmask, a.npat, lds_plane,                     \
                                        xcd_remap(blockIdx.x, gridDim.x), Zv);                                \
    _Pragma("unroll") for (int e_ = 0; e_ < MAXLEN; ++e_) {                                                   \
        PM.ps[e_] = a.pslot[e_];                                                                              \
        PM.cv[e_] = a.cval[e_];                                                                               \
    }                                                                                                         \
    PM.slots();

// SpMV (with the Newton shift) on the plane march, bit-identical to k_spmv /
// k_spmv_pair.  One 16-B store per row pair (8-B aligned on the odd planes
// of an odd P).
__device__ __forceinline__ void st16(double* p, double2 v) { __builtin_memcpy(p, &v, 16); }
__device__ __forceinline__ double2 ld16g(const double* p) {
    double2 v;
    __builtin_memcpy(&v, p, 16);
    return v;
}

// waves per SIMD the plane-march kernels are compiled for: 5 (96 VGPRs, no
// spills) measured faster than the 6 the LDS (26 KB per block) would allow
// (80 VGPRs with spill reloads in the loop): lap3d_215 in the loop 40.4-41.0
// -> 37.9-38.0 us per SpMV, 845-848 -> 862 outer-it/s (profiles/r05/ab/)
#ifndef CAL_SPMV_WPE
#define CAL_SPMV_WPE 5
#endif
#ifndef CAL_RESID_WPE
#define CAL_RESID_WPE 5
#endif

template <int MODE, int MAXLEN, int Z, int KM, bool LN, bool NEG1>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(CAL_SPMV_WPE))) void k_spmv_planes(PatArgs a) {
    extern __shared__ __attribute__((aligned(16))) double lds_plane[];
    CAL_PLANE_MARCH(pm, a.x, Z)
    const double2 xp0 = pm.ld2((pm.z0 - 1) * pm.P + pm.xy0 + 2 * pm.tid);
    auto run = [&](auto fullc) {
        constexpr bool FULL = decltype(fullc)::value;
        pm.march(xp0, [&](int j, auto bc, const double2& xp, const double2& xc, const double2& xn, unsigned wm) {
            constexpr int B = decltype(bc)::value;
            const int r = (pm.z0 + j) * pm.P + pm.xy0 + 2 * pm.tid;
            const bool v0 = FULL || (pm.in0 && r < pm.n), v1 = FULL || (pm.in1 && r + 1 < pm.n);
            double y0, y1;
            pm.template sums<true, B>(pm.z0 + j, xp, xc, xn, wm, y0, y1);
            if (MODE != 0) {
                const double u0 = a.shift * xc.x, u1 = a.shift * xc.y;
                y0 = y0 - u0;
                y1 = y1 - u1;
                if (MODE == 2) {
                    double2 q;
                    if (FULL) q = ld16g(a.xprev + r);
                    else q = make_double2(a.xprev[v0 ? r : 0], a.xprev[v1 ? r + 1 : 0]);
                    const double w0 = a.im2 * q.x, w1 = a.im2 * q.y;
                    y0 = y0 + w0;
                    y1 = y1 + w1;
                }
            }
            if (v0 && v1) st16(a.y + r, make_double2(y0, y1));
            else if (v0) a.y[r] = y0;
        });
    };
    if (pm.full) run(std::true_type{});
    else run(std::false_type{});
}

// the plane march applies to a whole single slab (pat_args sets the tables)
static bool planes_ok(const PatArgs& a) {
    return a.rzval && a.rzmask && a.wavemask && a.plane_P >= 256 && a.plane_H <= 256 && a.pmaxlen >= 2 &&
           a.pmaxlen <= 8 && a.pcanon && a.gap == 0 && a.xlo == 0 && a.ld >= a.n + 2 &&
           a.ld < ((int64_t)1 << 28) && (a.cuniform ? a.rowmask != nullptr : (a.npat > 256 || a.rowkey8));
}
static int planes_blocks(const PatArgs& a, int Z) {
    const int64_t nxy = (a.plane_P + kPlaneBlockRows - 1) / kPlaneBlockRows;
    const int64_t nz = (a.n + a.plane_P - 1) / a.plane_P;
    return (int)(nxy * ((nz + Z - 1) / Z));
}
// the key mode of the plane march: 0 mask bytes, 1 / 2 pattern ids of 1 / 2 B
static int planes_km(const PatArgs& a) { return a.cuniform ? 0 : (a.npat <= 256 ? 1 : 2); }
static size_t planes_lds(const PatArgs& a) {
    switch (planes_km(a)) {
        case 0: return PlaneMarch<8, 0, false, false>::lds_bytes(a.npat);
        case 1: return PlaneMarch<8, 1, false, false>::lds_bytes(a.npat);
        default: return PlaneMarch<8, 2, false, false>::lds_bytes(a.npat);
    }
}
// slots MID - 1, MID, MID + 1 (MID = L / 2, L odd) are the offsets -1, 0, +1
static bool planes_ln(const PatArgs& a) {
    const int L = a.pmaxlen, m = L / 2;
    return (L & 1) && L >= 5 && a.pslot[m - 1] == -1 && a.pslot[m] == 0 && a.pslot[m + 1] == 1;
}
// uniform slot values, -1 at every slot but the middle (the Laplacians)
static bool planes_neg1(const PatArgs& a) {
    if (!a.cuniform || !planes_ln(a)) return false;
    for (int e = 0; e < a.pmaxlen; ++e)
        if (e != a.pmaxlen / 2 && a.cval[e] != -1.0) return false;
    return true;
}
// dispatch f(MAXLEN, KM, LN, NEG1) over the plane march's instantiations
template <typename F>
static void planes_dispatch(const PatArgs& a, F&& f) {
    auto km = [&](auto ml, auto ln) {
        switch (planes_km(a)) {
            case 0: f(ml, std::integral_constant<int, 0>{}, ln, std::false_type{}); break;
            case 1: f(ml, std::integral_constant<int, 1>{}, ln, std::false_type{}); break;
            default: f(ml, std::integral_constant<int, 2>{}, ln, std::false_type{}); break;
        }
    };
    const bool ln = planes_ln(a), ng = planes_neg1(a);
    using T = std::true_type;
    using N = std::false_type;
    using K0 = std::integral_constant<int, 0>;
    switch (a.pmaxlen) {
        case 2: km(std::integral_constant<int, 2>{}, N{}); break;
        case 3: km(std::integral_constant<int, 3>{}, N{}); break;
        case 4: km(std::integral_constant<int, 4>{}, N{}); break;
        case 5:
            if (ng) f(std::integral_constant<int, 5>{}, K0{}, T{}, T{});
            else if (ln) km(std::integral_constant<int, 5>{}, T{});
            else km(std::integral_constant<int, 5>{}, N{});
            break;
        case 6: km(std::integral_constant<int, 6>{}, N{}); break;
        case 7:
            if (ng) f(std::integral_constant<int, 7>{}, K0{}, T{}, T{});
            else if (ln) km(std::integral_constant<int, 7>{}, T{});
            else km(std::integral_constant<int, 7>{}, N{});
            break;
        default: km(std::integral_constant<int, 8>{}, N{}); break;
    }
}

// planes per block of the plane-march SpMV (round 4, lap3d_215 in the loop:
// 16 -> 40.5 us per SpMV, 32.8 back to back; 8 -> 40.3 / 34.3; 32 -> 47.7 /
// 42.1; the row-pair kernel 41.4 / 34.5)
#ifndef CAL_SPMV_PLANES
#define CAL_SPMV_PLANES 8
#endif
constexpr int kSpmvPlanes = CAL_SPMV_PLANES;

// Small grids (few planes of few blocks: lap2d_1000 has 2 blocks per plane,
// 250 blocks at 8 planes each, a quarter of the chip) march 2 planes per
// block instead, at the price of re-reading 2 halo planes of x per 2.
#ifndef CAL_SPMV_PLANES_MIN_BLOCKS
#define CAL_SPMV_PLANES_MIN_BLOCKS 1024
#endif
static int spmv_planes_z(const PatArgs& a) {
    return planes_blocks(a, kSpmvPlanes) >= CAL_SPMV_PLANES_MIN_BLOCKS ? kSpmvPlanes : 2;
}

template <int MODE>
static hipError_t launch_spmv_planes(const PatArgs& a, hipStream_t st) {
    const size_t lds = planes_lds(a);
    const int z = spmv_planes_z(a);
    dim3 g((unsigned)planes_blocks(a, z)), b(256);
    planes_dispatch(a, [&](auto ml, auto km, auto ln, auto ng) {
        constexpr int ML = decltype(ml)::value, KM = decltype(km)::value;
        constexpr bool LN = decltype(ln)::value, NEG1 = decltype(ng)::value;
        if (z == kSpmvPlanes) hipLaunchKernelGGL((k_spmv_planes<MODE, ML, kSpmvPlanes, KM, LN, NEG1>), g, b, lds, st, a);
        else hipLaunchKernelGGL((k_spmv_planes<MODE, ML, 2, KM, LN, NEG1>), g, b, lds, st, a);
    });
    return hipGetLastError();
}

template <int MODE>
static hipError_t launch_pat_mode(const PatArgs& a, hipStream_t st) {
    if (planes_ok(a)) return launch_spmv_planes<MODE>(a, st);
    const size_t lds = (size_t)a.npat * 8 + (size_t)a.nent * 12 + 16;
    const size_t lds2 = (size_t)a.npent * 20 + (size_t)a.nppat * 8 + 16;
    if (spmv_pat_pair_path(a)) {
        const int64_t npairs = (a.n + 1) / 2;
        // 512 threads per block (1024 rows; half the table stagings of 256
        // threads: lap3d_215 in the loop 45.2 -> 42.7 us per SpMV, 809 -> 825
        // outer-it/s; 1024 measured no better)
        constexpr int tb = 512;
        dim3 g((unsigned)((npairs + tb - 1) / tb)), b(tb);
#define CAL_PR(ML)                                                                                                    \
    if (a.pcanon) hipLaunchKernelGGL((k_spmv_pair<MODE, ML, true, tb>), g, b, lds2, st, a, a.ppat, a.ppinfo, a.ppoff, \
                                     a.ppval);                                                                        \
    else hipLaunchKernelGGL((k_spmv_pair<MODE, ML, false, tb>), g, b, lds2, st, a, a.ppat, a.ppinfo, a.ppoff, a.ppval);
        switch (a.pmaxlen) {
            case 1: CAL_PR(1); break;
            case 2: CAL_PR(2); break;
            case 3: CAL_PR(3); break;
            case 4: CAL_PR(4); break;
            case 5: CAL_PR(5); break;
            case 6: CAL_PR(6); break;
            case 7: CAL_PR(7); break;
            case 8: CAL_PR(8); break;
            default: CAL_PR(16); break;
        }
#undef CAL_PR
        return hipGetLastError();
    }
    if (lds <= kPatLdsMax) {
        const int blocks = a.nblk < 2048 ? a.nblk : 2048;
        const int cpb = (a.nblk + blocks - 1) / blocks;
        dim3 g(blocks), b(256);
#define CAL_PL(ML) hipLaunchKernelGGL((k_spmv_pat_lds<MODE, ML>), g, b, lds, st, a, a.npat, a.nent, cpb)
        switch (a.maxlen) {
            case 1: CAL_PL(1); break;
            case 2: CAL_PL(2); break;
            case 3: CAL_PL(3); break;
            case 4: CAL_PL(4); break;
            case 5: CAL_PL(5); break;
            case 6: CAL_PL(6); break;
            case 7: CAL_PL(7); break;
            case 8: CAL_PL(8); break;
            case 16: CAL_PL(16); break;
            default: CAL_PL(32); break;
        }
#undef CAL_PL
        return hipGetLastError();
    }
    dim3 g(a.nblk), b(256);
    switch (a.maxlen) {
        case 1: case 2: case 3: case 4: hipLaunchKernelGGL((k_spmv_pat<MODE, 4>), g, b, 0, st, a); break;
        case 5: case 6: case 7: case 8: hipLaunchKernelGGL((k_spmv_pat<MODE, 8>), g, b, 0, st, a); break;
        case 16: hipLaunchKernelGGL((k_spmv_pat<MODE, 16>), g, b, 0, st, a); break;
        default: hipLaunchKernelGGL((k_spmv_pat<MODE, 32>), g, b, 0, st, a); break;
    }
    return hipGetLastError();
}

// blocks of the pair residual launch (0: the pair path does not apply)
int spmv_pair_resid_blocks(const PatArgs& a) {
    if (!spmv_pat_pair_path(a) || !a.pcanon || a.gap != 0) return 0;
    return (int)(((a.n + 1) / 2 + 255) / 256);
}

hipError_t launch_spmv_pair_resid(const PatArgs& a, double lr, double* partial, hipStream_t st) {
    PatArgs b = a;
    b.shift = lr;
    const int blocks = spmv_pair_resid_blocks(b);
    if (blocks <= 0) return hipErrorInvalidValue;
    const size_t lds = (size_t)b.npent * 20 + 16;
    dim3 g(blocks), bl(256);
#define CAL_PRR(ML) \
    hipLaunchKernelGGL((k_spmv_pair_resid<ML>), g, bl, lds, st, b, b.ppat, b.ppoff, b.ppval, partial)
    switch (b.pmaxlen) {
        case 1: CAL_PRR(1); break;
        case 2: CAL_PRR(2); break;
        case 3: CAL_PRR(3); break;
        case 4: CAL_PRR(4); break;
        case 5: CAL_PRR(5); break;
        case 6: CAL_PRR(6); break;
        case 7: CAL_PRR(7); break;
        case 8: CAL_PRR(8); break;
        default: return hipErrorInvalidValue;
    }
#undef CAL_PRR
    return hipGetLastError();
}

// Ritz residual partials of many real Ritz pairs in one launch
// (compute_ritz_rnorm, ca_lanczos.m:88-97): blockIdx.y takes pairs
// [CPB y, CPB y + CPB) of the list (x = X + col[i] * ldx, l = lam[i]).  Each
// thread takes PPT row pairs of the block's contiguous run (pair
// b*256*PPT + j*256 + tid) and, per row pair, serves all CPB Ritz pairs with
// work done once: the pair id, the slot offsets and the table entries.  The
// kernel is built to issue few VALU instructions per (row pair, Ritz pair),
// which is what bounded its predecessor (≈170 per row pair and Ritz pair:
// 64-bit address clamps and per-entry selects redone for every Ritz pair):
//   * x is read through one buffer descriptor per Ritz pair (wave-uniform,
//     SGPRs) with the row pair's 32-bit slot offsets computed once; a slot
//     outside the column's range returns 0 from the range check instead of
//     being clamped.  A slot a row uses is always inside (the pair build
//     checks both halves, runtime.cpp build_pair_patterns);
//   * the pair table is staged with the entries a row does not use set to
//     +0.0, so every slot is a plain multiply-add: the running sum of a row
//     starts at +0.0 and gains ±0 terms only where the reference adds
//     nothing, which leaves its bits unchanged (a sum that starts at +0.0 is
//     never -0.0; x + ±0 = x for x != 0).  Each row therefore still adds its
//     own entries in CSR column order, and y = A x - l x has the bits of
//     k_spmv_pair's MODE 1 (the Ritz vectors are finite);
//   * the centre slot (offset 0) doubles as the shift operand when present.
// Split pairs and a row pair whose second row lies past the local rows (an
// odd distributed slab's last row pairs with the first ghost row) take the
// per-row path.  The block's two sums of Ritz pair i go to
// partial[(2 out[i] + e) * pstride + b], as before.
template <int MAXLEN, int CPB, int PPT, bool MID, bool LANE>
__global__ __launch_bounds__(256) void k_resid_pairs(PatArgs a, const uint16_t* __restrict__ ppat,
                                                    const int* __restrict__ ppoff, const double2* __restrict__ ppval,
                                                    const double* __restrict__ X, int64_t ldx,
                                                    const int* __restrict__ col, const double* __restrict__ lam,
                                                    const int* __restrict__ out, int npairs_ritz,
                                                    double* __restrict__ partial, int64_t pstride) {
    extern __shared__ __attribute__((aligned(16))) double lds_pair[];
    double2* s_pz = reinterpret_cast<double2*>(lds_pair);
    // per pair pattern: bit e set when row 2t or 2t+1 uses slot e; a slot
    // neither row uses is loaded at an offset past the descriptor's range
    // (it reads 0), so a padding or non-received ghost position is never
    // read, whatever it holds
    uint32_t* s_um = reinterpret_cast<uint32_t*>(s_pz + a.npent);
    __shared__ double ws[CPB][2][4];
    const int tid = threadIdx.x;
    const int64_t npairs = (a.n + 1) >> 1;
    const int64_t b0 = (int64_t)xcd_remap(blockIdx.x, gridDim.x) * 256 * PPT;
    for (int i = tid; i < a.npent; i += 256) {
        const int code = ppoff[i];
        const double2 v = ppval[i];
        s_pz[i] = make_double2((code & 1) ? v.x : 0.0, (code & 2) ? v.y : 0.0);
    }
    for (int q = tid; q < a.nppat; q += 256) {
        uint32_t um = 0;
        for (int e = 0; e < MAXLEN; ++e) um |= (ppoff[q * MAXLEN + e] & 3) ? (1u << e) : 0u;
        s_um[q] = um;
    }
    const int i0 = blockIdx.y * CPB;
    const int nq = npairs_ritz - i0 < CPB ? npairs_ritz - i0 : CPB;  // uniform over the block
    // one descriptor per Ritz pair over its column's addressable range [xlo, xhi)
    const uint32_t nbytes = (uint32_t)((a.xhi - a.xlo) * 8);
    __amdgpu_buffer_rsrc_t rs[CPB];
    const double* xq[CPB];
    double lq[CPB], num[CPB], den[CPB];
#pragma unroll
    for (int q = 0; q < CPB; ++q) {
        const int qq = q < nq ? q : 0;
        const double* xb = X + (int64_t)col[i0 + qq] * ldx;
        xq[q] = xb;
        const double* lo = xb + a.xlo;
        const uint64_t pl = (uint64_t)(uintptr_t)lo;
        const uint32_t plo = __builtin_amdgcn_readfirstlane((uint32_t)pl);
        const uint32_t phi = __builtin_amdgcn_readfirstlane((uint32_t)(pl >> 32));
        rs[q] = __builtin_amdgcn_make_buffer_rsrc((void*)(uintptr_t)(((uint64_t)phi << 32) | plo), (short)0,
                                                  (int)__builtin_amdgcn_readfirstlane(nbytes), 0x00020000);
        lq[q] = lam[i0 + qq];
        num[q] = 0.0;
        den[q] = 0.0;
    }
    __syncthreads();
    for (int j = 0; j < PPT; ++j) {
        const int64_t t = b0 + (int64_t)j * 256 + tid;
        if (b0 + (int64_t)j * 256 >= npairs) break;  // uniform over the block
        const int64_t tcl = t < npairs ? t : npairs - 1;
        const int id = ppat[tcl];
        const int64_t r0 = 2 * tcl;
        const bool pairpath = id != kPairSplit && r0 + 1 < a.n;
        const int base = pairpath ? id * MAXLEN : 0;
        uint32_t off[MAXLEN];
        const uint32_t um = pairpath ? s_um[id] : 0xFFFFFFFFu;
#pragma unroll
        for (int e = 0; e < MAXLEN; ++e)
            off[e] = ((um >> e) & 1u) ? (uint32_t)(r0 + a.pslot[e] - a.xlo) * 8u : 0xFFFFFFF0u;
        const uint32_t offc = (uint32_t)(r0 - a.xlo) * 8u;
        double2 z[MAXLEN];
#pragma unroll
        for (int e = 0; e < MAXLEN; ++e) z[e] = s_pz[base + e];
        // y = A x - l x of both rows from the zeroed table (see above)
        // run: the wave's 64 lanes hold 64 consecutive row pairs (the fast
        // path), so with LANE the -1 / +1 slots are the neighbouring lanes'
        // centre loads moved over by one DPP wave shift, and the wave's two
        // outer values come from scalar loads (pair_slot_loads' scheme)
        auto pair_sums = [&](int q, double& nu, double& de, bool run) {
            typedef unsigned int u4 __attribute__((ext_vector_type(4)));
            constexpr int Z = MAXLEN / 2;
            constexpr bool LN = LANE && MID && MAXLEN >= 3;
            double2 xc[MAXLEN];
#pragma unroll
            for (int e = 0; e < MAXLEN; ++e) {
                if (LN && run && (e == Z - 1 || e == Z + 1)) continue;
                const u4 w = __builtin_amdgcn_raw_buffer_load_b128(rs[q], (int)off[e], 0, 0);
                xc[e] = make_double2(__builtin_bit_cast(double, ((uint64_t)w.y << 32) | w.x),
                                     __builtin_bit_cast(double, ((uint64_t)w.w << 32) | w.z));
            }
            if constexpr (LN) {
                if (run) {
                    const int64_t tw = (int64_t)__builtin_amdgcn_readfirstlane((unsigned)(t & 0xffffffff)) |
                                       ((int64_t)__builtin_amdgcn_readfirstlane((unsigned)((uint64_t)t >> 32)) << 32);
                    int64_t el = 2 * tw - 1, er = 2 * tw + 128;  // x[lane 0's r0 - 1], x[lane 63's r0 + 2]
                    el = el < a.xlo ? a.xlo : (el > a.xhi - 1 ? a.xhi - 1 : el);
                    er = er < a.xlo ? a.xlo : (er > a.xhi - 1 ? a.xhi - 1 : er);
                    const double xl = xq[q][el], xr = xq[q][er];
                    xc[Z - 1] = make_double2(dpp_wave_shift<kDppWaveShr1>(xc[Z].y, xl), xc[Z].x);
                    xc[Z + 1] = make_double2(xc[Z].y, dpp_wave_shift<kDppWaveShl1>(xc[Z].x, xr));
                }
            }
            double2 xs;
            if constexpr (MID) {
                xs = xc[MAXLEN / 2];
            } else {
                const u4 w = __builtin_amdgcn_raw_buffer_load_b128(rs[q], (int)offc, 0, 0);
                xs = make_double2(__builtin_bit_cast(double, ((uint64_t)w.y << 32) | w.x),
                                  __builtin_bit_cast(double, ((uint64_t)w.w << 32) | w.z));
            }
            double y0 = 0.0, y1 = 0.0;
#pragma unroll
            for (int e = 0; e < MAXLEN; ++e) {
                const double t0 = z[e].x * xc[e].x, t1 = z[e].y * xc[e].y;
                y0 = y0 + t0;
                y1 = y1 + t1;
            }
            const double u0 = lq[q] * xs.x, u1 = lq[q] * xs.y;
            y0 = y0 - u0;
            y1 = y1 - u1;
            nu = y0 * y0 + y1 * y1;
            de = u0 * u0 + u1 * u1;
        };
        const bool fast = pairpath && t < npairs;
        if (__builtin_amdgcn_ballot_w64(!fast) == 0) {  // the whole wave on the pair path (wave-uniform)
#pragma unroll
            for (int q = 0; q < CPB; ++q) {
                if (q >= nq) break;
                double nu, de;
                pair_sums(q, nu, de, true);
                num[q] = num[q] + nu;
                den[q] = den[q] + de;
            }
        } else {
#pragma unroll
            for (int q = 0; q < CPB; ++q) {
                if (q >= nq) break;
                if (t >= npairs) continue;
                double nu = 0.0, de = 0.0;
                if (pairpath) {
                    pair_sums(q, nu, de, false);
                } else {
                    const double* x = xq[q];
                    for (int k = 0; k < 2 && r0 + k < a.n; ++k) {
                        const int64_t rr = r0 + k;
                        const int2 pi = a.pinfo[a.pat[rr]];
                        double sum = 0.0;
                        for (int e = 0; e < pi.y; ++e) {
                            const double tv = a.pval[pi.x + e] * x[rr + a.pdelta[pi.x + e]];
                            sum = sum + tv;
                        }
                        const double u = lq[q] * x[rr];
                        const double y = sum - u;
                        nu = nu + y * y;
                        de = de + u * u;
                    }
                }
                num[q] = num[q] + nu;
                den[q] = den[q] + de;
            }
        }
    }
    const int lane = tid & 63, wave = tid >> 6;
#pragma unroll
    for (int q = 0; q < CPB; ++q) {
        if (q < nq) {
            const double nu = wave_sum(num[q]), de = wave_sum(den[q]);
            if (lane == 0) {
                ws[q][0][wave] = nu;
                ws[q][1][wave] = de;
            }
        }
    }
    __syncthreads();
    if (tid < 2 * CPB) {
        const int q = tid >> 1, e = tid & 1;
        if (i0 + q < npairs_ritz)
            partial[(2 * (int64_t)out[i0 + q] + e) * pstride + blockIdx.x] =
                ((ws[q][e][0] + ws[q][e][1]) + ws[q][e][2]) + ws[q][e][3];
    }
}

// Ritz residual partials on the plane march (the geometry above): one Ritz
// pair per block row (blockIdx.y), kResidPlanes planes per block; y = A x -
// l x of each row with the SpMV's bits, then the block's sums of y^2 and,
// times l^2, of x^2 (||l x||^2 = l^2 ||x||^2: one accumulator less than
// summing (l x)^2, the same value to rounding).
template <int MAXLEN, int KM, bool LN, bool NEG1>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(CAL_RESID_WPE))) void k_resid_planes(
    PatArgs a, const double* __restrict__ X, int64_t ldx, const int* __restrict__ col, const double* __restrict__ lam,
    const int* __restrict__ out, double* __restrict__ partial, int64_t pstride) {
    extern __shared__ __attribute__((aligned(16))) double lds_plane[];
    __shared__ double ws[2][4];
    const int i = blockIdx.y;
    CAL_PLANE_MARCH(pm, X + (int64_t)col[i] * ldx, kResidPlanes)
    const double l = lam[i];
    const double2 xp0 = pm.ld2((pm.z0 - 1) * pm.P + pm.xy0 + 2 * pm.tid);
    double num = 0.0, den = 0.0;
    auto run = [&](auto fullc) {
        constexpr bool FULL = decltype(fullc)::value;
        pm.march(xp0, [&](int j, auto bc, const double2& xp, const double2& xc, const double2& xn, unsigned wm) {
            constexpr int B = decltype(bc)::value;
            double y0, y1;
            pm.template sums<false, B>(pm.z0 + j, xp, xc, xn, wm, y0, y1);
            const double u0 = l * xc.x, u1 = l * xc.y;
            y0 = y0 - u0;
            y1 = y1 - u1;
            if (FULL) {
                num = __builtin_fma(y0, y0, num);
                num = __builtin_fma(y1, y1, num);
                den = __builtin_fma(xc.x, xc.x, den);
                den = __builtin_fma(xc.y, xc.y, den);
            } else {
                const int r = (pm.z0 + j) * pm.P + pm.xy0 + 2 * pm.tid;
                const bool v0 = pm.in0 && r < pm.n, v1 = pm.in1 && r + 1 < pm.n;
                const double a0 = v0 ? y0 : 0.0, a1 = v1 ? y1 : 0.0;
                const double b0 = v0 ? xc.x : 0.0, b1 = v1 ? xc.y : 0.0;
                num = __builtin_fma(a0, a0, num);
                num = __builtin_fma(a1, a1, num);
                den = __builtin_fma(b0, b0, den);
                den = __builtin_fma(b1, b1, den);
            }
            // the sums before the step's LDS stores (PlaneMarch::step)
            asm volatile("" : "+v"(num), "+v"(den));
        });
    };
    if (pm.full) run(std::true_type{});
    else run(std::false_type{});
    num = wave_sum(num);
    den = wave_sum(den);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (lane == 0) {
        ws[0][wave] = num;
        ws[1][wave] = den;
    }
    __syncthreads();
    if (threadIdx.x < 2) {
        const double v = ((ws[threadIdx.x][0] + ws[threadIdx.x][1]) + ws[threadIdx.x][2]) + ws[threadIdx.x][3];
        partial[(2 * (int64_t)out[i] + threadIdx.x) * pstride + blockIdx.x] = threadIdx.x == 0 ? v : (l * l) * v;
    }
}

// the batched residual kernel's shape: one Ritz pair per block, 8 row pairs
// per thread, the +-1 slots from the neighbouring lanes (the same-box sweep
// of round 4, diagnostics-only lap3d_215: 1x8 with lane slots 43.2 ms per
// 15 iterations against 44.3-51.4 ms for 1x2 .. 8x2 and 4x4 with or without)
constexpr int kResidCpb = 1, kResidPpt = 8;

int spmv_pair_resid_multi_blocks(const PatArgs& a) {
    const int nb = spmv_pair_resid_blocks(a);
    if (nb <= 0) return 0;
    if (planes_ok(a)) return planes_blocks(a, kResidPlanes);
    return (nb + kResidPpt - 1) / kResidPpt;
}

hipError_t launch_spmv_pair_resid_multi(const PatArgs& a, const double* X, int64_t ldx, const int* col,
                                        const double* lam, const int* out, int npr, double* partial,
                                        int64_t pstride, hipStream_t st) {
    const int blocks = spmv_pair_resid_multi_blocks(a);
    if (blocks <= 0 || pstride < blocks) return hipErrorInvalidValue;
    if (npr <= 0) return hipSuccess;
    if (a.pmaxlen > 8 || !a.pcanon) return hipErrorInvalidValue;
    // 32-bit slot offsets: the column's range must fit the descriptor
    if ((a.xhi - a.xlo) * 8 >= ((int64_t)1 << 31)) return hipErrorInvalidValue;
    if (planes_ok(a)) {
        const size_t lds = planes_lds(a);
        dim3 g(blocks, npr), bl(256);
        planes_dispatch(a, [&](auto ml, auto km, auto ln, auto ng) {
            constexpr int ML = decltype(ml)::value, KM = decltype(km)::value;
            constexpr bool LN = decltype(ln)::value, NEG1 = decltype(ng)::value;
            hipLaunchKernelGGL((k_resid_planes<ML, KM, LN, NEG1>), g, bl, lds, st, a, X, ldx, col, lam, out, partial,
                               pstride);
        });
        return hipGetLastError();
    }
    const size_t lds = (size_t)a.npent * 16 + (size_t)a.nppat * 4 + 16;
    const bool mid = (a.pmaxlen & 1) && a.pslot[a.pmaxlen / 2] == 0;
    const bool lane = mid && a.pmaxlen >= 3 && a.pslot[a.pmaxlen / 2 - 1] == -1 &&
                      a.pslot[a.pmaxlen / 2 + 1] == 1;
    auto go = [&](auto cpb_c, auto ppt_c) {
        constexpr int CPB = decltype(cpb_c)::value, PPT = decltype(ppt_c)::value;
        dim3 g(blocks, (npr + CPB - 1) / CPB), bl(256);
#define CAL_PRM(ML, M, LN)                                                                                          \
    hipLaunchKernelGGL((k_resid_pairs<ML, CPB, PPT, M, LN>), g, bl, lds, st, a, a.ppat, a.ppoff, a.ppval, X, ldx, col, \
                       lam, out, npr, partial, pstride)
#define CAL_PRM_ODD(ML)                 \
    if (lane) CAL_PRM(ML, true, true);  \
    else if (mid) CAL_PRM(ML, true, false); \
    else CAL_PRM(ML, false, false)
        switch (a.pmaxlen) {
            case 1: if (mid) CAL_PRM(1, true, false); else CAL_PRM(1, false, false); break;
            case 2: CAL_PRM(2, false, false); break;
            case 3: CAL_PRM_ODD(3); break;
            case 4: CAL_PRM(4, false, false); break;
            case 5: CAL_PRM_ODD(5); break;
            case 6: CAL_PRM(6, false, false); break;
            case 7: CAL_PRM_ODD(7); break;
            default: CAL_PRM(8, false, false); break;
        }
#undef CAL_PRM_ODD
#undef CAL_PRM
    };
    go(std::integral_constant<int, kResidCpb>{}, std::integral_constant<int, kResidPpt>{});
    return hipGetLastError();
}

hipError_t launch_spmv_pat(const PatArgs& a, hipStream_t st) {
    if (a.nblk <= 0) return hipSuccess;
    if (a.gap != 0 && !spmv_pat_pair_path(a)) {  // the row kernels take one range: two launches
        PatArgs b = a, h = a;
        b.gap_at = b.gap = h.gap_at = h.gap = 0;
        b.n = 2 * a.gap_at;
        b.nblk = (int)((b.n + 255) / 256);
        const int64_t sh = 2 * (a.gap_at + a.gap);
        h.n = a.n - 2 * a.gap_at;
        h.nblk = (int)((h.n + 255) / 256);
        h.pat += sh;
        h.x += sh;
        h.y += sh;
        if (h.xprev) h.xprev += sh;
        if (h.ppat) h.ppat += sh / 2;
        h.xlo -= sh;
        h.xhi -= sh;
        hipError_t e = launch_spmv_pat(b, st);
        return e != hipSuccess ? e : launch_spmv_pat(h, st);
    }
    switch (a.mode) {
        case 0: return launch_pat_mode<0>(a, st);
        case 1: return launch_pat_mode<1>(a, st);
        default: return launch_pat_mode<2>(a, st);
    }
}

// --------------------------------------------------------------------------
// Gram: C = A^T B (MFMA f64 16x16x4).  A: up to 16*NTA columns, B: <= 16.
// Lane l owns column (l&15) of every 16-column tile and rows g*RUN..g*RUN+RUN-1
// (g = l>>4) of each 4*RUN-row wave step: MFMA k index = g, so A-operand
// A[i][k] = A(row_k, i) and B-operand B[k][j] = B(row_k, j) are plain loads.
// Output tile layout (f64 16x16x4): lane l, reg r -> C[(l>>4)+4r][l&15].
// Block partial: column-major 16*NTA x 16 (ld 16*NTA).
// --------------------------------------------------------------------------
template <int NTA, int RUN>
__global__ __launch_bounds__(256) void k_gram(Panel A, Panel B, int64_t n, double* __restrict__ partial) {
    __shared__ double red[3][NTA][64][4];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int c16 = lane & 15, g = lane >> 4;
    const double* ac[NTA];
    bool aon[NTA];
#pragma unroll
    for (int t = 0; t < NTA; ++t) {
        const int c = t * 16 + c16;
        aon[t] = c < A.total;
        ac[t] = pcol(A, aon[t] ? c : 0);
    }
    const bool bon = c16 < B.total;
    const double* bc = pcol(B, bon ? c16 : 0);
    d4 acc[NTA];
#pragma unroll
    for (int t = 0; t < NTA; ++t) acc[t] = d4{0.0, 0.0, 0.0, 0.0};

    const int64_t wstep = 4 * RUN;
    const int64_t stride = (int64_t)gridDim.x * 4 * wstep;
    for (int64_t r0 = ((int64_t)blockIdx.x * 4 + wave) * wstep; r0 < n; r0 += stride) {
        const int64_t rb = r0 + g * RUN;
        double av[NTA][RUN], bv[RUN];
        if (r0 + wstep <= n) {
            if (RUN % 2 == 0) {
#pragma unroll
                for (int m = 0; m < RUN; m += 2) {
                    d2 x = *reinterpret_cast<const d2*>(bc + rb + m);
                    bv[m] = bon ? x[0] : 0.0;
                    bv[m + 1] = bon ? x[1] : 0.0;
#pragma unroll
                    for (int t = 0; t < NTA; ++t) {
                        d2 y = *reinterpret_cast<const d2*>(ac[t] + rb + m);
                        av[t][m] = aon[t] ? y[0] : 0.0;
                        av[t][m + 1] = aon[t] ? y[1] : 0.0;
                    }
                }
            } else {
#pragma unroll
                for (int m = 0; m < RUN; ++m) {
                    bv[m] = bon ? bc[rb + m] : 0.0;
#pragma unroll
                    for (int t = 0; t < NTA; ++t) av[t][m] = aon[t] ? ac[t][rb + m] : 0.0;
                }
            }
        } else {
#pragma unroll
            for (int m = 0; m < RUN; ++m) {
                const bool in = rb + m < n;
                const int64_t rr = in ? rb + m : 0;
                double x = bc[rr];
                bv[m] = (bon && in) ? x : 0.0;
#pragma unroll
                for (int t = 0; t < NTA; ++t) {
                    double y = ac[t][rr];
                    av[t][m] = (aon[t] && in) ? y : 0.0;
                }
            }
        }
#pragma unroll
        for (int m = 0; m < RUN; ++m)
#pragma unroll
            for (int t = 0; t < NTA; ++t) acc[t] = mfma64(av[t][m], bv[m], acc[t]);
    }
    // deterministic block reduction: waves 1..3 park, wave 0 adds in order
    if (wave > 0) {
#pragma unroll
        for (int t = 0; t < NTA; ++t)
#pragma unroll
            for (int r = 0; r < 4; ++r) red[wave - 1][t][lane][r] = acc[t][r];
    }
    __syncthreads();
    if (wave == 0) {
        const int ldc = 16 * NTA;
        // entry-major partials: entry e of block b at partial[e * nblocks + b]
        double* out = partial + blockIdx.x;
        const int64_t nb = gridDim.x;
#pragma unroll
        for (int t = 0; t < NTA; ++t)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                double v = acc[t][r];
                v = v + red[0][t][lane][r];
                v = v + red[1][t][lane][r];
                v = v + red[2][t][lane][r];
                const int i = t * 16 + g + 4 * r, j = c16;
                out[(int64_t)(j * ldc + i) * nb] = v;
            }
    }
}

// k_gram with coalesced loads: the same rows feed the same MFMAs in the same
// order (so the same bits), but a block's 16 RUN rows (its four waves' row
// runs of one grid step) are first loaded column by column with one row per
// lane -- 512 contiguous bytes per wave instruction instead of 16 column
// pieces -- and staged in LDS ([row][col], odd leading dimension), then read
// back in k_gram's operand layout: lane (c16, g) of wave w takes row
// w*4RUN + g*RUN + m of column 16t + c16 for MFMA m of tile t.  U grid steps
// (rows rb0 + u*stride, u < U) share one staging round, so one barrier
// covers U*16*RUN rows; the MFMAs still take the steps in order.  The B tile
// is read once per round into registers; A goes through LDS 16 columns at a
// time, the next chunk's loads in flight during the current MFMAs.
template <int NTA, int RUN, int U>
__global__ __launch_bounds__(256) void k_gram_lds(Panel A, Panel B, int64_t n, double* __restrict__ partial) {
    constexpr int R = 16 * RUN;   // rows per grid step of a block
    constexpr int LD = 17;        // [row][col] leading dimension (odd: conflict-free row-major writes)
    constexpr int PER = R / 16;   // values per thread per 16-column chunk and step
    constexpr int BUF = U * R * LD;
    // dynamic LDS: the two staging buffers, later reused for the wave partials
    extern __shared__ __attribute__((aligned(16))) double lds_g[];
    auto red = reinterpret_cast<double (*)[NTA][64][4]>(lds_g);  // [3][NTA][64][4]
    const int tid = threadIdx.x;
    const int lane = tid & 63, wave = tid >> 6;
    const int c16 = lane & 15, g = lane >> 4;
    // loader mapping: chunk element e = tid + 256 q -> column e / R (uniform
    // over a wave, R >= 64: scalar pointer arithmetic), row e % R
    const int lrow0 = tid % R;
    d4 acc[NTA];
#pragma unroll
    for (int t = 0; t < NTA; ++t) acc[t] = d4{0.0, 0.0, 0.0, 0.0};
    const int orow = wave * 4 * RUN + g * RUN;  // this lane's operand rows: orow + m
    const int64_t stride = (int64_t)gridDim.x * R;
    double v[U][PER];
    auto load = [&](int c, int64_t rb) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t rr = rb + u * stride + lrow0;
            const bool in = rr < n;
#pragma unroll
            for (int q = 0; q < PER; ++q) {
                const int cc = __builtin_amdgcn_readfirstlane((tid + 256 * q) / R) + (c > 0 ? 16 * (c - 1) : 0);
                const bool on = cc < (c == 0 ? B.total : A.total);
                const double* pc = c == 0 ? pcol(B, on ? cc : 0) : pcol(A, on ? cc : 0);
                const double x = pc[in ? rr : 0];
                v[u][q] = (on && in) ? x : 0.0;
            }
        }
    };
    int64_t rb0 = (int64_t)blockIdx.x * R;
    if (rb0 < n) load(0, rb0);
    for (; rb0 < n; rb0 += U * stride) {
        double bv[U][RUN];
#pragma unroll
        for (int c = 0; c <= NTA; ++c) {
            // buffer c & 1: its last reader was chunk c - 2, done before the
            // barrier after chunk c - 1's write (and the round-end barrier)
            double* s = lds_g + (c & 1) * BUF;
#pragma unroll
            for (int u = 0; u < U; ++u)
#pragma unroll
                for (int q = 0; q < PER; ++q) s[(u * R + lrow0) * LD + (tid + 256 * q) / R] = v[u][q];
            // the next chunk's loads are in flight across the barrier and the MFMAs
            if (c < NTA) load(c + 1, rb0);
            else if (rb0 + U * stride < n) load(0, rb0 + U * stride);
            __syncthreads();
#pragma unroll
            for (int u = 0; u < U; ++u) {
                if (rb0 + u * stride >= n) break;  // block-uniform: k_gram has no such step
                const double* su = s + u * R * LD;
                if (c == 0) {
#pragma unroll
                    for (int m = 0; m < RUN; ++m) bv[u][m] = su[(orow + m) * LD + c16];
                } else {
#pragma unroll
                    for (int m = 0; m < RUN; ++m)
                        acc[c - 1] = mfma64(su[(orow + m) * LD + c16], bv[u][m], acc[c - 1]);
                }
            }
        }
        __syncthreads();  // the next round's chunk 0 rewrites buffer 0
    }
    __syncthreads();  // (no round ran) the staging buffers become the partials
    if (wave > 0) {
#pragma unroll
        for (int t = 0; t < NTA; ++t)
#pragma unroll
            for (int r = 0; r < 4; ++r) red[wave - 1][t][lane][r] = acc[t][r];
    }
    __syncthreads();
    if (wave == 0) {
        const int ldc = 16 * NTA;
        double* out = partial + blockIdx.x;
        const int64_t nb = gridDim.x;
#pragma unroll
        for (int t = 0; t < NTA; ++t)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                double v = acc[t][r];
                v = v + red[0][t][lane][r];
                v = v + red[1][t][lane][r];
                v = v + red[2][t][lane][r];
                const int i = t * 16 + g + 4 * r, j = c16;
                out[(int64_t)(j * ldc + i) * nb] = v;
            }
    }
}

// The narrow Grams (A <= 32 columns, B <= 16: the block projections and the
// s + 1-column normalisations of every outer iteration) with all columns of a
// round staged at once: per round a block loads R = 16 RUN rows of B's 16 and
// A's 16 NTA columns, one column per wave instruction (R contiguous doubles:
// 512 B per wave), into LDS [row][col] (odd leading dimension), one barrier,
// then lane (c16, g) of wave w feeds MFMA m of tile t with row
// w*4RUN + g*RUN + m of A column 16t + c16 and of B column c16.  k_gram's
// row-group loads touch 64 cache lines per wave instruction (16 columns x 4
// row groups) and ran the IRL's narrow Grams at 3-3.5 TB/s.  Two rounds of
// loads are in flight (register slots 0/1, the loop unrolled by two), the LDS
// double buffered: buffer b was last read by round r - 2's MFMAs, which every
// wave finished before passing round r - 1's barrier.  The row order within
// a block's MFMAs differs from k_gram<NTA, 16>'s (RUN = 4 vs 16), so the
// Grams differ from k_gram's in the last bits; the kernel itself is
// deterministic (fixed rounds per block, fixed block reduction).  Taken up to
// 64 A columns (NTA 4: 83 KB of LDS, one block per CU); 512 blocks.  IRL
// driver (circuit_1259, n = 1.58 M, A 4..48 x B 8 columns): Gram class
// 3.29 -> 4.27 TB/s, 31.3 -> 34.5 solves/s (profiles/r05/ab_gram).
#ifndef CAL_GRAM_ROWS
#define CAL_GRAM_ROWS 1
#endif
#ifndef CAL_GRAM_ROWS_RUN
#define CAL_GRAM_ROWS_RUN 4
#endif
#ifndef CAL_GRAM_ROWS_BLOCKS
#define CAL_GRAM_ROWS_BLOCKS 512
#endif
#ifndef CAL_GRAM_ROWS_MAXNTA
#define CAL_GRAM_ROWS_MAXNTA 4
#endif
// NSLOT rounds of loads in flight per thread (register slots), the LDS
// double buffered: round r loads into slot r % NSLOT, stages into buffer
// r % 2 and issues round r + NSLOT's loads into the slot it just drained.
// One block per CU (83 KB at NTA 4), so the bytes in flight per CU are
// NSLOT x 256 threads x PER x 8 B: 80 KB with 2 slots.
#ifndef CAL_GRAM_ROWS_NSLOT
#define CAL_GRAM_ROWS_NSLOT 2
#endif
// LDS stage buffers: 2 (one barrier per round) or 1 (a second barrier before
// the stage is rewritten; half the LDS, so more blocks per CU)
#ifndef CAL_GRAM_ROWS_LDSBUF
#define CAL_GRAM_ROWS_LDSBUF 2
#endif
// BW: B columns staged (16, or 8 when B has <= 8: the MFMA lanes of B
// columns 8..15 take zeros without LDS).  With BW = 8 the NTA = 4 stage is
// 75 KB, so two blocks share a CU: a 64 + 8-column sweep reads at the
// two-block rate (6.0 against 5.1-5.3 TB/s at lap3d_215's n,
// tools/wide_read_probe.hip, profiles/r06/wide_read_probe.json).
template <int NTA, int RUN, bool BB, int BW = 16>
__global__ __launch_bounds__(256) void k_gram_rows(Panel A, Panel B, int64_t n, double* __restrict__ partial,
                                                   int ldc_out, int a_off) {
    static_assert(BW == 8 || BW == 16, "k_gram_rows B width");
    constexpr int R = 16 * RUN;         // rows per round
    constexpr int NC = BW + 16 * NTA;   // staged columns: B's BW, then A's
    constexpr int LD = NC + 1;
    constexpr int CPI = 256 / R;        // columns per block-wide load instruction
    constexpr int PER = NC / CPI;       // loads per thread and round
    constexpr int NS = CAL_GRAM_ROWS_NSLOT;
    static_assert(R >= 64 && 256 % R == 0 && NC % CPI == 0, "k_gram_rows geometry");
    static_assert(NS >= 2 && NS <= 4, "k_gram_rows slots");
    extern __shared__ __attribute__((aligned(16))) double lds_gr[];  // [2][R][LD], then the partials
    constexpr int NT = NTA + (BB ? 1 : 0);                             // output tiles (B'B last)
    auto red = reinterpret_cast<double (*)[NT][64][4]>(lds_gr);        // [3][NT][64][4]
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, c16 = lane & 15, g = lane >> 4;
    const int lrow = tid % R, lcol0 = __builtin_amdgcn_readfirstlane(tid / R);
    // column q of this thread: lcol0 + CPI q (wave-uniform); absent columns
    // are not loaded (zeros staged), rows past n read row 0 and are zeroed
    const double* pc[PER];
    bool on[PER];
#pragma unroll
    for (int q = 0; q < PER; ++q) {
        const int cc = lcol0 + CPI * q;
        if (cc < BW) {
            on[q] = cc < B.total;
            pc[q] = pcol(B, on[q] ? cc : 0);
        } else {
            on[q] = cc - BW < A.total;
            pc[q] = pcol(A, on[q] ? cc - BW : 0);
        }
    }
    d4 acc[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[t] = d4{0.0, 0.0, 0.0, 0.0};
    const int orow = wave * 4 * RUN + g * RUN;
    const int64_t stride = (int64_t)gridDim.x * R;
    double v[NS][PER];
    bool vin[NS];
#pragma unroll
    for (int q = 0; q < NS; ++q) vin[q] = false;
    // (slot and buffer indices are constants once the loops below unroll)
    auto load = [&](int S, int64_t rb) {
        const int64_t rr = rb + lrow;
        vin[S] = rr < n;
        const int64_t ro = vin[S] ? rr : 0;
#pragma unroll
        for (int q = 0; q < PER; ++q) v[S][q] = on[q] ? pc[q][ro] : 0.0;  // on[q] wave-uniform
    };
    auto round = [&](int S, int L, int64_t rb) {
        double* s = lds_gr + (CAL_GRAM_ROWS_LDSBUF == 2 ? L : 0) * (R * LD);
        if (CAL_GRAM_ROWS_LDSBUF == 1) __syncthreads();  // the previous round's MFMAs read the stage
#pragma unroll
        for (int q = 0; q < PER; ++q) s[lrow * LD + lcol0 + CPI * q] = vin[S] ? v[S][q] : 0.0;
        if (rb + NS * stride < n) load(S, rb + NS * stride);
        __syncthreads();
#pragma unroll
        for (int m = 0; m < RUN; ++m) {
            const double* row = s + (orow + m) * LD + c16;
            const double b = BW == 16 || c16 < BW ? row[0] : 0.0;
#pragma unroll
            for (int t = 0; t < NTA; ++t) acc[t] = mfma64(row[BW + 16 * t], b, acc[t]);
            if constexpr (BB) acc[NTA] = mfma64(b, b, acc[NTA]);
        }
    };
    // rounds of one unrolled pass: slot i % NS, LDS buffer i % 2
    constexpr int U = NS % 2 == 0 ? NS : 2 * NS;
    int64_t rb = (int64_t)blockIdx.x * R;
#pragma unroll
    for (int i = 0; i < NS; ++i)
        if (rb + i * stride < n) load(i, rb + i * stride);
    while (rb < n) {
#pragma unroll
        for (int i = 0; i < U; ++i) {
            if (rb >= n) break;
            round(i % NS, i % 2, rb);
            rb += stride;
        }
    }
    __syncthreads();  // the staging buffers become the partials
    if (wave > 0) {
#pragma unroll
        for (int t = 0; t < NT; ++t)
#pragma unroll
            for (int r = 0; r < 4; ++r) red[wave - 1][t][lane][r] = acc[t][r];
    }
    __syncthreads();
    if (wave == 0) {
        const int ldc = ldc_out;  // 16 NTA, or the whole Gram's when A is one column range of it
        double* out = partial + blockIdx.x;
        const int64_t nb = gridDim.x;
#pragma unroll
        for (int t = 0; t < NT; ++t)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                double x = acc[t][r];
                x = x + red[0][t][lane][r];
                x = x + red[1][t][lane][r];
                x = x + red[2][t][lane][r];
                const int i = g + 4 * r, j = c16;
                // A'B entry (a_off + 16t + i, j) at j ldc + a_off + 16t + i;
                // B'B (i, j) after them at 16 ldc + j 16 + i
                const int e = t < NTA ? j * ldc + a_off + 16 * t + i : 16 * ldc + j * 16 + i;
                out[(int64_t)e * nb] = x;
            }
    }
}

template <int NTA, bool BB = false>
static void launch_gram_rows(const Panel& A, const Panel& B, int64_t n, int blocks, double* partial, hipStream_t st,
                             int ldc_out = 16 * NTA, int a_off = 0) {
    constexpr int RUN = CAL_GRAM_ROWS_RUN, R = 16 * RUN;
    const int bw = B.total <= 8 ? 8 : 16, LD = bw + 16 * NTA + 1;
    const size_t lds = std::max((size_t)CAL_GRAM_ROWS_LDSBUF * R * LD, (size_t)3 * (NTA + 1) * 64 * 4) * sizeof(double);
    if (bw == 8)
        hipLaunchKernelGGL((k_gram_rows<NTA, RUN, BB, 8>), dim3(blocks), dim3(256), lds, st, A, B, n, partial,
                           ldc_out, a_off);
    else
        hipLaunchKernelGGL((k_gram_rows<NTA, RUN, BB, 16>), dim3(blocks), dim3(256), lds, st, A, B, n, partial,
                           ldc_out, a_off);
}

// Columns c0 .. c0 + nc - 1 of a panel (host side)
static Panel gram_panel_slice(const Panel& P, int c0, int nc) {
    Panel out = panel();
    int base = 0;
    for (int q = 0; q < P.nseg; ++q) {
        const int lo = std::max(c0, base), hi = std::min(c0 + nc, base + P.ncol[q]);
        if (hi > lo) panel_add(out, P.ptr[q] + (int64_t)(lo - base) * P.ld[q], P.ld[q], hi - lo);
        base += P.ncol[q];
    }
    return out;
}

// A'B for 65 .. 128 A columns on the row-staged kernel: A's first 64 columns
// and the rest in two launches writing their column ranges of one partial
// layout (ldc = 16 nta, the layout of k_gram_lds), reduced as one Gram.  B
// is read twice (<= 16 of 80 .. 144 columns).  Used when CAL_GRAM_ROWS_SPLIT.
#ifndef CAL_GRAM_ROWS_SPLIT
#define CAL_GRAM_ROWS_SPLIT 1
#endif
#ifndef CAL_GRAM_SPLIT_NTA
#define CAL_GRAM_SPLIT_NTA CAL_GRAM_ROWS_MAXNTA  // A columns per launch / 16
#endif
static hipError_t launch_gram_rows_split(const Panel& A, const Panel& B, int64_t n, const GramPlan& pl,
                                         double* partial, hipStream_t st) {
    // the fewest launches of <= CAL_GRAM_SPLIT_NTA tiles, the tiles spread
    // evenly over them (72 columns: 48 + 24, not 64 + 8 -- a launch of 8 + 8
    // columns streams at a fraction of the rate, profiles/r06/gram3)
    const int tiles = (A.total + 15) / 16;
    const int nl = (tiles + CAL_GRAM_SPLIT_NTA - 1) / CAL_GRAM_SPLIT_NTA;
    const int W0 = 16 * ((tiles + nl - 1) / nl);
    const int ldc = 16 * pl.nta;
    for (int a0 = 0; a0 < A.total; a0 += W0) {
        const int na = std::min(W0, A.total - a0), nt = (na + 15) / 16;
        const Panel As = gram_panel_slice(A, a0, na);
        switch (nt) {
            case 1: launch_gram_rows<1>(As, B, n, pl.blocks, partial, st, ldc, a0); break;
            case 2: launch_gram_rows<2>(As, B, n, pl.blocks, partial, st, ldc, a0); break;
#if CAL_GRAM_ROWS_MAXNTA >= 3
            case 3: launch_gram_rows<3>(As, B, n, pl.blocks, partial, st, ldc, a0); break;
#endif
#if CAL_GRAM_ROWS_MAXNTA >= 4
            case 4: launch_gram_rows<4>(As, B, n, pl.blocks, partial, st, ldc, a0); break;
#endif
            default: return hipErrorInvalidValue;
        }
    }
    return hipGetLastError();
}

bool gram_bb_ok(int wa, int wb) { return CAL_GRAM_ROWS && wb <= 16 && wa >= 1 && (wa + 15) / 16 <= CAL_GRAM_ROWS_MAXNTA; }

hipError_t launch_gram_bb(const Panel& A, const Panel& B, int64_t n, const GramPlan& pl, double* partial,
                          hipStream_t st) {
    if (!gram_bb_ok(A.total, B.total)) return hipErrorInvalidValue;
    switch (pl.nta) {
        case 1: launch_gram_rows<1, true>(A, B, n, pl.blocks, partial, st); break;
        case 2: launch_gram_rows<2, true>(A, B, n, pl.blocks, partial, st); break;
#if CAL_GRAM_ROWS_MAXNTA >= 3
        case 3: launch_gram_rows<3, true>(A, B, n, pl.blocks, partial, st); break;
#endif
#if CAL_GRAM_ROWS_MAXNTA >= 4
        case 4: launch_gram_rows<4, true>(A, B, n, pl.blocks, partial, st); break;
#endif
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

GramPlan gram_plan(int wa, int wb, int64_t n) {
    GramPlan p;
    p.nta = (wa + 15) / 16;
    if (p.nta < 1) p.nta = 1;
    const bool rows = CAL_GRAM_ROWS && (p.nta <= CAL_GRAM_ROWS_MAXNTA ||
                                        (CAL_GRAM_ROWS_SPLIT && wb <= 16 && p.nta <= 2 * CAL_GRAM_ROWS_MAXNTA));
    const int run = rows ? CAL_GRAM_ROWS_RUN : (p.nta <= 2 ? 16 : (p.nta <= 4 ? 8 : 4));
    int64_t blocks = (n + 16 * run - 1) / (16 * run);
    if (rows && blocks > CAL_GRAM_ROWS_BLOCKS) blocks = CAL_GRAM_ROWS_BLOCKS;
    if (blocks > 2048) blocks = 2048;
    if (blocks < 1) blocks = 1;
    p.blocks = (int)blocks;
    p.entries = (int64_t)16 * p.nta * 16;
    return p;
}

template <int NTA, int RUN>
static void launch_gram_lds(const Panel& A, const Panel& B, int64_t n, int blocks, double* partial, hipStream_t st) {
    // grid steps per staging round: U = 2 / 4 (fewer barriers, twice / four
    // times the LDS) measured 5-20 % slower than U = 1 (occupancy)
    constexpr int U = 1;
    const size_t lds = std::max((size_t)2 * U * 16 * RUN * 17, (size_t)3 * NTA * 64 * 4) * sizeof(double);
    hipLaunchKernelGGL((k_gram_lds<NTA, RUN, U>), dim3(blocks), dim3(256), lds, st, A, B, n, partial);
}

// One-pass Gram of the w <= 16 NT columns of Q (column c at Q + c ld), the
// 16 x 16 tile pairs ta <= tb only (the block-upper part of Q'Q): the
// orthogonality errors of every deferred iteration of a run from one sweep
// over Q (compute_orth_err, ca_lanczos.m:99-107; lanczos.cpp: oe_flush),
// where the per-iteration Grams re-read Q(:,1:s(k-1)) every iteration.
// Per grid step a block stages R = 32 rows of all columns in LDS ([row][col],
// odd leading dimension; half a wave loads 32 rows of one column), double
// buffered, the next step's loads in flight across the barrier and the
// MFMAs.  Wave v owns the pairs p = v + 4i of the upper pairs in row order
// (compile-time per wave: the operand reads are fixed LDS offsets) and feeds
// v_mfma_f64_16x16x4f64 from the staged rows, 4 rows per MFMA.  The pairs of
// one wave are its own, so there is no block reduction: lane l of the wave
// owning pair p writes register r of it to entry (p * 64 + l) * 4 + r of
// the block's partials (entry-major, e * nblocks + block).
__host__ __device__ constexpr int gw_pair_a(int nt, int p) {
    int ta = 0;
    while (p >= nt - ta) {
        p -= nt - ta;
        ++ta;
    }
    return ta;
}
__host__ __device__ constexpr int gw_pair_b(int nt, int p) {
    int ta = 0;
    while (p >= nt - ta) {
        p -= nt - ta;
        ++ta;
    }
    return ta + p;
}

// pair P = WV + 4 I of the wave, register I (constant-evaluated indices)
template <int NT, int P, int I, int PW>
__device__ __forceinline__ void gram_wide_mfma(const double* __restrict__ row, d4 (&acc)[PW]) {
    if constexpr (P < NT * (NT + 1) / 2) {
        constexpr int ta = gw_pair_a(NT, P), tb = gw_pair_b(NT, P);
        acc[I] = mfma64(row[16 * ta], row[16 * tb], acc[I]);
    }
}

template <int NT, int WV, int PW, int R, int LDW, int... I>
__device__ __forceinline__ void gram_wide_step(const double* __restrict__ s, d4 (&acc)[PW], int g, int c16,
                                               std::integer_sequence<int, I...>) {
#pragma unroll
    for (int q = 0; q < R / 4; ++q) {
        const double* row = s + (4 * q + g) * LDW + c16;
        (gram_wide_mfma<NT, WV + 4 * I, I, PW>(row, acc), ...);
    }
}

template <int NT>
__global__ __launch_bounds__(256) void k_gram_wide(const double* __restrict__ Q, int64_t ld, int w, int64_t n,
                                                  double* __restrict__ partial) {
    constexpr int R = 32, LDW = 16 * NT + 1, NP = NT * (NT + 1) / 2, PW = (NP + 3) / 4;
    constexpr int PER = R * 16 * NT / 256;  // staged values per thread and step
    extern __shared__ __attribute__((aligned(16))) double lds_gw[];  // [2][R][LDW]
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, c16 = lane & 15, g = lane >> 4;
    const int lrow = tid & (R - 1), lcol = tid / R;  // loader: column lcol + (256 / R) q, row lrow
    d4 acc[PW];
#pragma unroll
    for (int i = 0; i < PW; ++i) acc[i] = d4{0.0, 0.0, 0.0, 0.0};
    const int64_t stride = (int64_t)gridDim.x * R;
    // columns past w are clamped to column 0 (only entries no caller reads
    // see them); rows past n are zeroed at the LDS write, so nothing waits
    // on the loads before the barrier and the MFMAs
    double v[PER];
    bool vin = false;
    auto load = [&](int64_t rb) {
        const int64_t rr = rb + lrow;
        vin = rr < n;
        const int64_t ro = vin ? rr : 0;
#pragma unroll
        for (int q = 0; q < PER; ++q) {
            const int c = lcol + (256 / R) * q;
            v[q] = Q[(int64_t)(c < w ? c : 0) * ld + ro];
        }
    };
    int64_t rb = (int64_t)blockIdx.x * R;
    if (rb < n) load(rb);
    for (int buf = 0; rb < n; rb += stride, buf ^= 1) {
        double* sb = lds_gw + buf * (R * LDW);
#pragma unroll
        for (int q = 0; q < PER; ++q) sb[lrow * LDW + lcol + (256 / R) * q] = vin ? v[q] : 0.0;
        if (rb + stride < n) load(rb + stride);
        __syncthreads();
        constexpr auto seq = std::make_integer_sequence<int, PW>{};
        switch (wave) {  // wave-uniform: each wave's pairs at fixed offsets
            case 0: gram_wide_step<NT, 0, PW, R, LDW>(sb, acc, g, c16, seq); break;
            case 1: gram_wide_step<NT, 1, PW, R, LDW>(sb, acc, g, c16, seq); break;
            case 2: gram_wide_step<NT, 2, PW, R, LDW>(sb, acc, g, c16, seq); break;
            default: gram_wide_step<NT, 3, PW, R, LDW>(sb, acc, g, c16, seq); break;
        }
        // buffer buf is rewritten two steps on, after the next step's barrier,
        // which every wave passes only once its MFMAs on buf have issued
    }
    const int64_t nb = gridDim.x;
#pragma unroll
    for (int i = 0; i < PW; ++i) {
        const int p = wave + 4 * i;
        if (p < NP)
#pragma unroll
            for (int r = 0; r < 4; ++r) partial[((int64_t)(p * 64 + lane) * 4 + r) * nb + blockIdx.x] = acc[i][r];
    }
}

int gram_wide_entries(int w) {
    const int nt = (w + 15) / 16;
    return nt * (nt + 1) / 2 * 256;
}

int gram_wide_blocks(int64_t n) {
    const int64_t b = (n + 31) / 32;
    return (int)std::max<int64_t>(1, std::min<int64_t>(512, b));
}

void gram_wide_entry(int w, int e, int* i, int* j) {
    const int nt = (w + 15) / 16;
    const int p = e / 256, lane = (e / 4) % 64, r = e % 4;
    *i = 16 * gw_pair_a(nt, p) + (lane >> 4) + 4 * r;
    *j = 16 * gw_pair_b(nt, p) + (lane & 15);
}

hipError_t launch_gram_wide(const double* Q, int64_t ld, int w, int64_t n, double* partial, hipStream_t st) {
    if (w < 1 || w > 128) return hipErrorInvalidValue;
    const int nt = (w + 15) / 16, blocks = gram_wide_blocks(n);
    const size_t lds = (size_t)2 * 32 * (16 * nt + 1) * sizeof(double);
#define CAL_GW(NT)                                                                                          \
    case NT: hipLaunchKernelGGL(k_gram_wide<NT>, dim3(blocks), dim3(256), lds, st, Q, ld, w, n, partial); break
    switch (nt) {
        CAL_GW(1);
        CAL_GW(2);
        CAL_GW(3);
        CAL_GW(4);
        CAL_GW(5);
        CAL_GW(6);
        CAL_GW(7);
        CAL_GW(8);
        default: return hipErrorInvalidValue;
    }
#undef CAL_GW
    return hipGetLastError();
}

hipError_t launch_gram(const Panel& A, const Panel& B, int64_t n, const GramPlan& pl, double* partial,
                       hipStream_t st) {
    dim3 g(pl.blocks), b(256);
    // the staged loads pay from 33 A columns on (tools/gram_probe.hip: +5-15 %
    // at 48-128 columns; RUN = 16 stages 256-row blocks in 70 KB of LDS and
    // loses to the direct loads at <= 32 columns)
    if (CAL_GRAM_ROWS && pl.nta <= CAL_GRAM_ROWS_MAXNTA) {
        switch (pl.nta) {
            case 1: launch_gram_rows<1>(A, B, n, pl.blocks, partial, st); break;
            case 2: launch_gram_rows<2>(A, B, n, pl.blocks, partial, st); break;
#if CAL_GRAM_ROWS_MAXNTA >= 3
            case 3: launch_gram_rows<3>(A, B, n, pl.blocks, partial, st); break;
#endif
#if CAL_GRAM_ROWS_MAXNTA >= 4
            case 4: launch_gram_rows<4>(A, B, n, pl.blocks, partial, st); break;
#endif
            default: return hipErrorInvalidValue;
        }
        return hipGetLastError();
    }
    if (CAL_GRAM_ROWS && CAL_GRAM_ROWS_SPLIT && B.total <= 16 && pl.nta <= 2 * CAL_GRAM_ROWS_MAXNTA)
        return launch_gram_rows_split(A, B, n, pl, partial, st);
    if (pl.nta >= 3) {
        switch (pl.nta) {
            case 3: launch_gram_lds<3, 8>(A, B, n, pl.blocks, partial, st); break;
            case 4: launch_gram_lds<4, 8>(A, B, n, pl.blocks, partial, st); break;
            case 5: launch_gram_lds<5, 4>(A, B, n, pl.blocks, partial, st); break;
            case 6: launch_gram_lds<6, 4>(A, B, n, pl.blocks, partial, st); break;
            case 7: launch_gram_lds<7, 4>(A, B, n, pl.blocks, partial, st); break;
            case 8: launch_gram_lds<8, 4>(A, B, n, pl.blocks, partial, st); break;
            default: return hipErrorInvalidValue;
        }
        return hipGetLastError();
    }
    switch (pl.nta) {
        case 1: hipLaunchKernelGGL((k_gram<1, 16>), g, b, 0, st, A, B, n, partial); break;
        case 2: hipLaunchKernelGGL((k_gram<2, 16>), g, b, 0, st, A, B, n, partial); break;
        case 3: hipLaunchKernelGGL((k_gram<3, 8>), g, b, 0, st, A, B, n, partial); break;
        case 4: hipLaunchKernelGGL((k_gram<4, 8>), g, b, 0, st, A, B, n, partial); break;
        case 5: hipLaunchKernelGGL((k_gram<5, 4>), g, b, 0, st, A, B, n, partial); break;
        case 6: hipLaunchKernelGGL((k_gram<6, 4>), g, b, 0, st, A, B, n, partial); break;
        case 7: hipLaunchKernelGGL((k_gram<7, 4>), g, b, 0, st, A, B, n, partial); break;
        case 8: hipLaunchKernelGGL((k_gram<8, 4>), g, b, 0, st, A, B, n, partial); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

// --------------------------------------------------------------------------
// Apply: Y = P M (+ optional Y^T Y and Psub^T Y).  MFMA A-operand = P rows:
// lane l holds P(row r0 + (l&15)*RUN + t, col 4*kc + (l>>4)) for tile t; the
// B-operand M(4*kc + (l>>4), 16*ty + (l&15)) comes from LDS.  Accumulator
// tile (ty,t) reg r holds Y(row r0 + ((l>>4)+4r)*RUN + t, col 16*ty + (l&15)),
// which is directly the A and B operand of the fused Gram MFMAs (k = l>>4).
// --------------------------------------------------------------------------
template <int NTY, int RUN, bool GRAM, bool GRAMP, bool STORE>
__global__ __launch_bounds__(256) void k_apply(Panel P, const double* __restrict__ M, int wp, int wy,
                                               PanelOut Y, int wq, int64_t n,
                                               double* __restrict__ partial) {
    extern __shared__ __attribute__((aligned(16))) double smem[];
    const int wpp = (wp + 3) & ~3;
    const int ldm = 16 * NTY;
    double* Ms = smem;                      // [wpp][ldm]
    double* red = smem + (size_t)wpp * ldm;  // [3][2][64][4]
    for (int e = threadIdx.x; e < wpp * ldm; e += 256) {
        const int k = e / ldm, j = e % ldm;
        Ms[e] = (k < wp && j < wy) ? M[(int64_t)j * wp + k] : 0.0;
    }
    __syncthreads();
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int c16 = lane & 15, g = lane >> 4;
    const int nkc = wpp / 4;
    d4 gacc = d4{0.0, 0.0, 0.0, 0.0}, gpacc = d4{0.0, 0.0, 0.0, 0.0};
    const bool qon = c16 < wq;
    const double* qc = pcol(P, qon ? c16 : 0);

    const int64_t wstep = 16 * RUN;
    const int64_t stride = (int64_t)gridDim.x * 4 * wstep;
    for (int64_t r0 = ((int64_t)blockIdx.x * 4 + wave) * wstep; r0 < n; r0 += stride) {
        const bool full = r0 + wstep <= n;
        d4 acc[NTY][RUN];
#pragma unroll
        for (int ty = 0; ty < NTY; ++ty)
#pragma unroll
            for (int t = 0; t < RUN; ++t) acc[ty][t] = d4{0.0, 0.0, 0.0, 0.0};
        const int64_t ra = r0 + (int64_t)c16 * RUN;  // this lane's A-operand rows
        for (int kc = 0; kc < nkc; ++kc) {
            const int c = kc * 4 + g;
            const bool con = c < wp;
            const double* pc = pcol(P, con ? c : 0);
            double av[RUN];
            if (full && RUN % 2 == 0) {
#pragma unroll
                for (int t = 0; t < RUN; t += 2) {
                    d2 x = *reinterpret_cast<const d2*>(pc + ra + t);
                    av[t] = con ? x[0] : 0.0;
                    av[t + 1] = con ? x[1] : 0.0;
                }
            } else {
#pragma unroll
                for (int t = 0; t < RUN; ++t) {
                    const bool in = ra + t < n;
                    double x = pc[in ? ra + t : 0];
                    av[t] = (con && in) ? x : 0.0;
                }
            }
#pragma unroll
            for (int ty = 0; ty < NTY; ++ty) {
                const double bm = Ms[(kc * 4 + g) * ldm + ty * 16 + c16];
#pragma unroll
                for (int t = 0; t < RUN; ++t) acc[ty][t] = mfma64(av[t], bm, acc[ty][t]);
            }
        }
        if (STORE) {
#pragma unroll
            for (int ty = 0; ty < NTY; ++ty) {
                const int j = ty * 16 + c16;
                if (j < wy) {
                    double* yc = pcol_out(Y, j);
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const int64_t rr = r0 + (int64_t)(g + 4 * r) * RUN;
                        if (full && RUN % 2 == 0) {
#pragma unroll
                            for (int t = 0; t < RUN; t += 2) {
                                d2 x;
                                x[0] = acc[ty][t][r];
                                x[1] = acc[ty][t + 1][r];
                                *reinterpret_cast<d2*>(yc + rr + t) = x;
                            }
                        } else {
#pragma unroll
                            for (int t = 0; t < RUN; ++t)
                                if (rr + t < n) yc[rr + t] = acc[ty][t][r];
                        }
                    }
                }
            }
        }
        if (GRAM) {
#pragma unroll
            for (int t = 0; t < RUN; ++t)
#pragma unroll
                for (int r = 0; r < 4; ++r) gacc = mfma64(acc[0][t][r], acc[0][t][r], gacc);
        }
        if (GRAMP) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int64_t rr = r0 + (int64_t)(g + 4 * r) * RUN;
#pragma unroll
                for (int t = 0; t < RUN; ++t) {
                    const bool in = rr + t < n;
                    double x = qc[in ? rr + t : 0];
                    const double qv = (qon && in) ? x : 0.0;
                    gpacc = mfma64(qv, acc[0][t][r], gpacc);
                }
            }
        }
    }
    if (GRAM || GRAMP) {
        __syncthreads();
        if (wave > 0) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                red[(((wave - 1) * 2 + 0) * 64 + lane) * 4 + r] = gacc[r];
                red[(((wave - 1) * 2 + 1) * 64 + lane) * 4 + r] = gpacc[r];
            }
        }
        __syncthreads();
        if (wave == 0) {
            const int nent = 256 * ((GRAM ? 1 : 0) + (GRAMP ? 1 : 0));
            double* out = partial + blockIdx.x;  // entry-major: [entry][block]
            const int64_t nb = gridDim.x;
            (void)nent;
            int base = 0;
#pragma unroll
            for (int which = 0; which < 2; ++which) {
                if ((which == 0 && !GRAM) || (which == 1 && !GRAMP)) continue;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    double v = which == 0 ? gacc[r] : gpacc[r];
                    v = v + red[((0 * 2 + which) * 64 + lane) * 4 + r];
                    v = v + red[((1 * 2 + which) * 64 + lane) * 4 + r];
                    v = v + red[((2 * 2 + which) * 64 + lane) * 4 + r];
                    const int i = g + 4 * r, j = c16;
                    out[(int64_t)(base + j * 16 + i) * nb] = v;
                }
                base += 256;
            }
        }
    }
}

ApplyPlan apply_plan(int wp, int wy, int64_t n, bool gram, int wq) {
    ApplyPlan p;
    p.nty = wy <= 16 ? 1 : (wy <= 32 ? 2 : (wy <= 64 ? 4 : 8));
    p.run = p.nty == 1 ? 4 : (p.nty == 2 ? 2 : 1);
    p.gram = gram && p.nty == 1;
    p.gramp = wq > 0 && p.nty == 1;
    int64_t blocks = (n + 64 * p.run - 1) / (64 * p.run);
    if (blocks > 2048) blocks = 2048;
    if (blocks < 1) blocks = 1;
    p.blocks = (int)blocks;
    const int wpp = (wp + 3) & ~3;
    p.lds_bytes = sizeof(double) * ((size_t)wpp * 16 * p.nty + 3 * 2 * 64 * 4);
    p.entries = 256 * ((p.gram ? 1 : 0) + (p.gramp ? 1 : 0));
    return p;
}

// Store-only apply Y = P M with one row per lane: every column load and
// store is a contiguous 512-B wave access (the tile layout of k_apply reads
// 16 row runs per instruction and reaches 3.3-3.8 TB/s on the restart
// drivers' wide panels; tools/wide_probe.hip).  M (wp x wy, column-major) is
// staged row-major in LDS for broadcast reads.  y_j = fma(p_c, M(c,j), y_j)
// over c ascending.  Y may alias columns of P: a lane reads all of its row
// before it writes it.
#ifndef CAL_APPLY_ROWS_G
#define CAL_APPLY_ROWS_G 8
#endif
#ifndef CAL_APPLY_ROWS_GRID
#define CAL_APPLY_ROWS_GRID 0  // blocks cap (grid-stride rows); 0: one 256-row tile per block
#endif
template <int WY>
__global__ __launch_bounds__(256) void k_apply_rows(Panel P, const double* __restrict__ M, int wp, int wy,
                                                    PanelOut Y, int64_t n) {
    extern __shared__ __attribute__((aligned(16))) double Mr[];  // [wp][WY]
    for (int e = threadIdx.x; e < wp * WY; e += 256) {
        const int c = e / WY, j = e % WY;
        Mr[e] = j < wy ? M[(int64_t)j * wp + c] : 0.0;
    }
    __syncthreads();
    // segment tables copied field by field with static indices (a reference
    // to the by-value kernel argument would copy it to scratch per thread)
    const double* sp[kMaxSeg];
    int64_t sl[kMaxSeg];
    int sb[kMaxSeg + 1];
    sb[0] = 0;
#pragma unroll
    for (int q = 0; q < kMaxSeg; ++q) {
        sp[q] = P.ptr[q];
        sl[q] = P.ld[q];
        sb[q + 1] = sb[q] + (q < P.nseg ? P.ncol[q] : 0);
    }
    double* yp[kMaxSeg];
    int64_t yl[kMaxSeg];
    int yb[kMaxSeg + 1];
    yb[0] = 0;
#pragma unroll
    for (int q = 0; q < kMaxSeg; ++q) {
        yp[q] = Y.ptr[q];
        yl[q] = Y.ld[q];
        yb[q + 1] = yb[q] + (q < Y.nseg ? Y.ncol[q] : 0);
    }
    const int64_t stride = (int64_t)gridDim.x * 256;
    for (int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x; r < n; r += stride) {
        auto colp = [&](int c) {
            const double* res = sp[0] + r;
#pragma unroll
            for (int q = 0; q < kMaxSeg; ++q)
                if (c >= sb[q] && c < sb[q + 1]) res = sp[q] + (int64_t)(c - sb[q]) * sl[q] + r;
            return res;
        };
        double y[WY];
#pragma unroll
        for (int j = 0; j < WY; ++j) y[j] = 0.0;
        constexpr int G = CAL_APPLY_ROWS_G;  // columns whose loads are in flight together
        for (int c0 = 0; c0 < wp; c0 += G) {
            double p[G];
#pragma unroll
            for (int u = 0; u < G; ++u) p[u] = *colp(c0 + u < wp ? c0 + u : c0);
#pragma unroll
            for (int u = 0; u < G; ++u) {
                if (c0 + u < wp) {
                    const double* mrow = Mr + (c0 + u) * WY;
#pragma unroll
                    for (int j = 0; j < WY; ++j) y[j] = __builtin_fma(p[u], mrow[j], y[j]);
                }
            }
        }
#pragma unroll
        for (int j = 0; j < WY; ++j) {
            if (j < wy) {
                double* dst = yp[0] + r;
#pragma unroll
                for (int q = 0; q < kMaxSeg; ++q)
                    if (j >= yb[q] && j < yb[q + 1]) dst = yp[q] + (int64_t)(j - yb[q]) * yl[q] + r;
                *dst = y[j];
            }
        }
    }
}

// One block-MGS step of project.m fused with the next block's Gram:
//   Y = P M (P = [Q{i} | X], M = [-R{i}; I]: X - Q{i} R{i}, stored), and
//   G = Qn' Y (Qn = Q{i+1}: the next step's R{i+1}), in one pass over the rows.
// Staged like k_gram_rows: per round a block loads 64 rows of P's and Qn's
// columns, one column per wave instruction (lane = row, 512 B), into LDS
// [row][col] (the loads of the next round in flight across the round);
// barrier; thread (row = lane, wave w) forms y_j = fma(p_c, M(c,j), y_j) over
// c ascending for its WY/4 columns j (k_apply_rows' order: the same Y bits),
// stores them (lane = row again) and parks them in LDS; barrier; lane (c16,
// g) of wave w feeds MFMA m with row w*16 + g*4 + m of Qn column c16 and of
// Y column c16.  Buffer b is rewritten two rounds on, after both barriers of
// the round between.  GRAM = false is the plain staged apply (one barrier).
// The four waves' accumulators are added in order at the end (entry-major
// partials as k_gram's: A = Qn, B = Y, ldc = 16).  Replaces apply (read P,
// write Y) + Gram (read Qn, re-read Y): 8 n (wp + wq) read and 8 n wy written
// instead of 8 n (wp + wq + wy) read and 8 n wy written, and one launch.
// GRAM: 0 none, 1 Qn'Y as above, 2 Y'Y (the last MGS step fused with the
// normalize's first Gram sweep, P1 of blockorth.cpp orth_device: its 272-entry
// tile layout, the extra column's 16 entries zero).
template <int WY, int NCP, int GRAM>
__global__ __launch_bounds__(256) void k_apply_stage(Panel P, const double* __restrict__ M, int wp, int wy,
                                                     PanelOut Y, Panel Qn, int64_t n, double* __restrict__ partial) {
    constexpr int R = 64;
    constexpr int NQ = GRAM == 1 ? 16 : 0;
    constexpr int NS = NCP + NQ;             // staged global columns
    constexpr int PER = NS / 4;              // loads per thread and round
    constexpr int LD = NS + (GRAM ? WY : 0) + 1;
    constexpr int JW = WY / 4;               // y columns per thread
    static_assert(NS % 4 == 0 && WY % 4 == 0, "k_apply_stage geometry");
    extern __shared__ __attribute__((aligned(16))) double lds_as[];
    double* Mr = lds_as;                     // [NCP][WY]
    double* buf = lds_as + NCP * WY;         // [2][R][LD]
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, c16 = lane & 15, g = lane >> 4;
    for (int e = tid; e < NCP * WY; e += 256) {
        const int c = e / WY, j = e % WY;
        Mr[e] = (j < wy && c < wp) ? M[(int64_t)j * wp + c] : 0.0;
    }
    const int wq = GRAM == 1 ? Qn.total : 0;
    // loader: column wave + 4 q (wave-uniform), row lane
    const double* pc[PER];
    bool on[PER];
#pragma unroll
    for (int q = 0; q < PER; ++q) {
        const int cc = wave + 4 * q;
        if (cc < NCP) {
            on[q] = cc < wp;
            pc[q] = pcol(P, on[q] ? cc : 0);
        } else {
            on[q] = cc - NCP < wq;
            pc[q] = pcol(Qn, on[q] ? cc - NCP : 0);
        }
    }
    double* yc[JW];
    bool yon[JW];
#pragma unroll
    for (int u = 0; u < JW; ++u) {
        const int j = wave * JW + u;
        yon[u] = j < wy;
        yc[u] = pcol_out(Y, yon[u] ? j : 0);
    }
    d4 acc = d4{0.0, 0.0, 0.0, 0.0};
    const int64_t stride = (int64_t)gridDim.x * R;
    double v[PER];
    bool vin = false;
    auto load = [&](int64_t rb) {
        const int64_t rr = rb + lane;
        vin = rr < n;
        const int64_t ro = vin ? rr : 0;
#pragma unroll
        for (int q = 0; q < PER; ++q) v[q] = on[q] ? pc[q][ro] : 0.0;
    };
    int64_t rb = (int64_t)blockIdx.x * R;
    if (rb < n) load(rb);
    __syncthreads();  // Mr
    for (int b = 0; rb < n; rb += stride, b ^= 1) {
        double* sb = buf + b * (R * LD);
        const bool in = vin;
#pragma unroll
        for (int q = 0; q < PER; ++q) sb[lane * LD + wave + 4 * q] = in ? v[q] : 0.0;
        if (rb + stride < n) load(rb + stride);
        __syncthreads();
        // Y rows: this thread's row `lane`, columns wave*JW + u
        double y[JW];
#pragma unroll
        for (int u = 0; u < JW; ++u) y[u] = 0.0;
        const double* prow = sb + lane * LD;
        for (int c = 0; c < wp; ++c) {
            const double pv = prow[c];
#pragma unroll
            for (int u = 0; u < JW; ++u) y[u] = __builtin_fma(pv, Mr[c * WY + wave * JW + u], y[u]);
        }
        const int64_t r = rb + lane;
#pragma unroll
        for (int u = 0; u < JW; ++u)
            if (yon[u] && r < n) yc[u][r] = y[u];
        if constexpr (GRAM) {
#pragma unroll
            for (int u = 0; u < JW; ++u) sb[lane * LD + NS + wave * JW + u] = (yon[u] && r < n) ? y[u] : 0.0;
            __syncthreads();
#pragma unroll
            for (int m = 0; m < 4; ++m) {
                const double* row = sb + (wave * 16 + g * 4 + m) * LD;
                const double yb = c16 < WY ? row[NS + (c16 < WY ? c16 : 0)] : 0.0;
                acc = mfma64(GRAM == 1 ? row[NCP + c16] : yb, yb, acc);
            }
        }
    }
    if constexpr (GRAM) {
        __syncthreads();  // the staging buffers become the partials
        auto red = reinterpret_cast<double (*)[64][4]>(buf);  // [3][64][4]
        if (wave > 0)
#pragma unroll
            for (int q = 0; q < 4; ++q) red[wave - 1][lane][q] = acc[q];
        __syncthreads();
        if (wave == 0) {
            double* out = partial + blockIdx.x;
            const int64_t nb = gridDim.x;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                double x = acc[q];
                x = x + red[0][lane][q];
                x = x + red[1][lane][q];
                x = x + red[2][lane][q];
                const int i = g + 4 * q, j = c16;
                out[(int64_t)(j * 16 + i) * nb] = x;
            }
            if (GRAM == 2 && g == 0) out[(int64_t)(256 + c16) * nb] = 0.0;
        }
    }
}

#ifndef CAL_APPLY_GRAM_BLOCKS
#define CAL_APPLY_GRAM_BLOCKS 1024
#endif
bool apply_gram_ok(int wp, int wy, int wq) { return wp >= 1 && wp <= 32 && wy >= 1 && wy <= 16 && wq >= 1 && wq <= 16; }
int apply_gram_blocks(int64_t n) {
    return (int)std::max<int64_t>(1, std::min<int64_t>(CAL_APPLY_GRAM_BLOCKS, (n + 63) / 64));
}

template <int GRAM>
static hipError_t launch_apply_stage(const Panel& P, const double* dM, int wp, int wy, const PanelOut& Y,
                                     const Panel& Qn, int64_t n, double* partial, hipStream_t st) {
    const int blocks = apply_gram_blocks(n);
    auto go = [&](auto WY_, auto NCP_) {
        constexpr int WY = decltype(WY_)::value, NCP = decltype(NCP_)::value;
        constexpr int LD = NCP + (GRAM == 1 ? 16 : 0) + (GRAM ? WY : 0) + 1;
        const size_t lds = sizeof(double) * std::max((size_t)NCP * WY + 2 * 64 * LD, (size_t)3 * 64 * 4);
        hipLaunchKernelGGL((k_apply_stage<WY, NCP, GRAM>), dim3(blocks), dim3(256), lds, st, P, dM, wp, wy, Y, Qn,
                           n, partial);
    };
    using I8 = std::integral_constant<int, 8>;
    using I16 = std::integral_constant<int, 16>;
    using I24 = std::integral_constant<int, 24>;
    using I32 = std::integral_constant<int, 32>;
    using I64 = std::integral_constant<int, 64>;
    if (wy <= 8) {
        if (wp <= 24) go(I8{}, I24{});
        else if (wp <= 32 || GRAM) go(I8{}, I32{});
        else go(I8{}, I64{});
    } else {
        if (wp <= 24) go(I16{}, I24{});
        else if (wp <= 32 || GRAM) go(I16{}, I32{});
        else go(I16{}, I64{});
    }
    return hipGetLastError();
}

hipError_t launch_apply_gram(const Panel& P, const double* dM, int wp, int wy, const PanelOut& Y, const Panel& Qn,
                             int64_t n, double* partial, hipStream_t st) {
    if (!apply_gram_ok(wp, wy, Qn.total)) return hipErrorInvalidValue;
    return launch_apply_stage<1>(P, dM, wp, wy, Y, Qn, n, partial, st);
}

bool apply_selfgram_ok(int wp, int wy) { return wp >= 1 && wp <= 32 && wy >= 1 && wy <= 16; }

hipError_t launch_apply_selfgram(const Panel& P, const double* dM, int wp, int wy, const PanelOut& Y, int64_t n,
                                 double* partial, int* blocks, hipStream_t st) {
    if (!apply_selfgram_ok(wp, wy)) return hipErrorInvalidValue;
    *blocks = apply_gram_blocks(n);
    return launch_apply_stage<2>(P, dM, wp, wy, Y, Panel{}, n, partial, st);
}

// the row-parallel store-only apply: <= 16 outputs for any panel up to 256
// columns, wider output chunks (32, 64) while M fits 64 KB of LDS
int apply_rows_max_wy(int wp) {
    if (wp < 1 || wp > 256) return 0;
    int wy = 16;
    while (wy < 64 && (size_t)wp * (2 * wy) * sizeof(double) <= 65536) wy *= 2;
    return wy;
}
bool apply_rows_ok(int wp, int wy) { return wy >= 1 && wy <= apply_rows_max_wy(wp); }

#ifndef CAL_APPLY_STAGE
#define CAL_APPLY_STAGE 1  // plain applies (wp <= CAL_APPLY_STAGE_WP, wy <= 16) on k_apply_stage<GRAM = false>
#endif
#ifndef CAL_APPLY_STAGE_WP
#define CAL_APPLY_STAGE_WP 32
#endif
hipError_t launch_apply(const Panel& P, const double* dM, int wp, int wy, const PanelOut& Y, bool store,
                        int wq, int64_t n, const ApplyPlan& pl, double* partial, hipStream_t st) {
    if (CAL_APPLY_STAGE && store && !pl.gram && !pl.gramp && wp <= CAL_APPLY_STAGE_WP && wy <= 16 && wp >= 1 &&
        wy >= 1 && n > 0)
        return launch_apply_stage<0>(P, dM, wp, wy, Y, Panel{}, n, nullptr, st);
    if (store && !pl.gram && !pl.gramp && apply_rows_ok(wp, wy)) {
        int64_t nbk = (n + 255) / 256;
        if (CAL_APPLY_ROWS_GRID > 0 && nbk > CAL_APPLY_ROWS_GRID) nbk = CAL_APPLY_ROWS_GRID;
        const dim3 g((unsigned)nbk), b(256);
        const int WY = wy <= 1 ? 1 : (wy <= 2 ? 2 : (wy <= 4 ? 4 : (wy <= 8 ? 8 : (wy <= 16 ? 16 : (wy <= 32 ? 32 : 64)))));
        const size_t sh = sizeof(double) * (size_t)wp * WY;
        if (n <= 0) return hipSuccess;
        switch (WY) {
            case 1: hipLaunchKernelGGL((k_apply_rows<1>), g, b, sh, st, P, dM, wp, wy, Y, n); break;
            case 2: hipLaunchKernelGGL((k_apply_rows<2>), g, b, sh, st, P, dM, wp, wy, Y, n); break;
            case 4: hipLaunchKernelGGL((k_apply_rows<4>), g, b, sh, st, P, dM, wp, wy, Y, n); break;
            case 8: hipLaunchKernelGGL((k_apply_rows<8>), g, b, sh, st, P, dM, wp, wy, Y, n); break;
            case 16: hipLaunchKernelGGL((k_apply_rows<16>), g, b, sh, st, P, dM, wp, wy, Y, n); break;
            case 32: hipLaunchKernelGGL((k_apply_rows<32>), g, b, sh, st, P, dM, wp, wy, Y, n); break;
            default: hipLaunchKernelGGL((k_apply_rows<64>), g, b, sh, st, P, dM, wp, wy, Y, n); break;
        }
        return hipGetLastError();
    }
    dim3 g(pl.blocks), b(256);
    const size_t sh = pl.lds_bytes;
#define CAL_APPLY(NTY, RUN, G, GP, S) \
    hipLaunchKernelGGL((k_apply<NTY, RUN, G, GP, S>), g, b, sh, st, P, dM, wp, wy, Y, wq, n, partial)
    if (pl.nty == 1) {
        const int key = (pl.gram ? 4 : 0) | (pl.gramp ? 2 : 0) | (store ? 1 : 0);
        switch (key) {
            case 1: CAL_APPLY(1, 4, false, false, true); break;
            case 2: CAL_APPLY(1, 4, false, true, false); break;
            case 3: CAL_APPLY(1, 4, false, true, true); break;
            case 4: CAL_APPLY(1, 4, true, false, false); break;
            case 5: CAL_APPLY(1, 4, true, false, true); break;
            case 6: CAL_APPLY(1, 4, true, true, false); break;
            case 7: CAL_APPLY(1, 4, true, true, true); break;
            default: return hipErrorInvalidValue;
        }
    } else {
        if (!store) return hipErrorInvalidValue;
        switch (pl.nty) {
            case 2: CAL_APPLY(2, 2, false, false, true); break;
            case 4: CAL_APPLY(4, 1, false, false, true); break;
            case 8: CAL_APPLY(8, 1, false, false, true); break;
            default: return hipErrorInvalidValue;
        }
    }
#undef CAL_APPLY
    return hipGetLastError();
}

// Store-only Y = P M for wide outputs (the Ritz vectors X = Q(:,1:sk) Vp of
// compute_ritz_rnorm, ca_lanczos.m:93) on the matrix cores with the operand
// roles transposed: D = M^T P^T.  Lane l feeds A = M(4kc + (l>>4), 16ty +
// (l&15)) from LDS and B = P(r0 + 2(l&15) + t, 4kc + (l>>4)) (one 16-B load
// per lane for t = 0, 1), so accumulator register r of tile (ty, t) holds
// Y(r0 + 2(l&15) + t, 16ty + (l>>4) + 4r): every store writes 256 contiguous
// bytes of one column.  The k_apply_rows kernel above pays one LDS broadcast
// read per two FMAs and stalls on the LDS return path at ~25 TF; here one LDS
// read feeds two 16x16x4 MFMAs (tools/ritz_apply_probe.hip, n = 9.94 M:
// 120 x 120 in 6.6 ms vs 12.5 ms).  Each output is the k-ascending FMA chain
// starting from 0, as k_apply_rows computes it (the probe compares bitwise).
// One segment each; Y must not alias P.  Grid: blockIdx.y = 16*NT-column group.
template <int NT, int WAVES, int KG>
__device__ __forceinline__ void apply_mt_body(const double* __restrict__ P, int64_t ldp, const double* __restrict__ M,
                                              int wp, int wy, double* __restrict__ Y, int64_t ldy, int64_t n) {
    extern __shared__ __attribute__((aligned(16))) double Ms[];  // [wpp][16 NT]
    constexpr int ldm = 16 * NT;
    const int wpp = (wp + 3) & ~3;
    const int c0 = blockIdx.y * ldm;
    for (int e = threadIdx.x; e < wpp * ldm; e += 64 * WAVES) {
        const int k = e / ldm, j = e % ldm;
        Ms[e] = (k < wp && c0 + j < wy) ? M[(int64_t)(c0 + j) * wp + k] : 0.0;
    }
    __syncthreads();
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int c16 = lane & 15, g = lane >> 4;
    const int nkc = wpp / 4;
    const int64_t stride = (int64_t)gridDim.x * WAVES * 32;
    // B operands in groups of KG k-steps, the next group's loads issued before
    // this group's MFMAs (KG per NT from tools/ritz_apply_probe.hip); the last
    // group of a row tile issues the NEXT row tile's first group, so its load
    // latency hides behind this tile's last MFMAs and stores.  Full 32-row
    // tiles load branch-free (a column past wp reads column wp - 1, whose
    // coefficient rows in Ms are zero): a per-load branch between a 16-B and
    // a guarded path made the compiler join the two with vmcnt(0) after every
    // group, i.e. no load was in flight across the MFMAs.  The one partial
    // tile of the grid runs after the loop with guarded loads.
    auto load_full = [&](int64_t rt, int kc0, double (&b)[KG][2]) {
        const int64_t rbt = rt + 2 * c16;
#pragma unroll
        for (int u = 0; u < KG; ++u) {
            const int c = 4 * (kc0 + u) + g;
            const d2 x = *reinterpret_cast<const d2*>(P + (int64_t)(c < wp ? c : wp - 1) * ldp + rbt);
            b[u][0] = x[0];
            b[u][1] = x[1];
        }
    };
    auto load_part = [&](int64_t rt, int kc0, double (&b)[KG][2]) {
        const int64_t rbt = rt + 2 * c16;
#pragma unroll
        for (int u = 0; u < KG; ++u) {
            const int c = 4 * (kc0 + u) + g;
            const double* pc = P + (int64_t)(c < wp ? c : wp - 1) * ldp;
            b[u][0] = rbt < n ? pc[rbt] : 0.0;
            b[u][1] = rbt + 1 < n ? pc[rbt + 1] : 0.0;
        }
    };
    auto mfma_group = [&](int kc0, const double (&b)[KG][2], d4 (&acc)[NT][2]) {
#pragma unroll
        for (int u = 0; u < KG; ++u) {
            const int c = 4 * (kc0 + u) + g;  // rows of Ms past wpp are never read: kc0 + u < nkc below
            if (kc0 + u < nkc) {
#pragma unroll
                for (int ty = 0; ty < NT; ++ty) {
                    const double a = Ms[c * ldm + 16 * ty + c16];
                    acc[ty][0] = mfma64(a, b[u][0], acc[ty][0]);
                    acc[ty][1] = mfma64(a, b[u][1], acc[ty][1]);
                }
            }
        }
    };
    auto store_tile = [&](int64_t r0, bool full, const d4 (&acc)[NT][2]) {
        const int64_t rb = r0 + 2 * c16;
#pragma unroll
        for (int ty = 0; ty < NT; ++ty)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int j = c0 + 16 * ty + g + 4 * r;
                if (j < wy) {
                    double* yc = Y + (int64_t)j * ldy;
                    if (full) {
                        d2 x;
                        x[0] = acc[ty][0][r];
                        x[1] = acc[ty][1][r];
                        *reinterpret_cast<d2*>(yc + rb) = x;
                    } else {
                        if (rb < n) yc[rb] = acc[ty][0][r];
                        if (rb + 1 < n) yc[rb + 1] = acc[ty][1][r];
                    }
                }
            }
    };
    double bcur[KG][2], bnxt[KG][2];
    int64_t r0 = ((int64_t)blockIdx.x * WAVES + wave) * 32;
    if (r0 + 32 <= n) load_full(r0, 0, bcur);
    for (; r0 + 32 <= n; r0 += stride) {
        d4 acc[NT][2];
#pragma unroll
        for (int ty = 0; ty < NT; ++ty) acc[ty][0] = acc[ty][1] = d4{0.0, 0.0, 0.0, 0.0};
        for (int kc0 = 0; kc0 < nkc; kc0 += KG) {
            if (kc0 + KG < nkc) load_full(r0, kc0 + KG, bnxt);
            else if (r0 + stride + 32 <= n) load_full(r0 + stride, 0, bnxt);
            mfma_group(kc0, bcur, acc);
#pragma unroll
            for (int u = 0; u < KG; ++u) {
                bcur[u][0] = bnxt[u][0];
                bcur[u][1] = bnxt[u][1];
            }
        }
        store_tile(r0, true, acc);
    }
    if (r0 < n) {  // the partial tile
        d4 acc[NT][2];
#pragma unroll
        for (int ty = 0; ty < NT; ++ty) acc[ty][0] = acc[ty][1] = d4{0.0, 0.0, 0.0, 0.0};
        for (int kc0 = 0; kc0 < nkc; kc0 += KG) {
            load_part(r0, kc0, bcur);
            mfma_group(kc0, bcur, acc);
        }
        store_tile(r0, false, acc);
    }
}

template <int NT, int WAVES, int KG>
__global__ __launch_bounds__(64 * WAVES) void k_apply_mt(const double* __restrict__ P, int64_t ldp,
                                                         const double* __restrict__ M, int wp, int wy,
                                                         double* __restrict__ Y, int64_t ldy, int64_t n) {
    apply_mt_body<NT, WAVES, KG>(P, ldp, M, wp, wy, Y, ldy, n);
}

// k-steps per load group of k_apply_mt by tile count
// (6 k-steps from 3 tiles on, now that the group's loads stay in flight: 5-8 %
// faster than 4 at 5-7 tiles; at 8 tiles 6 spill and 4 stays)
constexpr int apply_mt_kg(int nt) { return nt <= 2 ? 2 : (nt <= 7 ? 6 : 4); }

// 16-column tiles per block: ceil(wy / 16) up to 8 (no idle tiles), fewer
// until M (wpp x 16 NT doubles) fits the 160 KB of LDS of one CU (0: never)
static int apply_mt_nt(int wp, int wy) {
    const size_t wpp = (size_t)((wp + 3) & ~3);
    int nt = std::min(8, (wy + 15) / 16);
    while (nt > 1 && wpp * 16 * nt * sizeof(double) > 160 * 1024) --nt;
    return wpp * 16 * nt * sizeof(double) <= 160 * 1024 ? nt : 0;
}

bool apply_mt_ok(int wp, int wy) { return wp >= 1 && wy >= 1 && apply_mt_nt(wp, wy) > 0; }

hipError_t launch_apply_mt(const double* P, int64_t ldp, const double* dM, int wp, int wy, double* Y, int64_t ldy,
                           int64_t n, hipStream_t st) {
    if (!apply_mt_ok(wp, wy) || (((uintptr_t)P | (uintptr_t)Y | (uintptr_t)(ldp * 8) | (uintptr_t)(ldy * 8)) & 15))
        return hipErrorInvalidValue;
    if (n <= 0) return hipSuccess;
    const int wpp = (wp + 3) & ~3;
    // probe (n = 9.94 M): <= 32 outputs 4 waves, 4 blocks per CU; wider 8
    // waves, 2 blocks per CU (1 at 128 outputs); fewer when M does not fit
    auto go = [&](auto nt_c, auto waves_c, int per_cu) {
        constexpr int NT = decltype(nt_c)::value, WAVES = decltype(waves_c)::value;
        constexpr int KG = apply_mt_kg(NT);
        const size_t lds = (size_t)wpp * 16 * NT * sizeof(double);
        const int fit = (int)((160 * 1024) / lds);
        const int bpc = std::max(1, std::min(per_cu, fit));
        int64_t blocks = (n + 32 * WAVES - 1) / (32 * WAVES);
        if (blocks > 256 * bpc) blocks = 256 * bpc;
        const unsigned groups = (unsigned)((wy + 16 * NT - 1) / (16 * NT));
        hipLaunchKernelGGL((k_apply_mt<NT, WAVES, KG>), dim3((unsigned)blocks, groups), dim3(64 * WAVES), lds, st, P, ldp,
                           dM, wp, wy, Y, ldy, n);
    };
    using I = std::integral_constant<int, 4>;
    using E = std::integral_constant<int, 8>;
    switch (apply_mt_nt(wp, wy)) {
        case 1: go(std::integral_constant<int, 1>{}, I{}, 4); break;
        case 2: go(std::integral_constant<int, 2>{}, I{}, 4); break;
        case 3: go(std::integral_constant<int, 3>{}, E{}, 2); break;
        case 4: go(std::integral_constant<int, 4>{}, E{}, 2); break;
        case 5: go(std::integral_constant<int, 5>{}, E{}, 2); break;
        case 6: go(std::integral_constant<int, 6>{}, E{}, 2); break;
        case 7: go(std::integral_constant<int, 7>{}, E{}, 2); break;
        default: go(std::integral_constant<int, 8>{}, E{}, 1); break;
    }
    return hipGetLastError();
}

// --------------------------------------------------------------------------
// Hot-shape kernels (block width s <= 8, projection block w <= 9).
//
// k_tilegram: G = T^T T for a tile T of <= 16 columns (one v_mfma_f64_16x16x4
// per 4 rows, A and B the same register: no padding MFMAs) plus E^T T for
// up to one extra column E (VALU).  Lane layout as k_gram.
// Partials (entry-major): [0,256) tile Gram (col-major 16x16), [256,272)
// E^T T.
// --------------------------------------------------------------------------
template <int RUN>
__global__ __launch_bounds__(256) void k_tilegram(Panel T, const double* __restrict__ E, int64_t n,
                                                  double* __restrict__ partial) {
    __shared__ double red[3][64][5];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int c16 = lane & 15, g = lane >> 4;
    const bool on = c16 < T.total;
    const double* tc = pcol(T, on ? c16 : 0);
    const bool eon = E != nullptr;
    const double* ec = eon ? E : tc;
    d4 acc = d4{0.0, 0.0, 0.0, 0.0};
    double eacc = 0.0;
    const int64_t wstep = 4 * RUN;
    const int64_t stride = (int64_t)gridDim.x * 4 * wstep;
    for (int64_t r0 = ((int64_t)blockIdx.x * 4 + wave) * wstep; r0 < n; r0 += stride) {
        const int64_t rb = r0 + g * RUN;
        double av[RUN], ev[RUN];
        if (r0 + wstep <= n) {
#pragma unroll
            for (int m = 0; m < RUN; m += 2) {
                d2 x = *reinterpret_cast<const d2*>(tc + rb + m);
                d2 y = *reinterpret_cast<const d2*>(ec + rb + m);
                av[m] = on ? x[0] : 0.0;
                av[m + 1] = on ? x[1] : 0.0;
                ev[m] = eon ? y[0] : 0.0;
                ev[m + 1] = eon ? y[1] : 0.0;
            }
        } else {
#pragma unroll
            for (int m = 0; m < RUN; ++m) {
                const bool in = rb + m < n;
                const int64_t rr = in ? rb + m : 0;
                const double x = tc[rr], y = ec[rr];
                av[m] = (on && in) ? x : 0.0;
                ev[m] = (eon && in) ? y : 0.0;
            }
        }
#pragma unroll
        for (int m = 0; m < RUN; ++m) {
            acc = mfma64(av[m], av[m], acc);
            eacc = eacc + ev[m] * av[m];
        }
    }
    if (wave > 0) {
#pragma unroll
        for (int r = 0; r < 4; ++r) red[wave - 1][lane][r] = acc[r];
        red[wave - 1][lane][4] = eacc;
    }
    __syncthreads();
    if (wave == 0) {
        const int64_t nb = gridDim.x;
        double* out = partial + blockIdx.x;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            double v = acc[r];
            v = v + red[0][lane][r];
            v = v + red[1][lane][r];
            v = v + red[2][lane][r];
            const int i = g + 4 * r, j = c16;
            out[(int64_t)(j * 16 + i) * nb] = v;
        }
        // E^T T: reduce the four row groups g of column c16 in a fixed order
        double e = eacc;
        e = e + red[0][lane][4];
        e = e + red[1][lane][4];
        e = e + red[2][lane][4];
        const double e1 = __shfl(e, c16 + 16, 64), e2 = __shfl(e, c16 + 32, 64), e3 = __shfl(e, c16 + 48, 64);
        if (g == 0) out[(int64_t)(256 + c16) * nb] = ((e + e1) + e2) + e3;
    }
}

hipError_t launch_tilegram(const Panel& T, const double* E, int64_t n, int blocks, double* partial,
                           hipStream_t st) {
    hipLaunchKernelGGL((k_tilegram<16>), dim3(blocks), dim3(256), 0, st, T, E, n, partial);
    return hipGetLastError();
}

// k_rowapply: lane <-> row.  Y = P * M with P of wp <= WPMAX columns and
// M zero-padded to WPMAX x MOUT (row-major), staged in LDS and read as
// broadcasts (scalar loads of M measured 9 us faster for pass A alone but
// slower for pass B, and no different in the loop).  Every column load is a
// contiguous 512-B wave access; padded columns reload a valid column (cache
// hit) times zero.
// GRAM: the stored rows [Qp(0:nq) | Y(0:m)] (nq = min(wq, 8)) are
// transposed through LDS into one 16-column tile and accumulated with
// v_mfma_f64_16x16x4 (tile^T tile); Qp column 8 (if wq == 9) is the extra
// column.  Partials as k_tilegram.
// APPLY = false: Gram only (no M, no store): tile = P columns 0..m-1, extra
// column = P column 16 when wq > 0 (the row-parallel form of k_tilegram).
// STORE = false: the Grams of Y without writing Y (pass A of two_pass).
// CHAIN: Y2 = [P(0:wq) | Y] * M2 with Y = P * M1 recomputed bit-identically
// in registers (pass B of two_pass without a stored intermediate block);
// M = [M1 (WPMAX x MOUT) | M2p (WPMAX x MOUT, rows >= wq zero) | M2y (MOUT x MOUT)].
// LDS hand-off inside one wave: the wave's LDS operations retire in order;
// the fences keep the compiler from moving LDS accesses across.
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// gate (CHAIN only, may be null): the coefficient step's two failure flags
// (k_orth_coef out[512..513]); when either is set the sweep stores nothing.
// A failed Cholesky leaves M1 or M2 unwritten (stale scratch) and the host
// redoes the block from its input -- which, in ca_lanczos's first block, is
// the same storage as the output (q = Q(:,1)).
template <int WPMAX, int MOUT, bool GRAM, bool APPLY = true, bool STORE = true, bool CHAIN = false, bool NTS = false>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) void k_rowapply(ColList P, const double* __restrict__ M, int wp, int m,
                                                  OutList Y, int wq, int64_t n, double* __restrict__ partial,
                                                  const double* __restrict__ gate) {
    if (CHAIN && gate && (gate[0] != 0.0 || gate[1] != 0.0)) return;  // block-uniform
    constexpr int TLD = 17;  // padded LDS row (doubles)
    constexpr int MSZ = WPMAX * MOUT * (CHAIN ? 2 : 1) + (CHAIN ? MOUT * MOUT : 0);
    // tile: 256 rows x 16 Gram columns, the pad column 16 holds the extra
    // column; after the row loop the same LDS holds the cross-wave partials
    // (38 KB per block -> 4 blocks per CU)
    __shared__ double tile[GRAM ? 256 * TLD : 1];
    double* const red = tile;
    __shared__ __attribute__((aligned(16))) double Ms[MSZ];  // broadcast reads
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int c16 = lane & 15, g = lane >> 4;
    const int nq = wq < 8 ? wq : 8;
    const bool has_ext = wq > 8;
    if (APPLY)
        for (int e = tid; e < MSZ; e += 256) Ms[e] = M[e];
    if (GRAM)
        for (int e = tid; e < 256 * TLD; e += 256) tile[e] = 0.0;
    __syncthreads();
    d4 acc = d4{0.0, 0.0, 0.0, 0.0};
    double eacc = 0.0;
    // (host pads P.p[c >= wp] with a valid column and Y.p[j >= m] unused)
    const double* const* pc = P.p;
    double* const* yc = Y.p;
    // without the Gram one row per thread and no loop (nothing for the
    // compiler to hoist the M broadcasts out of); with it a grid-stride loop
    // whose LDS reads are pinned inside the iteration by a compiler barrier.
    // Gram kinds: each wave transposes only its own 64 rows through the tile,
    // so wave-level syncs suffice, and the next iteration's rows are loaded
    // before this iteration's MFMA phase.
    const int64_t nch = (n + 255) / 256;
    const int64_t cstride = GRAM ? (int64_t)gridDim.x : nch;
    auto chunk_base = [&](int64_t ci) { return ci * 256; };
    double pn[WPMAX];
    auto load_rows = [&](int64_t b, double* dst) {
        const int64_t r = b + tid;
        const int64_t rr = r < n ? r : n - 1;
#pragma unroll
        for (int c = 0; c < WPMAX; ++c) dst[c] = pc[c][rr];
    };
    load_rows(chunk_base(blockIdx.x), pn);
    for (int64_t ci = blockIdx.x; ci < nch; ci += cstride) {
        asm volatile("" ::: "memory");
        const int64_t base = chunk_base(ci);
        const int64_t r = base + tid;
        const bool in = r < n;
        double p[WPMAX];
#pragma unroll
        for (int c = 0; c < WPMAX; ++c) p[c] = in ? pn[c] : 0.0;
        if (GRAM && ci + cstride < nch) load_rows(chunk_base(ci + cstride), pn);
        double y[MOUT];
#pragma unroll
        for (int j = 0; j < MOUT; ++j) y[j] = 0.0;
#pragma unroll
        for (int c = 0; c < (APPLY ? WPMAX : 0); ++c) {
            // one M row per column, read right before use: the barrier takes
            // the accumulators as operands, so column c's FMAs retire before
            // column c+1's broadcasts issue (otherwise the scheduler keeps all
            // WPMAX*MOUT M values live and spills)
#pragma unroll
            for (int j = 0; j < MOUT; ++j) asm volatile("" : "+v"(y[j])::"memory");
            double mrow[MOUT];
#pragma unroll
            for (int j = 0; j < MOUT; j += 2) {
                const d2 t = *reinterpret_cast<const d2*>(&Ms[c * MOUT + j]);
                mrow[j] = t[0];
                if (j + 1 < MOUT) mrow[j + 1] = t[1];
            }
#pragma unroll
            for (int j = 0; j < MOUT; ++j) y[j] = __builtin_fma(p[c], mrow[j], y[j]);
        }
        if (CHAIN) {
            // y2 = P(0:wq) * M2p + y * M2y  (same pinning as above)
            const double* M2p = Ms + WPMAX * MOUT;
            const double* M2y = Ms + 2 * WPMAX * MOUT;
            double y2[MOUT];
#pragma unroll
            for (int j = 0; j < MOUT; ++j) y2[j] = 0.0;
#pragma unroll
            for (int c = 0; c < WPMAX + MOUT; ++c) {
#pragma unroll
                for (int j = 0; j < MOUT; ++j) asm volatile("" : "+v"(y2[j])::"memory");
                const double src = c < WPMAX ? p[c < WPMAX ? c : 0] : y[c >= WPMAX ? c - WPMAX : 0];
                const double* row = c < WPMAX ? M2p + c * MOUT : M2y + (c - WPMAX) * MOUT;
                double mrow[MOUT];
#pragma unroll
                for (int j = 0; j < MOUT; j += 2) {
                    const d2 t = *reinterpret_cast<const d2*>(&row[j]);
                    mrow[j] = t[0];
                    if (j + 1 < MOUT) mrow[j + 1] = t[1];
                }
#pragma unroll
                for (int j = 0; j < MOUT; ++j) y2[j] = __builtin_fma(src, mrow[j], y2[j]);
            }
#pragma unroll
            for (int j = 0; j < MOUT; ++j) y[j] = y2[j];
        }
        if (APPLY && STORE && in) {
#pragma unroll
            for (int j = 0; j < MOUT; ++j) {
                if (j < m) {
                    if constexpr (NTS) __builtin_nontemporal_store(y[j], &yc[j][r]);
                    else yc[j][r] = y[j];
                }
            }
        }
        if (GRAM) {
            double* trow = tile + tid * TLD;
            if (APPLY) {
#pragma unroll
                for (int c = 0; c < 8; ++c)
                    if (c < nq) trow[c] = p[c < WPMAX ? c : 0];
#pragma unroll
                for (int j = 0; j < MOUT; ++j)
                    if (j < m) trow[nq + j] = y[j];
                trow[16] = has_ext ? p[8 < WPMAX ? 8 : 0] : 0.0;
            } else {  // Gram only: tile = P columns 0..m-1, extra = column 16
#pragma unroll
                for (int c = 0; c < 16; ++c)
                    if (c < m) trow[c] = p[c < WPMAX ? c : 0];
                trow[16] = wq > 0 ? p[16 < WPMAX ? 16 : 0] : 0.0;
            }
            wave_lds_sync();
#pragma unroll
            for (int k = 0; k < 16; ++k) {
                const int row = wave * 64 + 4 * k + g;
                const double a = tile[row * TLD + c16];
                acc = mfma64(a, a, acc);
                eacc = eacc + tile[row * TLD + 16] * a;
            }
            wave_lds_sync();
        }
    }
    if (GRAM) __syncthreads();  // the partials below reuse the tile across waves
    if (GRAM) {
        if (wave > 0) {
#pragma unroll
            for (int r = 0; r < 4; ++r) red[((wave - 1) * 64 + lane) * 5 + r] = acc[r];
            red[((wave - 1) * 64 + lane) * 5 + 4] = eacc;
        }
        __syncthreads();
        if (wave == 0) {
            const int64_t nb = gridDim.x;
            double* out = partial + blockIdx.x;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                double v = acc[r];
                v = v + red[(0 * 64 + lane) * 5 + r];
                v = v + red[(1 * 64 + lane) * 5 + r];
                v = v + red[(2 * 64 + lane) * 5 + r];
                out[(int64_t)(c16 * 16 + g + 4 * r) * nb] = v;
            }
            double e = eacc;
            e = e + red[(0 * 64 + lane) * 5 + 4];
            e = e + red[(1 * 64 + lane) * 5 + 4];
            e = e + red[(2 * 64 + lane) * 5 + 4];
            const double e1 = __shfl(e, c16 + 16, 64), e2 = __shfl(e, c16 + 32, 64), e3 = __shfl(e, c16 + 48, 64);
            if (g == 0) out[(int64_t)(256 + c16) * nb] = ((e + e1) + e2) + e3;
        }
    }
}

int rowapply_wpmax(int wp) { return wp <= 5 ? 5 : (wp <= 9 ? 9 : (wp <= 17 ? 17 : 0)); }
int rowapply_mout(int m) { return m <= 4 ? 4 : (m <= 8 ? 8 : (m <= 16 ? 16 : 0)); }

// kind: 0 store only, 1 store + Gram, 2 Gram without store (pass A),
// 3 chained store (pass B).  Instantiated for the shapes of s = 4 and s = 8
// ('full' with s = 4 reaches 10..17 projection columns with 4 outputs).
hipError_t launch_rowapply(const ColList& P, const double* dM, int wp, int m, const OutList& Y, int kind, int wq,
                           int64_t n, int blocks, double* partial, hipStream_t st, const double* gate) {
    const int WP = rowapply_wpmax(wp), MO = rowapply_mout(m);
    dim3 g(blocks), b(256);
    // pass B's block Q is read again only after the next step's matrix powers
    // have streamed through the Infinity Cache (256 MB): when the sweep's
    // columns do not fit it, Q is stored non-temporally, so its lines are not
    // written back out of the cache during the powers (lap3d_215, same-box
    // A/Bs: 817/818 -> 828/829 and 847/847/846 -> 855/854/855 outer-it/s,
    // profiles/r04/passb_nt/)
    const bool nts = (int64_t)n * 8 * (wp + m) > ((int64_t)256 << 20);
#define CAL_RA(W, MM, G, S, C) \
    hipLaunchKernelGGL((k_rowapply<W, MM, G, true, S, C>), g, b, 0, st, P, dM, wp, m, Y, wq, n, partial, gate)
#define CAL_RA_NT(W, MM) \
    hipLaunchKernelGGL((k_rowapply<W, MM, false, true, true, true, true>), g, b, 0, st, P, dM, wp, m, Y, wq, n, partial, \
                       gate)
#define CAL_RA_SHAPE(W, MM)                                  \
    case W * 100 + MM:                                       \
        switch (kind) {                                      \
            case 0: CAL_RA(W, MM, false, true, false); break; \
            case 1: CAL_RA(W, MM, true, true, false); break;  \
            case 2: CAL_RA(W, MM, true, false, false); break; \
            default:                                         \
                if (nts) CAL_RA_NT(W, MM);                   \
                else CAL_RA(W, MM, false, true, true);       \
                break;                                       \
        }                                                    \
        break;
    switch (WP * 100 + MO) {
        CAL_RA_SHAPE(5, 4)
        CAL_RA_SHAPE(5, 8)
        CAL_RA_SHAPE(9, 4)
        CAL_RA_SHAPE(9, 8)
        CAL_RA_SHAPE(9, 16)
        CAL_RA_SHAPE(17, 4)
        CAL_RA_SHAPE(17, 8)
        case 1716:
            if (kind != 0) return hipErrorInvalidValue;
            CAL_RA(17, 16, false, true, false);
            break;
        default: return hipErrorInvalidValue;
    }
#undef CAL_RA_SHAPE
#undef CAL_RA_NT
#undef CAL_RA
    return hipGetLastError();
}

// k_passb_wide: pass B of the s = 8 block orthogonalisation (k_rowapply<17,
// 8, CHAIN>: the same FMA sequence, so the same Q bits) fused with the Gram
// the 'full' orthogonalisation needs next (ca_lanczos.m:197:
// projectAndNormalize({Q(:,1:(k-1)s+1)}, Q_new)): G = A' Q_new with
// A = [Qp (9) | Q_new (8) | Qold (wold)] -- the block's own columns from
// registers, only Qold = Q(:,1:(k-2)s) loaded -- so the wide Gram sweep no
// longer re-reads Qp and Q_new.  One row per lane, grid-stride; per 64-row
// wave group the 16-column A groups go through the wave's LDS rows onto
// v_mfma_f64_16x16x4f64 with B = Q_new (columns 8..15 zero), the next
// group's Qold loads in flight during the current group's MFMAs.  Partials
// entry-major: entry j (16 NTW) + a (a = A column, j < 8) of block b at
// partial[entry * nblocks + b]; entries a >= 17 + wold are padding.  gate: as
// k_rowapply's.
template <int NTW, bool NTS>
__global__ __launch_bounds__(256) void k_passb_wide(ColList P, const double* __restrict__ M, OutList Y,
                                                    const double* __restrict__ qold, int64_t ldq, int wold,
                                                    int64_t n, double* __restrict__ partial,
                                                    const double* __restrict__ gate) {
    constexpr int WPMAX = 17, MOUT = 8, WQ = 9;
    constexpr int MSZ = WPMAX * MOUT * 2 + MOUT * MOUT;
    constexpr int TLD = 17;
    constexpr int WTILE = 64 * TLD;  // a wave's rows: Q_new (for B), then each A group
    constexpr int RT = 4;            // tiles per step of the cross-wave reduction (3 x RT x 256 <= 4 WTILE)
    constexpr int LDSZ = 4 * WTILE;  // 35 KB: four blocks per CU
    if (gate && (gate[0] != 0.0 || gate[1] != 0.0)) return;  // block-uniform
    __shared__ __attribute__((aligned(16))) double Ms[MSZ];
    __shared__ double lds[LDSZ];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, c16 = lane & 15, g = lane >> 4;
    for (int e = tid; e < MSZ; e += 256) Ms[e] = M[e];
    __syncthreads();
    double* const tw = lds + wave * WTILE;
    d4 acc[NTW];
#pragma unroll
    for (int t = 0; t < NTW; ++t) acc[t] = d4{0.0, 0.0, 0.0, 0.0};
    const double* const* pc = P.p;
    double* const* yc = Y.p;
    const int64_t nch = (n + 255) / 256;
    for (int64_t ci = blockIdx.x; ci < nch; ci += gridDim.x) {
        asm volatile("" ::: "memory");
        const int64_t r = ci * 256 + tid;
        const bool in = r < n;
        const int64_t rr = in ? r : n - 1;
        double p[WPMAX];
#pragma unroll
        for (int c = 0; c < WPMAX; ++c) p[c] = pc[c][rr];
#pragma unroll
        for (int c = 0; c < WPMAX; ++c) p[c] = in ? p[c] : 0.0;
        // Q1 = P M1, then Q_new = [P(0:9) | Q1] [M2p; M2y] (k_rowapply CHAIN)
        double y[MOUT];
#pragma unroll
        for (int j = 0; j < MOUT; ++j) y[j] = 0.0;
#pragma unroll
        for (int c = 0; c < WPMAX; ++c) {
#pragma unroll
            for (int j = 0; j < MOUT; ++j) asm volatile("" : "+v"(y[j])::"memory");
            double mrow[MOUT];
#pragma unroll
            for (int j = 0; j < MOUT; j += 2) {
                const d2 t = *reinterpret_cast<const d2*>(&Ms[c * MOUT + j]);
                mrow[j] = t[0];
                mrow[j + 1] = t[1];
            }
#pragma unroll
            for (int j = 0; j < MOUT; ++j) y[j] = __builtin_fma(p[c], mrow[j], y[j]);
        }
        {
            const double* M2p = Ms + WPMAX * MOUT;
            const double* M2y = Ms + 2 * WPMAX * MOUT;
            double y2[MOUT];
#pragma unroll
            for (int j = 0; j < MOUT; ++j) y2[j] = 0.0;
#pragma unroll
            for (int c = 0; c < WPMAX + MOUT; ++c) {
#pragma unroll
                for (int j = 0; j < MOUT; ++j) asm volatile("" : "+v"(y2[j])::"memory");
                const double src = c < WPMAX ? p[c < WPMAX ? c : 0] : y[c >= WPMAX ? c - WPMAX : 0];
                const double* row = c < WPMAX ? M2p + c * MOUT : M2y + (c - WPMAX) * MOUT;
                double mrow[MOUT];
#pragma unroll
                for (int j = 0; j < MOUT; j += 2) {
                    const d2 t = *reinterpret_cast<const d2*>(&row[j]);
                    mrow[j] = t[0];
                    mrow[j + 1] = t[1];
                }
#pragma unroll
                for (int j = 0; j < MOUT; ++j) y2[j] = __builtin_fma(src, mrow[j], y2[j]);
            }
#pragma unroll
            for (int j = 0; j < MOUT; ++j) y[j] = y2[j];
        }
        if (in) {
#pragma unroll
            for (int j = 0; j < MOUT; ++j) {
                if constexpr (NTS) __builtin_nontemporal_store(y[j], &yc[j][r]);
                else yc[j][r] = y[j];
            }
        }
        // the Gram: Q_new rows (B) through the wave's rows, then the A groups
        // [Qp | Q_new | Qold] through the same rows
#pragma unroll
        for (int j = 0; j < MOUT; ++j) tw[lane * TLD + j] = y[j];
        double nxt[16];  // the next group's Qold values (two groups ahead measured slower: registers)
        // unconditional loads of a valid row and a valid column, no select: a
        // load under a condition became a branch per load, and a select right
        // after the load a full vmcnt wait per load.  Rows past n have Q_new =
        // 0, so their (finite) A values add nothing; the padding columns past
        // Qold (clamped to its last column) give Gram entries a >= 17 + wold,
        // which no caller reads.
        auto load_old = [&](int t) {
#pragma unroll
            for (int c = 0; c < 16; ++c) {
                const int k = 16 * t + c - (WQ + MOUT);  // Qold column (wave-uniform)
                const int kc = k < 0 ? 0 : (k < wold ? k : wold - 1);
                nxt[c] = qold[(int64_t)kc * ldq + rr];
            }
        };
        load_old(1);
        wave_lds_sync();
        double bv[16];
#pragma unroll
        for (int kk = 0; kk < 16; ++kk) bv[kk] = c16 < MOUT ? tw[(4 * kk + g) * TLD + c16] : 0.0;
        wave_lds_sync();
#pragma unroll
        for (int t = 0; t < NTW; ++t) {
            // group t into the wave's rows first, then group t + 1's loads into
            // the registers group t just left (loading first made the compiler
            // wait for every load before reusing its register)
            if (t == 0) {  // [Qp (9) | Q_new (0:7)]
#pragma unroll
                for (int c = 0; c < 16; ++c) tw[lane * TLD + c] = c < WQ ? p[c < WQ ? c : 0] : y[c >= WQ ? c - WQ : 0];
            } else {
#pragma unroll
                for (int c = 0; c < 16; ++c) tw[lane * TLD + c] = (t == 1 && c == 0) ? y[7] : nxt[c];  // col 16 = Q_new(:, 7)
                if (t + 1 < NTW) load_old(t + 1);
            }
            wave_lds_sync();
#pragma unroll
            for (int kk = 0; kk < 16; ++kk) acc[t] = mfma64(tw[(4 * kk + g) * TLD + c16], bv[kk], acc[t]);
            wave_lds_sync();
        }
    }
    // the block's partials, RT tiles at a time through the tiles' LDS
    auto red = reinterpret_cast<double (*)[RT][64][4]>(lds);  // [3][RT][64][4]
    const int64_t nb = gridDim.x;
    double* out = partial + blockIdx.x;
#pragma unroll
    for (int t0 = 0; t0 < NTW; t0 += RT) {
        __syncthreads();  // the tiles (or the previous step's partials) are read
        if (wave > 0) {
#pragma unroll
            for (int t = t0; t < (t0 + RT < NTW ? t0 + RT : NTW); ++t)
#pragma unroll
                for (int q = 0; q < 4; ++q) red[wave - 1][t - t0][lane][q] = acc[t][q];
        }
        __syncthreads();
        if (wave == 0 && c16 < MOUT) {
#pragma unroll
            for (int t = t0; t < (t0 + RT < NTW ? t0 + RT : NTW); ++t)
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    double v = acc[t][q];
                    v = v + red[0][t - t0][lane][q];
                    v = v + red[1][t - t0][lane][q];
                    v = v + red[2][t - t0][lane][q];
                    const int a = 16 * t + g + 4 * q, j = c16;
                    out[(int64_t)(j * 16 * NTW + a) * nb] = v;
                }
        }
    }
}

int passb_wide_tiles(int wold) { return (9 + 8 + wold + 15) / 16; }

hipError_t launch_passb_wide(const ColList& P, const double* dM, const OutList& Y, const Panel& Qold, int64_t n,
                             int blocks, double* partial, const double* gate, hipStream_t st) {
    if (Qold.total > 0 && Qold.nseg != 1) return hipErrorInvalidValue;  // one column block (Q(:,1:(k-2)s))
    const int ntw = passb_wide_tiles(Qold.total);
    // (no Qold: column 0 of P stands in; only padding columns read it)
    const double* qold = Qold.total > 0 ? Qold.ptr[0] : P.p[0];
    const int64_t ldq = Qold.total > 0 ? Qold.ld[0] : 0;
    const int wold = Qold.total;
    const bool nts = (int64_t)n * 8 * (17 + 8) > ((int64_t)256 << 20);  // as launch_rowapply's pass B
    dim3 g(blocks), b(256);
#define CAL_PBW(T)                                                                                              \
    case T:                                                                                                     \
        if (nts) hipLaunchKernelGGL((k_passb_wide<T, true>), g, b, 0, st, P, dM, Y, qold, ldq, wold, n, partial, \
                                    gate);                                                                      \
        else hipLaunchKernelGGL((k_passb_wide<T, false>), g, b, 0, st, P, dM, Y, qold, ldq, wold, n, partial, \
                                gate);                                                                          \
        break;
    switch (ntw) {
        CAL_PBW(2)
        CAL_PBW(3)
        CAL_PBW(4)
        CAL_PBW(5)
        CAL_PBW(6)
        CAL_PBW(7)
        CAL_PBW(8)
        CAL_PBW(9)
        CAL_PBW(10)
        CAL_PBW(11)
        CAL_PBW(12)
        default: return hipErrorInvalidValue;
    }
#undef CAL_PBW
    return hipGetLastError();
}

// Row-parallel tile Gram: tile = P.p[0..nt) (nt <= 16), extra = P.p[16] if
// has_extra.  Same partial layout as k_tilegram.
hipError_t launch_rowgram(const ColList& P, int nt, bool has_extra, int64_t n, int blocks, double* partial,
                          hipStream_t st) {
    OutList none{};
    hipLaunchKernelGGL((k_rowapply<17, 4, true, false>), dim3(blocks), dim3(256), 0, st, P, nullptr, 17, nt, none,
                       has_extra ? 1 : 0, n, partial, nullptr);
    return hipGetLastError();
}

// --------------------------------------------------------------------------
// fixed-order partial reduction and small vector kernels
// --------------------------------------------------------------------------

// One block per entry: partials are entry-major (part[e*nparts + p]), so the
// 256 threads read one contiguous run; fixed-order strided sums, then a fixed
// butterfly and a fixed wave order -> bitwise reproducible.
__global__ __launch_bounds__(256) void k_reduce(const double* __restrict__ part, int nparts,
                                                double* __restrict__ out) {
    __shared__ double ws[4];
    const int64_t e = blockIdx.x;
    const double* p = part + e * nparts;
    double s = 0.0;
    for (int i = threadIdx.x; i < nparts; i += 256) s = s + p[i];
    s = wave_sum(s);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (lane == 0) ws[wave] = s;
    __syncthreads();
    if (threadIdx.x == 0) out[e] = ((ws[0] + ws[1]) + ws[2]) + ws[3];
}

hipError_t launch_reduce(const double* partial, int nparts, int64_t nent, double* out, hipStream_t st) {
    if (nent <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_reduce, dim3((unsigned)nent), dim3(256), 0, st, partial, nparts, out);
    return hipGetLastError();
}

__global__ __launch_bounds__(256) void k_dot(const double* __restrict__ x, const double* __restrict__ y,
                                             int64_t n, double* __restrict__ partial) {
    __shared__ double ws[4];
    double s = 0.0;
    const int64_t stride = (int64_t)gridDim.x * 256;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) s = s + x[i] * y[i];
    s = wave_sum(s);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (lane == 0) ws[wave] = s;
    __syncthreads();
    if (threadIdx.x == 0) partial[blockIdx.x] = ((ws[0] + ws[1]) + ws[2]) + ws[3];
}

int dot_blocks(int64_t n) {
    int64_t b = (n + 255) / 256;
    if (b > 1024) b = 1024;
    if (b < 1) b = 1;
    return (int)b;
}

hipError_t launch_dot(const double* x, const double* y, int64_t n, double* partial, int blocks,
                      hipStream_t st) {
    hipLaunchKernelGGL(k_dot, dim3(blocks), dim3(256), 0, st, x, y, n, partial);
    return hipGetLastError();
}

__global__ __launch_bounds__(256) void k_axpy_sub(double* __restrict__ y, const double* __restrict__ x, double a,
                                                  int64_t n) {
    const int64_t stride = (int64_t)gridDim.x * 256;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) {
        const double t = a * x[i];
        y[i] = y[i] - t;
    }
}

__global__ __launch_bounds__(256) void k_div(double* __restrict__ y, const double* __restrict__ x, double b,
                                             int64_t n) {
    const int64_t stride = (int64_t)gridDim.x * 256;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) y[i] = x[i] / b;
}

__global__ __launch_bounds__(256) void k_gather(double* __restrict__ dst, const double* __restrict__ src,
                                                const int* __restrict__ idx, int64_t cnt) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < cnt) dst[i] = src[idx[i]];
}

static unsigned vec_blocks(int64_t n) {
    int64_t b = (n + 255) / 256;
    if (b > 4096) b = 4096;
    if (b < 1) b = 1;
    return (unsigned)b;
}

// Vector kernels whose every block first sums the previous dot's partials
// (k_nrm_div, k_pro_div: up to 2 x 1024 doubles per block): at most 1024
// blocks, so the partials are read 1024 times, not 4096.  The per-block sum
// and the elementwise update are unchanged: the same bits.
#ifndef CAL_REDVEC_BLOCKS
#define CAL_REDVEC_BLOCKS 1024
#endif
static unsigned redvec_blocks(int64_t n) {
    const unsigned b = vec_blocks(n);
    return b > CAL_REDVEC_BLOCKS ? CAL_REDVEC_BLOCKS : b;
}

hipError_t launch_axpy_sub(double* y, const double* x, double a, int64_t n, hipStream_t st) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_axpy_sub, dim3(vec_blocks(n)), dim3(256), 0, st, y, x, a, n);
    return hipGetLastError();
}

hipError_t launch_div(double* y, const double* x, double b, int64_t n, hipStream_t st) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_div, dim3(vec_blocks(n)), dim3(256), 0, st, y, x, b, n);
    return hipGetLastError();
}

hipError_t launch_gather(double* dst, const double* src, const int* idx, int64_t cnt, hipStream_t st) {
    if (cnt <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_gather, dim3((unsigned)((cnt + 255) / 256)), dim3(256), 0, st, dst, src, idx, cnt);
    return hipGetLastError();
}

// --------------------------------------------------------------------------
// Ritz residual (compute_ritz_rnorm, ca_lanczos.m:92-96) for one Ritz pair:
// x = xr + i xi, l = lr + i li; partial[2b] = sum |A x - l x|^2,
// partial[2b+1] = sum |l x|^2 over the rows of block b.
// --------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_spmv_resid(SpmvArgs a, const double* __restrict__ xi, double lr,
                                                    double li, int64_t nrows, double* __restrict__ partial) {
    __shared__ double ws[2][4];
    double s_num = 0.0, s_den = 0.0;
    const int64_t stride = (int64_t)gridDim.x * 256;
    for (int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x; r < nrows; r += stride) {
        double axr = 0.0, axi = 0.0;
        for (int j = a.rowptr[r]; j < a.rowptr[r + 1]; ++j) {
            const int c = a.col[j];
            axr = axr + a.val[j] * a.x[c];
            if (xi) axi = axi + a.val[j] * xi[c];
        }
        const double xr_ = a.x[r], xi_ = xi ? xi[r] : 0.0;
        const double lxr = lr * xr_ - li * xi_;
        const double lxi = lr * xi_ + li * xr_;
        const double er = axr - lxr, ei = axi - lxi;
        s_num = s_num + (er * er + ei * ei);
        s_den = s_den + (lxr * lxr + lxi * lxi);
    }
    s_num = wave_sum(s_num);
    s_den = wave_sum(s_den);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (lane == 0) {
        ws[0][wave] = s_num;
        ws[1][wave] = s_den;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        partial[blockIdx.x] = ((ws[0][0] + ws[0][1]) + ws[0][2]) + ws[0][3];
        partial[gridDim.x + blockIdx.x] = ((ws[1][0] + ws[1][1]) + ws[1][2]) + ws[1][3];
    }
}

hipError_t launch_spmv_resid(const SpmvArgs& a, const double* xi, double lr, double li, int64_t nrows,
                             double* partial, int blocks, hipStream_t st) {
    hipLaunchKernelGGL(k_spmv_resid, dim3(blocks), dim3(256), 0, st, a, xi, lr, li, nrows, partial);
    return hipGetLastError();
}

// --------------------------------------------------------------------------
// Block-orthogonalisation coefficients on the device (blockorth.cpp,
// orth_device).  The s x s algebra between the three sweeps of two_pass --
// Cholesky, triangular inverse, the coefficient blocks M1 / M2 and R, RY --
// runs in one 256-thread block right after the Gram reduction, so the sweeps
// are enqueued back to back without a host round trip.  Every quantity is
// computed with the same operation order as the host path in blockorth.cpp
// (right-looking Cholesky updates reproduce the left-looking host sums term
// for term; products and sums in the same sequence), so both paths give the
// same bits.
// --------------------------------------------------------------------------
// tools/coef_probe.hip builds with CAL_OC_PROF: clock64() marks per step
#ifdef CAL_OC_PROF
__device__ long long g_oc_marks[16];
#define OC_MARK(i)                                           \
    do {                                                     \
        __syncthreads();                                     \
        if (threadIdx.x == 0) g_oc_marks[i] = clock64();     \
    } while (0)
#else
#define OC_MARK(i) \
    do {           \
    } while (0)
#endif
namespace {
constexpr int kOcM = 16, kOcW = 9;
#ifndef CAL_OC_THREADS
#define CAL_OC_THREADS 256
#endif
constexpr int kOcThreads = CAL_OC_THREADS;  // >= kOcM * kOcM (oc_chol_inv8 clears R by thread)
constexpr int kOcOut = 516;   // R (<= 16 x 16) at 0, RY at 256, flags at 512

// Upper Cholesky of the m x m matrix in G (ld kOcM, destroyed) into R;
// returns false (block-uniform) on a non-positive or non-finite pivot.
__device__ bool oc_chol(int m, double* G, double* R, int* flag) {
    const int tid = threadIdx.x;
    for (int e = tid; e < kOcM * kOcM; e += blockDim.x) R[e] = 0.0;
    __syncthreads();
    for (int j = 0; j < m; ++j) {
        // G(j,j..m-1) already hold G - sum_{k<j} R(k,j) R(k,i) (host: chol_upper)
        if (tid == 0) {
            const double sj = G[j + j * kOcM];
            *flag = !(sj > 0.0) || !isfinite(sj);
            if (!*flag) R[j + j * kOcM] = sqrt(sj);
        }
        __syncthreads();
        if (*flag) return false;
        const double rjj = R[j + j * kOcM];
        for (int i = j + 1 + tid; i < m; i += blockDim.x) R[j + i * kOcM] = G[j + i * kOcM] / rjj;
        __syncthreads();
        // trailing update of rows/cols > j, one (r, i) entry per thread
        for (int e = tid; e < m * m; e += blockDim.x) {
            const int r = e % m, i = e / m;
            if (r > j && i >= r) {
                const double t = R[j + r * kOcM] * R[j + i * kOcM];
                G[r + i * kOcM] = G[r + i * kOcM] - t;
            }
        }
        __syncthreads();
    }
    return true;
}

// Ri = R^-1 (upper), column j by lane j with the host's back substitution
// (s = [i == j] - sum_{k=i+1..j} R(i,k) Ri(k,j), ascending k; Ri(i,j) = s /
// R(i,i)).  The lane's own column stays in registers; i descends in lockstep
// over all lanes, so the R(i,k) reads are LDS broadcasts.
__device__ void oc_trinv(int m, const double* R, double* Ri) {
    const int tid = threadIdx.x;
    if (tid < kOcM) {
        const int j = tid;
        double col[kOcM];
#pragma unroll
        for (int i = kOcM - 1; i >= 0; --i) {
            double s = (i == j) ? 1.0 : 0.0;
#pragma unroll
            for (int k = i + 1; k < kOcM; ++k) {
                const double t = R[i + k * kOcM] * col[k];
                const double u = s - t;
                s = k <= j ? u : s;
            }
            const double v = s / R[i + i * kOcM];
            col[i] = (i <= j && j < m && i < m) ? v : 0.0;
        }
#pragma unroll
        for (int i = 0; i < kOcM; ++i) Ri[i + j * kOcM] = col[i];
    }
    __syncthreads();
}

// m <= 8: Cholesky and inverse in wave 0 with the matrix in registers, lane
// l = r + 8c holding entry (r, c); same operations, in the same order, as
// oc_chol / oc_trinv (and dense::chol_upper / tri_inv_upper on the host):
//   R(j,j) = sqrt(G(j,j)), R(j,c) = G(j,c) / R(j,j),
//   G(r,c) -= R(j,r) * R(j,c) for j < r <= c (ascending j),
//   Ri(i,j) = ([i == j] - sum_{k=i+1..j} R(i,k) Ri(k,j)) / R(i,i).
// R and Ri are written to LDS (ld kOcM); returns false (block-uniform) on a
// non-positive or non-finite pivot.  Called by all threads of the block.
__device__ bool oc_chol_inv8(int m, const double* G, double* R, double* Ri, int* flag) {
    const int tid = threadIdx.x;
    if (tid < 64) {
        const int r = tid & 7, c = tid >> 3;
        double g = (r < m && c < m) ? G[r + c * kOcM] : 0.0;
        double rv = 0.0;  // R(r, c) once row r is final
        int bad = 0;
        for (int j = 0; j < m; ++j) {
            const double sj = __shfl(g, j + 8 * j, 64);
            if (!(sj > 0.0) || !isfinite(sj)) {
                bad = 1;
                break;
            }
            const double rjj = sqrt(sj);
            if (r == j) rv = c == j ? rjj : (c > j && c < m ? g / rjj : 0.0);
            const double rjr = __shfl(rv, j + 8 * r, 64);  // R(j, r)
            const double rjc = __shfl(rv, j + 8 * c, 64);  // R(j, c)
            if (r > j && c >= r) {
                const double t = rjr * rjc;
                g = g - t;
            }
        }
        R[r + c * kOcM] = (r <= c && r < m && c < m) ? rv : 0.0;
        if (tid == 0) *flag = bad;
    }
    __syncthreads();
    if (*flag) return false;
    if (tid < 8) {
        const int j = tid;
        double col[8];
#pragma unroll
        for (int i = 7; i >= 0; --i) {
            double s = (i == j) ? 1.0 : 0.0;
#pragma unroll
            for (int k = i + 1; k < 8; ++k) {
                const double t = R[i + k * kOcM] * col[k];
                const double u = s - t;
                s = k <= j ? u : s;
            }
            const double v = s / R[i + i * kOcM];
            col[i] = (i <= j && j < m && i < m) ? v : 0.0;
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) Ri[i + j * kOcM] = col[i];
#pragma unroll
        for (int i = 8; i < kOcM; ++i) Ri[i + j * kOcM] = 0.0;
    } else if (tid < kOcM) {
#pragma unroll
        for (int i = 0; i < kOcM; ++i) Ri[i + tid * kOcM] = 0.0;
    }
    if (tid < kOcM * kOcM && (tid & 15) >= 8) R[tid] = 0.0;  // rows 8.. of R (columns < 16)
    if (tid < kOcM * kOcM && (tid >> 4) >= 8) R[tid] = 0.0;
    __syncthreads();
    return true;
}
}  // namespace

// PHASE 0 (after the P1 Gram of [Qp(0:nq) | X] (+ Qp column 8)):
//   C = Qp'X, Y'Y = X'X - C'C, the reorth flag of projectAndNormalize.m:52,
//   Ra = chol(Y'Y), M1 = [-C; I] Ra^-1 -> row-kernel layout in mbuf[0 : WP*MO).
// PHASE 1 (after pass A's Grams of Q1):
//   Rb = chol(Q1'Q1 - C3'C3), M2 = [-C3 Rb^-1; Rb^-1] -> mbuf chain part,
//   R = Rb Ra, RY = C + C3 Ra -> out.
// st: C (kOcW x kOcM, ld w) at 0, Ra at 256.  out: R (m x m) at 0, RY
// (w x m) at 256, flags at 512: [0] phase-0 failure, [1] phase-1 failure,
// [2] reorth.
template <int PHASE>
__device__ void orth_coef_body(const double* __restrict__ tile, double* __restrict__ st, double* __restrict__ mbuf,
                               double* __restrict__ out, int w, int m, int WP, int MO, int doreorth) {
    __shared__ double G[kOcM * kOcM], R[kOcM * kOcM], Ri[kOcM * kOcM], C[kOcW * kOcM], Ra[kOcM * kOcM];
    __shared__ double C0[PHASE == 1 ? kOcW * kOcM : 1];  // phase 1: phase 0's C (from st)
    __shared__ double nb[kOcM];
    __shared__ int flag;
    const int tid = threadIdx.x, nq = w < 8 ? w : 8, wp = w + m;
    OC_MARK(0);
    // unpack the tile: G = block Gram (m x m), C = Qp' block (w x m)
    for (int e = tid; e < m * m; e += blockDim.x) {
        const int i = e % m, j = e / m;
        G[i + j * kOcM] = tile[(nq + i) + (nq + j) * 16];
    }
    for (int e = tid; e < w * m; e += blockDim.x) {
        const int i = e % w, j = e / w;
        C[e] = i < 8 ? tile[i + (nq + j) * 16] : tile[256 + nq + j];
    }
    if (PHASE == 1) {
        for (int e = tid; e < m * m; e += blockDim.x) Ra[e % m + (e / m) * kOcM] = st[256 + e];
        for (int e = tid; e < w * m; e += blockDim.x) C0[e] = st[e];
    }
    __syncthreads();
    OC_MARK(1);
    if (PHASE == 0 && tid < m) nb[tid] = sqrt(G[tid + tid * kOcM]);  // norms before (projectAndNormalize.m:17-22)
    // G -= C'C   (host: s = sum_k C(k,i) C(k,j); G(i,j) -= s)
    double upd[kOcM * kOcM / kOcThreads];
    for (int e = tid, q = 0; e < m * m; e += blockDim.x, ++q) {
        const int i = e % m, j = e / m;
        double s = 0.0;
        for (int k = 0; k < w; ++k) {
            const double t = C[k + i * w] * C[k + j * w];
            s = s + t;
        }
        upd[q] = G[i + j * kOcM] - s;
    }
    __syncthreads();
    for (int e = tid, q = 0; e < m * m; e += blockDim.x, ++q) G[e % m + (e / m) * kOcM] = upd[q];
    __syncthreads();
    OC_MARK(2);
    if (PHASE == 0) {
        // rel = |before - after| / before per column (lane i), then the
        // NaN-ignoring max in column order, reorth = max(rel) > 0.5
        if (tid < m) {
            const double after = sqrt(fmax(G[tid + tid * kOcM], 0.0));
            nb[tid] = fabs(nb[tid] - after) / nb[tid];
        }
        __syncthreads();
        if (tid == 0) {
            double mx = NAN;
            for (int i = 0; i < m; ++i) {
                const double rel = nb[i];
                if (!isnan(rel) && (isnan(mx) || rel > mx)) mx = rel;
            }
            out[512 + 2] = (doreorth && mx > 0.5) ? 1.0 : 0.0;
        }
    }
    const bool fast = m <= 8;
    const bool ok = fast ? oc_chol_inv8(m, G, R, Ri, &flag) : oc_chol(m, G, R, &flag);
    OC_MARK(3);
    if (tid == 0) out[512 + PHASE] = ok ? 0.0 : 1.0;
    if (!ok) return;  // block-uniform: the host redoes the block on its own path
    if (!fast) oc_trinv(m, R, Ri);
    OC_MARK(4);
    if (PHASE == 0) {
        // M1 = Mz Ri, Mz = [-C; I] (wp x m); host: dense::matmul, p = 0..m-1
        for (int e = tid; e < WP * MO; e += blockDim.x) {
            const int cc = e / MO, j = e % MO;
            double s = 0.0;
            if (cc < wp && j < m) {
                for (int p = 0; p < m; ++p) {
                    const double mz = cc < w ? -C[cc + p * w] : (cc - w == p ? 1.0 : 0.0);
                    const double t = mz * Ri[p + j * kOcM];
                    s = s + t;
                }
            }
            mbuf[e] = (cc < wp && j < m) ? s : 0.0;
        }
        for (int e = tid; e < w * m; e += blockDim.x) st[e] = C[e];
        for (int e = tid; e < m * m; e += blockDim.x) st[256 + e] = R[e % m + (e / m) * kOcM];
    } else {
        double* M2p = mbuf + WP * MO;
        double* M2y = M2p + WP * MO;
        // four independent products over one flattened index (all waves busy):
        //   M2p = -C3 Rb^-1 (WP x MO), M2y = Rb^-1 (MO x MO),
        //   RY = C + C3 Ra (w x m), R = Rb Ra (m x m, upper)
        const int n1 = WP * MO, n2 = n1 + MO * MO, n3 = n2 + w * m, n4 = n3 + m * m;
        for (int f = tid; f < n4; f += blockDim.x) {
            if (f < n1) {
                const int e = f, cc = e / MO, j = e % MO;
                double v = 0.0;
                if (cc < w && j < m) {
                    double s = 0.0;
                    for (int k = 0; k <= j; ++k) {
                        const double t = C[cc + k * w] * Ri[k + j * kOcM];
                        s = s + t;
                    }
                    v = -s;
                }
                M2p[e] = v;
            } else if (f < n2) {
                const int e = f - n1, i = e / MO, j = e % MO;
                M2y[e] = (i < m && j < m) ? Ri[i + j * kOcM] : 0.0;
            } else if (f < n3) {
                const int e = f - n2, i = e % w, j = e / w;
                double s = 0.0;
                for (int k = 0; k <= j; ++k) {
                    const double t = C[i + k * w] * Ra[k + j * kOcM];
                    s = s + t;
                }
                const double ctot = 0.0 + s;
                out[256 + e] = C0[e] + ctot;
            } else {
                const int e = f - n3, i = e % m, j = e / m;
                double s = 0.0;
                for (int p = 0; p < m; ++p) {
                    const double t = R[i + p * kOcM] * Ra[p + j * kOcM];
                    s = s + t;
                }
                out[e] = i > j ? 0.0 : s;
            }
        }
    }
    OC_MARK(5);
}

// Phase 1 publishes the block's results to pinned host memory: the 516
// doubles of out (R, RY, flags) are copied to hout, then the sequence number
// is stored with system-scope release semantics -- the host polls it
// (blockorth.cpp orth_device) instead of a device-to-host copy + event.
__device__ void orth_publish(const double* __restrict__ out, double* __restrict__ hout,
                             unsigned long long* __restrict__ hseq, unsigned long long seq) {
    __syncthreads();  // out was written by the whole block
    for (int e = threadIdx.x; e < kOcOut; e += blockDim.x) hout[e] = out[e];
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        __threadfence_system();
        __hip_atomic_store(hseq, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

template <int PHASE>
__global__ __launch_bounds__(kOcThreads) void k_orth_coef(const double* __restrict__ tile, double* __restrict__ st,
                                                   double* __restrict__ mbuf, double* __restrict__ out, int w, int m,
                                                   int WP, int MO, int doreorth, double* __restrict__ hout,
                                                   unsigned long long* __restrict__ hseq, unsigned long long seq) {
    orth_coef_body<PHASE>(tile, st, mbuf, out, w, m, WP, MO, doreorth);
    if (PHASE == 1 && hout) orth_publish(out, hout, hseq, seq);
}

hipError_t launch_orth_coef(int phase, const double* tile, double* st, double* mbuf, double* out, int w, int m,
                            int WP, int MO, int doreorth, double* hout, unsigned long long* hseq,
                            unsigned long long seq, hipStream_t stream) {
    if (m < 1 || m > kOcM || w < 0 || w > kOcW) return hipErrorInvalidValue;
    if (phase == 0)
        hipLaunchKernelGGL(k_orth_coef<0>, dim3(1), dim3(kOcThreads), 0, stream, tile, st, mbuf, out, w, m, WP, MO, doreorth,
                           hout, hseq, seq);
    else
        hipLaunchKernelGGL(k_orth_coef<1>, dim3(1), dim3(kOcThreads), 0, stream, tile, st, mbuf, out, w, m, WP, MO, doreorth,
                           hout, hseq, seq);
    return hipGetLastError();
}


// M = [-G(0:w, 0:m); I_m] ((w + m) x m, column-major) from a reduced Gram
// block G (ld ldg): the coefficients of X - Q R (project.m:30) formed on the
// device, the same values the host path stages (blockorth.cpp project_blocks).
__global__ __launch_bounds__(256) void k_form_projM(const double* __restrict__ G, int ldg, int w, int m,
                                                   double* __restrict__ M) {
    const int e = blockIdx.x * 256 + threadIdx.x, rows = w + m;
    if (e >= rows * m) return;
    const int r = e % rows, j = e / rows;
    M[e] = r < w ? -G[r + (int64_t)j * ldg] : (r - w == j ? 1.0 : 0.0);
}

hipError_t launch_form_projM(const double* G, int ldg, int w, int m, double* M, hipStream_t st) {
    const int cnt = (w + m) * m;
    if (cnt <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_form_projM, dim3((cnt + 255) / 256), dim3(256), 0, st, G, ldg, w, m, M);
    return hipGetLastError();
}

// y -= a * x with a = *pa (or sqrt(*pa)) still on the device: the Lanczos
// recurrence's alpha / beta updates without a host round trip (same ops as
// k_axpy_sub with the host's value)
__global__ __launch_bounds__(256) void k_axpy_sub_dev(double* __restrict__ y, const double* __restrict__ x,
                                                     const double* __restrict__ pa, int take_sqrt, int64_t n) {
    const double a = take_sqrt ? sqrt(*pa) : *pa;
    const int64_t stride = (int64_t)gridDim.x * 256;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) {
        const double t = a * x[i];
        y[i] = y[i] - t;
    }
}

// The Newton prologue's recurrence (lanczos.m:105-110) in three launches
// instead of seven, single rank: no reduce launches, each kernel sums the
// block partials of the dot before it itself (every block the same sum, in
// k_reduce's order; block 0 publishes it), so the bits are those of
// k_axpy_sub_dev / k_dot / k_reduce / k_div_sqrt:
//   k_pro_dot     y = y - sqrt(*pb) x (x may be null); partials of y'z
//   k_pro_update  a = sum(pin) -> dst; y = y - a x; partials of y'y
//   k_pro_div     b = sum(pin) -> dst; q = y / sqrt(b)
// The partial-producing kernels run on k_dot's grid (dot_blocks) with its
// per-thread order.  A kernel's own partials go to a buffer the next kernel
// reads, never the one it reads itself.
__device__ __forceinline__ double pro_block_sum(double s, double* ws) {
    s = wave_sum(s);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    __syncthreads();  // ws may still be read by a previous use
    if (lane == 0) ws[wave] = s;
    __syncthreads();
    return ((ws[0] + ws[1]) + ws[2]) + ws[3];
}
// k_reduce's sum of np partials, in every block
__device__ __forceinline__ double pro_reduce(const double* __restrict__ p, int np, double* ws) {
    double s = 0.0;
    for (int i = threadIdx.x; i < np; i += 256) s = s + p[i];
    return pro_block_sum(s, ws);
}
// y = y - a x (x non-null), then sum of y z (z null: y y), k_dot's order
__device__ __forceinline__ double pro_axpy_dot(double* __restrict__ y, const double* __restrict__ x, double a,
                                               const double* __restrict__ z, int64_t n) {
    const int64_t stride = (int64_t)gridDim.x * 256;
    double s = 0.0;
    int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    for (; i + stride < n; i += 2 * stride) {
        double y0 = y[i], y1 = y[i + stride];
        const double x0 = x ? x[i] : 0.0, x1 = x ? x[i + stride] : 0.0;
        const double z0 = z ? z[i] : 0.0, z1 = z ? z[i + stride] : 0.0;
        if (x) {
            const double t0 = a * x0, t1 = a * x1;
            y0 = y0 - t0;
            y1 = y1 - t1;
            y[i] = y0;
            y[i + stride] = y1;
        }
        s = s + y0 * (z ? z0 : y0);
        s = s + y1 * (z ? z1 : y1);
    }
    if (i < n) {
        double yi = y[i];
        const double zi = z ? z[i] : 0.0;
        if (x) {
            const double t = a * x[i];
            yi = yi - t;
            y[i] = yi;
        }
        s = s + yi * (z ? zi : yi);
    }
    return s;
}

__global__ __launch_bounds__(256) void k_pro_dot(double* __restrict__ y, const double* __restrict__ x,
                                                 const double* __restrict__ pb, const double* __restrict__ z,
                                                 int64_t n, double* __restrict__ pout) {
    __shared__ double ws[4];
    const double a = x ? sqrt(*pb) : 0.0;
    const double s = pro_block_sum(pro_axpy_dot(y, x, a, z, n), ws);
    if (threadIdx.x == 0) pout[blockIdx.x] = s;
}

__global__ __launch_bounds__(256) void k_pro_update(double* __restrict__ y, const double* __restrict__ x,
                                                    const double* __restrict__ pin, int np, double* __restrict__ dst,
                                                    int64_t n, double* __restrict__ pout) {
    __shared__ double ws[4];
    const double a = pro_reduce(pin, np, ws);
    if (blockIdx.x == 0 && threadIdx.x == 0) dst[0] = a;
    const double s = pro_block_sum(pro_axpy_dot(y, x, a, nullptr, n), ws);
    if (threadIdx.x == 0) pout[blockIdx.x] = s;
}

__global__ __launch_bounds__(256) void k_pro_div(double* __restrict__ q, const double* __restrict__ y,
                                                 const double* __restrict__ pin, int np, double* __restrict__ dst,
                                                 int64_t n) {
    __shared__ double ws[4];
    const double b = pro_reduce(pin, np, ws);
    if (blockIdx.x == 0 && threadIdx.x == 0) dst[0] = b;
    const double sb = sqrt(b);
    const int64_t stride = (int64_t)gridDim.x * 256;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) q[i] = y[i] / sb;
}

// normest's per-iteration norms (lanczos.cpp normest_dev), single rank: one
// launch for the partials of x'x and y'y (k_dot's grid and order for each),
// one that sums them in k_reduce's order (block 0 publishes both) and scales
// x by 1/sqrt(x'x) (k_div_sqrt's arithmetic) -- four launches fewer per
// iteration, the same bits.
__global__ __launch_bounds__(256) void k_norms2(const double* __restrict__ x, const double* __restrict__ y,
                                                int64_t n, double* __restrict__ px, double* __restrict__ py) {
    __shared__ double ws[4];
    const int64_t stride = (int64_t)gridDim.x * 256;
    double sx = 0.0, sy = 0.0;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) {
        const double a = x[i], b = y[i];
        sx = sx + a * a;
        sy = sy + b * b;
    }
    sx = pro_block_sum(sx, ws);
    sy = pro_block_sum(sy, ws);
    if (threadIdx.x == 0) {
        px[blockIdx.x] = sx;
        py[blockIdx.x] = sy;
    }
}

__global__ __launch_bounds__(256) void k_nrm_div(double* __restrict__ x, const double* __restrict__ px,
                                                 const double* __restrict__ py, int np, double* __restrict__ dst,
                                                 int64_t n) {
    __shared__ double ws[4];
    const double xx = pro_reduce(px, np, ws);
    const double yy = pro_reduce(py, np, ws);
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        dst[0] = xx;
        dst[1] = yy;
    }
    const double sx = sqrt(xx);
    const int64_t stride = (int64_t)gridDim.x * 256;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) x[i] = x[i] / sx;
}

__global__ __launch_bounds__(256) void k_nrm_pair(const double* __restrict__ px, const double* __restrict__ py, int np,
                                                  double* __restrict__ dst) {
    __shared__ double ws[4];
    const double xx = pro_reduce(px, np, ws);  // k_nrm_div's reduction
    const double yy = pro_reduce(py, np, ws);
    if (threadIdx.x == 0) {
        dst[0] = xx;
        dst[1] = yy;
    }
}

hipError_t launch_normest_norms_only(const double* x, const double* y, int64_t n, double* part, double* dst,
                                     hipStream_t st) {
    if (n <= 0) return hipErrorInvalidValue;
    const int nb = dot_blocks(n);
    hipLaunchKernelGGL(k_norms2, dim3(nb), dim3(256), 0, st, x, y, n, part, part + nb);
    hipLaunchKernelGGL(k_nrm_pair, dim3(1), dim3(256), 0, st, part, part + nb, nb, dst);
    return hipGetLastError();
}

hipError_t launch_normest_norms(double* x, const double* y, int64_t n, double* part, double* dst, hipStream_t st) {
    if (n <= 0) return hipErrorInvalidValue;
    const int nb = dot_blocks(n);
    hipLaunchKernelGGL(k_norms2, dim3(nb), dim3(256), 0, st, x, y, n, part, part + nb);
    hipLaunchKernelGGL(k_nrm_div, dim3(redvec_blocks(n)), dim3(256), 0, st, x, part, part + nb, nb, dst, n);
    return hipGetLastError();
}

hipError_t launch_pro_step(double* r, const double* qprev, const double* pb_prev, const double* q, double* qnext,
                           int64_t n, double* part, double* d_alpha, double* d_beta2, hipStream_t st) {
    if (n <= 0) return hipErrorInvalidValue;
    const int nb = dot_blocks(n);
    double* pa = part;       // alpha partials
    double* pb = part + nb;  // beta^2 partials
    hipLaunchKernelGGL(k_pro_dot, dim3(nb), dim3(256), 0, st, r, qprev, pb_prev, q, n, pa);
    hipLaunchKernelGGL(k_pro_update, dim3(nb), dim3(256), 0, st, r, q, pa, nb, d_alpha, n, pb);
    hipLaunchKernelGGL(k_pro_div, dim3(redvec_blocks(n)), dim3(256), 0, st, qnext, r, pb, nb, d_beta2, n);
    return hipGetLastError();
}

hipError_t launch_axpy_sub_dev(double* y, const double* x, const double* pa, bool take_sqrt, int64_t n,
                               hipStream_t st) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_axpy_sub_dev, dim3(vec_blocks(n)), dim3(256), 0, st, y, x, pa, take_sqrt ? 1 : 0, n);
    return hipGetLastError();
}

// ||x|| on the device: y = x / sqrt(*nn) (normest's x = x / norm(x) with the
// norm still on the device; sqrt and the division as the host would do them)
__global__ __launch_bounds__(256) void k_div_sqrt(double* __restrict__ y, const double* __restrict__ x,
                                                 const double* __restrict__ nn, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n) y[i] = x[i] / sqrt(*nn);
}

hipError_t launch_div_sqrt(double* y, const double* x, const double* nn, int64_t n, hipStream_t st) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_div_sqrt, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, y, x, nn, n);
    return hipGetLastError();
}

// y(r) = sum_j |A(r,j)| over the local CSR rows: the start vector of
// normest (sum(abs(S))' = row sums for a symmetric A).
__global__ __launch_bounds__(256) void k_abs_rowsum(const int* __restrict__ rowptr, const double* __restrict__ val,
                                                    int64_t n, double* __restrict__ y) {
    const int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (r >= n) return;
    double s = 0.0;
    for (int p = rowptr[r]; p < rowptr[r + 1]; ++p) s = s + fabs(val[p]);
    y[r] = s;
}

hipError_t launch_abs_rowsum(const int* rowptr, const double* val, int64_t n, double* y, hipStream_t st) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_abs_rowsum, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, rowptr, val, n, y);
    return hipGetLastError();
}

}  // namespace cal
