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
                const double e0 = x[tw + 128 - P - 1], e1 = x[tw + 128 - N - 1], e5 = x[tw + 128 + N - 1],
                             e6 = x[tw + 128 + P - 1];
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

int main(int argc, char** argv) {
    const int nvec = argc > 1 ? atoi(argv[1]) : 32;
    const int64_t pad = P + 128;
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
    CK(hipMalloc(&part, (size_t)nvec * 20000 * 8));
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
    RUN(0, 4, 4);
    RUN(0, 1, 1);
    RUN(0, 1, 2);
    RUN(0, 1, 4);
    RUN(0, 1, 8);
    RUN(0, 2, 4);
    RUN(1, 1, 2);
    RUN(1, 1, 4);
    RUN(1, 1, 8);
    RUN(2, 1, 2);
    RUN(2, 1, 4);
    RUN(2, 1, 8);
    RUN(2, 2, 4);
    return 0;
}
