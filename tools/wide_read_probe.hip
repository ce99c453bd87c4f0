// Probe: the read floor of a W-column sweep at lap3d_215's n (9,938,375 rows,
// column-major, ld padded to 64) against the library's row-staged Gram
// (k_gram_rows) on the same columns -- is the 'full' mode's wide Gram
// (65..121 Q columns against the 8-column block) at the memory system's
// floor for that many concurrent column streams?  Not part of the library.
//   hipcc -O3 -std=c++17 -ffp-contract=off --offload-arch=gfx950 -Iinclude \
//         -Ica_lanczos_amd/csrc tools/wide_read_probe.hip -o tools/wide_read_probe
// Floors (a sum per lane, nothing stored but one double per thread):
//   rows<NS>: k_gram_rows' load pattern -- per round a block reads 64 rows of
//             all W columns, one column per wave instruction (512 B), NS
//             rounds in flight per thread; no LDS, so several blocks per CU;
//   lane:     k_rowapply's -- one row per lane, every column of it, a
//             256-row chunk per block and grid-stride.
//   panel16:  the W columns as W/16 sequential sweeps of 16 (fewer streams
//             in flight), one launch each.
#include "../ca_lanczos_amd/csrc/kernels.hip"

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

template <int NS>
__global__ __launch_bounds__(256) void k_floor_rows(const double* __restrict__ X, int64_t ld, int w, int64_t n,
                                                    double* __restrict__ out) {
    const int tid = threadIdx.x, lrow = tid & 63, c0 = tid >> 6;
    const int64_t stride = (int64_t)gridDim.x * 64;
    double s = 0.0;
    for (int64_t rb = (int64_t)blockIdx.x * 64; rb < n; rb += NS * stride) {
        double v[NS][32];
#pragma unroll
        for (int k = 0; k < NS; ++k) {
            const int64_t r = rb + k * stride + lrow;
            const int64_t ro = r < n ? r : 0;
#pragma unroll
            for (int q = 0; q < 32; ++q) {
                const int c = c0 + 4 * q;
                v[k][q] = c < w ? X[(int64_t)c * ld + ro] : 0.0;
            }
        }
#pragma unroll
        for (int k = 0; k < NS; ++k)
#pragma unroll
            for (int q = 0; q < 32; ++q) s += v[k][q];
    }
    out[(int64_t)blockIdx.x * 256 + tid] = s;
}

__global__ __launch_bounds__(256) void k_floor_lane(const double* __restrict__ X, int64_t ld, int w, int64_t n,
                                                    double* __restrict__ out) {
    double s = 0.0;
    for (int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x; r < n; r += (int64_t)gridDim.x * 256) {
        double v[128];
#pragma unroll
        for (int c = 0; c < 128; ++c) v[c] = c < w ? X[(int64_t)c * ld + r] : 0.0;
#pragma unroll
        for (int c = 0; c < 128; ++c) s += v[c];
    }
    out[(int64_t)blockIdx.x * 256 + threadIdx.x] = s;
}

int main() {
    using namespace cal;
    const int64_t n = 9938375, ld = (n + 63) / 64 * 64;
    const int WMAX = 128;
    double* buf;
    CK(hipMalloc(&buf, (size_t)WMAX * ld * 8));
    CK(hipMemset(buf, 0, (size_t)WMAX * ld * 8));
    double *part, *out;
    CK(hipMalloc(&part, (size_t)2048 * 16 * 16 * 9 * 8));
    CK(hipMalloc(&out, (size_t)4096 * 256 * 8));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    auto time = [&](auto launch) -> double {
        for (int i = 0; i < 2; ++i) launch();
        CK(hipEventRecord(a));
        const int reps = 10;
        for (int i = 0; i < reps; ++i) launch();
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        return ms * 1e3 / reps;
    };
    for (int w : {17, 24, 32, 48, 64, 72, 80, 96, 112, 128}) {
        const double gb = (double)w * n * 8 / 1e9;
        auto rate = [&](double us) { return gb / (us * 1e-6); };
        printf("{\"w\": %d", w);
        for (int blocks : {512, 1024, 2048}) {
            printf(", \"rows2_b%d\": %.0f", blocks, rate(time([&] {
                       hipLaunchKernelGGL(k_floor_rows<2>, dim3(blocks), dim3(256), 0, 0, buf, ld, w, n, out); })));
            printf(", \"rows4_b%d\": %.0f", blocks, rate(time([&] {
                       hipLaunchKernelGGL(k_floor_rows<4>, dim3(blocks), dim3(256), 0, 0, buf, ld, w, n, out); })));
        }
        for (int blocks : {1024, 2048, 4096})
            printf(", \"lane_b%d\": %.0f", blocks, rate(time([&] {
                       hipLaunchKernelGGL(k_floor_lane, dim3(blocks), dim3(256), 0, 0, buf, ld, w, n, out); })));
        printf(", \"panel16_b1024\": %.0f", rate(time([&] {
                   for (int c = 0; c < w; c += 16)
                       hipLaunchKernelGGL(k_floor_rows<2>, dim3(1024), dim3(256), 0, 0, buf + (int64_t)c * ld, ld,
                                          std::min(16, w - c), n, out);
               })));
        // the library's Gram: A = columns 16.., B = the first min(16, w) (the
        // 'full' shape has B = 8; here B is 16 wide when w allows)
        if (w > 16) {
            Panel A{}, B{};
            const int wb = w >= 24 ? 8 : w - 16;
            const int wa = w - wb;
            B.nseg = 1; B.ptr[0] = buf; B.ld[0] = ld; B.ncol[0] = wb; B.total = wb;
            A.nseg = 1; A.ptr[0] = buf + (int64_t)wb * ld; A.ld[0] = ld; A.ncol[0] = wa; A.total = wa;
            const GramPlan pl = gram_plan(wa, wb, n);
            printf(", \"gram_wa\": %d, \"gram_wb\": %d, \"gram_blocks\": %d, \"gram_launch\": %.0f", wa, wb, pl.blocks,
                   rate(time([&] { CK(launch_gram(A, B, n, pl, part, 0)); })));
        }
        printf("}\n");
        fflush(stdout);
    }
    return 0;
}
