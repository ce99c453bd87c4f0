// Probe: the block-orthogonalisation sweeps (k_rowapply kinds) back to back
// on a 215^3-row, 17-column panel, beside stripped-down variants, to see what
// each part of pass A costs.  Not part of the library.
//   hipcc -O3 -std=c++17 -ffp-contract=off --offload-arch=gfx950 -Iinclude \
//         -Ica_lanczos_amd/csrc tools/rowapply_probe.hip -o tools/rowapply_probe
#include "../ca_lanczos_amd/csrc/kernels.hip"

#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

// loads + the 17x8 apply from LDS broadcasts (pass A without the Gram)
template <bool SGPR_M>
__global__ __launch_bounds__(256) void k_apply_only(cal::ColList P, const double* __restrict__ M, int64_t n,
                                                    double* out) {
    __shared__ __attribute__((aligned(16))) double Ms[17 * 8];
    for (int e = threadIdx.x; e < 17 * 8; e += 256) Ms[e] = M[e];
    __syncthreads();
    double acc = 0;
    for (int64_t base = (int64_t)blockIdx.x * 256; base < n; base += (int64_t)gridDim.x * 256) {
        const int64_t r = base + threadIdx.x < n ? base + threadIdx.x : n - 1;
        double p[17];
#pragma unroll
        for (int c = 0; c < 17; ++c) p[c] = P.p[c][r];
        double y[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
        for (int c = 0; c < 17; ++c)
#pragma unroll
            for (int j = 0; j < 8; ++j) y[j] = __builtin_fma(p[c], SGPR_M ? M[c * 8 + j] : Ms[c * 8 + j], y[j]);
#pragma unroll
        for (int j = 0; j < 8; ++j) acc += y[j];
    }
    if (acc == 1.2345) out[0] = acc;
}

int main() {
    using namespace cal;
    const int64_t n = 215LL * 215 * 215, ld = (n + 63) / 64 * 64;
    double* buf;
    CK(hipMalloc(&buf, 26 * ld * 8));
    CK(hipMemset(buf, 0, 26 * ld * 8));
    ColList cl;
    for (int c = 0; c < 17; ++c) cl.p[c] = buf + c * ld;
    OutList ol;
    for (int j = 0; j < 16; ++j) ol.p[j] = buf + (17 + (j < 8 ? j : 0)) * ld;
    double *dM, *part;
    CK(hipMalloc(&dM, 4096 * 8));
    CK(hipMemset(dM, 0, 4096 * 8));
    CK(hipMalloc(&part, (size_t)1024 * 272 * 8));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    auto time = [&](const char* name, auto launch) {
        for (int i = 0; i < 3; ++i) launch();
        CK(hipEventRecord(a));
        const int reps = 20;
        for (int i = 0; i < reps; ++i) launch();
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        printf("{\"kernel\": \"%s\", \"us\": %.1f}\n", name, ms * 1e3 / reps);
        return 0;
    };
    time("P1 rowgram (17 cols, MFMA tile)", [&] { launch_rowgram(cl, 16, true, n, 1024, part, 0); });
    time("pass A (apply + Grams, no store)", [&] { launch_rowapply(cl, dM, 17, 8, ol, 2, 9, n, 1024, part, 0); });
    time("pass B (chained apply, store)", [&] { launch_rowapply(cl, dM, 17, 8, ol, 3, 9, n, (int)((n + 255) / 256), part, 0); });
    time("apply only, M in LDS", [&] { hipLaunchKernelGGL(k_apply_only<false>, dim3(1024), dim3(256), 0, 0, cl, dM, n, buf); });
    time("apply only, M scalar loads", [&] { hipLaunchKernelGGL(k_apply_only<true>, dim3(1024), dim3(256), 0, 0, cl, dM, n, buf); });
    time("apply only, M in LDS, 2048 blocks", [&] { hipLaunchKernelGGL(k_apply_only<false>, dim3(2048), dim3(256), 0, 0, cl, dM, n, buf); });
    CK(hipDeviceSynchronize());
    return 0;
}
