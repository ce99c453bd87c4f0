// Probe: the headline's P1 Gram ([Qp(0:8) | X]'X plus Qp's ninth column,
// lap3d_215: n = 9,938,375, 17 columns) on the row Gram sweep the library runs
// (launch_rowgram, k_rowapply<17,4,Gram-only>) against the row-staged Gram
// (k_gram_rows<1,4,B'B>: A = Qp's 9 columns, B = X's 8 -> Qp'X and X'X, the
// same entries) for several grid sizes, back to back (1.35 GB per launch, five
// times the Infinity Cache).  Not part of the library.
//   hipcc -O3 -std=c++17 -ffp-contract=off --offload-arch=gfx950 -Iinclude \
//         -Ica_lanczos_amd/csrc tools/p1_probe.hip -o tools/p1_probe
#include "../ca_lanczos_amd/csrc/kernels.hip"

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

int main() {
    using namespace cal;
    const int64_t n = 9938375, ld = (n + 2 + 63) / 64 * 64;
    const int w = 9, m = 8;
    double* buf;
    CK(hipMalloc(&buf, (size_t)(w + m) * ld * 8));
    {
        std::vector<double> h((size_t)ld);
        for (int c = 0; c < w + m; ++c) {
            for (int64_t i = 0; i < ld; ++i) h[i] = ((i * 7919 + c * 104729) % 2003) / 1001.0 - 1.0;
            CK(hipMemcpy(buf + (size_t)c * ld, h.data(), ld * 8, hipMemcpyHostToDevice));
        }
    }
    double* part;
    CK(hipMalloc(&part, (size_t)4096 * 1024 * 8));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    auto time = [&](auto launch) -> double {
        for (int i = 0; i < 3; ++i) launch();
        CK(hipEventRecord(a));
        const int reps = 20;
        for (int i = 0; i < reps; ++i) launch();
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms = 0.f;
        CK(hipEventElapsedTime(&ms, a, b));
        return ms * 1e3 / reps;
    };
    const double gb = 8.0 * n * (w + m) / 1e3;
    // the library's P1: T = [Qp(0:8) | X] (16 columns) + Qp column 8 as the extra column
    ColList ct{};
    for (int cc = 0; cc < 16; ++cc) ct.p[cc] = buf + (size_t)(cc < 8 ? cc : cc + 1) * ld;
    ct.p[16] = buf + (size_t)8 * ld;
    printf("{\"n\": %lld", (long long)n);
    for (int blocks : {512, 1024, 2048}) {
        const double us = time([&] { launch_rowgram(ct, 16, true, n, blocks, part, 0); });
        printf(", \"rowgram_b%d_us\": %.1f, \"rowgram_b%d_GBps\": %.0f", blocks, us, blocks, gb / us);
    }
    Panel A = panel(), B = panel();
    panel_add(A, buf, ld, w);
    panel_add(B, buf + (size_t)w * ld, ld, m);
    for (int blocks : {512, 1024, 2048}) {
        const double us = time([&] {
            const size_t lds = std::max((size_t)2 * 64 * 33, (size_t)3 * 2 * 64 * 4) * 8;
            hipLaunchKernelGGL((k_gram_rows<1, 4, true>), dim3(blocks), dim3(256), lds, 0, A, B, n, part, 16, 0);
        });
        printf(", \"gram_rows_bb_b%d_us\": %.1f, \"gram_rows_bb_b%d_GBps\": %.0f", blocks, us, blocks, gb / us);
    }
    printf("}\n");
    return 0;
}
