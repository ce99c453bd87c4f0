// Probe: the generic tall-skinny Gram / apply kernels (k_gram, k_apply) of
// the 'full' projections at the IRL's shapes (n = 1.58 M rows, A up to 57
// columns, B / Y 8 columns), back to back.  Not part of the library.
//   hipcc -O3 -std=c++17 -ffp-contract=off --offload-arch=gfx950 -Iinclude \
//         -Ica_lanczos_amd/csrc tools/wide_probe.hip -o tools/wide_probe
#include "../ca_lanczos_amd/csrc/kernels.hip"

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

int main() {
    using namespace cal;
    const int64_t n = 1585081, ld = (n + 63) / 64 * 64;
    double* buf;
    CK(hipMalloc(&buf, (size_t)80 * ld * 8));
    CK(hipMemset(buf, 0, (size_t)80 * ld * 8));
    double *dM, *part;
    CK(hipMalloc(&dM, 65536 * 8));
    CK(hipMemset(dM, 0, 65536 * 8));
    CK(hipMalloc(&part, (size_t)2048 * 4096 * 8));
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
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        return ms * 1e3 / reps;
    };
    for (int wa : {8, 9, 16, 24, 32, 40, 48, 57}) {
        Panel A{}, B{};
        A.nseg = 1; A.ptr[0] = buf; A.ld[0] = ld; A.ncol[0] = wa; A.total = wa;
        B.nseg = 1; B.ptr[0] = buf + (size_t)64 * ld; B.ld[0] = ld; B.ncol[0] = 8; B.total = 8;
        const GramPlan pl = gram_plan(wa, 8, n);
        const double tg = time([&] { launch_gram(A, B, n, pl, part, 0); });
        // apply: Y(8) = [A | B] M, wp = wa + 8
        Panel P{};
        P.nseg = 2; P.ptr[0] = buf; P.ld[0] = ld; P.ncol[0] = wa; P.ptr[1] = B.ptr[0]; P.ld[1] = ld; P.ncol[1] = 8;
        P.total = wa + 8;
        PanelOut Y{};
        Y.nseg = 1; Y.ptr[0] = buf + (size_t)72 * ld; Y.ld[0] = ld; Y.ncol[0] = 8; Y.total = 8;
        const ApplyPlan ap = apply_plan(wa + 8, 8, n, false, 0);
        const double ta = time([&] { launch_apply(P, dM, wa + 8, 8, Y, true, 0, n, ap, part, 0); });
        const double bg = (wa + 8) * 8.0 * n, ba = (wa + 16) * 8.0 * n;
        printf("{\"wa\": %d, \"gram_us\": %.1f, \"gram_GBps\": %.0f, \"gram_blocks\": %d, \"apply_us\": %.1f, \"apply_GBps\": %.0f}\n",
               wa, tg, bg / (tg * 1e-6) / 1e9, pl.blocks, ta, ba / (ta * 1e-6) / 1e9);
    }
    return 0;
}
