// Probe: the tall-skinny Gram C = A'B (k_gram, direct loads) against
// k_gram_lds (coalesced loads staged through LDS, same MFMA order) at the
// IRL (n = 1.58 M) and bench (n = 9.94 M) sizes: time per launch and a
// bitwise comparison of the block partials.  Not part of the library.
//   hipcc -O3 -std=c++17 -ffp-contract=off --offload-arch=gfx950 -Iinclude \
//         -Ica_lanczos_amd/csrc tools/gram_probe.hip -o tools/gram_probe
#include "../ca_lanczos_amd/csrc/kernels.hip"

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

int main() {
    using namespace cal;
    const int64_t nmax = 9938375, ldmax = (nmax + 63) / 64 * 64;
    double* buf;
    CK(hipMalloc(&buf, (size_t)144 * ldmax * 8));
    {
        std::vector<double> h((size_t)ldmax);
        for (int c = 0; c < 144; ++c) {
            for (int64_t i = 0; i < ldmax; ++i) h[i] = ((i * 7919 + c * 104729) % 2003) / 1001.0 - 1.0;
            CK(hipMemcpy(buf + (size_t)c * ldmax, h.data(), ldmax * 8, hipMemcpyHostToDevice));
        }
    }
    double *p1, *p2;
    CK(hipMalloc(&p1, (size_t)2048 * 4096 * 8));
    CK(hipMalloc(&p2, (size_t)2048 * 4096 * 8));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    auto time = [&](auto launch) -> double {
        for (int i = 0; i < 3; ++i) launch();
        CK(hipEventRecord(a));
        const int reps = 10;
        for (int i = 0; i < reps; ++i) launch();
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        return ms * 1e3 / reps;
    };
    for (int64_t n : {(int64_t)1585081, nmax}) {
        const int64_t ld = (n + 63) / 64 * 64;
        for (int wb : {8, 9, 16}) {
            for (int wa : {9, 16, 24, 32, 48, 57, 64, 96, 120, 128}) {
                Panel A{}, B{};
                A.nseg = 1; A.ptr[0] = buf; A.ld[0] = ld; A.ncol[0] = wa; A.total = wa;
                B.nseg = 1; B.ptr[0] = buf + (size_t)128 * ld; B.ld[0] = ld; B.ncol[0] = wb; B.total = wb;
                const GramPlan pl = gram_plan(wa, wb, n);
                setenv("CAL_GRAM_LDS", "0", 1);
                auto old = [&] {
                    dim3 g(pl.blocks), bl(256);
                    switch (pl.nta) {
                        case 1: hipLaunchKernelGGL((k_gram<1, 16>), g, bl, 0, 0, A, B, n, p1); break;
                        case 2: hipLaunchKernelGGL((k_gram<2, 16>), g, bl, 0, 0, A, B, n, p1); break;
                        case 3: hipLaunchKernelGGL((k_gram<3, 8>), g, bl, 0, 0, A, B, n, p1); break;
                        case 4: hipLaunchKernelGGL((k_gram<4, 8>), g, bl, 0, 0, A, B, n, p1); break;
                        case 5: hipLaunchKernelGGL((k_gram<5, 4>), g, bl, 0, 0, A, B, n, p1); break;
                        case 6: hipLaunchKernelGGL((k_gram<6, 4>), g, bl, 0, 0, A, B, n, p1); break;
                        case 7: hipLaunchKernelGGL((k_gram<7, 4>), g, bl, 0, 0, A, B, n, p1); break;
                        default: hipLaunchKernelGGL((k_gram<8, 4>), g, bl, 0, 0, A, B, n, p1); break;
                    }
                };
                auto neu = [&] {
                    switch (pl.nta) {
                        case 1: launch_gram_lds<1, 16>(A, B, n, pl.blocks, p2, 0); break;
                        case 2: launch_gram_lds<2, 16>(A, B, n, pl.blocks, p2, 0); break;
                        case 3: launch_gram_lds<3, 8>(A, B, n, pl.blocks, p2, 0); break;
                        case 4: launch_gram_lds<4, 8>(A, B, n, pl.blocks, p2, 0); break;
                        case 5: launch_gram_lds<5, 4>(A, B, n, pl.blocks, p2, 0); break;
                        case 6: launch_gram_lds<6, 4>(A, B, n, pl.blocks, p2, 0); break;
                        case 7: launch_gram_lds<7, 4>(A, B, n, pl.blocks, p2, 0); break;
                        default: launch_gram_lds<8, 4>(A, B, n, pl.blocks, p2, 0); break;
                    }
                };
                const double t1 = time(old);
                const double t2 = time(neu);
                CK(hipGetLastError());
                const size_t cnt = (size_t)pl.blocks * pl.entries;
                std::vector<double> h1(cnt), h2(cnt);
                CK(hipMemcpy(h1.data(), p1, cnt * 8, hipMemcpyDeviceToHost));
                CK(hipMemcpy(h2.data(), p2, cnt * 8, hipMemcpyDeviceToHost));
                const bool same = std::memcmp(h1.data(), h2.data(), cnt * 8) == 0;
                const double by = (double)(wa + wb) * 8.0 * n;
                printf("{\"n\": %ld, \"wa\": %d, \"wb\": %d, \"k_gram_us\": %.1f, \"k_gram_GBps\": %.0f, \"lds_us\": %.1f, "
                       "\"lds_GBps\": %.0f, \"bitwise_equal\": %s}\n",
                       (long)n, wa, wb, t1, by / (t1 * 1e-6) / 1e9, t2, by / (t2 * 1e-6) / 1e9, same ? "true" : "false");
                fflush(stdout);
            }
        }
    }
    return 0;
}
