// Probe: the library's Ritz-vector apply (k_apply_mt, kernels.hip) at the
// bench size, by sk, with its k-step group KG swept, bitwise against the
// row-parallel apply.  Not part of the library.
//   hipcc -O3 -std=c++17 -ffp-contract=off --offload-arch=gfx950 -Iinclude tools/apply_probe2.hip -o tools/apply_probe2
#include "../ca_lanczos_amd/csrc/kernels.hip"

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

int main() {
    using namespace cal;
    const int64_t n = 9938375, ld = (n + 63) / 64 * 64;
    double *Pbuf, *Ybuf, *dM, *Yref;
    CK(hipMalloc(&Pbuf, (size_t)128 * ld * 8));
    CK(hipMalloc(&Ybuf, (size_t)128 * ld * 8));
    CK(hipMalloc(&Yref, (size_t)128 * ld * 8));
    CK(hipMalloc(&dM, 128 * 128 * 8));
    {
        std::vector<double> h((size_t)ld);
        for (int c = 0; c < 128; ++c) {
            for (int64_t i = 0; i < ld; ++i) h[i] = ((i * 7919 + c * 104729) % 2003) / 1001.0 - 1.0;
            CK(hipMemcpy(Pbuf + (size_t)c * ld, h.data(), ld * 8, hipMemcpyHostToDevice));
        }
        std::vector<double> m(128 * 128);
        for (int i = 0; i < 128 * 128; ++i) m[i] = ((i * 31) % 97) / 97.0 - 0.5;
        CK(hipMemcpy(dM, m.data(), m.size() * 8, hipMemcpyHostToDevice));
    }
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    auto time = [&](auto launch) -> double {
        for (int i = 0; i < 2; ++i) launch();
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(a));
        const int reps = 10;
        for (int i = 0; i < reps; ++i) launch();
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        return ms * 1e3 / reps;
    };
    auto maxdiff = [&](int wy) {
        std::vector<double> h1(4096), h2(4096);
        double md = 0.0;
        for (int c = 0; c < wy; c += 7)
            for (int64_t off : {(int64_t)0, n / 2, n - 4096}) {
                CK(hipMemcpy(h1.data(), Ybuf + (size_t)c * ld + off, 4096 * 8, hipMemcpyDeviceToHost));
                CK(hipMemcpy(h2.data(), Yref + (size_t)c * ld + off, 4096 * 8, hipMemcpyDeviceToHost));
                for (int i = 0; i < 4096; ++i) md = std::max(md, std::fabs(h1[i] - h2[i]));
            }
        return md;
    };
    for (int sk : {48, 96, 120}) {
        Panel P{};
        P.nseg = 1; P.ptr[0] = Pbuf; P.ld[0] = ld; P.ncol[0] = sk; P.total = sk;
        for (int j0 = 0; j0 < sk; j0 += 64) {  // reference: the row-parallel apply (same FMA chains)
            const int wy = std::min(64, sk - j0);
            PanelOut Y{};
            Y.nseg = 1; Y.ptr[0] = Yref + (size_t)j0 * ld; Y.ld[0] = ld; Y.ncol[0] = wy; Y.total = wy;
            const ApplyPlan ap = apply_plan(sk, wy, n, false, 0);
            CK(launch_apply(P, dM + (size_t)j0 * sk, sk, wy, Y, true, 0, n, ap, nullptr, 0));
        }
        CK(hipDeviceSynchronize());
        const double fl = 2.0 * sk * sk * n;
        const double tlib = time([&] { launch_apply_mt(Pbuf, ld, dM, sk, sk, Ybuf, ld, n, 0); });
        const double dlib = maxdiff(sk);
        auto kg_time = [&](auto kg_c) {
            constexpr int KG = decltype(kg_c)::value;
            constexpr int NT = 8, W = 8;
            const size_t lds = (size_t)((sk + 3) & ~3) * 16 * NT * 8;
            const int64_t blocks = std::min<int64_t>((n + 32 * W - 1) / (32 * W), 256);
            return time([&] {
                hipLaunchKernelGGL((cal::k_apply_mt<NT, W, KG>), dim3((unsigned)blocks, (sk + 16 * NT - 1) / (16 * NT)),
                                   dim3(64 * W), lds, 0, Pbuf, ld, dM, sk, sk, Ybuf, ld, n);
            });
        };
        const double k2 = kg_time(std::integral_constant<int, 2>{}), k4 = kg_time(std::integral_constant<int, 4>{}),
                     k6 = kg_time(std::integral_constant<int, 6>{}), k8 = kg_time(std::integral_constant<int, 8>{});
        const double dk8 = maxdiff(sk);
        printf("{\"sk\": %d, \"lib_us\": %.0f, \"lib_TF\": %.1f, \"diff_vs_rows\": %.2e, \"nt8_kg2_us\": %.0f, "
               "\"kg4_us\": %.0f, \"kg6_us\": %.0f, \"kg8_us\": %.0f, \"diff_kg8\": %.2e}\n",
               sk, tlib, fl / (tlib * 1e-6) / 1e12, dlib, k2, k4, k6, k8, dk8);
        fflush(stdout);
    }
    return 0;
}
