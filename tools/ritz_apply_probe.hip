// Probe: the Ritz-vector apply X = Q(:,1:sk) * V (sk x sk) of the
// diagnostics (ca_lanczos.m:88-97) at the bench size (n = 9.94 M): the
// library's row-parallel apply, rocBLAS dgemm, and an MFMA kernel with the
// transposed operand roles (D = M^T P^T, so each accumulator register holds
// 16 consecutive rows of one output column: full 128-B lines per store).
// Not part of the library.
//   hipcc -O3 -std=c++17 -ffp-contract=off --offload-arch=gfx950 -Iinclude \
//         -Ica_lanczos_amd/csrc tools/ritz_apply_probe.hip -lrocblas -o tools/ritz_apply_probe
#include "../ca_lanczos_amd/csrc/kernels.hip"

#include <rocblas/rocblas.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

namespace probe {
using cal::d2;
using cal::d4;
using cal::mfma64;

template <int NT, int WAVES>
__global__ __launch_bounds__(64 * WAVES) void k_apply_mt(const double* __restrict__ P, int64_t ldp,
                                                         const double* __restrict__ M, int wp, int wy,
                                                         double* __restrict__ Y, int64_t ldy, int64_t n) {
    extern __shared__ __attribute__((aligned(16))) double Ms[];
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
    for (int64_t r0 = ((int64_t)blockIdx.x * WAVES + wave) * 32; r0 < n; r0 += stride) {
        const bool full = r0 + 32 <= n;
        const int64_t rb = r0 + 2 * c16;
        d4 acc[NT][2];
#pragma unroll
        for (int ty = 0; ty < NT; ++ty) acc[ty][0] = acc[ty][1] = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll 4
        for (int kc = 0; kc < nkc; ++kc) {
            const int c = 4 * kc + g;
            const bool con = c < wp;
            const double* pc = P + (int64_t)(con ? c : 0) * ldp;
            double b0, b1;
            if (full) {
                const d2 x = *reinterpret_cast<const d2*>(pc + rb);
                b0 = x[0];
                b1 = x[1];
            } else {
                b0 = rb < n ? pc[rb] : 0.0;
                b1 = rb + 1 < n ? pc[rb + 1] : 0.0;
            }
            b0 = con ? b0 : 0.0;
            b1 = con ? b1 : 0.0;
#pragma unroll
            for (int ty = 0; ty < NT; ++ty) {
                const double a = Ms[c * ldm + 16 * ty + c16];
                acc[ty][0] = mfma64(a, b0, acc[ty][0]);
                acc[ty][1] = mfma64(a, b1, acc[ty][1]);
            }
        }
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
    }
}

template <int NT, int WAVES>
void launch_mt(const double* P, int64_t ldp, const double* M, int wp, int wy, double* Y, int64_t ldy, int64_t n,
               int bpc) {
    const int wpp = (wp + 3) & ~3;
    const size_t lds = (size_t)wpp * 16 * NT * sizeof(double);
    const int groups = (wy + 16 * NT - 1) / (16 * NT);
    int64_t blocks = (n + 32 * WAVES - 1) / (32 * WAVES);
    if (blocks > 256 * bpc) blocks = 256 * bpc;
    hipLaunchKernelGGL((k_apply_mt<NT, WAVES>), dim3((unsigned)blocks, groups), dim3(64 * WAVES), lds, 0, P, ldp, M,
                       wp, wy, Y, ldy, n);
}
}  // namespace probe

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
    rocblas_handle hb;
    rocblas_create_handle(&hb);
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
        for (int c = 0; c < wy; c += 7) {
            for (int64_t off : {(int64_t)0, n / 2, n - 4096}) {
                CK(hipMemcpy(h1.data(), Ybuf + (size_t)c * ld + off, 4096 * 8, hipMemcpyDeviceToHost));
                CK(hipMemcpy(h2.data(), Yref + (size_t)c * ld + off, 4096 * 8, hipMemcpyDeviceToHost));
                for (int i = 0; i < 4096; ++i) md = std::max(md, std::fabs(h1[i] - h2[i]));
            }
        }
        return md;
    };
    for (int sk : {16, 32, 48, 64, 96, 120, 128}) {
        Panel P{};
        P.nseg = 1; P.ptr[0] = Pbuf; P.ld[0] = ld; P.ncol[0] = sk; P.total = sk;
        // library path: <= 64 output chunks (as ritz_diagnostics' apply_host)
        auto lib = [&] {
            for (int j0 = 0; j0 < sk; j0 += 64) {
                const int wy = std::min(64, sk - j0);
                PanelOut Y{};
                Y.nseg = 1; Y.ptr[0] = Yref + (size_t)j0 * ld; Y.ld[0] = ld; Y.ncol[0] = wy; Y.total = wy;
                const ApplyPlan ap = apply_plan(sk, wy, n, false, 0);
                launch_apply(P, dM + (size_t)j0 * sk, sk, wy, Y, true, 0, n, ap, nullptr, 0);
            }
        };
        const double tl = time(lib);
        const double one = 1.0, zero = 0.0;
        const double tr = time([&] {
            rocblas_dgemm(hb, rocblas_operation_none, rocblas_operation_none, (rocblas_int)n, sk, sk, &one, Pbuf,
                          (rocblas_int)ld, dM, sk, &zero, Ybuf, (rocblas_int)ld);
        });
        const double dr = maxdiff(sk);
        const double t84 = time([&] { probe::launch_mt<8, 4>(Pbuf, ld, dM, sk, sk, Ybuf, ld, n, 1); });
        const double d84 = maxdiff(sk);
        const double t88 = time([&] { probe::launch_mt<8, 8>(Pbuf, ld, dM, sk, sk, Ybuf, ld, n, 1); });
        const double t44 = time([&] { probe::launch_mt<4, 4>(Pbuf, ld, dM, sk, sk, Ybuf, ld, n, 2); });
        const double t48 = time([&] { probe::launch_mt<4, 8>(Pbuf, ld, dM, sk, sk, Ybuf, ld, n, 2); });
        const double t24 = time([&] { probe::launch_mt<2, 4>(Pbuf, ld, dM, sk, sk, Ybuf, ld, n, 4); });
        const double d24 = maxdiff(sk);
        const double tlib = time([&] { cal::launch_apply_mt(Pbuf, ld, dM, sk, sk, Ybuf, ld, n, 0); });
        const double dlib = maxdiff(sk);
        // k-step grouping of the library kernel (KG) at this sk's tile count
        auto kg_time = [&](auto kg_c) {
            constexpr int KG = decltype(kg_c)::value;
            auto one = [&](auto nt_c, auto w_c, int per_cu) {
                constexpr int NT = decltype(nt_c)::value, W = decltype(w_c)::value;
                const size_t lds = (size_t)((sk + 3) & ~3) * 16 * NT * 8;
                const int bpc = std::max(1, std::min(per_cu, (int)((160 * 1024) / lds)));
                int64_t blocks = std::min<int64_t>((n + 32 * W - 1) / (32 * W), 256 * bpc);
                return time([&] {
                    hipLaunchKernelGGL((cal::k_apply_mt<NT, W, KG>), dim3((unsigned)blocks, (sk + 16 * NT - 1) / (16 * NT)),
                                       dim3(64 * W), lds, 0, Pbuf, ld, dM, sk, sk, Ybuf, ld, n);
                });
            };
            using I = std::integral_constant<int, 4>;
            using E = std::integral_constant<int, 8>;
            switch (std::min(8, (sk + 15) / 16)) {
                case 1: return one(std::integral_constant<int, 1>{}, I{}, 4);
                case 2: return one(std::integral_constant<int, 2>{}, I{}, 4);
                case 3: return one(std::integral_constant<int, 3>{}, E{}, 2);
                case 4: return one(std::integral_constant<int, 4>{}, E{}, 2);
                case 6: return one(std::integral_constant<int, 6>{}, E{}, 2);
                default: return one(std::integral_constant<int, 8>{}, E{}, 1);
            }
        };
        printf("{\"sk\": %d, \"kg1_us\": %.0f, \"kg2_us\": %.0f, \"kg4_us\": %.0f}\n", sk,
               kg_time(std::integral_constant<int, 1>{}), kg_time(std::integral_constant<int, 2>{}),
               kg_time(std::integral_constant<int, 4>{}));
        const double fl = 2.0 * sk * sk * n, by = 2.0 * sk * 8.0 * n;
        printf("{\"sk\": %d, \"launch_apply_mt_us\": %.0f, \"TF\": %.1f, \"diff_vs_rows\": %.2e}\n", sk, tlib,
               fl / (tlib * 1e-6) / 1e12, dlib);
        auto rate = [&](double us) { return fl / (us * 1e-6) / 1e12; };
        auto bw = [&](double us) { return by / (us * 1e-6) / 1e9; };
        printf("{\"sk\": %d, \"lib_us\": %.0f, \"lib_TF\": %.1f, \"rocblas_us\": %.0f, \"rocblas_TF\": %.1f, \"rocblas_GBps\": %.0f, "
               "\"mt84_us\": %.0f, \"mt88_us\": %.0f, \"mt44_us\": %.0f, \"mt48_us\": %.0f, \"mt24_us\": %.0f, \"best_mt_TF\": %.1f, "
               "\"diff_rocblas\": %.2e, \"diff_mt84\": %.2e, \"diff_mt24\": %.2e}\n",
               sk, tl, rate(tl), tr, rate(tr), bw(tr), t84, t88, t44, t48, t24,
               rate(std::min(std::min(std::min(t84, t88), std::min(t44, t48)), t24)), dr, d84, d24);
        fflush(stdout);
    }
    return 0;
}
