// Probe: the row-staged narrow Gram (k_gram_rows<NTA, RUN>) at the IRL shapes
// (n = 1.58 M, A 4..48 columns, B 8) against a bare read of the same columns
// (one column per wave instruction, 2 or 4 rounds in flight, a sum per lane:
// the read floor of the shape), for several grid sizes.  Not part of the library.
//   hipcc -O3 -std=c++17 -ffp-contract=off --offload-arch=gfx950 -Iinclude \
//         -Ica_lanczos_amd/csrc tools/gram_rows_probe.hip -o tools/gram_rows_probe
#include "../ca_lanczos_amd/csrc/kernels.hip"

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

// floor: W columns (column-major, ld), lane = row, DEPTH rows-of-256 rounds in flight
template <int DEPTH>
__global__ __launch_bounds__(256) void k_read_floor(const double* __restrict__ X, int64_t ld, int w, int64_t n,
                                                    double* __restrict__ out) {
    double s = 0.0;
    const int64_t stride = (int64_t)gridDim.x * 256;
    for (int c = 0; c < w; ++c) {
        const double* col = X + (int64_t)c * ld;
        int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x;
        for (; r + (DEPTH - 1) * stride < n; r += DEPTH * stride) {
            double v[DEPTH];
#pragma unroll
            for (int d = 0; d < DEPTH; ++d) v[d] = col[r + d * stride];
#pragma unroll
            for (int d = 0; d < DEPTH; ++d) s += v[d];
        }
        for (; r < n; r += stride) s += col[r];
    }
    out[(int64_t)blockIdx.x * 256 + threadIdx.x] = s;
}

int main() {
    using namespace cal;
    const int64_t n = 1585081, ld = (n + 63) / 64 * 64;
    const int wmax = 64;
    double* buf;
    CK(hipMalloc(&buf, (size_t)wmax * ld * 8));
    {
        std::vector<double> h((size_t)ld);
        for (int c = 0; c < wmax; ++c) {
            for (int64_t i = 0; i < ld; ++i) h[i] = ((i * 7919 + c * 104729) % 2003) / 1001.0 - 1.0;
            CK(hipMemcpy(buf + (size_t)c * ld, h.data(), ld * 8, hipMemcpyHostToDevice));
        }
    }
    double* p1;
    CK(hipMalloc(&p1, (size_t)4096 * 4096 * 8));
    // a 512 MB buffer swept between launches so the Infinity Cache holds none of the panels
    double* flush;
    const size_t fl = (size_t)64 << 20;
    CK(hipMalloc(&flush, fl * 8));
    CK(hipMemset(flush, 0, fl * 8));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    auto time = [&](auto launch) -> double {
        double tot = 0.0;
        for (int i = 0; i < 12; ++i) {
            CK(hipMemsetAsync(flush, i, fl * 8));
            CK(hipEventRecord(a));
            launch();
            CK(hipEventRecord(b));
            CK(hipEventSynchronize(b));
            float ms = 0.f;
            CK(hipEventElapsedTime(&ms, a, b));
            if (i >= 2) tot += ms;
        }
        return tot / 10 * 1e3;  // us
    };
    const int shapes[][2] = {{9, 8}, {8, 8}, {4, 8}, {12, 8}, {16, 8}, {20, 8}, {28, 8}, {32, 8}, {36, 8}, {44, 8}, {48, 8}};
    for (auto& sh : shapes) {
        const int wa = sh[0], wb = sh[1];
        Panel A = panel(), B = panel();
        panel_add(A, buf, ld, wa);
        panel_add(B, buf + (size_t)wa * ld, ld, wb);
        const double gb = 8.0 * n * (wa + wb) / 1e3;  // bytes / 1e3 -> GB/s with us
        const int nta = (wa + 15) / 16;
        printf("{\"wa\": %d, \"wb\": %d", wa, wb);
        for (int depth : {2, 4}) {
            for (int blocks : {1024, 2048}) {
                double us = time([&] {
                    if (depth == 2) hipLaunchKernelGGL(k_read_floor<2>, dim3(blocks), dim3(256), 0, 0, buf, ld, wa + wb, n, p1);
                    else hipLaunchKernelGGL(k_read_floor<4>, dim3(blocks), dim3(256), 0, 0, buf, ld, wa + wb, n, p1);
                });
                printf(", \"floor_d%d_b%d\": %.0f", depth, blocks, gb / us);
            }
        }
        for (int run : {4, 8}) {
            for (int blocks : {512, 1024, 2048}) {
                const int R = 16 * run;
                if (blocks > (n + R - 1) / R) continue;
                auto go = [&](auto NTA_, auto RUN_) {
                    constexpr int NTA = decltype(NTA_)::value, RUN = decltype(RUN_)::value;
                    const size_t lds = std::max((size_t)2 * 16 * RUN * (16 * (NTA + 1) + 1), (size_t)3 * NTA * 64 * 4) * 8;
                    hipLaunchKernelGGL((k_gram_rows<NTA, RUN, false>), dim3(blocks), dim3(256), lds, 0, A, B, n, p1, 16 * NTA, 0);
                };
                using I1 = std::integral_constant<int, 1>;
                using I2 = std::integral_constant<int, 2>;
                using I3 = std::integral_constant<int, 3>;
                using I4 = std::integral_constant<int, 4>;
                using R4 = std::integral_constant<int, 4>;
                using R8 = std::integral_constant<int, 8>;
                double us = time([&] {
                    if (run == 4) {
                        if (nta == 1) go(I1{}, R4{}); else if (nta == 2) go(I2{}, R4{}); else if (nta == 3) go(I3{}, R4{}); else go(I4{}, R4{});
                    } else {
                        if (nta == 1) go(I1{}, R8{}); else if (nta == 2) go(I2{}, R8{}); else if (nta == 3) go(I3{}, R8{}); else go(I4{}, R8{});
                    }
                });
                printf(", \"rows_r%d_b%d\": %.0f", run, blocks, gb / us);
            }
        }
        if (nta >= 3) {
            GramPlan pl = gram_plan(wa, wb, n);
            double us = time([&] {
                if (nta == 3) launch_gram_lds<3, 8>(A, B, n, pl.blocks, p1, 0);
                else launch_gram_lds<4, 8>(A, B, n, pl.blocks, p1, 0);
            });
            printf(", \"lds_r8\": %.0f", gb / us);
        } else {
            double us = time([&] {
                if (nta == 1) hipLaunchKernelGGL((k_gram<1, 16>), dim3(2048), dim3(256), 0, 0, A, B, n, p1);
                else hipLaunchKernelGGL((k_gram<2, 16>), dim3(2048), dim3(256), 0, 0, A, B, n, p1);
            });
            printf(", \"k_gram\": %.0f", gb / us);
        }
        printf("}\n");
        fflush(stdout);
    }
    return 0;
}
