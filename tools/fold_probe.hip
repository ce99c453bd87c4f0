// Probe: the fused-TSQR kernels (ca_lanczos_amd/csrc/tsqr_fold.hip) at the
// bench's shape (n = 215^3 rows, Qp 9 columns, X 8 columns), timed with HIP
// events, with FOLD_PROBE switching parts of k_fold_up off (see kProbe).
// Not part of the library.  Build (one binary per switch value):
//   hipcc -O3 -std=c++17 -ffp-contract=off --offload-arch=gfx950 -Iinclude \
//     -mllvm -pragma-unroll-threshold=4000000 -DFOLD_PROBE=<bits> tools/fold_probe.hip -o tools/fold_probe_<bits>
#include "../ca_lanczos_amd/csrc/tsqr_fold.hip"

#include <cstdio>
#include <vector>

#define CK(x)                                                                      \
    do {                                                                           \
        hipError_t e_ = (x);                                                       \
        if (e_ != hipSuccess) {                                                    \
            printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__);           \
            return 1;                                                              \
        }                                                                          \
    } while (0)

__global__ void k_fill(double* p, int64_t cnt, unsigned long long seed, double scale) {
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < cnt; i += (int64_t)gridDim.x * 256) {
        unsigned long long z = (unsigned long long)i * 0x9E3779B97F4A7C15ull + seed;
        z ^= z >> 31;
        z *= 0xBF58476D1CE4E5B9ull;
        z ^= z >> 29;
        p[i] = scale * ((double)(z >> 11) * 0x1p-53 - 0.5);
    }
}

int main(int argc, char** argv) {
    using namespace cal;
    const int64_t n = 9938375;
    const int m = 8, w = 9, reps = 30;
    const int64_t ld = (n + 63) / 64 * 64;
    double *P, *Q, *F;
    CK(hipMalloc((void**)&P, (size_t)17 * ld * sizeof(double)));
    CK(hipMalloc((void**)&Q, (size_t)8 * ld * sizeof(double)));
    const int64_t n0 = fold_tiles(n), nblk = fold_blocks(n);
    const std::vector<int> nu = fold_levels(n);
    size_t off = 0;
    auto take = [&](size_t cnt) {
        const size_t o = off;
        off += (cnt + 7) & ~size_t(7);
        return o;
    };
    const size_t t0 = fold_l0_tile_doubles(), tu = fold_tile_doubles();
    const size_t oV0 = take(n0 * t0), otb0 = take(n0 * 16), oR0 = take(n0 * 64);
    size_t oVu[3], oRu[3], oMu[3];
    for (size_t L = 0; L < nu.size(); ++L) {
        oVu[L] = take((size_t)nu[L] * tu);
        oRu[L] = take((size_t)nu[L] * 64);
        oMu[L] = take((size_t)nu[L] * 64);
    }
    const size_t oRrm = take(64), oK = take(72), oOut = take(520), oPart = take((size_t)272 * nblk);
    const size_t oT1 = take(272), oG = take(72), oSb = take(64), oSm = take(64), oRt = take(64);
    CK(hipMalloc((void**)&F, off * sizeof(double)));
    hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, P, (int64_t)17 * ld, 1ull, 1.0);
    hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, F, (int64_t)off, 7ull, 0.2);
    CK(hipDeviceSynchronize());
    std::vector<double> flags(520, 0.0);
    flags[514] = 1.0;
    CK(hipMemcpy(F + oOut, flags.data(), 520 * sizeof(double), hipMemcpyHostToDevice));
    FoldArgs fa;
    fa.n = n;
    fa.m = m;
    fa.w = w;
    fa.nblk = (int)nblk;
    fa.n0 = (int)n0;
    fa.nlev = (int)nu.size();
    fa.C = F + oOut;  // any 272 doubles stand in for the P1 tile
    fa.flags = F + oOut + 512;
    fa.K = F + oK;
    fa.V0 = F + oV0;
    fa.tb0 = F + otb0;
    fa.R0 = F + oR0;
    for (size_t L = 0; L < nu.size(); ++L) {
        fa.nu[L] = nu[L];
        fa.Vu[L] = F + oVu[L];
        fa.Ru[L] = F + oRu[L];
        fa.Mu[L] = F + oMu[L];
    }
    fa.Stop = F + oRrm;
    fa.lds = 8;
    fa.Rroot_m = F + oRrm;
    fa.partial = F + oPart;
    ColList cu{};
    for (int k = 0; k < 17; ++k) cu.p[k] = P + (size_t)k * ld;
    OutList qo{};
    for (int j = 0; j < 16; ++j) qo.p[j] = Q + (size_t)(j < 8 ? j : 0) * ld;
    hipStream_t st;
    CK(hipStreamCreate(&st));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    auto timeit = [&](const char* name, double bytes, auto&& launch) -> int {
        for (int i = 0; i < 5; ++i) CK(launch());
        float tot = 0.0f, mn = 1e30f;
        for (int i = 0; i < reps; ++i) {
            CK(hipEventRecord(a, st));
            CK(launch());
            CK(hipEventRecord(b, st));
            CK(hipEventSynchronize(b));
            float ms;
            CK(hipEventElapsedTime(&ms, a, b));
            tot += ms;
            mn = ms < mn ? ms : mn;
        }
        const double avg = tot / reps;
        printf("probe=%d wpe=%d/%d %-10s avg %8.1f us  min %8.1f us  %6.2f TB/s (algorithmic %.3f GB)\n", FOLD_PROBE, FOLD_UP_WPE, FOLD_DOWN_WPE, name,
               avg * 1e3, mn * 1e3, bytes / (avg * 1e-3) / 1e12, bytes / 1e9);
        return 0;
    };
    const double b_up = 25.0 * 8.0 * n, b_down = 25.0 * 8.0 * n;
    if (timeit("up", b_up, [&] { return launch_fold_up(cu, fa, st); })) return 1;
    if (timeit("tree", 0.0, [&] { return launch_fold_tree(fa, st); })) return 1;
    {
        FoldArgs fred = fa;  // level 1 also reducing the C2 partials
        fred.red_out = F + oG;
        if (timeit("tree_red", 0.0, [&] { return launch_fold_tree(fred, st); })) return 1;
    }
    if (timeit("down", b_down, [&] { return launch_fold_down(cu, qo, fa, st); })) return 1;
    // the coefficient step on inputs that take its whole path (second
    // projection, Cholesky, no decline): X'X = I on the diagonal, C = 0.9,
    // C2 = 1e-8, root R = 2 I + 0.1 strictly upper
    {
        std::vector<double> t1(272, 0.0), g(72, 1e-8), rt(64, 0.0);
        for (int j = 0; j < 8; ++j) {
            t1[(8 + j) + (8 + j) * 16] = 1.0;
            for (int i = 0; i < 8; ++i) t1[i + (8 + j) * 16] = 0.9 / 3.0;
            t1[256 + 8 + j] = 0.9 / 3.0;
            for (int i = 0; i <= j; ++i) rt[i + j * 8] = i == j ? 2.0 : 0.1;
        }
        CK(hipMemcpy(F + oT1, t1.data(), 272 * 8, hipMemcpyHostToDevice));
        CK(hipMemcpy(F + oG, g.data(), 72 * 8, hipMemcpyHostToDevice));
        CK(hipMemcpy(F + oRt, rt.data(), 64 * 8, hipMemcpyHostToDevice));
    }
    double* hpin = nullptr;
    CK(hipHostMalloc((void**)&hpin, 1024 * sizeof(double), hipHostMallocDefault));
    unsigned long long* hseq = reinterpret_cast<unsigned long long*>(hpin + 516);
    unsigned long long sq = 0;
    if (timeit("coef1", 0.0, [&] {
            return launch_fold_coef1(F + oT1, F + oG, F + oRt, 8, F + oOut, F + oSb, F + oSm, F + oK, w, m, 1,
                                     (double)n, kFoldTol, nullptr, nullptr, 0, st);
        }))
        return 1;
    if (timeit("coef1_pub", 0.0, [&] {
            return launch_fold_coef1(F + oT1, F + oG, F + oRt, 8, F + oOut, F + oSb, F + oSm, F + oK, w, m, 1,
                                     (double)n, kFoldTol, hpin, hseq, ++sq, st);
        }))
        return 1;
    if (timeit("root_pub", 0.0, [&] {
            return launch_fold_root(fa, F + oT1, F + oG, F + oOut, F + oSb, F + oSm, F + oK, w, 1, (double)n, hpin,
                                    hseq, ++sq, st);
        }))
        return 1;
    if (timeit("root", 0.0, [&] {
            return launch_fold_root(fa, F + oT1, F + oG, F + oOut, F + oSb, F + oSm, F + oK, w, 1, (double)n,
                                    nullptr, nullptr, 0, st);
        }))
        return 1;
    {
        std::vector<double> o(520);
        CK(hipMemcpy(o.data(), F + oOut, 520 * 8, hipMemcpyDeviceToHost));
        printf("coef flags: reorth %g fail %g est %g\n", o[514], o[513], o[515]);
    }
    FoldArgs fr = fa;
    fr.V0 = nullptr;  // up without the tile store
    if (timeit("up_nost", 17.0 * 8.0 * n, [&] { return launch_fold_up(cu, fr, st); })) return 1;
    CK(hipDeviceSynchronize());
    return 0;
}
