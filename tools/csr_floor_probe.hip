// Probe: the floor of the CSR SpMV's access pattern on lap3d_215 (n = 9.94 M,
// nnz = 68.6 M).  Times, with HIP events over 20 launches
// each (the 1 GB working set is 4x the Infinity Cache, so no flush is needed):
//   read    a contiguous read of 12 nnz + 16 n bytes (the CSR byte count: col,
//           val, x and rowptr/y), 16-B loads -- the HBM read rate;
//   colval  the col (int32) and val (f64) streams alone, 12 B per nonzero;
//   gather  col/val streams + x[col] gathers, sums per lane (no rows);
//   spmv    gather + the row structure: rowptr reads, one y store per row
//           (one row per lane, the simplest CSR kernel -- scalar CSR);
// and prints each as GB/s on the CSR's algorithmic bytes (12 nnz + 8 n x
// + 8 n y + 4 n rowptr), the unit of bench.py's spmv_csr_kernel.gbps.
// Not part of the library.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/csr_floor_probe.hip -o tools/csr_floor_probe
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

typedef double d2 __attribute__((ext_vector_type(2)));

__global__ __launch_bounds__(256) void k_read(const d2* __restrict__ a, int64_t n2, double* __restrict__ out) {
    double s = 0.0;
    const int64_t stride = (int64_t)gridDim.x * 256;
    int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    for (; i + 3 * stride < n2; i += 4 * stride) {
        const d2 v0 = __builtin_nontemporal_load(a + i), v1 = __builtin_nontemporal_load(a + i + stride);
        const d2 v2 = __builtin_nontemporal_load(a + i + 2 * stride), v3 = __builtin_nontemporal_load(a + i + 3 * stride);
        s += v0[0] + v0[1] + v1[0] + v1[1] + v2[0] + v2[1] + v3[0] + v3[1];
    }
    for (; i < n2; i += stride) s += a[i][0] + a[i][1];
    out[(int64_t)blockIdx.x * 256 + threadIdx.x] = s;
}

template <bool GATHER>
__global__ __launch_bounds__(256) void k_colval(const int* __restrict__ col, const double* __restrict__ val,
                                                const double* __restrict__ x, int64_t nnz, double* __restrict__ out) {
    double s = 0.0;
    const int64_t stride = (int64_t)gridDim.x * 256;
    int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    for (; i + 3 * stride < nnz; i += 4 * stride) {
        int c[4];
        double v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            c[u] = __builtin_nontemporal_load(col + i + u * stride);
            v[u] = __builtin_nontemporal_load(val + i + u * stride);
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) s += v[u] * (GATHER ? x[c[u]] : (double)c[u]);
    }
    for (; i < nnz; i += stride) s += val[i] * (GATHER ? x[col[i]] : (double)col[i]);
    out[(int64_t)blockIdx.x * 256 + threadIdx.x] = s;
}

__global__ __launch_bounds__(256) void k_scalar_csr(const int* __restrict__ rp, const int* __restrict__ col,
                                                    const double* __restrict__ val, const double* __restrict__ x,
                                                    int64_t n, double* __restrict__ y) {
    const int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (r >= n) return;
    double s = 0.0;
    for (int k = rp[r]; k < rp[r + 1]; ++k) s += val[k] * x[col[k]];
    y[r] = s;
}

int main() {
    const int N = 215;
    const int64_t n = (int64_t)N * N * N;
    std::vector<int> rp(n + 1);
    std::vector<int> ci;
    std::vector<double> cv;
    ci.reserve(7 * n);
    cv.reserve(7 * n);
    rp[0] = 0;
    for (int64_t r = 0; r < n; ++r) {
        const int i = r % N, j = (r / N) % N, k = r / ((int64_t)N * N);
        auto add = [&](int64_t c, double v) { ci.push_back((int)c); cv.push_back(v); };
        if (k > 0) add(r - (int64_t)N * N, -1.0);
        if (j > 0) add(r - N, -1.0);
        if (i > 0) add(r - 1, -1.0);
        add(r, 6.0);
        if (i < N - 1) add(r + 1, -1.0);
        if (j < N - 1) add(r + N, -1.0);
        if (k < N - 1) add(r + (int64_t)N * N, -1.0);
        rp[r + 1] = (int)ci.size();
    }
    const int64_t nnz = ci.size();
    int *drp, *dci;
    double *dcv, *dx, *dy, *dout, *dbig;
    CK(hipMalloc(&drp, (n + 1) * 4));
    CK(hipMalloc(&dci, nnz * 4));
    CK(hipMalloc(&dcv, nnz * 8));
    CK(hipMalloc(&dx, n * 8));
    CK(hipMalloc(&dy, n * 8));
    CK(hipMemcpy(drp, rp.data(), (n + 1) * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(dci, ci.data(), nnz * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(dcv, cv.data(), nnz * 8, hipMemcpyHostToDevice));
    {
        std::vector<double> hx(n);
        for (int64_t i = 0; i < n; ++i) hx[i] = (i % 1013) / 1013.0;
        CK(hipMemcpy(dx, hx.data(), n * 8, hipMemcpyHostToDevice));
    }
    const double alg = 12.0 * nnz + 8.0 * n + 8.0 * n + 4.0 * n;  // bench.py's CSR bytes
    const int64_t nbig2 = (int64_t)((12.0 * nnz + 16.0 * n) / 16);
    CK(hipMalloc(&dbig, nbig2 * 16));
    CK(hipMemset(dbig, 0, nbig2 * 16));
    CK(hipMalloc(&dout, (size_t)8192 * 256 * 8));
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
    printf("{\"n\": %lld, \"nnz\": %lld, \"alg_bytes\": %.0f", (long long)n, (long long)nnz, alg);
    for (int blocks : {2048, 4096, 8192}) {
        const double t = time([&] { hipLaunchKernelGGL(k_read, dim3(blocks), dim3(256), 0, 0, (const d2*)dbig, nbig2, dout); });
        printf(", \"read_b%d_us\": %.1f, \"read_b%d_GBps\": %.0f", blocks, t, blocks, nbig2 * 16.0 / t / 1e3);
    }
    for (int blocks : {2048, 4096, 8192}) {
        const double t = time([&] { hipLaunchKernelGGL(k_colval<false>, dim3(blocks), dim3(256), 0, 0, dci, dcv, dx, nnz, dout); });
        printf(", \"colval_b%d_us\": %.1f, \"colval_b%d_GBps\": %.0f", blocks, t, blocks, 12.0 * nnz / t / 1e3);
    }
    for (int blocks : {2048, 4096, 8192}) {
        const double t = time([&] { hipLaunchKernelGGL(k_colval<true>, dim3(blocks), dim3(256), 0, 0, dci, dcv, dx, nnz, dout); });
        printf(", \"gather_b%d_us\": %.1f, \"gather_b%d_algGBps\": %.0f", blocks, t, blocks, (12.0 * nnz + 8.0 * n) / t / 1e3);
    }
    {
        const double t = time([&] {
            hipLaunchKernelGGL(k_scalar_csr, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, 0, drp, dci, dcv, dx, n, dy);
        });
        printf(", \"scalar_csr_us\": %.1f, \"scalar_csr_algGBps\": %.0f", t, alg / t / 1e3);
    }
    printf("}\n");
    return 0;
}
