// Probe: a 17-column read sweep (the Gram sweeps' traffic, n = 215^3) at 8, 16 and 32 bytes per lane
// per column, one-shot grid and the persistent grid-stride form of k_rowapply (one-ahead prefetch).
// Output: one JSON line per variant, median of 20 timed launches.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <vector>

#define CK(x)                                                                 \
    do {                                                                      \
        hipError_t e_ = (x);                                                  \
        if (e_ != hipSuccess) {                                               \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            return 1;                                                         \
        }                                                                     \
    } while (0)

struct Col17 { const double* p[17]; };

template <int W>
struct VecT;
template <> struct VecT<1> { typedef double t; };
template <> struct VecT<2> { typedef double __attribute__((ext_vector_type(2))) t; };
template <> struct VecT<4> { typedef double __attribute__((ext_vector_type(4))) t; };

template <int W>
__device__ __forceinline__ double hsum(typename VecT<W>::t v) {
    if constexpr (W == 1) return v;
    else if constexpr (W == 2) return v[0] + v[1];
    else return (v[0] + v[1]) + (v[2] + v[3]);
}

// one-shot: one thread per W rows
template <int W>
__global__ __launch_bounds__(256) void k_rd(Col17 P, int64_t n, double* out) {
    typedef typename VecT<W>::t V;
    const int64_t r = ((int64_t)blockIdx.x * 256 + threadIdx.x) * W;
    if (r + W > n) return;
    double s = 0.0;
#pragma unroll
    for (int c = 0; c < 17; ++c) s += hsum<W>(*reinterpret_cast<const V*>(P.p[c] + r));
    if (s == 1.2345) out[0] = s;
}

// persistent grid-stride with a one-ahead prefetch of all 17 columns (k_rowapply's loop shape)
template <int W>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) void k_rd_gs(Col17 P, int64_t n,
                                                                                         double* out) {
    typedef typename VecT<W>::t V;
    const int64_t nch = n / (256 * W);
    V pn[17];
    auto load = [&](int64_t ci, V* dst) {
        const int64_t r = (ci * 256 + threadIdx.x) * W;
#pragma unroll
        for (int c = 0; c < 17; ++c) dst[c] = *reinterpret_cast<const V*>(P.p[c] + r);
    };
    double s = 0.0;
    if ((int64_t)blockIdx.x < nch) load(blockIdx.x, pn);
    for (int64_t ci = blockIdx.x; ci < nch; ci += gridDim.x) {
        asm volatile("" ::: "memory");
        V p[17];
#pragma unroll
        for (int c = 0; c < 17; ++c) p[c] = pn[c];
        if (ci + gridDim.x < nch) load(ci + gridDim.x, pn);
#pragma unroll
        for (int c = 0; c < 17; ++c) s += hsum<W>(p[c]);
    }
    if (s == 1.2345) out[0] = s;
}

template <typename F>
static float time_med(F launch, hipEvent_t a, hipEvent_t b) {
    for (int i = 0; i < 3; ++i) launch();
    std::vector<float> t;
    for (int i = 0; i < 20; ++i) {
        hipEventRecord(a, 0);
        launch();
        hipEventRecord(b, 0);
        hipEventSynchronize(b);
        float ms = 0;
        hipEventElapsedTime(&ms, a, b);
        t.push_back(ms);
    }
    std::sort(t.begin(), t.end());
    return t[t.size() / 2];
}

int main() {
    const int64_t n = (int64_t)215 * 215 * 215 / 1024 * 1024;  // a multiple of 1024 rows
    Col17 P;
    std::vector<double*> bufs(17);
    for (int c = 0; c < 17; ++c) {
        CK(hipMalloc(&bufs[c], n * 8));
        CK(hipMemset(bufs[c], 0x3f, n * 8));
        P.p[c] = bufs[c];
    }
    double* out;
    CK(hipMalloc(&out, 64));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    const double bytes = 17.0 * 8.0 * (double)n;
    auto report = [&](const char* name, float ms) {
        printf("{\"variant\": \"%s\", \"us\": %.1f, \"TBps\": %.3f}\n", name, ms * 1e3, bytes / (ms * 1e-3) / 1e12);
        fflush(stdout);
    };
    report("oneshot_8B", time_med([&] { hipLaunchKernelGGL(k_rd<1>, dim3(n / 256), dim3(256), 0, 0, P, n, out); }, a, b));
    report("oneshot_16B", time_med([&] { hipLaunchKernelGGL(k_rd<2>, dim3(n / 512), dim3(256), 0, 0, P, n, out); }, a, b));
    report("oneshot_32B", time_med([&] { hipLaunchKernelGGL(k_rd<4>, dim3(n / 1024), dim3(256), 0, 0, P, n, out); }, a, b));
    for (int g : {1024, 2048}) {
        char nm[64];
        snprintf(nm, sizeof nm, "gridstride_8B_g%d", g);
        report(nm, time_med([&] { hipLaunchKernelGGL(k_rd_gs<1>, dim3(g), dim3(256), 0, 0, P, n, out); }, a, b));
        snprintf(nm, sizeof nm, "gridstride_16B_g%d", g);
        report(nm, time_med([&] { hipLaunchKernelGGL(k_rd_gs<2>, dim3(g), dim3(256), 0, 0, P, n, out); }, a, b));
    }
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
    return 0;
}
