// Probe: the s = 8 matrix powers of config 2 (lap2d_1000,
// n = 10^6, every power 8 MB, the whole chain Infinity-Cache resident) as
// eight dependent launches against ONE persistent launch whose blocks meet at
// a grid barrier between powers.  The SpMV is a plain 5-point stencil with the
// Newton shift (y = A x - l x, A = the Dirichlet Laplacian, one row per lane:
// the library's plane-march kernel moves the same 16 B per row), so the two
// forms differ only in what separates the powers.  Also timed: the grid
// barrier alone (eight barriers, no work) and one launch boundary alone (eight
// empty launches).  Not part of the library.
//   hipcc -O3 -std=c++17 -ffp-contract=off --offload-arch=gfx950 \
//         tools/persistent_powers_probe.hip -o tools/persistent_powers_probe
// Safety: the persistent grid is sized from the occupancy query so every block
// is resident, and every spin is bounded (a block that waits past the bound
// sets a flag and leaves): the kernel always drains.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

constexpr int S = 8;

__device__ __forceinline__ double stencil_row(const double* __restrict__ x, int64_t i, int N, int64_t n, double lam) {
    const int64_t r = i / N, c = i - r * N;
    double s = 0.0;
    if (r > 0) s = s - x[i - N];
    if (c > 0) s = s - x[i - 1];
    s = s + 4.0 * x[i];
    if (c < N - 1) s = s - x[i + 1];
    if (r < N - 1) s = s - x[i + N];
    const double t = lam * x[i];
    return s - t;
}

__global__ __launch_bounds__(256) void k_power(const double* __restrict__ x, double* __restrict__ y, int N, int64_t n,
                                               double lam) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n) y[i] = stencil_row(x, i, N, n, lam);
}

__global__ __launch_bounds__(256) void k_empty(int* __restrict__ p) {
    if (p && threadIdx.x == 0 && blockIdx.x == 0) p[0] = 0;
}

// sense-free barrier on a monotone generation word: the last arriver resets
// the count and bumps the generation; everybody else polls the generation
// (bounded).  Agent-scope release before arriving, acquire after leaving:
// the powers written on other XCDs reach this XCD's loads.
__device__ __forceinline__ void grid_barrier(unsigned* count, unsigned* gen, unsigned nblocks, unsigned target,
                                             unsigned* timeout_flag) {
    __syncthreads();
    if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        const unsigned prev = __hip_atomic_fetch_add(count, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
        if (prev == nblocks - 1) {
            __hip_atomic_store(count, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(gen, target, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        } else {
            unsigned spins = 0;
            while (__hip_atomic_load(gen, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) < target) {
                if (++spins > (1u << 22)) {
                    __hip_atomic_store(timeout_flag, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    }
    __syncthreads();
}

// the S powers in one launch: V[0] = q, V[j] = (A - lam_j) V[j-1]; grid-stride
// rows, a grid barrier after each power but the last
__global__ __launch_bounds__(256) void k_powers_persistent(double* __restrict__ V, int64_t ldv, int N, int64_t n,
                                                           const double* __restrict__ lam, unsigned* bar,
                                                           unsigned gen0, int work) {
    const unsigned nb = gridDim.x;
    for (int j = 1; j <= S; ++j) {
        if (work) {
            const double* x = V + (int64_t)(j - 1) * ldv;
            double* y = V + (int64_t)j * ldv;
            const double l = lam[j - 1];
            for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)nb * 256)
                y[i] = stencil_row(x, i, N, n, l);
        }
        if (j < S) grid_barrier(bar, bar + 1, nb, gen0 + (unsigned)j, bar + 2);
    }
}

int main() {
    int dev = 0, ncu = 0;
    CK(hipGetDevice(&dev));
    CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
    int occ = 0;
    CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k_powers_persistent, 256, 0));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    double lam_h[S];
    for (int j = 0; j < S; ++j) lam_h[j] = 0.5 + j;
    double* lam;
    CK(hipMalloc(&lam, sizeof lam_h));
    CK(hipMemcpy(lam, lam_h, sizeof lam_h, hipMemcpyHostToDevice));
    unsigned* bar;
    CK(hipMalloc(&bar, 64));
    CK(hipMemset(bar, 0, 64));
    unsigned gen = 0;
    for (int N : {1000, 2000, 3162}) {
        const int64_t n = (int64_t)N * N, ldv = (n + 63) / 64 * 64;
        double* V;
        CK(hipMalloc(&V, (size_t)(S + 1) * ldv * 8));
        std::vector<double> q(n);
        for (int64_t i = 0; i < n; ++i) q[i] = 1.0 / (1.0 + (double)(i % 977));
        CK(hipMemcpy(V, q.data(), n * 8, hipMemcpyHostToDevice));
        const int nblk = (int)((n + 255) / 256);
        auto chain = [&]() {
            for (int j = 1; j <= S; ++j)
                hipLaunchKernelGGL(k_power, dim3(nblk), dim3(256), 0, 0, V + (int64_t)(j - 1) * ldv,
                                   V + (int64_t)j * ldv, N, n, lam_h[j - 1]);
        };
        auto time = [&](auto f, int reps) -> double {
            for (int i = 0; i < 3; ++i) f();
            CK(hipDeviceSynchronize());
            CK(hipEventRecord(a));
            for (int i = 0; i < reps; ++i) f();
            CK(hipEventRecord(b));
            CK(hipEventSynchronize(b));
            float ms;
            CK(hipEventElapsedTime(&ms, a, b));
            return ms * 1e3 / reps;
        };
        const double t_chain = time(chain, 50);
        std::vector<double> ref((size_t)S * n);
        CK(hipMemcpy2D(ref.data(), n * 8, V + ldv, ldv * 8, n * 8, S, hipMemcpyDeviceToHost));
        printf("{\"N\": %d, \"n\": %lld, \"cus\": %d, \"occupancy\": %d, \"eight_launches_us\": %.2f", N, (long long)n,
               ncu, occ, t_chain);
        for (int per_cu : {1, 2, 4}) {
            if (per_cu > occ) continue;
            const int grid = ncu * per_cu;
            CK(hipMemset(V + ldv, 0, (size_t)S * ldv * 8));
            auto pers = [&](int work) {
                return [&, work]() {
                    hipLaunchKernelGGL(k_powers_persistent, dim3(grid), dim3(256), 0, 0, V, ldv, N, n, lam, bar, gen,
                                       work);
                    gen += S - 1;
                };
            };
            const double t_p = time(pers(1), 50);
            std::vector<double> got((size_t)S * n);
            CK(hipMemcpy2D(got.data(), n * 8, V + ldv, ldv * 8, n * 8, S, hipMemcpyDeviceToHost));
            unsigned flags[3];
            CK(hipMemcpy(flags, bar, sizeof flags, hipMemcpyDeviceToHost));
            const bool same = got == ref;
            const double t_b = time(pers(0), 50);
            printf(", \"persistent_%dpercu_us\": %.2f, \"bitwise_equal_%d\": %s, \"barriers_only_%dpercu_us\": %.2f, "
                   "\"timeout_%d\": %u",
                   per_cu, t_p, per_cu, same ? "true" : "false", per_cu, t_b, per_cu, flags[2]);
            if (flags[2]) {  // a bounded spin expired: stop here
                printf("}\n");
                return 1;
            }
        }
        const double t_empty = time([&]() {
            for (int j = 0; j < S; ++j) hipLaunchKernelGGL(k_empty, dim3(nblk), dim3(256), 0, 0, (int*)nullptr);
        }, 50);
        printf(", \"eight_empty_launches_us\": %.2f, \"bytes_per_power\": %lld}\n", t_empty, (long long)(16 * n));
        fflush(stdout);
        CK(hipFree(V));
    }
    return 0;
}
