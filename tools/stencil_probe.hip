// Probe: what a 7-point gather SpMV can reach on this GPU (n = 215^3), to
// bound the row-pattern SpMV.  Not part of the library.
//   hipcc -O3 --offload-arch=gfx950 tools/stencil_probe.hip -o /tmp/probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

__global__ void k_copy(const double* __restrict__ x, double* __restrict__ y, int64_t n) {
    int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (r < n) y[r] = x[r];
}
__global__ void k_copy2(const double* __restrict__ x, double* __restrict__ y, int64_t n) {
    int64_t r = 2 * ((int64_t)blockIdx.x * 256 + threadIdx.x);
    if (r + 1 < n) {
        double2 v = *reinterpret_cast<const double2*>(x + r);
        *reinterpret_cast<double2*>(y + r) = v;
    }
}
// fixed 7-point stencil on an origin-offset x (halo of N*N each side)
template <bool IDS>
__global__ void k_st7(const double* __restrict__ x, double* __restrict__ y, const uint16_t* __restrict__ id,
                      int64_t n, int N) {
    int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (r >= n) return;
    const int64_t P = (int64_t)N * N;
    double s = 6.0 * x[r] - x[r - 1] - x[r + 1] - x[r - N] - x[r + N] - x[r - P] - x[r + P];
    if (IDS) s += (double)id[r];
    y[r] = s;
}
// two rows per lane, 16-B x/y accesses where aligned
__global__ void k_st7x2(const double* __restrict__ x, double* __restrict__ y, int64_t n, int N) {
    int64_t r = 2 * ((int64_t)blockIdx.x * 256 + threadIdx.x);
    if (r + 1 >= n) return;
    const int64_t P = (int64_t)N * N;
    double2 c = *reinterpret_cast<const double2*>(x + r);
    double2 zm = *reinterpret_cast<const double2*>(x + r - P);
    double2 zp = *reinterpret_cast<const double2*>(x + r + P);
    double l = x[r - 1], rr = x[r + 2];
    double ym0 = x[r - N], ym1 = x[r + 1 - N], yp0 = x[r + N], yp1 = x[r + 1 + N];
    double2 o;
    o.x = 6.0 * c.x - l - c.y - ym0 - yp0 - zm.x - zp.x;
    o.y = 6.0 * c.y - c.x - rr - ym1 - yp1 - zm.y - zp.y;
    *reinterpret_cast<double2*>(y + r) = o;
}

// generic gather kernel: NO offsets from `off`, optional XCD-contiguous block order
struct Offs { int64_t d[8]; };
template <int NO, bool XCD>
__global__ void k_gen(const double* __restrict__ x, double* __restrict__ y, int64_t n, Offs off) {
    int b = blockIdx.x;
    if (XCD) {
        const int G = gridDim.x, q = G >> 3, rm = G & 7, xi = b & 7, i = b >> 3;
        b = (xi < rm ? xi * (q + 1) : rm * (q + 1) + (xi - rm) * q) + i;
    }
    int64_t r = (int64_t)b * 256 + threadIdx.x;
    if (r >= n) return;
    double s = 0.0;
#pragma unroll
    for (int e = 0; e < NO; ++e) s += x[r + off.d[e]];
    y[r] = s;
}

// k_gen<7, XCD> plus a 2-B id per row (added), and/or a persistent grid
// sweeping the XCD's chunk range interleaved (as k_spmv_pat_lds)
template <bool IDS, bool PERSIST>
__global__ void k_gen7x(const double* __restrict__ x, double* __restrict__ y, const uint16_t* __restrict__ id,
                        int64_t n, Offs off, int nchunk) {
    const int G = gridDim.x, q = G >> 3, rm = G & 7, xi = blockIdx.x & 7, i = blockIdx.x >> 3;
    const int nbx = q + (xi < rm ? 1 : 0);
    const int b0 = xi < rm ? xi * (q + 1) : rm * (q + 1) + (xi - rm) * q;
    int c0, c1, cs;
    if (PERSIST) {
        c0 = (int)((int64_t)nchunk * b0 / G) + i;
        c1 = (int)((int64_t)nchunk * (b0 + nbx) / G);
        cs = nbx;
    } else {
        c0 = b0 + i;
        c1 = c0 + 1;
        cs = 1;
    }
    for (int c = c0; c < c1; c += cs) {
        const int64_t r = (int64_t)c * 256 + threadIdx.x;
        if (r >= n) break;
        double s = IDS ? (double)id[r] : 0.0;
#pragma unroll
        for (int e = 0; e < 7; ++e) s += x[r + off.d[e]];
        y[r] = s;
    }
}

// 2 rows per lane (r even), every offset one 16-B load (8-B aligned when the
// offset is odd), XCD-contiguous block order
template <bool XCD>
__global__ void k_gen7_pair(const double* __restrict__ x, double* __restrict__ y, int64_t n, Offs off) {
    int b = blockIdx.x;
    if (XCD) {
        const int G = gridDim.x, q = G >> 3, rm = G & 7, xi = b & 7, i = b >> 3;
        b = (xi < rm ? xi * (q + 1) : rm * (q + 1) + (xi - rm) * q) + i;
    }
    const int64_t r = 2 * ((int64_t)b * 256 + threadIdx.x);
    if (r + 1 >= n) return;
    double s0 = 0.0, s1 = 0.0;
#pragma unroll
    for (int e = 0; e < 7; ++e) {
        const double* p = x + r + off.d[e];
        double2 v;
        __builtin_memcpy(&v, p, 16);
        s0 += v.x;
        s1 += v.y;
    }
    double2 o;
    o.x = s0;
    o.y = s1;
    *reinterpret_cast<double2*>(y + r) = o;
}

// pair kernel with the table machinery of k_spmv_pair: per-pair uint16 id,
// LDS (offset code, value pair) table, MODE-1 centre load; ID: load ids,
// TAB: offsets/values from the LDS table (else from kernel args)
template <bool ID, bool TAB, bool CENTER, bool GFILL = false, bool NTST = false>
__global__ __launch_bounds__(256) void k_pairtab(const double* __restrict__ x, double* __restrict__ y,
                                                 const uint16_t* __restrict__ ids, int64_t n, Offs off,
                                                 const int* __restrict__ gtab_off = nullptr,
                                                 const double2* __restrict__ gtab_v = nullptr) {
    __shared__ int s_off[256];
    __shared__ double2 s_v[256];
    if (GFILL) {  // stage a 256-entry table (4.6 KB) from global memory, as k_spmv_pair does
        s_off[threadIdx.x] = gtab_off[threadIdx.x];
        s_v[threadIdx.x] = gtab_v[threadIdx.x];
    } else if (threadIdx.x < 7) {
        s_off[threadIdx.x] = (int)off.d[threadIdx.x] * 4 + 3;
        s_v[threadIdx.x] = make_double2(threadIdx.x == 3 ? 6.0 : -1.0, threadIdx.x == 3 ? 6.0 : -1.0);
    }
    __syncthreads();
    const int G = gridDim.x, q = G >> 3, rm = G & 7, xi = blockIdx.x & 7, i = blockIdx.x >> 3;
    const int b = (xi < rm ? xi * (q + 1) : rm * (q + 1) + (xi - rm) * q) + i;
    const int64_t t = (int64_t)b * 256 + threadIdx.x;
    const int64_t r = 2 * t;
    if (r + 1 >= n) return;
    int base = 0;
    if (ID) base = ids[t];  // 0
    double y0 = 0.0, y1 = 0.0;
    int code[7];
    double2 xv[7];
#pragma unroll
    for (int e = 0; e < 7; ++e) {
        code[e] = TAB ? s_off[base + e] : (int)off.d[e] * 4 + 3;
        double2 v;
        __builtin_memcpy(&v, x + r + (code[e] >> 2), 16);
        xv[e] = v;
    }
#pragma unroll
    for (int e = 0; e < 7; ++e) {
        const double2 v = TAB ? s_v[base + e] : make_double2(-1.0, -1.0);
        const double t0 = v.x * xv[e].x, t1 = v.y * xv[e].y;
        const double a0 = y0 + t0, a1 = y1 + t1;
        y0 = (code[e] & 1) ? a0 : y0;
        y1 = (code[e] & 2) ? a1 : y1;
    }
    if (CENTER) {
        double2 c;
        __builtin_memcpy(&c, x + r, 16);
        y0 -= 0.5 * c.x;
        y1 -= 0.5 * c.y;
    }
    if (NTST) {
        __builtin_nontemporal_store(y0, y + r);
        __builtin_nontemporal_store(y1, y + r + 1);
    } else {
        double2 o;
        o.x = y0;
        o.y = y1;
        *reinterpret_cast<double2*>(y + r) = o;
    }
}

// the streaming sweeps between the powers: 17 columns read (Gram-like) or
// 17 read + 8 written (apply-like); NTQ: non-temporal stores for all but the
// last output column
struct Col17 { const double* p[17]; };
struct Col8 { double* p[8]; };
template <bool STORE, bool NTQ>
__global__ __launch_bounds__(256) void k_sweep17(Col17 P, Col8 Y, int64_t n) {
    const int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (r >= n) return;
    double v[17];
#pragma unroll
    for (int c = 0; c < 17; ++c) v[c] = P.p[c][r];
    double acc[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        acc[j] = 0;
#pragma unroll
        for (int c = 0; c < 17; ++c) acc[j] += v[c] * (0.01 * (c + j));
    }
    if (STORE) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            if (NTQ && j < 7) __builtin_nontemporal_store(acc[j], Y.p[j] + r);
            else Y.p[j][r] = acc[j];
        }
    } else if (acc[0] == 1.2345) {
        Y.p[0][r] = acc[1];
    }
}

int main() {
    const int N = 215;
    const int64_t n = (int64_t)N * N * N, P = (int64_t)N * N;
    double *xb, *y;
    uint16_t* id;
    CK(hipMalloc(&xb, (n + 2 * P + 64) * 8));
    CK(hipMalloc(&y, n * 8));
    CK(hipMalloc(&id, n * 2));
    CK(hipMemset(xb, 0, (n + 2 * P + 64) * 8));
    CK(hipMemset(id, 0, n * 2));
    double* x = xb + P + 32;  // 256-B aligned origin
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    auto time = [&](const char* name, double bytes, auto launch) {
        for (int i = 0; i < 5; ++i) launch();
        hipEventRecord(a);
        const int reps = 100;
        for (int i = 0; i < reps; ++i) launch();
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        const double us = ms * 1e3 / reps;
        printf("{\"kernel\": \"%s\", \"us\": %.2f, \"GBps\": %.0f}\n", name, us, bytes / (us * 1e-6) / 1e9);
    };
    const int g1 = (int)((n + 255) / 256), g2 = (int)((n / 2 + 255) / 256);
    time("copy 8B/lane", 16.0 * n, [&] { hipLaunchKernelGGL(k_copy, dim3(g1), dim3(256), 0, 0, x, y, n); });
    time("copy 16B/lane", 16.0 * n, [&] { hipLaunchKernelGGL(k_copy2, dim3(g2), dim3(256), 0, 0, x, y, n); });
    time("st7 8B/lane", 16.0 * n, [&] { hipLaunchKernelGGL((k_st7<false>), dim3(g1), dim3(256), 0, 0, x, y, id, n, N); });
    time("st7+ids 8B/lane", 18.0 * n, [&] { hipLaunchKernelGGL((k_st7<true>), dim3(g1), dim3(256), 0, 0, x, y, id, n, N); });
    time("st7 2 rows/lane", 16.0 * n, [&] { hipLaunchKernelGGL(k_st7x2, dim3(g2), dim3(256), 0, 0, x, y, n, N); });
    auto gen = [&](const char* name, std::vector<int64_t> o, bool xcd) {
        Offs off{};
        for (size_t i = 0; i < o.size(); ++i) off.d[i] = o[i];
        const int no = (int)o.size();
        time(name, 16.0 * n, [&] {
            if (no == 1 && !xcd) hipLaunchKernelGGL((k_gen<1, false>), dim3(g1), dim3(256), 0, 0, x, y, n, off);
            if (no == 3 && !xcd) hipLaunchKernelGGL((k_gen<3, false>), dim3(g1), dim3(256), 0, 0, x, y, n, off);
            if (no == 3 && xcd) hipLaunchKernelGGL((k_gen<3, true>), dim3(g1), dim3(256), 0, 0, x, y, n, off);
            if (no == 5 && !xcd) hipLaunchKernelGGL((k_gen<5, false>), dim3(g1), dim3(256), 0, 0, x, y, n, off);
            if (no == 7 && !xcd) hipLaunchKernelGGL((k_gen<7, false>), dim3(g1), dim3(256), 0, 0, x, y, n, off);
            if (no == 7 && xcd) hipLaunchKernelGGL((k_gen<7, true>), dim3(g1), dim3(256), 0, 0, x, y, n, off);
        });
    };
    gen("gen c", {0}, false);
    gen("gen c,+-1", {-1, 0, 1}, false);
    gen("gen c,+-1 aligned-ish(0,+256,+512)", {0, 256, 512}, false);
    gen("gen c,+-N", {-N, 0, N}, false);
    gen("gen c,+-N xcd", {-N, 0, N}, true);
    gen("gen c,+-P", {-P, 0, P}, false);
    gen("gen c,+-P xcd", {-P, 0, P}, true);
    gen("gen c,+-1,+-N", {-N, -1, 0, 1, N}, false);
    gen("gen 7pt", {-P, -N, -1, 0, 1, N, P}, false);
    gen("gen 7pt xcd", {-P, -N, -1, 0, 1, N, P}, true);
    gen("gen 7 x aligned 0..6*64", {0, 64, 128, 192, 256, 320, 384}, false);
    {
        Offs off{};
        const int64_t o7[7] = {-P, -N, -1, 0, 1, N, P};
        for (int e = 0; e < 7; ++e) off.d[e] = o7[e];
        const int nch = g1;
        time("7pt pair 16B", 16.0 * n, [&] { hipLaunchKernelGGL((k_gen7_pair<false>), dim3(g2), dim3(256), 0, 0, x, y, n, off); });
        time("7pt pair 16B xcd", 16.0 * n, [&] { hipLaunchKernelGGL((k_gen7_pair<true>), dim3(g2), dim3(256), 0, 0, x, y, n, off); });
        time("pairtab none", 16.0 * n, [&] { hipLaunchKernelGGL((k_pairtab<false, false, false>), dim3(g2), dim3(256), 0, 0, x, y, id, n, off); });
        time("pairtab center", 16.0 * n, [&] { hipLaunchKernelGGL((k_pairtab<false, false, true>), dim3(g2), dim3(256), 0, 0, x, y, id, n, off); });
        time("pairtab ids", 17.0 * n, [&] { hipLaunchKernelGGL((k_pairtab<true, false, false>), dim3(g2), dim3(256), 0, 0, x, y, id, n, off); });
        time("pairtab lds", 16.0 * n, [&] { hipLaunchKernelGGL((k_pairtab<false, true, false>), dim3(g2), dim3(256), 0, 0, x, y, id, n, off); });
        time("pairtab ids+lds", 17.0 * n, [&] { hipLaunchKernelGGL((k_pairtab<true, true, false>), dim3(g2), dim3(256), 0, 0, x, y, id, n, off); });
        time("pairtab ids+lds+center", 17.0 * n, [&] { hipLaunchKernelGGL((k_pairtab<true, true, true>), dim3(g2), dim3(256), 0, 0, x, y, id, n, off); });
        {
            std::vector<int> ho(256, 0);
            std::vector<double2> hv(256, make_double2(0.0, 0.0));
            for (int e = 0; e < 7; ++e) {
                ho[e] = (int)o7[e] * 4 + 3;
                hv[e] = make_double2(e == 3 ? 6.0 : -1.0, e == 3 ? 6.0 : -1.0);
            }
            int* go;
            double2* gv;
            CK(hipMalloc(&go, 256 * 4));
            CK(hipMalloc(&gv, 256 * 16));
            CK(hipMemcpy(go, ho.data(), 256 * 4, hipMemcpyHostToDevice));
            CK(hipMemcpy(gv, hv.data(), 256 * 16, hipMemcpyHostToDevice));
            time("pairtab ids+lds+center gfill", 17.0 * n, [&] { hipLaunchKernelGGL((k_pairtab<true, true, true, true>), dim3(g2), dim3(256), 0, 0, x, y, id, n, off, go, gv); });
        }
        time("7pt xcd + ids", 18.0 * n, [&] { hipLaunchKernelGGL((k_gen7x<true, false>), dim3(g1), dim3(256), 0, 0, x, y, id, n, off, nch); });
        time("7pt xcd persistent 2048", 16.0 * n, [&] { hipLaunchKernelGGL((k_gen7x<false, true>), dim3(2048), dim3(256), 0, 0, x, y, id, n, off, nch); });
        time("7pt xcd persistent 2048 + ids", 18.0 * n, [&] { hipLaunchKernelGGL((k_gen7x<true, true>), dim3(2048), dim3(256), 0, 0, x, y, id, n, off, nch); });
        time("7pt xcd persistent 8192 + ids", 18.0 * n, [&] { hipLaunchKernelGGL((k_gen7x<true, true>), dim3(8192), dim3(256), 0, 0, x, y, id, n, off, nch); });
    }
    // in-loop emulation: 8 powers rotating through 9 vectors, then a Gram-like
    // read sweep, an apply-like read sweep and an apply sweep writing the new
    // block whose last column is the next q
    {
        const int64_t ldv = ((n + 2 * P + 64) + 63) / 64 * 64;
        double* pool;
        CK(hipMalloc(&pool, (size_t)(9 + 17) * ldv * 8));
        CK(hipMemset(pool, 0, (size_t)(9 + 17) * ldv * 8));
        auto V = [&](int j) { return pool + (size_t)j * ldv + P + 32; };
        auto Qc = [&](int j) { return pool + (size_t)(9 + j) * ldv + P + 32; };
        std::vector<int> ho(256, 0);
        std::vector<double2> hv(256, make_double2(0.0, 0.0));
        const int64_t o7[7] = {-P, -N, -1, 0, 1, N, P};
        Offs off{};
        for (int e = 0; e < 7; ++e) {
            off.d[e] = o7[e];
            ho[e] = (int)o7[e] * 4 + 3;
            hv[e] = make_double2(e == 3 ? 6.0 : -1.0, e == 3 ? 6.0 : -1.0);
        }
        int* go;
        double2* gv;
        CK(hipMalloc(&go, 256 * 4));
        CK(hipMalloc(&gv, 256 * 16));
        CK(hipMemcpy(go, ho.data(), 256 * 4, hipMemcpyHostToDevice));
        CK(hipMemcpy(gv, hv.data(), 256 * 16, hipMemcpyHostToDevice));
        std::vector<hipEvent_t> ev(12);
        for (auto& evk : ev) CK(hipEventCreate(&evk));
        const int masks[] = {0x00, 0xFF, 0x80, 0xC0, 0xE0, 0xF0, 0xF8, 0x81, 0xE1};
        for (int variant = 0; variant < (int)(sizeof(masks) / sizeof(int)); ++variant) {
            const int ntmask = masks[variant];
            const bool ntq = false;
            double acc[11] = {0};
            const int steps = 6;
            for (int stp = 0; stp < steps; ++stp) {
                CK(hipEventRecord(ev[0]));
                for (int j = 0; j < 8; ++j) {
                    if ((ntmask >> j) & 1)
                        hipLaunchKernelGGL((k_pairtab<true, true, true, true, true>), dim3(g2), dim3(256), 0, 0, V(j), V(j + 1), id, n, off, go, gv);
                    else
                        hipLaunchKernelGGL((k_pairtab<true, true, true, true, false>), dim3(g2), dim3(256), 0, 0, V(j), V(j + 1), id, n, off, go, gv);
                    CK(hipEventRecord(ev[j + 1]));
                }
                Col17 Pc;
                Col8 Yc;
                for (int c = 0; c < 9; ++c) Pc.p[c] = Qc(c);
                for (int c = 0; c < 8; ++c) Pc.p[9 + c] = V(c + 1);
                for (int c = 0; c < 7; ++c) Yc.p[c] = Qc(9 + c);
                Yc.p[7] = V(0);
                hipLaunchKernelGGL((k_sweep17<false, false>), dim3(g1), dim3(256), 0, 0, Pc, Yc, n);
                CK(hipEventRecord(ev[9]));
                hipLaunchKernelGGL((k_sweep17<false, false>), dim3(g1), dim3(256), 0, 0, Pc, Yc, n);
                CK(hipEventRecord(ev[10]));
                if (ntq) hipLaunchKernelGGL((k_sweep17<true, true>), dim3(g1), dim3(256), 0, 0, Pc, Yc, n);
                else hipLaunchKernelGGL((k_sweep17<true, false>), dim3(g1), dim3(256), 0, 0, Pc, Yc, n);
                CK(hipEventRecord(ev[11]));
                CK(hipEventSynchronize(ev[11]));
                if (stp == 0) continue;
                for (int k = 0; k < 11; ++k) {
                    float ms;
                    CK(hipEventElapsedTime(&ms, ev[k], ev[k + 1]));
                    acc[k] += ms * 1e3 / (steps - 1);
                }
            }
            double tot = 0;
            for (int k = 0; k < 11; ++k) tot += acc[k];
            printf("{\"inloop\": \"spmv nt mask 0x%02x\", \"spmv_us\": [", ntmask);
            for (int k = 0; k < 8; ++k) printf("%.1f%s", acc[k], k < 7 ? ", " : "");
            printf("], \"gram_us\": %.1f, \"gram2_us\": %.1f, \"apply_us\": %.1f, \"total_us\": %.1f}\n", acc[8], acc[9],
                   acc[10], tot);
        }
    }
    CK(hipDeviceSynchronize());
    return 0;
}
