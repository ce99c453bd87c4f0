// host_api.cpp -- the host-only entry points of calanczos_host.h (no HIP):
// the T-matrix eigen-analysis (ca_lanczos.m:229), qrstep
// (impl_restarted_ca_lanczos.m:623-678), the prologue's tridiagonal eig and
// MATLAB's rand.  Built into libcalanczos.so with the rest, and on its own
// with g++ -fsanitize=address,undefined into the host checker
// (csrc/Makefile `host-san`, tests/test_host_sanitized.py), together with
// dense.cpp, leja.cpp and the TSQR tree plan.
#include <atomic>
#include <random>

#include "../../include/calanczos_host.h"
#include "dense.hpp"

using namespace cal;

extern "C" {

int cal_eig(int n, const double* T, int ldt, double* wr, double* wi, double* V) {
    if (n < 0 || !T || !wr || !wi || !V) return CAL_ERR_ARG;
    bool sym = true;
    for (int j = 0; j < n && sym; ++j)
        for (int i = 0; i < j; ++i)
            if (T[i + (size_t)j * ldt] != T[j + (size_t)i * ldt]) {
                sym = false;
                break;
            }
    if (sym) {
        dense::eig_symmetric(n, T, ldt, wr, V, n);
        for (int i = 0; i < n; ++i) wi[i] = 0.0;
        return 0;
    }
    return dense::eig_general(n, T, ldt, wr, wi, V, n) ? 0 : CAL_ERR_NUMERIC;
}

int cal_qrstep(int m, double* H, int ldh, double* W, int ldw, double mu) {
    if (m < 1 || !H || !W || ldh < m || ldw < m) return CAL_ERR_ARG;
    dense::hess_qrstep(m, H, ldh, W, ldw, mu);
    return 0;
}

int cal_tridiag_eigvals(int n, const double* alpha, const double* beta, double* w) {
    if (n < 0 || !alpha || (n > 1 && !beta) || !w) return CAL_ERR_ARG;
    return dense::tridiag_eigvals(n, alpha, beta, w) ? 0 : CAL_ERR_NUMERIC;
}

// MATLAB rand (MT19937 genrand_res53) of a fresh stream seeded `seed`
int cal_matlab_rand(int64_t count, unsigned seed, double* out) {
    if (count < 0 || (count > 0 && !out)) return CAL_ERR_ARG;
    std::mt19937 g(seed);
    dense::matlab_rand(g, count, out);
    return 0;
}

static std::atomic<long long> g_residency_gen{0};

long long cal_residency_generation(void) { return g_residency_gen.load(std::memory_order_acquire); }

long long cal_residency_invalidate(void) { return g_residency_gen.fetch_add(1, std::memory_order_acq_rel) + 1; }

}  // extern "C"
