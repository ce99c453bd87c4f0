// host_check.cpp -- driver for the sanitized build of the library's host code
// ("Host: -fsanitize=address,undefined").  TEST INFRASTRUCTURE.
//
// Built by `make -C ca_lanczos_amd/csrc host-san` with g++ -fsanitize=address,
// undefined together with dense.cpp, leja.cpp, host_api.cpp and
// tsqr_plan.cpp (the library's index-heavy host code, no HIP), and driven by
// tests/test_host_sanitized.py: commands on stdin, results on stdout as
// %.17g (exact round trip), any sanitizer report ends the process non-zero.
//
//   leja n  x_re[n] x_im[n]            -> y_re[n] y_im[n] idx[n]
//   nbm s modifiedp  re[s] im[s]       -> B[(s+1)*s]
//   eig n  T[n*n]                      -> status wr[n] wi[n] V[n*n]
//   qrstep m mu  H[m*m] W[m*m]         -> H[m*m] W[m*m]
//   tridiag n  a[n] b[n-1]             -> status w[n]
//   chol m  G[m*m]                     -> ok R[m*m]
//   triinv m  R[m*m]                   -> Ri[m*m]
//   svd m  A[m*m]                      -> U[m*m] S[m] V[m*m]
//   rand count seed                    -> values[count]
//   plan n m TR form P me              -> checks the workspace layout; prints
//                                         need, levels, then per level
//                                         src rows tiles in up down S
#include <cstdio>
#include <cstdlib>
#include <iostream>
#include <string>
#include <vector>

#include "../../include/calanczos_host.h"
#include "../../ca_lanczos_amd/csrc/dense.hpp"
#include "../../ca_lanczos_amd/csrc/tsqr_plan.hpp"

namespace {

std::vector<double> readv(size_t n) {
    std::vector<double> v(n);
    for (size_t i = 0; i < n; ++i) std::cin >> v[i];
    return v;
}

void put(const double* v, size_t n) {
    for (size_t i = 0; i < n; ++i) std::printf("%.17g%c", v[i], i + 1 == n ? '\n' : ' ');
    if (n == 0) std::printf("\n");
}

void puti(const int* v, size_t n) {
    for (size_t i = 0; i < n; ++i) std::printf("%d%c", v[i], i + 1 == n ? '\n' : ' ');
    if (n == 0) std::printf("\n");
}

// every level's buffers inside [0, need), the UP / DOWN / gathered regions
// pairwise disjoint, each stack input the previous level's UP output (or the
// gathered region), each S the parent's DOWN output
int check_plan(const cal::TsqrPlan& p, int m, int P, int me) {
    const int64_t mm = (int64_t)m * m;
    struct R {
        int64_t a, b;
    };
    std::vector<R> regs;
    auto add = [&](int64_t off, int64_t len) {
        if (off < 0 || len < 0 || off + len > (int64_t)p.need) return false;
        regs.push_back({off, off + len});
        return true;
    };
    for (size_t l = 0; l < p.lv.size(); ++l) {
        const cal::TsqrLevelPlan& L = p.lv[l];
        if (L.tiles < 1 || L.rows < 1) return 1;
        if (!add(L.up, L.tiles * mm)) return 2;
        if (L.src == 0 && !add(L.down, (L.rows / m) * mm)) return 3;
        if (L.src != 0 && L.down != -1) return 4;
        if (P > 1 && l == p.nlocal && !add(L.in, (int64_t)P * mm)) return 5;
        if (l > 0 && !(P > 1 && l == p.nlocal) && L.in != p.lv[l - 1].up) return 6;
        if (l + 1 < p.lv.size() && l + 1 != p.nlocal && L.S != p.lv[l + 1].down) return 7;
        if (l > 0 && L.rows != p.lv[l - 1].tiles * m && !(P > 1 && l == p.nlocal)) return 8;
    }
    if (p.lv.back().tiles != 1 || p.lv.back().S != -1) return 9;
    if (P > 1) {
        if (p.lv[p.nlocal - 1].S != p.lv[p.nlocal].down + me * mm) return 10;
        if (p.lv[p.nlocal].rows != (int64_t)P * m || p.lv[p.nlocal - 1].tiles != 1) return 11;
    } else if (p.nlocal != p.lv.size()) {
        return 12;
    }
    for (size_t i = 0; i < regs.size(); ++i)
        for (size_t j = i + 1; j < regs.size(); ++j)
            if (regs[i].a < regs[j].b && regs[j].a < regs[i].b) return 13;
    return 0;
}

}  // namespace

int main() {
    std::string cmd;
    while (std::cin >> cmd) {
        if (cmd == "leja") {
            int n;
            std::cin >> n;
            auto re = readv(n), im = readv(n);
            std::vector<double> yr(n), yi(n);
            std::vector<int> idx(n);
            const int st = cal_leja(n, re.data(), im.data(), yr.data(), yi.data(), idx.data());
            std::printf("%d\n", st);
            put(yr.data(), n);
            put(yi.data(), n);
            puti(idx.data(), n);
        } else if (cmd == "nbm") {
            int s, mod;
            std::cin >> s >> mod;
            auto re = readv(s), im = readv(s);
            std::vector<double> B((size_t)(s + 1) * s);
            const int st = cal_newton_basis_matrix(s, re.data(), im.data(), mod, B.data());
            std::printf("%d\n", st);
            put(B.data(), B.size());
        } else if (cmd == "eig") {
            int n;
            std::cin >> n;
            auto T = readv((size_t)n * n);
            std::vector<double> wr(n), wi(n), V((size_t)n * n);
            const int st = cal_eig(n, T.data(), n, wr.data(), wi.data(), V.data());
            std::printf("%d\n", st);
            put(wr.data(), n);
            put(wi.data(), n);
            put(V.data(), V.size());
        } else if (cmd == "qrstep") {
            int m;
            double mu;
            std::cin >> m >> mu;
            auto H = readv((size_t)m * m), W = readv((size_t)m * m);
            const int st = cal_qrstep(m, H.data(), m, W.data(), m, mu);
            std::printf("%d\n", st);
            put(H.data(), H.size());
            put(W.data(), W.size());
        } else if (cmd == "eigsym") {  // vectors and values, then the values alone
            int n;
            std::cin >> n;
            auto T = readv((size_t)n * n);
            std::vector<double> w(n), w2(n), V((size_t)n * n);
            cal::dense::eig_symmetric(n, T.data(), n, w.data(), V.data(), n);
            cal::dense::eig_symmetric(n, T.data(), n, w2.data(), nullptr, n);
            std::printf("0\n");
            put(w.data(), n);
            put(w2.data(), n);
            put(V.data(), V.size());
        } else if (cmd == "qrsteps") {  // count batched steps, then the same one at a time
            int m, count;
            std::cin >> m >> count;
            auto mu = readv(count);
            auto H = readv((size_t)m * m), W = readv((size_t)m * m);
            auto H1 = H, W1 = W;
            cal::dense::hess_qrsteps(m, H.data(), m, W.data(), m, mu.data(), count);
            for (int t = 0; t < count; ++t) cal::dense::hess_qrstep(m, H1.data(), m, W1.data(), m, mu[t]);
            std::printf("0\n");
            put(H.data(), H.size());
            put(W.data(), W.size());
            put(H1.data(), H1.size());
            put(W1.data(), W1.size());
        } else if (cmd == "tridiag") {
            int n;
            std::cin >> n;
            auto a = readv(n), b = readv(n > 0 ? n - 1 : 0);
            std::vector<double> w(n);
            const int st = cal_tridiag_eigvals(n, a.data(), b.data(), w.data());
            std::printf("%d\n", st);
            put(w.data(), n);
        } else if (cmd == "chol") {
            int m;
            std::cin >> m;
            auto G = readv((size_t)m * m);
            std::vector<double> R((size_t)m * m, 0.0);
            const bool ok = cal::dense::chol_upper(m, G.data(), m, R.data(), m);
            std::printf("%d\n", ok ? 1 : 0);
            put(R.data(), R.size());
        } else if (cmd == "triinv") {
            int m;
            std::cin >> m;
            auto Rm = readv((size_t)m * m);
            std::vector<double> Ri((size_t)m * m, 0.0);
            cal::dense::tri_inv_upper(m, Rm.data(), m, Ri.data(), m);
            std::printf("0\n");
            put(Ri.data(), Ri.size());
        } else if (cmd == "svd") {
            int m;
            std::cin >> m;
            auto A = readv((size_t)m * m);
            std::vector<double> U((size_t)m * m), S(m), V((size_t)m * m);
            cal::dense::svd(m, A.data(), m, U.data(), S.data(), V.data());
            std::printf("0\n");
            put(U.data(), U.size());
            put(S.data(), S.size());
            put(V.data(), V.size());
        } else if (cmd == "rand") {
            long long count;
            unsigned seed;
            std::cin >> count >> seed;
            std::vector<double> v((size_t)count);
            const int st = cal_matlab_rand(count, seed, v.data());
            std::printf("%d\n", st);
            put(v.data(), v.size());
        } else if (cmd == "plan") {
            long long n, TR;
            int m, form, P, me;
            std::cin >> n >> m >> TR >> form >> P >> me;
            const cal::TsqrPlan p = cal::tsqr_plan(n, m, TR, form != 0, P, me);
            std::printf("%d\n", check_plan(p, m, P, me));
            std::printf("%zu %zu %zu\n", p.need, p.lv.size(), p.nlocal);
            for (const auto& L : p.lv)
                std::printf("%d %lld %lld %lld %lld %lld %lld\n", L.src, (long long)L.rows, (long long)L.tiles,
                            (long long)L.in, (long long)L.up, (long long)L.down, (long long)L.S);
        } else {
            std::fprintf(stderr, "unknown command %s\n", cmd.c_str());
            return 2;
        }
        std::fflush(stdout);
    }
    return 0;
}
