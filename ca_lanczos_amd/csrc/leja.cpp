// leja.cpp -- Newton-basis set-up on the host:
// real_leja.m:18-87 -> count_multiplicities.m:5-41 -> modified_leja.m:24-196,
// and newton_basis_matrix.m:13-60.  Op-for-op restatement (including the
// capacity rescaling of modified_leja.m:95-117 and the final unscaling at
// :192) so the shifts are bit-identical to the oracle's for the same input.
#include <algorithm>
#include <cmath>
#include <complex>
#include <string>
#include <vector>

#include "../../include/calanczos_host.h"
#include "leja.hpp"

namespace cal {
namespace leja {

using cd = std::complex<double>;

static bool is_conj_pair(cd a, cd b) { return a.real() == b.real() && a.imag() == -b.imag() && a.imag() != 0; }

// |z| exactly as MATLAB/NumPy/glibc compute it (hypot); clang may lower
// std::abs(std::complex) to an inline sqrt(re^2 + im^2) that rounds differently.
static double cabs_h(cd z) { return std::hypot(z.real(), z.imag()); }

// permutation of MATLAB [~,ix] = sort(x) (stable; complex: |x| then angle)
static std::vector<int> sort_perm(const std::vector<cd>& x, bool cplx) {
    std::vector<int> idx(x.size());
    for (size_t i = 0; i < x.size(); ++i) idx[i] = (int)i;
    auto key_less = [&](int a, int b) {
        if (!cplx) return x[a].real() < x[b].real();
        const double aa = cabs_h(x[a]), ab = cabs_h(x[b]);
        if (aa != ab) return aa < ab;
        return std::atan2(x[a].imag(), x[a].real()) < std::atan2(x[b].imag(), x[b].real());
    };
    std::stable_sort(idx.begin(), idx.end(), key_less);
    return idx;
}

static int first_max(const std::vector<double>& v) {
    int bi = -1;
    double best = 0.0;
    for (size_t i = 0; i < v.size(); ++i) {
        if (std::isnan(v[i])) continue;
        if (bi < 0 || v[i] > best) {
            best = v[i];
            bi = (int)i;
        }
    }
    return bi < 0 ? 0 : bi;
}

int count_multiplicities(const std::vector<cd>& x, int n, bool cplx, std::vector<cd>& y, std::vector<double>& mults) {
    const std::vector<int> p = sort_perm(x, cplx);
    std::vector<cd> xs(x.size());
    for (size_t i = 0; i < x.size(); ++i) xs[i] = x[p[i]];
    std::vector<int> ii;
    y.clear();
    for (size_t i = 0; i < xs.size(); ++i)
        if (i == 0 || xs[i] != xs[i - 1]) {
            y.push_back(xs[i]);
            ii.push_back((int)i);
        }
    const int nu = (int)y.size();
    mults.assign(nu, 1.0);
    if (nu == n) return nu;  // count_multiplicities.m:18-21
    for (int k = 0; k < nu - 1; ++k) mults[k] = ii[k + 1] - ii[k];
    mults[nu - 1] = n - ii[nu - 1];
    return nu;
}

static double seq_prod(const std::vector<double>& v) {
    double p = 1.0;
    for (double t : v) p = p * t;
    return p;
}

int modified_leja(std::vector<cd> x, int n, const std::vector<double>& mults, std::vector<cd>& y,
                  std::vector<int>& outidx, std::string& err) {
    if ((int)x.size() < n) {
        err = "modified_leja: fewer unique shifts than n (repeated shifts)";
        return -1;
    }
    y.clear();
    outidx.clear();
    if (n < 1) return 0;
    if (n == 1) {
        y.push_back(x[0]);
        outidx.push_back(0);
    } else {  // modified_leja_start (modified_leja.m:41-78)
        std::vector<double> ax(n);
        for (int i = 0; i < n; ++i) ax[i] = cabs_h(x[i]);
        const int j = first_max(ax);
        if (x[j].imag() == 0) {
            y.push_back(x[j]);
            outidx.push_back(j);
        } else if (j > 0 && is_conj_pair(x[j - 1], x[j])) {
            if (x[j - 1].imag() < 0) {
                err = "Complex conjugate pair out of order";
                return -1;
            }
            y = {x[j - 1], x[j]};
            outidx = {j - 1, j};
        } else if (j < n - 1 && is_conj_pair(x[j], x[j + 1])) {
            if (x[j].imag() < 0) {
                x[j] = cd(x[j].real(), 0.0);
                x[j + 1] = cd(x[j + 1].real(), 0.0);
            }
            y = {x[j], x[j + 1]};
            outidx = {j, j + 1};
        } else {
            err = j == 0 ? "Complex shift, not in a pair, occurs at beginning of input"
                         : "Complex shift, not in a pair, occurs at end of input";
            return -1;
        }
    }
    std::vector<int> inidx;
    for (int i = 0; i < n; ++i) {
        bool used = false;
        for (int o : outidx) used = used || (o == i);
        if (!used) inidx.push_back(i);
    }
    double capacity = 1.0;
    int num_points = (int)outidx.size();
    bool first = true;
    while (!inidx.empty()) {  // modified_leja_helper (modified_leja.m:80-181)
        if (!first && num_points > 1) {
            const double old_capacity = capacity;
            const cd y_last = y[num_points - 1];
            std::vector<double> terms;
            for (int t = 0; t < num_points - 1; ++t) {
                const int o = outidx[t];
                terms.push_back(std::pow(cabs_h(y_last - x[o]), mults[o] * (1.0 / num_points)));
            }
            capacity = seq_prod(terms);
            const double ratio = capacity / old_capacity;
            for (auto& v : x) v = v / ratio;
            for (auto& v : y) v = v / ratio;
        }
        first = false;
        std::vector<double> zprod;
        for (int j : inidx) {
            std::vector<double> terms;
            for (int o : outidx) terms.push_back(std::pow(cabs_h(x[j] - x[o]) / capacity, mults[o]));
            zprod.push_back(seq_prod(terms));
        }
        const int k = first_max(zprod);
        const double max_zprod = zprod[k];
        const int j = inidx[k];
        if (max_zprod == 0) {
            err = "Product to maximize is zero; either there are multiple shifts, or the product underflowed";
            return -1;
        }
        if (std::isinf(max_zprod)) {
            err = "Product to maximize is Inf; must have overflowed";
            return -1;
        }
        auto erase = [&](int v) {
            for (size_t i = 0; i < inidx.size(); ++i)
                if (inidx[i] == v) {
                    inidx.erase(inidx.begin() + i);
                    return;
                }
        };
        if (x[j].imag() == 0) {
            erase(j);
            outidx.push_back(j);
            y.push_back(x[j]);
            num_points += 1;
        } else if (j > 0 && is_conj_pair(x[j - 1], x[j])) {
            if (x[j - 1].imag() < 0) {
                err = "Complex conjugate pair out of order";
                return -1;
            }
            erase(j - 1);
            erase(j);
            outidx.push_back(j - 1);
            outidx.push_back(j);
            y.push_back(x[j - 1]);
            y.push_back(x[j]);
            num_points += 2;
        } else if (j < n - 1 && is_conj_pair(x[j], x[j + 1])) {
            if (x[j].imag() < 0) {
                err = "Complex conjugate pair out of order";
                return -1;
            }
            erase(j);
            erase(j + 1);
            outidx.push_back(j);
            outidx.push_back(j + 1);
            y.push_back(x[j]);
            y.push_back(x[j + 1]);
            num_points += 2;
        } else {
            err = "Complex shift, not in a pair";
            return -1;
        }
    }
    for (auto& v : y) v = v * capacity;  // modified_leja.m:192
    return 0;
}

int real_leja(const std::vector<cd>& x_in, std::vector<cd>& y, std::vector<int>& outidx, std::string& err) {
    const int n = (int)x_in.size();
    bool cplx = false;
    for (auto& v : x_in) cplx = cplx || v.imag() != 0;
    std::vector<cd> u;
    std::vector<double> mults;
    const int nu = count_multiplicities(x_in, n, cplx, u, mults);  // real_leja.m:44
    // stable sort by real part (real_leja.m:61-64)
    std::vector<cd> re(u.size());
    for (size_t i = 0; i < u.size(); ++i) re[i] = cd(u[i].real(), 0.0);
    const std::vector<int> p = sort_perm(re, false);
    std::vector<cd> ys(u.size());
    std::vector<double> ms(u.size());
    for (size_t i = 0; i < u.size(); ++i) {
        ys[i] = u[p[i]];
        ms[i] = mults[p[i]];
    }
    int k = 0;
    while (k < nu - 1) {  // real_leja.m:67-81
        if (ys[k].imag() != 0) {
            if (ys[k].real() == ys[k + 1].real() && ys[k].imag() == -ys[k + 1].imag()) {
                ys[k] = cd(ys[k].real(), std::fabs(ys[k].imag()));
                ys[k + 1] = cd(ys[k].real(), -std::fabs(ys[k].imag()));
                k += 2;
            } else {
                k += 1;  // reference prints 'Error in real_leja' and would spin; fail forward
            }
        } else {
            k += 1;
        }
    }
    return modified_leja(ys, n, ms, y, outidx, err);  // real_leja.m:86
}

int newton_basis_matrix(int s, const std::vector<cd>& lam, int modifiedp, std::vector<double>& B, std::string& err) {
    B.assign((size_t)(s + 1) * s, 0.0);
    auto at = [&](int i, int j) -> double& { return B[i + (size_t)j * (s + 1)]; };
    if ((int)lam.size() < s) {
        err = "newton_basis_matrix: fewer than s shifts";
        return -1;
    }
    for (int k = 0; k < s; ++k) {
        const cd shift = lam[k];
        if (modifiedp == 0) {
            if (shift.imag() != 0) {
                err = "newton_basis_matrix: complex shifts need the modified basis";
                return -1;
            }
            at(k, k) = shift.real();
        } else if (shift.imag() > 0) {
            if (k == s - 1) {
                err = "Complex shift occurs at end of shifts without its conjugate";
                return -1;
            }
            if (lam[k] != std::conj(lam[k + 1])) {
                err = "Modified Leja ordering broken";
                return -1;
            }
            at(k, k) = shift.real();
        } else if (shift.imag() < 0) {
            if (k == 0) {
                err = "newton_basis_matrix: imaginary part is negative for k = 1";
                return -1;
            }
            if (lam[k - 1] != std::conj(lam[k])) {
                err = "Modified Leja ordering broken";
                return -1;
            }
            at(k, k) = shift.real();
            at(k - 1, k) = -shift.imag() * shift.imag();
        } else {
            at(k, k) = shift.real();
        }
        at(k + 1, k) = 1.0;
    }
    return 0;
}

}  // namespace leja
}  // namespace cal

using namespace cal;

extern "C" {

int cal_leja(int n, const double* x_re, const double* x_im, double* y_re, double* y_im, int* outidx) {
    if (n < 0 || !x_re || !y_re) return CAL_ERR_ARG;
    std::vector<leja::cd> x(n);
    for (int i = 0; i < n; ++i) x[i] = leja::cd(x_re[i], x_im ? x_im[i] : 0.0);
    std::vector<leja::cd> y;
    std::vector<int> oi;
    std::string err;
    if (leja::real_leja(x, y, oi, err) != 0) return CAL_ERR_NUMERIC;
    for (size_t i = 0; i < y.size(); ++i) {
        y_re[i] = y[i].real();
        if (y_im) y_im[i] = y[i].imag();
        if (outidx) outidx[i] = oi[i];
    }
    return 0;
}

int cal_newton_basis_matrix(int s, const double* lam_re, const double* lam_im, int modifiedp, double* B) {
    if (s < 1 || !lam_re || !B) return CAL_ERR_ARG;
    std::vector<leja::cd> lam(s);
    for (int i = 0; i < s; ++i) lam[i] = leja::cd(lam_re[i], lam_im ? lam_im[i] : 0.0);
    std::vector<double> Bv;
    std::string err;
    if (leja::newton_basis_matrix(s, lam, modifiedp, Bv, err) != 0) return CAL_ERR_NUMERIC;
    for (size_t i = 0; i < Bv.size(); ++i) B[i] = Bv[i];
    return 0;
}

}  // extern "C"
