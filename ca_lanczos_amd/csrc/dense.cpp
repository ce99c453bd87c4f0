// dense.cpp -- small dense host linear algebra (see dense.hpp).
#include "dense.hpp"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <vector>

namespace cal {
namespace dense {

bool chol_upper(int m, const double* G, int ldg, double* R, int ldr) {
    for (int j = 0; j < m; ++j)
        for (int i = 0; i < m; ++i) R[i + (size_t)j * ldr] = 0.0;
    for (int j = 0; j < m; ++j) {
        double s = G[j + (size_t)j * ldg];
        for (int k = 0; k < j; ++k) s -= R[k + (size_t)j * ldr] * R[k + (size_t)j * ldr];
        if (!(s > 0.0) || !std::isfinite(s)) return false;
        const double rjj = std::sqrt(s);
        R[j + (size_t)j * ldr] = rjj;
        for (int i = j + 1; i < m; ++i) {
            double t = G[j + (size_t)i * ldg];
            for (int k = 0; k < j; ++k) t -= R[k + (size_t)j * ldr] * R[k + (size_t)i * ldr];
            R[j + (size_t)i * ldr] = t / rjj;
        }
    }
    return true;
}

void tri_inv_upper(int m, const double* R, int ldr, double* Ri, int ldi) {
    for (int j = 0; j < m; ++j)
        for (int i = 0; i < m; ++i) Ri[i + (size_t)j * ldi] = 0.0;
    // solve R * Ri(:,j) = e_j by back substitution
    for (int j = 0; j < m; ++j) {
        for (int i = j; i >= 0; --i) {
            double s = (i == j) ? 1.0 : 0.0;
            for (int k = i + 1; k <= j; ++k) s -= R[i + (size_t)k * ldr] * Ri[k + (size_t)j * ldi];
            Ri[i + (size_t)j * ldi] = s / R[i + (size_t)i * ldr];
        }
    }
}

void matmul(int m, int k, int n, const double* A, int lda, const double* B, int ldb, double* C, int ldc) {
    std::vector<double> tmp((size_t)m * n, 0.0);
    for (int j = 0; j < n; ++j)
        for (int i = 0; i < m; ++i) {
            double s = 0.0;
            for (int p = 0; p < k; ++p) s += A[i + (size_t)p * lda] * B[p + (size_t)j * ldb];
            tmp[i + (size_t)j * m] = s;
        }
    for (int j = 0; j < n; ++j)
        for (int i = 0; i < m; ++i) C[i + (size_t)j * ldc] = tmp[i + (size_t)j * m];
}

void rdiv_upper(int r, int m, double* X, int ldx, const double* R, int ldr) {
    // Y R = X  ->  Y(:,j) = (X(:,j) - sum_{k<j} Y(:,k) R(k,j)) / R(j,j)
    for (int j = 0; j < m; ++j) {
        for (int i = 0; i < r; ++i) {
            double s = X[i + (size_t)j * ldx];
            for (int k = 0; k < j; ++k) s -= X[i + (size_t)k * ldx] * R[k + (size_t)j * ldr];
            X[i + (size_t)j * ldx] = s / R[j + (size_t)j * ldr];
        }
    }
}

bool tridiag_eigvals(int n, const double* dd, const double* ee, double* w) {
    if (n <= 0) return true;
    std::vector<double> d(dd, dd + n), e(n, 0.0);
    for (int i = 0; i < n - 1; ++i) e[i] = ee[i];
    const double eps = std::ldexp(1.0, -52);
    for (int l = 0; l < n; ++l) {
        int iter = 0, m;
        do {
            for (m = l; m < n - 1; ++m) {
                const double dd2 = std::fabs(d[m]) + std::fabs(d[m + 1]);
                if (std::fabs(e[m]) <= eps * dd2) break;
            }
            if (m != l) {
                if (iter++ == 100) return false;
                double g = (d[l + 1] - d[l]) / (2.0 * e[l]);
                double r = std::hypot(g, 1.0);
                g = d[m] - d[l] + e[l] / (g + (g >= 0 ? std::fabs(r) : -std::fabs(r)));
                double s = 1.0, c = 1.0, p = 0.0;
                int i;
                bool early = false;
                for (i = m - 1; i >= l; --i) {
                    double f = s * e[i], b = c * e[i];
                    e[i + 1] = (r = std::hypot(f, g));
                    if (r == 0.0) {
                        d[i + 1] -= p;
                        e[m] = 0.0;
                        early = true;
                        break;
                    }
                    s = f / r;
                    c = g / r;
                    g = d[i + 1] - p;
                    r = (d[i] - g) * s + 2.0 * c * b;
                    d[i + 1] = g + (p = s * r);
                    g = c * r - b;
                }
                if (early) continue;
                d[l] -= p;
                e[l] = g;
                e[m] = 0.0;
            }
        } while (m != l);
    }
    std::sort(d.begin(), d.end());
    for (int i = 0; i < n; ++i) w[i] = d[i];
    return true;
}

void singular_values(int m, const double* A, int lda, double* sv) {
    std::vector<double> U((size_t)m * m);
    for (int j = 0; j < m; ++j)
        for (int i = 0; i < m; ++i) U[i + (size_t)j * m] = A[i + (size_t)j * lda];
    const double eps = std::ldexp(1.0, -52);
    for (int sweep = 0; sweep < 60; ++sweep) {
        double off = 0.0;
        for (int p = 0; p < m - 1; ++p)
            for (int q = p + 1; q < m; ++q) {
                double a = 0, b = 0, c = 0;
                for (int i = 0; i < m; ++i) {
                    const double up = U[i + (size_t)p * m], uq = U[i + (size_t)q * m];
                    a += up * up;
                    b += uq * uq;
                    c += up * uq;
                }
                if (std::fabs(c) <= eps * std::sqrt(a * b) || c == 0.0) continue;
                off = std::max(off, std::fabs(c) / std::sqrt(a * b));
                const double zeta = (b - a) / (2.0 * c);
                const double t = (zeta >= 0 ? 1.0 : -1.0) / (std::fabs(zeta) + std::sqrt(1.0 + zeta * zeta));
                const double cs = 1.0 / std::sqrt(1.0 + t * t), sn = cs * t;
                for (int i = 0; i < m; ++i) {
                    const double up = U[i + (size_t)p * m], uq = U[i + (size_t)q * m];
                    U[i + (size_t)p * m] = cs * up - sn * uq;
                    U[i + (size_t)q * m] = sn * up + cs * uq;
                }
            }
        if (off <= eps) break;
    }
    for (int j = 0; j < m; ++j) {
        double s = 0;
        for (int i = 0; i < m; ++i) s += U[i + (size_t)j * m] * U[i + (size_t)j * m];
        sv[j] = std::sqrt(s);
    }
    std::sort(sv, sv + m, [](double x, double y) { return x > y; });
}

// Full SVD of a small square matrix by one-sided Jacobi: A V = U S with the
// singular values descending; U's columns for zero singular values are
// completed to an orthonormal basis.
void svd(int m, const double* A, int lda, double* U, double* S, double* V) {
    std::vector<double> W((size_t)m * m), Vw((size_t)m * m, 0.0);
    for (int j = 0; j < m; ++j) {
        for (int i = 0; i < m; ++i) W[i + (size_t)j * m] = A[i + (size_t)j * lda];
        Vw[j + (size_t)j * m] = 1.0;
    }
    const double eps = std::ldexp(1.0, -52);
    for (int sweep = 0; sweep < 60; ++sweep) {
        double off = 0.0;
        for (int p = 0; p < m - 1; ++p)
            for (int q = p + 1; q < m; ++q) {
                double a = 0, b = 0, c = 0;
                for (int i = 0; i < m; ++i) {
                    const double up = W[i + (size_t)p * m], uq = W[i + (size_t)q * m];
                    a += up * up;
                    b += uq * uq;
                    c += up * uq;
                }
                if (std::fabs(c) <= eps * std::sqrt(a * b) || c == 0.0) continue;
                off = std::max(off, std::fabs(c) / std::sqrt(a * b));
                const double zeta = (b - a) / (2.0 * c);
                const double t = (zeta >= 0 ? 1.0 : -1.0) / (std::fabs(zeta) + std::sqrt(1.0 + zeta * zeta));
                const double cs = 1.0 / std::sqrt(1.0 + t * t), sn = cs * t;
                for (int i = 0; i < m; ++i) {
                    const double up = W[i + (size_t)p * m], uq = W[i + (size_t)q * m];
                    W[i + (size_t)p * m] = cs * up - sn * uq;
                    W[i + (size_t)q * m] = sn * up + cs * uq;
                    const double vp = Vw[i + (size_t)p * m], vq = Vw[i + (size_t)q * m];
                    Vw[i + (size_t)p * m] = cs * vp - sn * vq;
                    Vw[i + (size_t)q * m] = sn * vp + cs * vq;
                }
            }
        if (off <= eps) break;
    }
    std::vector<double> sv(m);
    std::vector<int> ord(m);
    for (int j = 0; j < m; ++j) {
        double s2 = 0;
        for (int i = 0; i < m; ++i) s2 += W[i + (size_t)j * m] * W[i + (size_t)j * m];
        sv[j] = std::sqrt(s2);
        ord[j] = j;
    }
    std::stable_sort(ord.begin(), ord.end(), [&](int x, int y) { return sv[x] > sv[y]; });
    const double small = sv[ord[0]] * m * eps;
    int nz = 0;
    for (int k = 0; k < m; ++k) {
        const int j = ord[k];
        S[k] = sv[j];
        for (int i = 0; i < m; ++i) V[i + (size_t)k * m] = Vw[i + (size_t)j * m];
        if (sv[j] > small && sv[j] > 0.0) {
            for (int i = 0; i < m; ++i) U[i + (size_t)k * m] = W[i + (size_t)j * m] / sv[j];
            nz = k + 1;
        } else {
            for (int i = 0; i < m; ++i) U[i + (size_t)k * m] = 0.0;
        }
    }
    // complete U: Gram-Schmidt (twice) of unit vectors against the columns so far
    int next_e = 0;
    for (int k = nz; k < m; ++k) {
        for (; next_e < m; ++next_e) {
            std::vector<double> u(m, 0.0);
            u[next_e] = 1.0;
            for (int pass = 0; pass < 2; ++pass)
                for (int c = 0; c < k; ++c) {
                    double d = 0;
                    for (int i = 0; i < m; ++i) d += U[i + (size_t)c * m] * u[i];
                    for (int i = 0; i < m; ++i) u[i] -= d * U[i + (size_t)c * m];
                }
            double nu = 0;
            for (int i = 0; i < m; ++i) nu += u[i] * u[i];
            nu = std::sqrt(nu);
            if (nu > 0.5) {
                for (int i = 0; i < m; ++i) U[i + (size_t)k * m] = u[i] / nu;
                ++next_e;
                break;
            }
        }
    }
}

// Symmetric eigenproblem: Householder reduction to tridiagonal form with the
// transformations accumulated (EISPACK tred2), then the implicit QL iteration
// with Wilkinson-type shifts applied to the accumulated vectors (tql2).
// O(n^3) with a small constant (0.6 ms at n = 60; the Jacobi sweeps it
// replaces took 50 ms).  Ascending eigenvalues, orthonormal vectors; V =
// NULL: the values alone (the same arithmetic on d and e, so the same bits,
// without the O(n^3) accumulation and the rotations of the vectors).
void eig_symmetric(int n, const double* A, int lda, double* w, double* V, int ldv) {
    if (n <= 0) return;
    std::vector<double> z((size_t)n * n), d(n, 0.0), e(n, 0.0);
    auto Z = [&](int i, int j) -> double& { return z[(size_t)i + (size_t)j * n]; };
    for (int j = 0; j < n; ++j)
        for (int i = 0; i < n; ++i) Z(i, j) = A[i + (size_t)j * lda];
    // tred2: rows i = n-1 .. 1 reduced with the lower triangle
    for (int i = n - 1; i > 0; --i) {
        const int l = i - 1;
        double h = 0.0;
        if (l > 0) {
            double scale = 0.0;
            for (int k = 0; k <= l; ++k) scale += std::fabs(Z(i, k));
            if (scale == 0.0) {
                e[i] = Z(i, l);
            } else {
                for (int k = 0; k <= l; ++k) {
                    Z(i, k) /= scale;
                    h += Z(i, k) * Z(i, k);
                }
                double f = Z(i, l);
                double g = f >= 0.0 ? -std::sqrt(h) : std::sqrt(h);
                e[i] = scale * g;
                h -= f * g;
                Z(i, l) = f - g;
                f = 0.0;
                for (int j = 0; j <= l; ++j) {
                    Z(j, i) = Z(i, j) / h;
                    g = 0.0;
                    for (int k = 0; k <= j; ++k) g += Z(j, k) * Z(i, k);
                    for (int k = j + 1; k <= l; ++k) g += Z(k, j) * Z(i, k);
                    e[j] = g / h;
                    f += e[j] * Z(i, j);
                }
                const double hh = f / (h + h);
                for (int j = 0; j <= l; ++j) {
                    f = Z(i, j);
                    e[j] = g = e[j] - hh * f;
                    for (int k = 0; k <= j; ++k) Z(j, k) -= f * e[k] + g * Z(i, k);
                }
            }
        } else {
            e[i] = Z(i, l);
        }
        d[i] = h;
    }
    d[0] = 0.0;
    e[0] = 0.0;
    for (int i = 0; i < n; ++i) {  // accumulate the transformations
        if (!V) {  // values only: the diagonal, which the accumulation leaves as it is
            d[i] = Z(i, i);
            continue;
        }
        const int l = i - 1;
        if (d[i] != 0.0) {
            for (int j = 0; j <= l; ++j) {
                double g = 0.0;
                for (int k = 0; k <= l; ++k) g += Z(i, k) * Z(k, j);
                for (int k = 0; k <= l; ++k) Z(k, j) -= g * Z(k, i);
            }
        }
        d[i] = Z(i, i);
        Z(i, i) = 1.0;
        for (int j = 0; j <= l; ++j) Z(j, i) = Z(i, j) = 0.0;
    }
    // tql2 on (d, e) with the vectors in z
    for (int i = 1; i < n; ++i) e[i - 1] = e[i];
    e[n - 1] = 0.0;
    const double eps = std::ldexp(1.0, -52);
    for (int l = 0; l < n; ++l) {
        int iter = 0, m;
        do {
            for (m = l; m < n - 1; ++m) {
                const double dd = std::fabs(d[m]) + std::fabs(d[m + 1]);
                if (std::fabs(e[m]) <= eps * dd) break;
            }
            if (m != l) {
                if (iter++ == 60) break;  // accept: never observed for Lanczos T
                double g = (d[l + 1] - d[l]) / (2.0 * e[l]);
                double r = std::hypot(g, 1.0);
                g = d[m] - d[l] + e[l] / (g + (g >= 0.0 ? r : -r));
                double s = 1.0, c = 1.0, p = 0.0;
                int i;
                bool early = false;
                for (i = m - 1; i >= l; --i) {
                    double f = s * e[i], b = c * e[i];
                    e[i + 1] = (r = std::hypot(f, g));
                    if (r == 0.0) {
                        d[i + 1] -= p;
                        e[m] = 0.0;
                        early = true;
                        break;
                    }
                    s = f / r;
                    c = g / r;
                    g = d[i + 1] - p;
                    r = (d[i] - g) * s + 2.0 * c * b;
                    d[i + 1] = g + (p = s * r);
                    g = c * r - b;
                    for (int k = 0; V && k < n; ++k) {
                        f = Z(k, i + 1);
                        Z(k, i + 1) = s * Z(k, i) + c * f;
                        Z(k, i) = c * Z(k, i) - s * f;
                    }
                }
                if (early) continue;
                d[l] -= p;
                e[l] = g;
                e[m] = 0.0;
            }
        } while (m != l);
    }
    std::vector<int> idx(n);
    for (int i = 0; i < n; ++i) idx[i] = i;
    std::stable_sort(idx.begin(), idx.end(), [&](int x, int y) { return d[x] < d[y]; });
    for (int j = 0; j < n; ++j) {
        w[j] = d[idx[j]];
        for (int i = 0; V && i < n; ++i) V[i + (size_t)j * ldv] = Z(i, idx[j]);
    }
}

// ---- general eigenproblem: orthes + hqr2 (EISPACK algorithm) -------------
namespace {

struct Mat {
    int n;
    std::vector<double> a;
    explicit Mat(int n_) : n(n_), a((size_t)n_ * n_, 0.0) {}
    double& operator()(int i, int j) { return a[i + (size_t)j * n]; }
};

inline void cdiv(double xr, double xi, double yr, double yi, double& cr, double& ci) {
    double r, d;
    if (std::fabs(yr) > std::fabs(yi)) {
        r = yi / yr;
        d = yr + r * yi;
        cr = (xr + r * xi) / d;
        ci = (xi - r * xr) / d;
    } else {
        r = yr / yi;
        d = yi + r * yr;
        cr = (r * xr + xi) / d;
        ci = (r * xi - xr) / d;
    }
}

void orthes(Mat& H, Mat& V) {
    const int n = H.n, low = 0, high = n - 1;
    std::vector<double> ort(n, 0.0);
    for (int m = low + 1; m <= high - 1; ++m) {
        double scale = 0.0;
        for (int i = m; i <= high; ++i) scale += std::fabs(H(i, m - 1));
        if (scale != 0.0) {
            double h = 0.0;
            for (int i = high; i >= m; --i) {
                ort[i] = H(i, m - 1) / scale;
                h += ort[i] * ort[i];
            }
            double g = std::sqrt(h);
            if (ort[m] > 0) g = -g;
            h = h - ort[m] * g;
            ort[m] = ort[m] - g;
            for (int j = m; j < n; ++j) {
                double f = 0.0;
                for (int i = high; i >= m; --i) f += ort[i] * H(i, j);
                f = f / h;
                for (int i = m; i <= high; ++i) H(i, j) -= f * ort[i];
            }
            for (int i = 0; i <= high; ++i) {
                double f = 0.0;
                for (int j = high; j >= m; --j) f += ort[j] * H(i, j);
                f = f / h;
                for (int j = m; j <= high; ++j) H(i, j) -= f * ort[j];
            }
            ort[m] = scale * ort[m];
            H(m, m - 1) = scale * g;
        }
    }
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < n; ++j) V(i, j) = (i == j ? 1.0 : 0.0);
    for (int m = high - 1; m >= low + 1; --m) {
        if (H(m, m - 1) != 0.0) {
            for (int i = m + 1; i <= high; ++i) ort[i] = H(i, m - 1);
            for (int j = m; j <= high; ++j) {
                double g = 0.0;
                for (int i = m; i <= high; ++i) g += ort[i] * V(i, j);
                g = (g / ort[m]) / H(m, m - 1);
                for (int i = m; i <= high; ++i) V(i, j) += g * ort[i];
            }
        }
    }
}

bool hqr2(Mat& H, Mat& V, std::vector<double>& d, std::vector<double>& e) {
    const int nn = H.n;
    int n = nn - 1;
    const int low = 0, high = nn - 1;
    const double eps = std::ldexp(1.0, -52);
    double exshift = 0.0;
    double p = 0, q = 0, r = 0, s = 0, z = 0, t, w, x, y;
    double norm = 0.0;
    for (int i = 0; i < nn; ++i)
        for (int j = std::max(i - 1, 0); j < nn; ++j) norm += std::fabs(H(i, j));
    int iter = 0, total_iter = 0;
    while (n >= low) {
        int l = n;
        while (l > low) {
            s = std::fabs(H(l - 1, l - 1)) + std::fabs(H(l, l));
            if (s == 0.0) s = norm;
            if (std::fabs(H(l, l - 1)) < eps * s) break;
            l--;
        }
        if (l == n) {
            H(n, n) = H(n, n) + exshift;
            d[n] = H(n, n);
            e[n] = 0.0;
            n--;
            iter = 0;
        } else if (l == n - 1) {
            w = H(n, n - 1) * H(n - 1, n);
            p = (H(n - 1, n - 1) - H(n, n)) / 2.0;
            q = p * p + w;
            z = std::sqrt(std::fabs(q));
            H(n, n) = H(n, n) + exshift;
            H(n - 1, n - 1) = H(n - 1, n - 1) + exshift;
            x = H(n, n);
            if (q >= 0) {
                z = (p >= 0) ? p + z : p - z;
                d[n - 1] = x + z;
                d[n] = d[n - 1];
                if (z != 0.0) d[n] = x - w / z;
                e[n - 1] = 0.0;
                e[n] = 0.0;
                x = H(n, n - 1);
                s = std::fabs(x) + std::fabs(z);
                p = x / s;
                q = z / s;
                r = std::sqrt(p * p + q * q);
                p = p / r;
                q = q / r;
                for (int j = n - 1; j < nn; ++j) {
                    z = H(n - 1, j);
                    H(n - 1, j) = q * z + p * H(n, j);
                    H(n, j) = q * H(n, j) - p * z;
                }
                for (int i = 0; i <= n; ++i) {
                    z = H(i, n - 1);
                    H(i, n - 1) = q * z + p * H(i, n);
                    H(i, n) = q * H(i, n) - p * z;
                }
                for (int i = low; i <= high; ++i) {
                    z = V(i, n - 1);
                    V(i, n - 1) = q * z + p * V(i, n);
                    V(i, n) = q * V(i, n) - p * z;
                }
            } else {
                d[n - 1] = x + p;
                d[n] = x + p;
                e[n - 1] = z;
                e[n] = -z;
            }
            n = n - 2;
            iter = 0;
        } else {
            x = H(n, n);
            y = 0.0;
            w = 0.0;
            if (l < n) {
                y = H(n - 1, n - 1);
                w = H(n, n - 1) * H(n - 1, n);
            }
            if (iter == 10) {
                exshift += x;
                for (int i = low; i <= n; ++i) H(i, i) -= x;
                s = std::fabs(H(n, n - 1)) + std::fabs(H(n - 1, n - 2));
                x = y = 0.75 * s;
                w = -0.4375 * s * s;
            }
            if (iter == 30) {
                s = (y - x) / 2.0;
                s = s * s + w;
                if (s > 0) {
                    s = std::sqrt(s);
                    if (y < x) s = -s;
                    s = x - w / ((y - x) / 2.0 + s);
                    for (int i = low; i <= n; ++i) H(i, i) -= s;
                    exshift += s;
                    x = y = w = 0.964;
                }
            }
            iter = iter + 1;
            if (++total_iter > 100 * nn) return false;
            int m = n - 2;
            while (m >= l) {
                z = H(m, m);
                r = x - z;
                s = y - z;
                p = (r * s - w) / H(m + 1, m) + H(m, m + 1);
                q = H(m + 1, m + 1) - z - r - s;
                r = H(m + 2, m + 1);
                s = std::fabs(p) + std::fabs(q) + std::fabs(r);
                p = p / s;
                q = q / s;
                r = r / s;
                if (m == l) break;
                if (std::fabs(H(m, m - 1)) * (std::fabs(q) + std::fabs(r)) <
                    eps * (std::fabs(p) * (std::fabs(H(m - 1, m - 1)) + std::fabs(z) + std::fabs(H(m + 1, m + 1)))))
                    break;
                m--;
            }
            for (int i = m + 2; i <= n; ++i) {
                H(i, i - 2) = 0.0;
                if (i > m + 2) H(i, i - 3) = 0.0;
            }
            for (int k = m; k <= n - 1; ++k) {
                const bool notlast = (k != n - 1);
                if (k != m) {
                    p = H(k, k - 1);
                    q = H(k + 1, k - 1);
                    r = notlast ? H(k + 2, k - 1) : 0.0;
                    x = std::fabs(p) + std::fabs(q) + std::fabs(r);
                    if (x == 0.0) continue;
                    p = p / x;
                    q = q / x;
                    r = r / x;
                }
                s = std::sqrt(p * p + q * q + r * r);
                if (p < 0) s = -s;
                if (s != 0) {
                    if (k != m)
                        H(k, k - 1) = -s * x;
                    else if (l != m)
                        H(k, k - 1) = -H(k, k - 1);
                    p = p + s;
                    x = p / s;
                    y = q / s;
                    z = r / s;
                    q = q / p;
                    r = r / p;
                    for (int j = k; j < nn; ++j) {
                        p = H(k, j) + q * H(k + 1, j);
                        if (notlast) {
                            p = p + r * H(k + 2, j);
                            H(k + 2, j) = H(k + 2, j) - p * z;
                        }
                        H(k, j) = H(k, j) - p * x;
                        H(k + 1, j) = H(k + 1, j) - p * y;
                    }
                    for (int i = 0; i <= std::min(n, k + 3); ++i) {
                        p = x * H(i, k) + y * H(i, k + 1);
                        if (notlast) {
                            p = p + z * H(i, k + 2);
                            H(i, k + 2) = H(i, k + 2) - p * r;
                        }
                        H(i, k) = H(i, k) - p;
                        H(i, k + 1) = H(i, k + 1) - p * q;
                    }
                    for (int i = low; i <= high; ++i) {
                        p = x * V(i, k) + y * V(i, k + 1);
                        if (notlast) {
                            p = p + z * V(i, k + 2);
                            V(i, k + 2) = V(i, k + 2) - p * r;
                        }
                        V(i, k) = V(i, k) - p;
                        V(i, k + 1) = V(i, k + 1) - p * q;
                    }
                }
            }
        }
    }
    if (norm == 0.0) return true;
    for (n = nn - 1; n >= 0; --n) {
        p = d[n];
        q = e[n];
        if (q == 0) {
            int l = n;
            H(n, n) = 1.0;
            for (int i = n - 1; i >= 0; --i) {
                w = H(i, i) - p;
                r = 0.0;
                for (int j = l; j <= n; ++j) r = r + H(i, j) * H(j, n);
                if (e[i] < 0.0) {
                    z = w;
                    s = r;
                } else {
                    l = i;
                    if (e[i] == 0.0) {
                        H(i, n) = (w != 0.0) ? -r / w : -r / (eps * norm);
                    } else {
                        x = H(i, i + 1);
                        y = H(i + 1, i);
                        q = (d[i] - p) * (d[i] - p) + e[i] * e[i];
                        t = (x * s - z * r) / q;
                        H(i, n) = t;
                        if (std::fabs(x) > std::fabs(z))
                            H(i + 1, n) = (-r - w * t) / x;
                        else
                            H(i + 1, n) = (-s - y * t) / z;
                    }
                    t = std::fabs(H(i, n));
                    if ((eps * t) * t > 1)
                        for (int j = i; j <= n; ++j) H(j, n) = H(j, n) / t;
                }
            }
        } else if (q < 0) {
            int l = n - 1;
            double cr, ci;
            if (std::fabs(H(n, n - 1)) > std::fabs(H(n - 1, n))) {
                H(n - 1, n - 1) = q / H(n, n - 1);
                H(n - 1, n) = -(H(n, n) - p) / H(n, n - 1);
            } else {
                cdiv(0.0, -H(n - 1, n), H(n - 1, n - 1) - p, q, cr, ci);
                H(n - 1, n - 1) = cr;
                H(n - 1, n) = ci;
            }
            H(n, n - 1) = 0.0;
            H(n, n) = 1.0;
            for (int i = n - 2; i >= 0; --i) {
                double ra = 0.0, sa = 0.0, vr, vi;
                for (int j = l; j <= n; ++j) {
                    ra = ra + H(i, j) * H(j, n - 1);
                    sa = sa + H(i, j) * H(j, n);
                }
                w = H(i, i) - p;
                if (e[i] < 0.0) {
                    z = w;
                    r = ra;
                    s = sa;
                } else {
                    l = i;
                    if (e[i] == 0) {
                        cdiv(-ra, -sa, w, q, cr, ci);
                        H(i, n - 1) = cr;
                        H(i, n) = ci;
                    } else {
                        x = H(i, i + 1);
                        y = H(i + 1, i);
                        vr = (d[i] - p) * (d[i] - p) + e[i] * e[i] - q * q;
                        vi = (d[i] - p) * 2.0 * q;
                        if (vr == 0.0 && vi == 0.0)
                            vr = eps * norm * (std::fabs(w) + std::fabs(q) + std::fabs(x) + std::fabs(y) + std::fabs(z));
                        cdiv(x * r - z * ra + q * sa, x * s - z * sa - q * ra, vr, vi, cr, ci);
                        H(i, n - 1) = cr;
                        H(i, n) = ci;
                        if (std::fabs(x) > (std::fabs(z) + std::fabs(q))) {
                            H(i + 1, n - 1) = (-ra - w * H(i, n - 1) + q * H(i, n)) / x;
                            H(i + 1, n) = (-sa - w * H(i, n) - q * H(i, n - 1)) / x;
                        } else {
                            cdiv(-r - y * H(i, n - 1), -s - y * H(i, n), z, q, cr, ci);
                            H(i + 1, n - 1) = cr;
                            H(i + 1, n) = ci;
                        }
                    }
                    t = std::max(std::fabs(H(i, n - 1)), std::fabs(H(i, n)));
                    if ((eps * t) * t > 1)
                        for (int j = i; j <= n; ++j) {
                            H(j, n - 1) = H(j, n - 1) / t;
                            H(j, n) = H(j, n) / t;
                        }
                }
            }
        }
    }
    for (int j = nn - 1; j >= low; --j)
        for (int i = low; i <= high; ++i) {
            z = 0.0;
            for (int k = low; k <= std::min(j, high); ++k) z = z + V(i, k) * H(k, j);
            V(i, j) = z;
        }
    return true;
}

}  // namespace

bool eig_general(int n, const double* A, int lda, double* wr, double* wi, double* V, int ldv) {
    if (n <= 0) return true;
    Mat H(n), Vm(n);
    for (int j = 0; j < n; ++j)
        for (int i = 0; i < n; ++i) H(i, j) = A[i + (size_t)j * lda];
    std::vector<double> d(n, 0.0), e(n, 0.0);
    orthes(H, Vm);
    const bool ok = hqr2(H, Vm, d, e);
    for (int i = 0; i < n; ++i) {
        wr[i] = d[i];
        wi[i] = e[i];
    }
    for (int j = 0; j < n; ++j)
        for (int i = 0; i < n; ++i) V[i + (size_t)j * ldv] = Vm(i, j);
    return ok;
}

// Explicit shifted QR steps on an upper-Hessenberg H (m x m), one per shift
// mu[t]: H - mu I = QR, H <- RQ + mu I = Q'HQ, W (m x m) <- WQ, with Q the
// product of m-1 Givens rotations (O(m^2) a step; the reference's qrstep
// forms the same Q, up to column signs, by a dense Householder QR and two m^3
// products).  W's rotations depend on H only through the (c, s) pairs, so
// they are applied after all the H steps, eight rows at a time with the
// rotated column carried in registers: every W entry sees the same
// operations in the same order as when applied step by step (the same bits),
// at a fraction of the loads and stores.
typedef double v2d __attribute__((vector_size(16)));

void hess_qrsteps(int m, double* H, int ldh, double* W, int ldw, const double* mu, int count) {
    if (m < 1 || count < 1) return;
    auto h = [&](int i, int j) -> double& { return H[i + (size_t)j * ldh]; };
    const int nr = m - 1;
    std::vector<double> cs((size_t)count * (nr > 0 ? nr : 1), 1.0), sn((size_t)count * (nr > 0 ? nr : 1), 0.0);
    for (int t = 0; t < count; ++t) {
        double* ct = cs.data() + (size_t)t * nr;
        double* st = sn.data() + (size_t)t * nr;
        for (int i = 0; i < m; ++i) h(i, i) -= mu[t];
        for (int j = 0; j + 1 < m; ++j) {  // R = G'_{m-2} ... G'_0 (H - mu I)
            const double a = h(j, j), b = h(j + 1, j);
            double c = 1.0, s = 0.0;
            if (b != 0.0) {
                const double r = std::hypot(a, b);
                c = a / r;
                s = b / r;
            }
            ct[j] = c;
            st[j] = s;
            // rows j, j+1 of a column are adjacent: one pair vector per column,
            // [c x + s y, c y + (-s) x] -- (-s) x = -(s x) and a + (-b) = a - b
            // exactly, so the same bits as the scalar rotation
            const v2d cc = {c, c}, ss = {s, -s};
            for (int col = j; col < m; ++col) {
                double* hp = &h(j, col);
                v2d v;
                std::memcpy(&v, hp, sizeof v);
                const v2d sw = {v[1], v[0]};
                const v2d a = cc * v, b = ss * sw;
                const v2d r = a + b;
                std::memcpy(hp, &r, sizeof r);
            }
            h(j + 1, j) = 0.0;
        }
        for (int j = 0; j + 1 < m; ++j) {  // RQ, Q = G_0 ... G_{m-2}
            const double c = ct[j], s = st[j];
            for (int row = 0; row < std::min(j + 2, m); ++row) {
                const double x = h(row, j), y = h(row, j + 1);
                h(row, j) = c * x + s * y;
                h(row, j + 1) = c * y - s * x;
            }
        }
        for (int i = 0; i < m; ++i) h(i, i) += mu[t];
    }
    if (nr < 1) return;
    constexpr int RB = 8;
    for (int r0 = 0; r0 < m; r0 += RB) {
        const int rows = std::min(RB, m - r0);
        for (int t = 0; t < count; ++t) {
            const double* ct = cs.data() + (size_t)t * nr;
            const double* st = sn.data() + (size_t)t * nr;
            double a[RB];
            for (int i = 0; i < rows; ++i) a[i] = W[r0 + i];
            for (int j = 0; j < nr; ++j) {
                const double c = ct[j], s = st[j];
                double* wj = W + (size_t)j * ldw + r0;
                const double* wj1 = W + (size_t)(j + 1) * ldw + r0;
                if (rows == RB) {
#pragma GCC unroll 8
                    for (int i = 0; i < RB; ++i) {
                        const double x = a[i], y = wj1[i];
                        wj[i] = c * x + s * y;
                        a[i] = c * y - s * x;
                    }
                } else {
                    for (int i = 0; i < rows; ++i) {
                        const double x = a[i], y = wj1[i];
                        wj[i] = c * x + s * y;
                        a[i] = c * y - s * x;
                    }
                }
            }
            for (int i = 0; i < rows; ++i) W[(size_t)nr * ldw + r0 + i] = a[i];
        }
    }
}

void hess_qrstep(int m, double* H, int ldh, double* W, int ldw, double mu) { hess_qrsteps(m, H, ldh, W, ldw, &mu, 1); }

void matlab_rand(std::mt19937& g, int64_t count, double* out) {
    for (int64_t i = 0; i < count; ++i) {
        const uint32_t a = g() >> 5, b = g() >> 6;
        out[i] = (a * 67108864.0 + b) / 9007199254740992.0;
    }
}

}  // namespace dense
}  // namespace cal
