/* ca_lanczos_omp.c -- multithreaded C restatement of the reference's
 * CA-Lanczos outer loop ('local' orthogonalisation, diagnostics off).
 *
 * TEST INFRASTRUCTURE ONLY (the CPU baseline of bench.py and a second oracle
 * checked against oracle/ca_lanczos_ref.py by tests/test_oracle_c.py).
 * Nothing in the product links it.  SURVEY §8d asks for this second CPU
 * number: the NumPy restatement's SpMV is single-threaded, this one runs
 * every n-length loop on all host cores with OpenMP.
 *
 * Follows, line by line in structure:
 *   ca_lanczos.m:150-245   ca_lanczos_basic, orth 'local' (k = 1 normalize,
 *                          k > 1 projectAndNormalize against the previous
 *                          block, T update :200-223)
 *   matrix_powers_newton.m:15-48 (real shifts, modifiedp = 1) and
 *   matrix_powers_monomial.m:6-12 (through ca_lanczos.m:110-118)
 *   projectAndNormalize.m:3-90 (doreorth = true, threshold 0.5 at :52)
 *   project.m:7-58 (one block, doreorth = false)
 *   normalize.m:3-36 / tsqr.m:7-12: Householder QR + sign fix.  The QR is a
 *   TSQR (Householder per 2048-row tile, Householder of the stacked R
 *   factors, explicit Q through the tree): R is unique once its diagonal is
 *   made positive, so it equals MATLAB's qr(A,0) R up to rounding.
 * The Newton shifts / change-of-basis matrix Bk come from the caller (the
 * NumPy oracle's prologue, ca_lanczos.m:66-72).
 */
#include <math.h>
#include <stdio.h>
#include <omp.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define IDX(i, j, ld) ((size_t)(i) + (size_t)(j) * (size_t)(ld))

/* ---- dense helpers (column-major) ---------------------------------------- */

/* LAPACK dlarfg on x[0..len): alpha = x[0]; returns tau, x[0] = beta,
 * x[1..] = v(2:end) */
static double house(double* x, size_t len, size_t inc) {
    double xn = 0.0;
#pragma omp simd reduction(+ : xn)
    for (size_t i = 1; i < len; ++i) xn += x[i * inc] * x[i * inc];
    xn = sqrt(xn);
    if (xn == 0.0) return 0.0;
    const double alpha = x[0];
    const double beta = -copysign(hypot(alpha, xn), alpha);
    const double sc = 1.0 / (alpha - beta);
    for (size_t i = 1; i < len; ++i) x[i * inc] *= sc;
    x[0] = beta;
    return (beta - alpha) / beta;
}

/* Householder QR in place of A (rows x m, ld); tau[m] */
static void geqr2(size_t rows, int m, double* A, size_t ld, double* tau) {
    for (int j = 0; j < m; ++j) {
        if ((size_t)j >= rows) {
            tau[j] = 0.0;
            continue;
        }
        double* col = A + IDX(j, j, ld);
        tau[j] = house(col, rows - j, 1);
        if (tau[j] == 0.0) continue;
        for (int c = j + 1; c < m; ++c) {
            double* cc = A + IDX(j, c, ld);
            double d = cc[0];
#pragma omp simd reduction(+ : d)
            for (size_t i = 1; i < rows - j; ++i) d += col[i] * cc[i];
            d *= tau[j];
            cc[0] -= d;
            for (size_t i = 1; i < rows - j; ++i) cc[i] -= d * col[i];
        }
    }
}

/* apply H(0) ... H(m-1) (reflectors in A, tau) to C (rows x m, ldc): C = Q C */
static void apply_q(size_t rows, int m, const double* A, size_t ld, const double* tau, double* C, size_t ldc,
                    int ncol) {
    for (int j = m - 1; j >= 0; --j) {
        if (tau[j] == 0.0 || (size_t)j >= rows) continue;
        const double* v = A + IDX(j, j, ld);
        for (int c = 0; c < ncol; ++c) {
            double* cc = C + IDX(j, c, ldc);
            double d = cc[0];
#pragma omp simd reduction(+ : d)
            for (size_t i = 1; i < rows - j; ++i) d += v[i] * cc[i];
            d *= tau[j];
            cc[0] -= d;
            for (size_t i = 1; i < rows - j; ++i) cc[i] -= d * v[i];
        }
    }
}

/* tsqr.m:7-12: [Q,R] = qr(X,0), d = sign(diag(R)), R = diag(d) R, Q = Q diag(d).
 * S (n x m, ld n) is the input, X (ld n) receives Q (S == X: in place; else
 * each tile is copied into X inside the parallel tile loop and S is left
 * untouched); R is m x m (ld m).  Two-level TSQR:
 * Householder QR of cache-sized row tiles (in parallel), Householder QR of
 * the stacked tile R factors, then each tile's Q applied to its block of the
 * stack's Q. */
#define TSQR_TILE 2048
static void tsqr(size_t n, int m, const double* S, double* X, double* R) {
    const size_t nt = (n + TSQR_TILE - 1) / TSQR_TILE, PR = nt * (size_t)m;
    double* Rs = calloc(PR * m, sizeof(double));
    double* taus = calloc(nt * m, sizeof(double));
#pragma omp parallel for schedule(dynamic, 4)
    for (size_t t = 0; t < nt; ++t) {
        const size_t r0 = t * TSQR_TILE, rows = (r0 + TSQR_TILE <= n ? TSQR_TILE : n - r0);
        double* Xb = X + r0;
        if (S != X)
            for (int j = 0; j < m; ++j) memcpy(Xb + (size_t)j * n, S + r0 + (size_t)j * n, rows * sizeof(double));
        geqr2(rows, m, Xb, n, taus + t * m);
        for (int j = 0; j < m; ++j)
            for (int i = 0; i <= j && (size_t)i < rows; ++i) Rs[IDX(t * m + i, j, PR)] = Xb[IDX(i, j, n)];
    }
    /* QR of the stacked R factors */
    double* ttop = calloc(m, sizeof(double));
    geqr2(PR, m, Rs, PR, ttop);
    for (int j = 0; j < m; ++j)
        for (int i = 0; i < m; ++i) R[IDX(i, j, m)] = i <= j ? Rs[IDX(i, j, PR)] : 0.0;
    double* Qtop = calloc(PR * m, sizeof(double));
    for (int j = 0; j < m; ++j) Qtop[IDX(j, j, PR)] = 1.0;
    apply_q(PR, m, Rs, PR, ttop, Qtop, PR, m);
    /* sign fix (sign(0) = 0, as MATLAB); Q's columns are scaled by d as the
     * tiles are written back below */
    double d[64];
    for (int j = 0; j < m; ++j) {
        const double rj = R[IDX(j, j, m)];
        d[j] = rj > 0.0 ? 1.0 : (rj < 0.0 ? -1.0 : 0.0);
        for (int c = 0; c < m; ++c) R[IDX(j, c, m)] *= d[j];
    }
    /* Q tile t = H_t [Qtop block t; 0] */
#pragma omp parallel
    {
        double* C = malloc((size_t)TSQR_TILE * m * sizeof(double));
#pragma omp for schedule(dynamic, 4)
        for (size_t t = 0; t < nt; ++t) {
            const size_t r0 = t * TSQR_TILE, rows = (r0 + TSQR_TILE <= n ? TSQR_TILE : n - r0);
            double* Xb = X + r0;
            memset(C, 0, rows * m * sizeof(double));
            for (int j = 0; j < m; ++j)
                for (int i = 0; i < m && (size_t)i < rows; ++i) C[IDX(i, j, rows)] = Qtop[IDX(t * m + i, j, PR)];
            apply_q(rows, m, Xb, n, taus + t * m, C, rows, m);
            for (int j = 0; j < m; ++j) {
                double* xc = Xb + (size_t)j * n;
                const double* cc = C + (size_t)j * rows;
                for (size_t i = 0; i < rows; ++i) xc[i] = cc[i] * d[j];
            }
        }
        free(C);
    }
    free(Rs);
    free(taus);
    free(ttop);
    free(Qtop);
}

/* G (w x m, ld w) = Qp' X, Qp n x w, X n x m (both ld n): row blocks, each a
 * set of contiguous column segments (dot products over the block) */
#define GEMM_BLK 1024
static void gemm_tn(size_t n, int w, int m, const double* Qp, const double* X, double* G) {
    memset(G, 0, (size_t)w * m * sizeof(double));
    const size_t nb = (n + GEMM_BLK - 1) / GEMM_BLK;
#pragma omp parallel
    {
        double* acc = calloc((size_t)w * m, sizeof(double));
#pragma omp for schedule(static)
        for (size_t b = 0; b < nb; ++b) {
            const size_t i0 = b * GEMM_BLK, i1 = i0 + GEMM_BLK < n ? i0 + GEMM_BLK : n;
            for (int j = 0; j < m; ++j) {
                const double* x = X + (size_t)j * n;
                for (int a = 0; a < w; ++a) {
                    const double* q = Qp + (size_t)a * n;
                    double sum = 0.0;
#pragma omp simd reduction(+ : sum)
                    for (size_t i = i0; i < i1; ++i) sum += q[i] * x[i];
                    acc[IDX(a, j, w)] += sum;
                }
            }
        }
#pragma omp critical
        for (size_t e = 0; e < (size_t)w * m; ++e) G[e] += acc[e];
        free(acc);
    }
}

/* Y = X - Qp G, by row blocks and columns (Y may be X) */
static void gemm_sub(size_t n, int w, int m, const double* Qp, const double* G, const double* X, double* Y) {
    const size_t nb = (n + GEMM_BLK - 1) / GEMM_BLK;
#pragma omp parallel for schedule(static)
    for (size_t b = 0; b < nb; ++b) {
        const size_t i0 = b * GEMM_BLK, i1 = i0 + GEMM_BLK < n ? i0 + GEMM_BLK : n;
        double s[GEMM_BLK];
        for (int j = 0; j < m; ++j) {
            for (size_t i = i0; i < i1; ++i) s[i - i0] = 0.0;
            for (int a = 0; a < w; ++a) {
                const double* q = Qp + (size_t)a * n;
                const double g = G[IDX(a, j, w)];
                for (size_t i = i0; i < i1; ++i) s[i - i0] += q[i] * g;
            }
            const double* x = X + (size_t)j * n;
            double* y = Y + (size_t)j * n;
            for (size_t i = i0; i < i1; ++i) y[i] = x[i] - s[i - i0];
        }
    }
}

static double col_norm(size_t n, const double* x) {
    double s = 0.0;
#pragma omp parallel for simd reduction(+ : s) schedule(static)
    for (size_t i = 0; i < n; ++i) s += x[i] * x[i];
    return sqrt(s);
}

/* X (r x m) <- X / R, R upper (m x m): forward substitution by columns */
static void rdiv_upper(int r, int m, double* X, int ldx, const double* R, int ldr) {
    for (int j = 0; j < m; ++j) {
        for (int k = 0; k < j; ++k) {
            const double f = R[IDX(k, j, ldr)];
            for (int i = 0; i < r; ++i) X[IDX(i, j, ldx)] -= X[IDX(i, k, ldx)] * f;
        }
        const double d = R[IDX(j, j, ldr)];
        for (int i = 0; i < r; ++i) X[IDX(i, j, ldx)] /= d;
    }
}

/* y = A x [- shift x] */
static void spmv(size_t n, const int64_t* rp, const int32_t* col, const double* val, const double* x, double* y,
                 double shift, int shifted) {
#pragma omp parallel for schedule(static)
    for (size_t i = 0; i < n; ++i) {
        double s = 0.0;
        for (int64_t p = rp[i]; p < rp[i + 1]; ++p) s += val[p] * x[col[p]];
        y[i] = shifted ? s - shift * x[i] : s;
    }
}

/* ca_lanczos_basic, orth 'local', diagnostics off (ca_lanczos.m:150-245).
 * q: normalised start vector; Bk (s+1) x s; T_out (st x st, ld st);
 * reorth_out[t]: 1 where projectAndNormalize took its second pass. */
/* per-phase wall time, printed to stderr when CAL_OMP_PROFILE is set */
static double g_ph[8], g_loop;
#define PH(i, stmt) do { double t0_ = omp_get_wtime(); stmt; g_ph[i] += omp_get_wtime() - t0_; } while (0)

int cal_omp_ca_lanczos_local(int64_t n_, const int64_t* rowptr, const int32_t* col, const double* val,
                             const double* q, const double* Bk, int s, int t, int newton, double* T_out,
                             int* reorth_out) {
    if (n_ < 1 || s < 1 || t < 1) return -1;
    const size_t n = (size_t)n_;
    const int s1 = s + 1, st = s * t;
    double* Q = malloc(n * (size_t)(st + 1) * sizeof(double));
    double* V = malloc(n * (size_t)s1 * sizeof(double));
    double* Y = malloc(n * (size_t)s * sizeof(double));
    double* T = calloc((size_t)(st + 1) * (st + 1), sizeof(double));
    double* b = calloc((size_t)t + 1, sizeof(double));
    if (!Q || !V || !Y || !T || !b) return -2;
    const int ldT = st + 1;
    /* first touch of the n-length buffers on all threads (the pages are
     * faulted here, in parallel, not inside the first iteration's kernels);
     * the loop below is what cal_omp_loop_seconds() reports, the analogue of
     * the GPU bench's resident buffers */
#pragma omp parallel for schedule(static)
    for (size_t i = 0; i < n; ++i) {
        for (int j = 0; j <= st; ++j) Q[IDX(i, j, n)] = 0.0;
        for (int j = 0; j <= s; ++j) V[IDX(i, j, n)] = 0.0;
        for (int j = 0; j < s; ++j) Y[IDX(i, j, n)] = 0.0;
    }
    const double t_loop = omp_get_wtime();
    memcpy(Q, q, n * sizeof(double));
    for (int k = 1; k <= t; ++k) {
        /* matrix powers (ca_lanczos.m:110-118) */
        /* V(:,1) = Q(:,(k-1)s+1); only k = 1 reads it back (the QR of all
         * s+1 columns), so later blocks start the recurrence from Q itself */
        const double* v0 = Q + (size_t)((k - 1) * s) * n;
        if (k == 1) PH(2, memcpy(V, v0, n * sizeof(double)));
        for (int i = 0; i < s; ++i)
            PH(0, spmv(n, rowptr, col, val, i == 0 ? v0 : V + (size_t)i * n, V + (size_t)(i + 1) * n,
                       newton ? Bk[IDX(i, i, s1)] : 0.0, newton));
        if (k == 1) {
            /* [Q(:,1:s+1),Rk] = normalize(V) ; T = Rk*Bk/Rk(1:s,1:s) (:176-182) */
            double Rk[17 * 17], RB[17 * 16], R11[16 * 16];
            PH(5, tsqr(n, s1, V, Q, Rk));
            for (int j = 0; j < s; ++j)
                for (int i = 0; i < s1; ++i) {
                    double a = 0.0;
                    for (int l = 0; l < s1; ++l) a += Rk[IDX(i, l, s1)] * Bk[IDX(l, j, s1)];
                    RB[IDX(i, j, s1)] = a;
                }
            for (int j = 0; j < s; ++j)
                for (int i = 0; i < s; ++i) R11[IDX(i, j, s)] = Rk[IDX(i, j, s1)];
            rdiv_upper(s1, s, RB, s1, R11, s);
            for (int j = 0; j < s; ++j)
                for (int i = 0; i < s1; ++i) T[IDX(i, j, ldT)] = RB[IDX(i, j, s1)];
            b[0] = RB[IDX(s, s - 1, s1)];
            reorth_out[0] = 0;
            continue;
        }
        /* [Q_,Rk_] = projectAndNormalize({Q(:,(k-2)s+1:(k-1)s+1)}, V(:,2:s+1), true) (:187) */
        const double* Qp = Q + (size_t)((k - 2) * s) * n;
        double* X = V + n;
        double before[16], after[16], RY[17 * 16], RZ[17 * 16], R[16 * 16];
        for (int j = 0; j < s; ++j) PH(1, before[j] = col_norm(n, X + (size_t)j * n)); /* :17-22 */
        double* Qk = Q + (size_t)((k - 1) * s + 1) * n;                               /* :188 */
        PH(3, gemm_tn(n, s1, s, Qp, X, RY));                                          /* project :25 */
        PH(4, gemm_sub(n, s1, s, Qp, RY, X, Y));                                      /* Y kept for :63 */
        PH(5, tsqr(n, s, Y, Qk, R));                                                  /* normalize :26 */
        double worst = -1.0;
        for (int j = 0; j < s; ++j) {
            double a = 0.0;
            for (int i = 0; i < s; ++i) a += R[IDX(i, j, s)] * R[IDX(i, j, s)];
            after[j] = sqrt(a);                                                        /* :45-48 */
            const double rel = fabs(before[j] - after[j]) / before[j];
            if (rel > worst || (worst != worst)) worst = rel;
        }
        int reorth = worst > 0.5;                                                      /* :52 */
        const double* Rkk_s = RY;
        if (reorth) {
            PH(3, gemm_tn(n, s1, s, Qp, Y, RZ));                                       /* :63 */
            PH(4, gemm_sub(n, s1, s, Qp, RZ, Y, Y));
            PH(5, tsqr(n, s, Y, Qk, R));                                               /* :64 */
            for (int e = 0; e < s1 * s; ++e) RZ[e] += RY[e];                           /* :71-73 */
            Rkk_s = RZ;
        }
        reorth_out[k - 1] = reorth;
        /* T update (:200-223) */
        double Rk[17 * 17], R11[16 * 16], Rkk11[16 * 16], t1[16 * 16], t3[16 * 16];
        memset(Rk, 0, sizeof(Rk));
        Rk[0] = 1.0;
        for (int j = 1; j <= s; ++j) {
            Rk[IDX(0, j, s1)] = Rkk_s[IDX(s, j - 1, s1)];
            for (int i = 1; i <= s; ++i) Rk[IDX(i, j, s1)] = R[IDX(i - 1, j - 1, s)];
        }
        memset(Rkk11, 0, sizeof(Rkk11));
        for (int j = 0; j < s; ++j)
            for (int i = 0; i < s; ++i) R11[IDX(i, j, s)] = Rk[IDX(i, j, s1)];
        for (int j = 1; j < s; ++j)
            for (int i = 0; i < s; ++i) Rkk11[IDX(i, j, s)] = Rkk_s[IDX(i, j - 1, s1)];
        const double rho = Rk[IDX(s, s, s1)], rho_t = Rk[IDX(s - 1, s - 1, s1)];
        const double bk = Bk[IDX(s, s - 1, s1)], bprev = b[k - 2];
        for (int j = 0; j < s; ++j)
            for (int i = 0; i < s; ++i) {
                double a = 0.0;
                for (int l = 0; l < s; ++l) a += R11[IDX(i, l, s)] * Bk[IDX(l, j, s1)];
                t1[IDX(i, j, s)] = a;
            }
        rdiv_upper(s, s, t1, s, R11, s);
        memset(t3, 0, sizeof(t3));
        for (int j = 0; j < s; ++j) t3[IDX(0, j, s)] = bprev * Rkk11[IDX(s - 1, j, s)];
        rdiv_upper(s, s, t3, s, R11, s);
        const int m0 = s * (k - 1);
        for (int j = 0; j < s; ++j)
            for (int i = 0; i < s; ++i) {
                double v = t1[IDX(i, j, s)];
                if (j == s - 1) v += (bk / rho_t) * Rk[IDX(i, s, s1)];
                v -= t3[IDX(i, j, s)];
                T[IDX(m0 + i, m0 + j, ldT)] = v;
            }
        b[k - 1] = bk * (rho / rho_t);                                                /* :214 */
        T[IDX(m0 - 1, m0, ldT)] = bprev;
        T[IDX(m0, m0 - 1, ldT)] = bprev;
        T[IDX(m0 + s, m0 + s - 1, ldT)] = b[k - 1];
    }
    g_loop = omp_get_wtime() - t_loop;
    for (int j = 0; j < st; ++j)
        for (int i = 0; i < st; ++i) T_out[IDX(i, j, st)] = T[IDX(i, j, ldT)];
    if (getenv("CAL_OMP_PROFILE"))
        fprintf(stderr, "cal_omp phases (s): spmv %.3f norms %.3f copies %.3f gram %.3f sub %.3f tsqr %.3f\n",
                g_ph[0], g_ph[1], g_ph[2], g_ph[3], g_ph[4], g_ph[5]);
    memset(g_ph, 0, sizeof(g_ph));
    free(Q);
    free(V);
    free(Y);
    free(T);
    free(b);
    return 0;
}

int cal_omp_threads(void) { return omp_get_max_threads(); }

/* the thread count of the following calls (bench.py sets it from the usable
 * CPUs: affinity and the cgroup quota) */
int cal_omp_set_threads(int n) {
    if (n < 1) return -1;
    omp_set_num_threads(n);
    return 0;
}

/* wall time of the last cal_omp_ca_lanczos_local's outer loop (allocation and
 * first touch excluded) */
double cal_omp_loop_seconds(void) { return g_loop; }
