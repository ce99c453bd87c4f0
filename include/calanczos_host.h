/*
 * calanczos_host.h -- host-only entry points of libcalanczos (no GPU needed).
 *
 * These are the reference's small host-side routines of the Newton basis
 * set-up and of the T-matrix eigen-analysis, exported so a MATLAB host can
 * keep calling them by name and so the CPU test suite can pin them against
 * the oracle bit for bit.
 */
#ifndef CALANCZOS_HOST_H
#define CALANCZOS_HOST_H

#include "calanczos.h"

#ifdef __cplusplus
extern "C" {
#endif

/* [y,idx] = leja(x,'nonmodified') -> real_leja -> modified_leja.
 *   x = x_re + i*x_im (x_im may be NULL).  Outputs have n entries; outidx is
 *   0-based into the uniquified, real-sorted shifts (real_leja.m:83-86).
 *                                   leja.m:23-31, real_leja.m:18-87,
 *                                   modified_leja.m:24-196 */
int cal_leja(int n, const double* x_re, const double* x_im, double* y_re, double* y_im, int* outidx);

/* B_ = newton_basis_matrix(lambda, s, modifiedp); B is (s+1) x s column-major.
 *                                   newton_basis_matrix.m:13-60 */
int cal_newton_basis_matrix(int s, const double* lam_re, const double* lam_im, int modifiedp, double* B);

/* MATLAB rand of a fresh session with rng(seed,'twister'): MT19937
 * genrand_res53, `count` values in column-major order. */
int cal_matlab_rand(int64_t count, unsigned seed, double* out);

/* [V,D] = eig(T) for the Ritz analysis (ca_lanczos.m:229): symmetric solver
 * when T is exactly symmetric, general (Hessenberg QR) otherwise.  V is n x n
 * column-major; complex pairs are stored as (real, imag) column pairs. */
int cal_eig(int n, const double* T, int ldt, double* wr, double* wi, double* V);

/* Eigenvalues of the symmetric tridiagonal T = diag(alpha) + diag(beta,+-1),
 * ascending (the Newton prologue's eig(T), ca_lanczos.m:69). */
int cal_tridiag_eigvals(int n, const double* alpha, const double* beta, double* w);

/* [V,H] = qrstep(V,H,mu,1,m) for a real shift on an upper-Hessenberg H
 * (impl_restarted_ca_lanczos.m:623-678): H <- Q'HQ, W <- WQ with H - mu I =
 * QR.  Q is built from Givens rotations (the reference's Householder Q up to
 * column signs).  H (ldh >= m) and W (ldw >= m) column-major, in place. */
int cal_qrstep(int m, double* H, int ldh, double* W, int ldw, double mu);

/* Residency generation of the MEX shims' device copies of A (mex/
 * cal_mex_common.h).  Every shim keeps A resident across calls and re-uploads
 * it when the pointers, nnz, a sampled digest of jc/ir/pr or this
 * process-wide generation change.  An in-place edit of A's values that the
 * sampled digest does not cover needs the explicit invalidation, which bumps
 * the generation for every shim of the process (MATLAB:
 * calanczos_invalidate(), or `clear mex`).  Thread-safe. */
long long cal_residency_generation(void);
long long cal_residency_invalidate(void); /* returns the new generation */

#ifdef __cplusplus
}
#endif
#endif /* CALANCZOS_HOST_H */
