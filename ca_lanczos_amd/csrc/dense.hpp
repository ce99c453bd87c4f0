// dense.hpp -- small dense host linear algebra for the s x s / (sk) x (sk)
// matrices of the CA-Lanczos outer loop (no LAPACK dependency).
// All matrices are column-major: A(i,j) = A[i + j*ld].
#pragma once

#include <cstdint>
#include <random>
#include <vector>

namespace cal {
namespace dense {

// Upper Cholesky G = R^T R (m x m).  Returns false if G is not positive
// definite (a non-positive or non-finite pivot).
bool chol_upper(int m, const double* G, int ldg, double* R, int ldr);
// Inverse of an upper-triangular R (m x m) into Ri (upper).
void tri_inv_upper(int m, const double* R, int ldr, double* Ri, int ldi);
// C = A (m x k) * B (k x n)
void matmul(int m, int k, int n, const double* A, int lda, const double* B, int ldb, double* C, int ldc);
// X (r x m) <- X / R for upper-triangular R (MATLAB right division).
void rdiv_upper(int r, int m, double* X, int ldx, const double* R, int ldr);
// Eigenvalues of the symmetric tridiagonal matrix (diag d, off-diagonal e,
// n-1 entries), ascending.  Implicit QL.
bool tridiag_eigvals(int n, const double* d, const double* e, double* w);
// Singular values of a small square matrix (one-sided Jacobi), descending.
void singular_values(int m, const double* A, int lda, double* sv);
// Full SVD A = U diag(S) V' of a small square matrix (one-sided Jacobi),
// singular values descending; U completed to orthonormal for zero values.
void svd(int m, const double* A, int lda, double* U, double* S, double* V);
// General real eigenproblem (Householder Hessenberg reduction + shifted QR,
// EISPACK orthes/hqr2 algorithm).  A (n x n) is not modified.  On return
// wr/wi hold the eigenvalues; V (n x n) holds real vectors in the column of a
// real eigenvalue, and for a complex pair (wi[j] > 0, wi[j+1] = -wi[j])
// columns j and j+1 hold the real and imaginary part of the eigenvector of
// wr[j] + i wi[j].  Returns false if QR failed to converge.
bool eig_general(int n, const double* A, int lda, double* wr, double* wi, double* V, int ldv);
// Symmetric eigenproblem (tred2 + tql2), ascending, orthonormal vectors;
// V = NULL computes the same values without the vectors.
void eig_symmetric(int n, const double* A, int lda, double* w, double* V, int ldv);
// One explicit shifted QR step on an upper-Hessenberg H: H <- Q'HQ,
// W <- WQ with H - mu I = QR (Givens rotations; qrstep of the implicit restart).
void hess_qrstep(int m, double* H, int ldh, double* W, int ldw, double mu);
// count such steps, shifts mu[0..count) in order (W's rotations batched:
// the same bits as count hess_qrstep calls)
void hess_qrsteps(int m, double* H, int ldh, double* W, int ldw, const double* mu, int count);
// `count` draws of MATLAB's rand from the MT19937 stream g (genrand_res53:
// two 32-bit words per double)
void matlab_rand(std::mt19937& g, int64_t count, double* out);

}  // namespace dense
}  // namespace cal
