/*
 * calanczos.h -- C ABI of the MI355X-native CA-Lanczos hot path.
 *
 * Drop-in boundary for the MATLAB reference (magnusgrandin/ca-lanczos).  The
 * reference resolves every hot-path function by file name, so a MEX file of
 * the same name shadows the .m file.  Each entry point below
 * is what such a MEX shim binds; the comment on each cites
 * the reference interface it replaces.
 *
 * Conventions
 *  - Dense matrices are column-major double (MATLAB layout).  Host-pointer
 *    entry points take leading dimension == rows.
 *  - A is the n x n sparse symmetric matrix.  It is handed over once per
 *    context (cal_set_matrix_*), kept resident in HBM and reused by every
 *    call, as the SURVEY §8b "two tiers" design prescribes.
 *  - Every function returns an int status: 0 ok, < 0 error, > 0 warning.
 *    cal_last_error(ctx) holds the message of the last non-zero status.
 *  - Calls are synchronous (outputs valid on return) and a context may be
 *    used by one host thread at a time, like mexFunction.
 *  - Cell arrays of blocks ({Q1,Q2,...}) are passed as (nblocks, const
 *    double* const* blocks, const int* widths); a block of width 0 is the
 *    MATLAB empty matrix [].
 */
#ifndef CALANCZOS_H
#define CALANCZOS_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CAL_OK 0
#define CAL_ERR_ARG (-1)          /* bad argument (reference: disp()+return)        */
#define CAL_ERR_HIP (-2)          /* HIP runtime failure                            */
#define CAL_ERR_NOMATRIX (-3)     /* no matrix set on the context                   */
#define CAL_ERR_NUMERIC (-4)      /* NaN/Inf, Leja error() cases                    */
#define CAL_ERR_COMM (-5)         /* collective / halo failure                      */
#define CAL_ERR_UNSUPPORTED (-6)  /* option outside the built scope                 */
#define CAL_WARN_RANK_DEFICIENT 1 /* reference: disp('Rank deficient'), continues   */
#define CAL_WARN_BREAKDOWN 2      /* rho_t == 0 or beta == 0 (reference divides)    */

typedef struct cal_ctx cal_ctx;

/* ---- context lifecycle ------------------------------------------------- */
int cal_version(void);
int cal_device_count(int* count);
/* Create a context on HIP device `device` with its own stream. */
int cal_create(int device, cal_ctx** out);
void cal_destroy(cal_ctx* ctx);
const char* cal_last_error(const cal_ctx* ctx);
int cal_synchronize(cal_ctx* ctx);
/* Kernel-duration timer (HIP events on the context stream).  kind: "spmv",
 * "gram", "apply", "other", "allreduce", "halo" (the RCCL calls), "normest"
 * (the span of the implicit restart's normest on its own stream), "all".
 * Returns the number of launches timed and their summed duration since the
 * last reset. */
int cal_timer_enable(cal_ctx* ctx, int on);
int cal_timer_read(cal_ctx* ctx, const char* kind, int64_t* count, double* total_ms);
/* The algorithmic HBM bytes of the timed launches of a kind
 * since the last reset (the roofline's numerator; 0 for launches that state
 * none). */
int cal_timer_bytes(cal_ctx* ctx, const char* kind, double* bytes);
int cal_timer_reset(cal_ctx* ctx);

/* ---- the sparse matrix A ------------------------------------------------ */
/* MATLAB mxArray sparse storage (CSC: jc colptr, ir rowidx, pr values, all
 * mwIndex = int64), transposed into CSR on the host, so the device holds A
 * (not A') for any A; rows keep ascending columns, MATLAB's accumulation
 * order.  Replaces the `A` argument of SpMV.m:6, ca_lanczos.m:24. */
int cal_set_matrix_csc(cal_ctx* ctx, int64_t n, const int64_t* jc, const int64_t* ir, const double* pr);
/* CSR with int64 row pointers and int32 column indices (SciPy layout). */
int cal_set_matrix_csr(cal_ctx* ctx, int64_t n, const int64_t* rowptr, const int32_t* colind, const double* val);
/* Row-slab of a distributed matrix: rows [row0, row0+nlocal) of the global
 * n_global x n_global matrix, global column indices.  Requires a communicator
 * (cal_comm_*) when nranks > 1. */
int cal_set_matrix_csr_dist(cal_ctx* ctx, int64_t n_global, int64_t row0, int64_t nlocal,
                            const int64_t* rowptr, const int64_t* colind_global, const double* val);
int cal_matrix_info(cal_ctx* ctx, int64_t* n_local, int64_t* nnz_local, int64_t* n_global, int64_t* nghost);
/* CA matrix-powers kernel of a distributed banded matrix (window halo layout,
 * row-pattern format): each slab also stores the rows of its (depth-1)-band
 * deep ghost zone, so the s <= depth powers of matrix_powers_* / one
 * CA-Lanczos outer iteration need ONE halo exchange of q's s-band deep ghost
 * zone instead of s (the reference's SpMV.m / matrix_powers_*.m
 * are serial, the powers are bit-identical either way).  Applies at the next
 * cal_set_matrix_csr_dist; depth 1 turns it off; default 8.  mpk_info reports
 * the active depth (1 = off), the global band and the stored row count. */
int cal_set_mpk_depth(cal_ctx* ctx, int depth);
int cal_mpk_info(cal_ctx* ctx, int* depth, int64_t* band_l, int64_t* band_r, int64_t* n_rows);
/* Schedule the last matrix-powers call took: 0 one halo exchange per SpMV,
 * 1 one deep exchange, 2 one deep exchange on the RCCL stream overlapped
 * with the interior powers, 3 the split schedule without an exchange (one
 * rank, CAL_MPK_FAKE_BAND), 4 the host-staged twin of 2 (the exchange's
 * copies on the communicator's stream, its callbacks on a comm thread, the
 * same ev_q / ev_halo event graph); -1 before the first call. */
int cal_mpk_schedule(cal_ctx* ctx, int* schedule);
/* SpMV-class kernel launches the last matrix-powers call made on this rank
 * (one per power: split schedules count their powers, not their two-range
 * pieces); 0 before the first call. */
int cal_powers_launches(cal_ctx* ctx, int* launches);
/* Device storage of A, chosen at the next cal_set_matrix_*: "auto" (default:
 * row patterns when A has <= 65535 distinct rows of <= 32 entries, else
 * CSR), "csr", or "pattern".  Both are lossless and give bit-identical SpMV
 * results (same per-row summation order). */
int cal_set_spmv_format(cal_ctx* ctx, const char* fmt);
int cal_spmv_format(cal_ctx* ctx, int* is_pattern, int* npatterns, int* nentries);
/* Pair patterns of the row-pattern format (two rows per lane): number of
 * merged pair patterns, their table entries, and pairs on the per-row path. */
int cal_spmv_pair_info(cal_ctx* ctx, int* npairpatterns, int* nentries, int64_t* nsplit);
/* The plane march of the row-pattern format (k_spmv_planes, k_resid_planes:
 * a single slab whose canonical slots are -P .. +P with P >= 256 and the
 * other slots within 256 rows): the plane stride P, the in-plane reach H and
 * the key mode (0: uniform slot values keyed by slot-mask bytes, 1 / 2: 1-
 * or 2-byte pattern ids); P = 0, key_mode = -1 when it is not in use. */
int cal_spmv_plane_info(cal_ctx* ctx, int64_t* plane_P, int* plane_H, int* key_mode);
/* Where the s x s algebra between the block-orthogonalisation sweeps runs:
 * "device" (default: one kernel, no host round trip inside a block) or
 * "host".  Both give bit-identical results; "host" exists for testing. */
int cal_set_orth_coef(cal_ctx* ctx, const char* where);
/* Backend of normalize (tsqr.m) on the device: "auto" (default: Householder
 * TSQR for the host-pointer calls cal_tsqr / cal_normalize /
 * cal_project_and_normalize; CholQR2 fused into the CA-Lanczos sweeps, with
 * Householder TSQR whenever its Cholesky fails, i.e. kappa > ~1e8), "tsqr"
 * (Householder TSQR everywhere, the reference's algorithm; multi-GPU: the
 * local trees' roots are all-gathered over RCCL), "cholqr2" (CholQR2
 * everywhere, shifted CholQR3 when its Cholesky fails).  cal_tsqr is always
 * Householder TSQR.  get: 0 auto, 1 tsqr, 2 cholqr2. */
int cal_set_normalize(cal_ctx* ctx, const char* kind);
int cal_get_normalize(cal_ctx* ctx, int* kind);
/* Counters of the fused TSQR projectAndNormalize (Householder TSQR of Y with
 * the second projection folded into the R factor; blockorth.cpp
 * pn_tsqr_fold): blocks run, blocks declined (the explicit-Z TSQR path was
 * taken because the fold's loss-of-orthogonality estimate exceeded 1e-14),
 * and the last block's estimate.  Any pointer may be null. */
int cal_tsqr_fold_stats(cal_ctx* ctx, long long* runs, long long* declined, double* last_est);
/* The fused TSQR's acceptance threshold on its loss-of-orthogonality estimate
 * (default 1e-14, also the maximum): a block whose estimate exceeds it is
 * declined and redone on the explicit-Z path (projectAndNormalize.m:63-64
 * literally), so lowering it keeps the results within the bars.  0 declines
 * every block that takes the second projection, a negative tol every block
 * (the fallback's test hooks); NaN or a tol above 1e-14 (which would accept
 * folds the default declines) is an error. */
int cal_set_tsqr_fold_tol(cal_ctx* ctx, double tol);
/* Device-resident SpMV timing: `reps` launches of y = (A - shift I) x on
 * HBM-resident vectors (x = ones), HIP events around each launch on the
 * context stream; returns the mean and the minimum kernel time. */
int cal_bench_spmv(cal_ctx* ctx, int reps, double shift, double* mean_ms, double* min_ms);

/* ---- a1-a4: SpMV and the s-step matrix-powers kernel -------------------- */
/* Av = SpMV(A,v)                                       SpMV.m:6-8           */
int cal_spmv(cal_ctx* ctx, const double* v, double* Av);
/* V = matrix_powers_monomial(A,q,s); V is n x s        matrix_powers_monomial.m:6-12 */
int cal_matrix_powers_monomial(cal_ctx* ctx, const double* q, int s, double* V);
/* V = matrix_powers_newton(A,v,s,lambda,modifiedp); V is n x (s+1).
 * lambda = lambda_re + i*lambda_im (lambda_im may be NULL: real shifts).
 *                                                      matrix_powers_newton.m:15-54 */
int cal_matrix_powers_newton(cal_ctx* ctx, const double* v, int s, const double* lambda_re,
                             const double* lambda_im, int modifiedp, double* V);

/* ---- a5-a9: tall-skinny block orthogonalisation ------------------------- */
/* [Q,R] = tsqr(A): A n x m -> Q n x m, R m x m upper, diag(R) >= 0.   tsqr.m:7-12
 * Householder TSQR (LAPACK reflectors per tile, reduction tree), m <= 32, n >= m. */
int cal_tsqr(cal_ctx* ctx, int64_t n, int m, const double* A, double* Q, double* R);
/* [Q,R] = cholqr(X): G = X'X, R = chol(G), Q = X/R.                  cholqr.m:3-8 */
int cal_cholqr(cal_ctx* ctx, int64_t n, int m, const double* X, double* Q, double* R);
/* [X,R] = project(Q,X,doreorth); Xout may alias X; R[i] is widths[i] x m.  project.m:7-58 */
int cal_project(cal_ctx* ctx, int64_t n, int nblocks, const double* const* Q, const int* widths,
                int m, const double* X, int doreorth, double* Xout, double* const* R);
/* [Q,R,rank] = normalize(X,'None',tol).                               normalize.m:3-36 */
int cal_normalize(cal_ctx* ctx, int64_t n, int m, const double* X, double tol, double* Q, double* R,
                  int* rank);
/* [Q,R,rank] = normalize(X,opt,tol), opt "None" or "randomizeNullSpace"
 * (normalize.m:28-31,38-51: when rank < m, R = S*W' and Q = Q*U from svd(R),
 * then the null-space columns are replaced by rand (a fresh MT19937 stream,
 * seed 5489 -- cal_matlab_rand), projected against Q(:,1:rank) and tsqr'd).
 * Returns CAL_WARN_RANK_DEFICIENT when rank < m.  m <= 32. */
int cal_normalize_opt(cal_ctx* ctx, int64_t n, int m, const double* X, const char* opt, double tol, double* Q,
                      double* R, int* rank);
/* [QZ,RZ] = projectAndNormalize(Q,X,doreorth); RZ has nblocks+1 entries:
 * RZ[i] widths[i] x m, RZ[nblocks] m x m.  *reorth = 1 when the reference
 * would disp('second').                                    projectAndNormalize.m:3-90 */
int cal_project_and_normalize(cal_ctx* ctx, int64_t n, int nblocks, const double* const* Q,
                              const int* widths, int m, const double* X, int doreorth, double* QZ,
                              double* const* RZ, int* reorth, int* rank);

/* ---- a10-a14: the CA-Lanczos driver ------------------------------------- */
typedef struct cal_lanczos_info {
    int t;              /* outer iterations run                                 */
    int s;
    int n_reorth;       /* projectAndNormalize second passes ('second')         */
    int n_rank_deficient;
    int breakdown;      /* 1 if rho_t == 0 / beta == 0 was hit                  */
    double shifts[64];  /* Newton shifts (first 2s, Leja order; re part)        */
    double shifts_im[64];
    double prologue_ms; /* Newton prologue wall time                            */
    double loop_ms;     /* outer loop wall time (incl. diagnostics)             */
    double diag_ms;     /* of which diagnostics                                 */
    int n_orth_breaks;  /* periodic: full reorthogonalisations; selective: QR rebuilds */
    int n_ritz_locked;  /* selective: converged Ritz vectors in QR               */
    double norm_A;      /* normest(A) (periodic / selective)                    */
    int n_ritz_complex; /* selective: of n_ritz_locked, members of complex pairs */
} cal_lanczos_info;

/* [T,Q,rn,oe] = ca_lanczos(A,r,s,iter,basis,orth).           ca_lanczos.m:24-86
 * basis in {"monomial","newton"}, orth in {"local","full","periodic","selective"}.
 * Outputs (any may be NULL): T (s*t x s*t), Q (n x s*t), rn (t x s*t),
 * oe (t), reorth_flags (t).  t = ceil(iter/s).  diagnostics=0 skips the
 * per-iteration Ritz residuals / orthogonality error (rn, oe left zero);
 * they never feed back into T or Q (ca_lanczos.m:228-236). */
int cal_ca_lanczos(cal_ctx* ctx, const double* r, int s, int iter, const char* basis, const char* orth,
                   int diagnostics, double* T, double* Q, double* rn, double* oe, int* reorth_flags,
                   cal_lanczos_info* info);

/* rn = compute_ritz_rnorm(A,Q,Vp,Dp) for a real eigen-decomposition.  ca_lanczos.m:88-97
 * Q: n_local x k (host, column-major), Vp: k x k, d: the k eigenvalues
 * diag(Dp).  [d,ix] = sort(d,'descend') (stable); rn(i) = ||A x - l x|| /
 * ||l x|| with x = Q*Vp(:,ix(i)), l = d(ix(i)).  The diagnostics' device
 * path: X = Q*Vp on the matrix cores, then the batched residual kernel. */
int cal_compute_ritz_rnorm(cal_ctx* ctx, const double* Q, int k, const double* Vp, const double* d, double* rn);

/* Step-wise, device-resident form of the same loop (benchmarks, restart
 * drivers).  begin() normalises r and runs the basis set-up (Newton
 * prologue); step() runs one outer iteration (s SpMVs + block orth + T
 * update); get() copies the current T (sk x sk, ldt >= sk) and flags.
 * With diagnostics the iteration's rn / oe are computed late (rn one
 * iteration behind; oe of 'local' / 'full' runs of <= 128 columns at the
 * last step, from one Gram of Q): get() finishes whatever is pending, so
 * its rn / oe are always complete for the iterations run so far.  eig(T) of
 * iteration k runs on a host worker thread and is joined one step later: a
 * non-converging eig(T) is reported (CAL_ERR_NUMERIC) by step k+1 or by get(),
 * after step k+1 has already extended T. */
int cal_lanczos_begin(cal_ctx* ctx, const double* r, int s, int max_outer, const char* basis,
                      const char* orth);
int cal_lanczos_step(cal_ctx* ctx, int diagnostics);
int cal_lanczos_state(cal_ctx* ctx, int* k, int* s, int* reorth_last);
int cal_lanczos_get(cal_ctx* ctx, double* T, int ldt, double* rn, double* oe, int* reorth_flags,
                    cal_lanczos_info* info);
int cal_lanczos_get_Q(cal_ctx* ctx, int64_t col0, int ncols, double* Q);
int cal_lanczos_end(cal_ctx* ctx);

/* ---- f2: explicit restart ------------------------------------------------ */
typedef struct cal_restart_info {
    int num_restarts;      /* restarts run (<= 200)                                */
    int nconv;             /* eigenpairs returned                                  */
    int converged;         /* 1 if n_wanted eigenpairs converged                   */
    double norm_A;         /* normest(A)                                           */
    double max_ritz_norm;  /* largest beta|y_m| estimate among the returned pairs  */
    double ms;             /* wall time                                            */
} cal_restart_info;

/* [E,V,nres,rnorms,orth_err] = restarted_ca_lanczos(A,r,max_lanczos,
 * n_wanted_eigs,s,basis,orth,tol)  (restarted_ca_lanczos.m:4-198, restart
 * strategy 'largest').  orth in {"local","full"} (the reference defines no
 * periodic/selective inner solver).  Outputs: conv_eigs (n_wanted, descending;
 * info->nconv valid), Q_conv (n x n_wanted, may be NULL), rnorms (200 x
 * n_wanted column-major, rows 1..num_restarts, may be NULL; needs
 * diagnostics), orth_err (200, may be NULL; needs diagnostics). */
int cal_restarted_ca_lanczos(cal_ctx* ctx, const double* r, int max_lanczos, int n_wanted, int s, const char* basis,
                             const char* orth, double tol, int diagnostics, double* conv_eigs, double* Q_conv,
                             double* rnorms, double* orth_err, cal_restart_info* info);

/* ---- f3: implicit restart ------------------------------------------------ */
/* [conv_eigs,Q_conv,num_restarts] = impl_restarted_ca_lanczos(A,r,max_lanczos,
 * n_wanted_eigs,s,basis,orth,tol)  (impl_restarted_ca_lanczos.m:4-226).  The
 * reference file does not run; this is the implicit restart it
 * sets out to implement: k = max(n_wanted+4, s) kept vectors, p = s*floor(
 * (max_lanczos-k)/s) exact shifts by qrstep (:623-678) per restart, CA blocks
 * of lanczos_basic (:333-426) with orth 'full' (the only branch that is
 * defined: others return CAL_ERR_UNSUPPORTED), at most 40 restarts (:7).
 * Converged when the n_wanted largest-modulus Ritz pairs of T_k all have
 * ||r_k|||e_k'y| < tol*normest(A).  Outputs: conv_eigs (n_wanted,
 * descending), Q_conv (n x n_wanted, may be NULL), ritz_est (40 x n_wanted
 * column-major: the estimates after each restart, may be NULL).
 * Parity unpinned (no runnable reference): checked against analytic spectra
 * and scipy eigsh. */
int cal_impl_restarted_ca_lanczos(cal_ctx* ctx, const double* r, int max_lanczos, int n_wanted, int s,
                                  const char* basis, const char* orth, double tol, double* conv_eigs,
                                  double* Q_conv, double* ritz_est, cal_restart_info* info);

/* ---- multi-GPU (row slabs, RCCL over xGMI) ------------------------------ */
/* 128-byte RCCL unique id; broadcast it out of band (e.g. torch.distributed). */
int cal_comm_unique_id(void* id128);
int cal_comm_init_rccl(cal_ctx* ctx, int nranks, int rank, const void* id128);
/* Communicator statistics since the last reset (reset != 0 zeroes them after
 * reading): stats[0] ranks, [1] kind (0 none, 1 RCCL, 2 host-staged), [2]
 * ncclCommCount (-1 unless RCCL), [3] all-reduces issued, [4] doubles they
 * carried, [5] halo exchanges, [6] doubles exchanged (sent + received), [7]
 * rows computed by SpMV launches (with the CA matrix powers: the slab's rows
 * plus the shrinking ghost-zone ranges).  nstats <= 8.  The timer kinds
 * "allreduce" and "halo" time the RCCL calls (cal_timer_read). */
int cal_comm_stats(cal_ctx* ctx, int64_t* stats, int nstats, int reset);
/* Host-staged communicator (tests, CPU rendezvous): device buffers are
 * staged through pinned host memory and handed to these callbacks.  The
 * callbacks run on the caller's thread, except with the opt-in overlapped
 * matrix-powers schedule (environment CAL_MPK_OVERLAP=1, a rehearsal of the
 * RCCL schedule): there the exchange callback runs on a library-owned thread
 * while the caller's thread enqueues the interior powers, so the transport
 * must allow calls from another thread (MPI_THREAD_MULTIPLE or
 * MPI_THREAD_SERIALIZED with no concurrent use by the caller). */
typedef int (*cal_allreduce_fn)(void* user, double* buf, int64_t count);
typedef int (*cal_exchange_fn)(void* user, int peer, const double* send, int64_t nsend, double* recv,
                               int64_t nrecv);
int cal_comm_init_host(cal_ctx* ctx, int nranks, int rank, cal_allreduce_fn allreduce,
                       cal_exchange_fn exchange, void* user);
int cal_comm_info(cal_ctx* ctx, int* nranks, int* rank, int* kind);

#ifdef __cplusplus
}
#endif
#endif /* CALANCZOS_H */
