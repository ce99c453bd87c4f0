/* cal_mex_common.h -- shared by every MEX shim in mex/ (a MEX file
 * of the same name shadows the reference's .m file).
 *
 * One cal_ctx per shim keeps A (and the CA-Lanczos state) resident in HBM
 * across calls; it is destroyed at mexAtExit (`clear mex` forces a fresh
 * upload).  The residency decision must cost far less than the call it
 * serves (SpMV.mexa64 is called s times per outer iteration from the
 * unchanged matrix_powers_newton.m:32, against ~1 ms of device work), so it
 * reads a bounded number of entries, independent of nnz:
 *   - the jc / ir / pr pointers, n and nnz;
 *   - a digest of a fixed sample of the arrays: the first and last 32
 *     entries of each and up to kCalMexSamples evenly spaced entries of jc,
 *     ir and pr (≈1 ms at nnz = 7e7, tests/test_mex_shims.py);
 *   - the library's process-wide residency generation
 *     (cal_residency_generation, calanczos_host.h).
 * A different matrix that MATLAB allocates at freed addresses with the same
 * nnz, or an edit of a sampled entry, re-uploads.  In the per-power shims
 * (SpMV, matrix_powers_*), an in-place edit A(i,j) = v of an existing nonzero
 * that the sample misses is not seen: after such an edit call
 * calanczos_invalidate() (mex/calanczos_invalidate_mex.c, which bumps the
 * generation for every shim of the process) or `clear mex`.  The solver shims
 * (ca_lanczos, restarted_ca_lanczos, impl_restarted_ca_lanczos) run once per
 * solve, so they digest every entry of jc / ir / pr (cal_mex_ctx_full: about
 * 0.1 s at nnz = 7e7, next to a solve of seconds) and see every edit, as the
 * reference's SpMV.m:8 reads the current A.
 * MATLAB calls mexFunction on one thread, which matches the ABI's
 * one-thread-per-context rule. */
#ifndef CAL_MEX_COMMON_H
#define CAL_MEX_COMMON_H
#include <stdint.h>
#include <string.h>

#include "mex.h"
#include "calanczos.h"
#include "calanczos_host.h"

#define kCalMexSamples 16384

static cal_ctx* g_ctx = NULL;
static const void* g_jc = NULL;
static const void* g_ir = NULL;
static const void* g_pr = NULL;
static mwSize g_n = 0;
static mwSize g_nnz = 0;
/* one digest per mode (0 sampled, 1 full), both taken at upload: a call
 * compares the digest of its own mode, so alternating per-power and solver
 * shims on an unchanged A never re-uploads it */
static uint64_t g_digest[2] = {0, 0};
static long long g_gen = -1;

/* order-sensitive 64-bit mix of one word */
static uint64_t cal_mex_mix(uint64_t h, uint64_t w) {
    h ^= w + 0x9e3779b97f4a7c15ULL + (h << 6) + (h >> 2);
    h *= 0xff51afd7ed558ccdULL;
    h ^= h >> 33;
    return h;
}

/* digest of an array of `count` 8-byte words: every word (full), or a
 * bounded sample: the first and last 32 and up to kCalMexSamples evenly
 * spaced ones */
static uint64_t cal_mex_sample(uint64_t h, const void* p, size_t count, int full) {
    const unsigned char* b = (const unsigned char*)p;
    uint64_t w;
    size_t i, edge = count < 64 ? count : 32;
    if (full) {
        for (i = 0; i < count; ++i) {
            memcpy(&w, b + 8 * i, 8);
            h = cal_mex_mix(h, w);
        }
        return h;
    }
    for (i = 0; i < edge; ++i) {
        memcpy(&w, b + 8 * i, 8);
        h = cal_mex_mix(h, w);
    }
    for (i = count > edge ? count - edge : edge; i < count; ++i) {
        memcpy(&w, b + 8 * i, 8);
        h = cal_mex_mix(h, w);
    }
    if (count > 64) {
        const size_t step = count / kCalMexSamples > 1 ? count / kCalMexSamples : 1;
        for (i = 0; i < count; i += step) {
            memcpy(&w, b + 8 * i, 8);
            h = cal_mex_mix(h, w);
        }
    }
    return h;
}

/* the residency decision: 1 when the device copy must be (re)uploaded */
static uint64_t cal_mex_digest(const mwIndex* jc, const mwIndex* ir, const double* pr, mwSize n, int full) {
    const mwSize nnz = jc[n];
    uint64_t d = cal_mex_sample(0xcbf29ce484222325ULL ^ (uint64_t)n, jc, n + 1, full);
    d = cal_mex_sample(d, ir, nnz, full);
    return cal_mex_sample(d, pr, nnz, full);
}

static int cal_mex_stale(const mwIndex* jc, const mwIndex* ir, const double* pr, mwSize n, long long gen,
                         int full, uint64_t* digest) {
    const mwSize nnz = jc[n];
    const uint64_t d = cal_mex_digest(jc, ir, pr, n, full);
    *digest = d;
    return jc != g_jc || ir != g_ir || pr != g_pr || n != g_n || nnz != g_nnz || gen != g_gen ||
           d != g_digest[full ? 1 : 0];
}

static void cal_mex_exit(void) {
    if (g_ctx) cal_destroy(g_ctx);
    g_ctx = NULL;
}

/* status < 0: MATLAB error (the reference's error()/disp+return); > 0: warning */
static void cal_mex_check(int st) {
    if (st < 0) mexErrMsgIdAndTxt("calanczos:error", "%s", cal_last_error(g_ctx));
    if (st > 0) mexWarnMsgIdAndTxt("calanczos:warning", "%s", cal_last_error(g_ctx));
}

static cal_ctx* cal_mex_plain_ctx(void) {
    if (!g_ctx) {
        cal_mex_check(cal_create(0, &g_ctx));
        mexAtExit(cal_mex_exit);
    }
    return g_ctx;
}

/* Make A resident (the `A` of SpMV.m:6 / ca_lanczos.m:24).  MATLAB sparse is
 * CSC with mwIndex (int64) jc / ir; cal_set_matrix_csc transposes it into CSR,
 * so the device holds A itself (SpMV.m:8 is a general A*v). */
static cal_ctx* cal_mex_ctx_mode(const mxArray* A, int full) {
    if (!mxIsSparse(A) || mxIsComplex(A) || mxGetM(A) != mxGetN(A))
        mexErrMsgIdAndTxt("calanczos:arg", "A must be a real square sparse matrix");
    cal_ctx* c = cal_mex_plain_ctx();
    const mwIndex* jc = mxGetJc(A);
    const mwSize n = mxGetN(A);
    const long long gen = cal_residency_generation();
    uint64_t d = 0;
    if (cal_mex_stale(jc, mxGetIr(A), mxGetPr(A), n, gen, full, &d)) {
        cal_mex_check(cal_set_matrix_csc(c, (int64_t)n, (const int64_t*)jc, (const int64_t*)mxGetIr(A),
                                         mxGetPr(A)));
        g_jc = jc;
        g_ir = mxGetIr(A);
        g_pr = mxGetPr(A);
        g_n = n;
        g_nnz = jc[n];
        g_digest[full ? 1 : 0] = d;
        g_digest[full ? 0 : 1] = cal_mex_digest(jc, mxGetIr(A), mxGetPr(A), n, !full);
        g_gen = gen;
    }
    return c;
}

/* the per-power shims: sampled digest + generation */
static cal_ctx* cal_mex_ctx(const mxArray* A) { return cal_mex_ctx_mode(A, 0); }
/* the solver shims: every entry digested */
static cal_ctx* cal_mex_ctx_full(const mxArray* A) { return cal_mex_ctx_mode(A, 1); }

/* a cell array {Q1, Q2, ...} -> (nblocks, blocks, widths); [] has width 0 */
static int cal_mex_cell(const mxArray* cell, const double*** Q, int** w) {
    if (!mxIsCell(cell)) mexErrMsgIdAndTxt("calanczos:arg", "Input Q (arg 1) must be cell (block) array.");
    const int B = (int)mxGetNumberOfElements(cell);
    *Q = (const double**)mxCalloc(B > 0 ? B : 1, sizeof(double*));
    *w = (int*)mxCalloc(B > 0 ? B : 1, sizeof(int));
    for (int i = 0; i < B; ++i) {
        const mxArray* Qi = mxGetCell(cell, i);
        (*w)[i] = (Qi && !mxIsEmpty(Qi)) ? (int)mxGetN(Qi) : 0;
        (*Q)[i] = (*w)[i] ? mxGetPr(Qi) : NULL;
    }
    return B;
}

static void cal_mex_opt_string(int nrhs, const mxArray* prhs[], int i, char* buf, mwSize len) {
    if (nrhs > i && mxIsChar(prhs[i])) mxGetString(prhs[i], buf, len);
}
#endif
