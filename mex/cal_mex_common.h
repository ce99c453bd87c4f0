/* cal_mex_common.h -- shared by every MEX shim in mex/ (a MEX file
 * of the same name shadows the reference's .m file).
 *
 * One cal_ctx per MATLAB session keeps A (and the CA-Lanczos state) resident
 * in HBM across calls; it is re-uploaded only when a different sparse matrix
 * arrives and destroyed at mexAtExit (`clear mex` forces a fresh upload).
 * "Different" compares the jc / ir / pr pointers, nnz AND a 64-bit digest of
 * the ir and pr contents: an in-place edit A(i,j)=v of an existing nonzero, or
 * a new matrix MATLAB allocates at freed addresses with the same nnz, keeps
 * all four equal, and must not run on the stale device copy.  The digest reads
 * 16 bytes per nonzero on the host (~0.1 s at nnz = 7e7, against ~1 s for the
 * upload and format analysis it saves).  MATLAB calls mexFunction on one thread, which matches the
 * ABI's one-thread-per-context rule. */
#ifndef CAL_MEX_COMMON_H
#define CAL_MEX_COMMON_H
#include <stdint.h>
#include <string.h>

#include "mex.h"
#include "calanczos.h"

static cal_ctx* g_ctx = NULL;
static const void* g_jc = NULL;
static const void* g_ir = NULL;
static const void* g_pr = NULL;
static mwSize g_nnz = 0;
static uint64_t g_digest = 0;

/* order-sensitive 64-bit digest of a byte range (multiply-xorshift per word) */
static uint64_t cal_mex_digest(uint64_t h, const void* p, size_t bytes) {
    const unsigned char* b = (const unsigned char*)p;
    size_t i = 0;
    for (; i + 8 <= bytes; i += 8) {
        uint64_t w;
        memcpy(&w, b + i, 8);
        h ^= w + 0x9e3779b97f4a7c15ULL + (h << 6) + (h >> 2);
        h *= 0xff51afd7ed558ccdULL;
        h ^= h >> 33;
    }
    for (; i < bytes; ++i) {
        h ^= b[i];
        h *= 0x100000001b3ULL;
    }
    return h;
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
static cal_ctx* cal_mex_ctx(const mxArray* A) {
    if (!mxIsSparse(A) || mxIsComplex(A) || mxGetM(A) != mxGetN(A))
        mexErrMsgIdAndTxt("calanczos:arg", "A must be a real square sparse matrix");
    cal_ctx* c = cal_mex_plain_ctx();
    const mwIndex* jc = mxGetJc(A);
    const mwSize n = mxGetN(A), nnz = jc[n];
    uint64_t d = cal_mex_digest(0xcbf29ce484222325ULL, jc, (n + 1) * sizeof(mwIndex));
    d = cal_mex_digest(d, mxGetIr(A), nnz * sizeof(mwIndex));
    d = cal_mex_digest(d, mxGetPr(A), nnz * sizeof(double));
    if (jc != g_jc || mxGetIr(A) != g_ir || mxGetPr(A) != g_pr || nnz != g_nnz || d != g_digest) {
        cal_mex_check(cal_set_matrix_csc(c, (int64_t)n, (const int64_t*)jc, (const int64_t*)mxGetIr(A),
                                         mxGetPr(A)));
        g_jc = jc;
        g_ir = mxGetIr(A);
        g_pr = mxGetPr(A);
        g_nnz = nnz;
        g_digest = d;
    }
    return c;
}

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
