/* cal_mex_common.h -- shared by every MEX shim in mex/ (a MEX file
 * of the same name shadows the reference's .m file).
 *
 * One cal_ctx per MATLAB session keeps A (and the CA-Lanczos state) resident
 * in HBM across calls; it is re-uploaded only when a different sparse matrix
 * arrives (jc / ir / pr pointers and nnz compared) and destroyed at
 * mexAtExit.  MATLAB calls mexFunction on one thread, which matches the
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
 * CSC with mwIndex (int64) jc / ir; A is symmetric, so cal_set_matrix_csc
 * consumes the CSC arrays as CSR. */
static cal_ctx* cal_mex_ctx(const mxArray* A) {
    if (!mxIsSparse(A) || mxIsComplex(A) || mxGetM(A) != mxGetN(A))
        mexErrMsgIdAndTxt("calanczos:arg", "A must be a real square sparse matrix");
    cal_ctx* c = cal_mex_plain_ctx();
    const mwIndex* jc = mxGetJc(A);
    const mwSize n = mxGetN(A), nnz = jc[n];
    if (jc != g_jc || mxGetIr(A) != g_ir || mxGetPr(A) != g_pr || nnz != g_nnz) {
        cal_mex_check(cal_set_matrix_csc(c, (int64_t)n, (const int64_t*)jc, (const int64_t*)mxGetIr(A),
                                         mxGetPr(A)));
        g_jc = jc;
        g_ir = mxGetIr(A);
        g_pr = mxGetPr(A);
        g_nnz = nnz;
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
