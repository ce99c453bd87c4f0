/* tsqr.mexa64 -- [Q, R] = tsqr(A): Householder TSQR, diag(R) >= 0  (tsqr.m:7-12) */
#include "cal_mex_common.h"

void mexFunction(int nlhs, mxArray* plhs[], int nrhs, const mxArray* prhs[]) {
    if (nrhs != 1) mexErrMsgIdAndTxt("calanczos:arg", "[Q,R] = tsqr(A)");
    cal_ctx* c = cal_mex_plain_ctx();
    const mwSize n = mxGetM(prhs[0]), m = mxGetN(prhs[0]);
    plhs[0] = mxCreateDoubleMatrix(n, m, mxREAL);
    mxArray* R = mxCreateDoubleMatrix(m, m, mxREAL);
    cal_mex_check(cal_tsqr(c, (int64_t)n, (int)m, mxGetPr(prhs[0]), mxGetPr(plhs[0]), mxGetPr(R)));
    if (nlhs > 1) plhs[1] = R;
}
