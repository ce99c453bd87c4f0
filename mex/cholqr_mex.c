/* cholqr.mexa64 -- [Q, R] = cholqr(X): G = X'X, R = chol(G), Q = X/R  (cholqr.m:3-8) */
#include "cal_mex_common.h"

void mexFunction(int nlhs, mxArray* plhs[], int nrhs, const mxArray* prhs[]) {
    if (nrhs != 1) mexErrMsgIdAndTxt("calanczos:arg", "[Q,R] = cholqr(X)");
    cal_ctx* c = cal_mex_plain_ctx();
    const mwSize n = mxGetM(prhs[0]), m = mxGetN(prhs[0]);
    plhs[0] = mxCreateDoubleMatrix(n, m, mxREAL);
    mxArray* R = mxCreateDoubleMatrix(m, m, mxREAL);
    cal_mex_check(cal_cholqr(c, (int64_t)n, (int)m, mxGetPr(prhs[0]), mxGetPr(plhs[0]), mxGetPr(R)));
    if (nlhs > 1) plhs[1] = R;
}
