/* SpMV.mexa64 -- Av = SpMV(A, v)                               (SpMV.m:6-8) */
#include "cal_mex_common.h"

void mexFunction(int nlhs, mxArray* plhs[], int nrhs, const mxArray* prhs[]) {
    (void)nlhs;
    if (nrhs != 2) mexErrMsgIdAndTxt("calanczos:arg", "Av = SpMV(A, v)");
    cal_ctx* c = cal_mex_ctx(prhs[0]);
    const mwSize n = mxGetN(prhs[0]);
    if (mxGetM(prhs[1]) != n || mxGetN(prhs[1]) != 1) mexErrMsgIdAndTxt("calanczos:arg", "v must be n x 1");
    plhs[0] = mxCreateDoubleMatrix(n, 1, mxREAL);
    cal_mex_check(cal_spmv(c, mxGetPr(prhs[1]), mxGetPr(plhs[0])));
}
