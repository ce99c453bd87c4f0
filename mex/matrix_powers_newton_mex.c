/* matrix_powers_newton.mexa64 -- V = matrix_powers_newton(A, v, s, lambda, modifiedp)
 * n x (s+1); complex shifts through the separate-complex API (mex -R2017b).
 *                                               (matrix_powers_newton.m:15-54) */
#include "cal_mex_common.h"

void mexFunction(int nlhs, mxArray* plhs[], int nrhs, const mxArray* prhs[]) {
    (void)nlhs;
    if (nrhs < 4) mexErrMsgIdAndTxt("calanczos:arg", "V = matrix_powers_newton(A,v,s,lambda[,modifiedp])");
    cal_ctx* c = cal_mex_ctx(prhs[0]);
    const mwSize n = mxGetN(prhs[0]);
    const int s = (int)mxGetScalar(prhs[2]);
    const int modifiedp = nrhs > 4 ? (int)mxGetScalar(prhs[4]) : 0;   /* :16-18 default */
    if ((int)mxGetNumberOfElements(prhs[3]) < s) mexErrMsgIdAndTxt("calanczos:arg", "lambda needs s entries");
    const double* lre = mxGetPr(prhs[3]);
    const double* lim = mxIsComplex(prhs[3]) ? mxGetPi(prhs[3]) : NULL;
    plhs[0] = mxCreateDoubleMatrix(n, s + 1, mxREAL);
    cal_mex_check(cal_matrix_powers_newton(c, mxGetPr(prhs[1]), s, lre, lim, modifiedp, mxGetPr(plhs[0])));
}
