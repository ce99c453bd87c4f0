/* matrix_powers_monomial.mexa64 -- V = matrix_powers_monomial(A, q, s), n x s
 *                                            (matrix_powers_monomial.m:6-12) */
#include "cal_mex_common.h"

void mexFunction(int nlhs, mxArray* plhs[], int nrhs, const mxArray* prhs[]) {
    (void)nlhs;
    if (nrhs != 3) mexErrMsgIdAndTxt("calanczos:arg", "V = matrix_powers_monomial(A,q,s)");
    cal_ctx* c = cal_mex_ctx(prhs[0]);
    const mwSize n = mxGetN(prhs[0]);
    const int s = (int)mxGetScalar(prhs[2]);
    if (mxGetM(prhs[1]) != n) mexErrMsgIdAndTxt("calanczos:arg", "q must be n x 1");
    plhs[0] = mxCreateDoubleMatrix(n, s, mxREAL);
    cal_mex_check(cal_matrix_powers_monomial(c, mxGetPr(prhs[1]), s, mxGetPr(plhs[0])));
}
