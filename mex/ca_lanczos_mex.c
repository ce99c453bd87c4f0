/* ca_lanczos.mexa64 -- [T, Q, rn, oe] = ca_lanczos(A, r, s, iter, basis, orth)
 * The whole outer loop device-resident (SURVEY §8b tier 2); diagnostics run
 * when rn / oe are requested (they never feed back into T, Q).
 *                                                          (ca_lanczos.m:24-86) */
#include "cal_mex_common.h"

void mexFunction(int nlhs, mxArray* plhs[], int nrhs, const mxArray* prhs[]) {
    if (nrhs < 5) mexErrMsgIdAndTxt("calanczos:arg", "[T,Q,rn,oe] = ca_lanczos(A,r,s,iter,basis[,orth])");
    cal_ctx* c = cal_mex_ctx_full(prhs[0]);
    const mwSize n = mxGetN(prhs[0]);
    const int s = (int)mxGetScalar(prhs[2]), iter = (int)mxGetScalar(prhs[3]);
    if (s < 1 || iter < 1) mexErrMsgIdAndTxt("calanczos:arg", "s and iter must be positive");
    const int t = (iter + s - 1) / s;                                  /* :52 */
    char basis[16] = "monomial", orth[16] = "local";
    cal_mex_opt_string(nrhs, prhs, 4, basis, sizeof basis);
    cal_mex_opt_string(nrhs, prhs, 5, orth, sizeof orth);
    const int st = s * t;
    plhs[0] = mxCreateDoubleMatrix(st, st, mxREAL);
    double* Q = NULL;
    double* rn = NULL;
    double* oe = NULL;
    if (nlhs > 1) {
        plhs[1] = mxCreateDoubleMatrix(n, st, mxREAL);
        Q = mxGetPr(plhs[1]);
    }
    if (nlhs > 2) {
        plhs[2] = mxCreateDoubleMatrix(t, st, mxREAL);
        rn = mxGetPr(plhs[2]);
    }
    if (nlhs > 3) {
        plhs[3] = mxCreateDoubleMatrix(t, 1, mxREAL);
        oe = mxGetPr(plhs[3]);
    }
    cal_lanczos_info info;
    cal_mex_check(cal_ca_lanczos(c, mxGetPr(prhs[1]), s, iter, basis, orth, nlhs > 2, mxGetPr(plhs[0]), Q, rn, oe,
                                 NULL, &info));
}
