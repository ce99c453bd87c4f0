/* normalize.mexa64 -- [Q, R, rank] = normalize(X, opt, tol)        (normalize.m:3-51)
 * opt 'None' (default) or 'randomizeNullSpace'; tol default 1e-8 (:5-10).
 * The reference only disp()s in randomizeNullSpace (:40-41); so does this. */
#include "cal_mex_common.h"

void mexFunction(int nlhs, mxArray* plhs[], int nrhs, const mxArray* prhs[]) {
    if (nrhs < 1 || nrhs > 3) mexErrMsgIdAndTxt("calanczos:arg", "[Q,R,rank] = normalize(X[,opt[,tol]])");
    cal_ctx* c = cal_mex_plain_ctx();
    char opt[32] = "None";
    cal_mex_opt_string(nrhs, prhs, 1, opt, sizeof opt);
    const double tol = nrhs > 2 ? mxGetScalar(prhs[2]) : 1.0e-8;
    const mwSize n = mxGetM(prhs[0]), m = mxGetN(prhs[0]);
    plhs[0] = mxCreateDoubleMatrix(n, m, mxREAL);
    mxArray* R = mxCreateDoubleMatrix(m, m, mxREAL);
    int rank = 0;
    const int st = cal_normalize_opt(c, (int64_t)n, (int)m, mxGetPr(prhs[0]), opt, tol, mxGetPr(plhs[0]),
                                     mxGetPr(R), &rank);
    if (st < 0) cal_mex_check(st);
    if (st == CAL_WARN_RANK_DEFICIENT && (opt[0] == 'r' || opt[0] == 'R')) {
        mexPrintf("Randomize null space.\n");
        mexPrintf("Rank %d\n", rank);
    }
    if (nlhs > 1) plhs[1] = R;
    if (nlhs > 2) plhs[2] = mxCreateDoubleScalar((double)rank);
}
