/* project.mexa64 -- [X, R] = project(Q, X, doreorth)                  (project.m:7-58)
 * Q is a cell of blocks ([] allowed); R a 1 x B cell of w_i x m blocks. */
#include "cal_mex_common.h"

void mexFunction(int nlhs, mxArray* plhs[], int nrhs, const mxArray* prhs[]) {
    if (nrhs < 2) mexErrMsgIdAndTxt("calanczos:arg", "[X,R] = project(Q,X[,doreorth])");
    cal_ctx* c = cal_mex_plain_ctx();
    const double** Q;
    int* w;
    const int B = cal_mex_cell(prhs[0], &Q, &w);
    const mxArray* X = prhs[1];
    if (mxIsCell(X)) mexErrMsgIdAndTxt("calanczos:arg", "Input X (arg 2) project() must be a column matrix.");
    const mwSize n = mxGetM(X), m = mxGetN(X);
    const int doreorth = nrhs > 2 ? (int)mxGetScalar(prhs[2]) : 0;    /* :21-23 default false */
    double** R = (double**)mxCalloc(B > 0 ? B : 1, sizeof(double*));
    mxArray* Rc = mxCreateCellMatrix(1, B);
    for (int i = 0; i < B; ++i) {
        mxArray* Ri = mxCreateDoubleMatrix(w[i], m, mxREAL);
        R[i] = mxGetPr(Ri);
        mxSetCell(Rc, i, Ri);
    }
    plhs[0] = mxCreateDoubleMatrix(n, m, mxREAL);
    cal_mex_check(cal_project(c, (int64_t)n, B, (const double* const*)Q, w, (int)m, mxGetPr(X), doreorth,
                              mxGetPr(plhs[0]), (double* const*)R));
    if (nlhs > 1) plhs[1] = Rc;
    mxFree(R);
    mxFree(Q);
    mxFree(w);
}
