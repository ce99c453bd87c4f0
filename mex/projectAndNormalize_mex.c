/* projectAndNormalize.mexa64 -- [QZ, RZ] = projectAndNormalize(Q, X, doreorth)
 * RZ is a 1 x (B+1) cell; disp('second') when the reference would
 * reorthogonalise.                                  (projectAndNormalize.m:3-90) */
#include "cal_mex_common.h"

void mexFunction(int nlhs, mxArray* plhs[], int nrhs, const mxArray* prhs[]) {
    if (nrhs < 2) mexErrMsgIdAndTxt("calanczos:arg", "[QZ,RZ] = projectAndNormalize(Q,X[,doreorth])");
    cal_ctx* c = cal_mex_plain_ctx();
    const double** Q;
    int* w;
    const int B = cal_mex_cell(prhs[0], &Q, &w);
    const mxArray* X = prhs[1];
    const mwSize n = mxGetM(X), m = mxGetN(X);
    const int doreorth = nrhs > 2 ? (int)mxGetScalar(prhs[2]) : 1;    /* :5-7 default true */
    double** RZ = (double**)mxCalloc(B + 1, sizeof(double*));
    mxArray* Rc = mxCreateCellMatrix(1, B + 1);
    for (int i = 0; i < B; ++i) {
        mxArray* Ri = mxCreateDoubleMatrix(w[i], m, mxREAL);
        RZ[i] = mxGetPr(Ri);
        mxSetCell(Rc, i, Ri);
    }
    mxArray* Rl = mxCreateDoubleMatrix(m, m, mxREAL);
    RZ[B] = mxGetPr(Rl);
    mxSetCell(Rc, B, Rl);
    plhs[0] = mxCreateDoubleMatrix(n, m, mxREAL);
    int reorth = 0, rank = 0;
    cal_mex_check(cal_project_and_normalize(c, (int64_t)n, B, (const double* const*)Q, w, (int)m, mxGetPr(X),
                                            doreorth, mxGetPr(plhs[0]), (double* const*)RZ, &reorth, &rank));
    if (reorth) mexPrintf("second\n");                                /* :53 */
    if (nlhs > 1) plhs[1] = Rc;
    mxFree(RZ);
    mxFree(Q);
    mxFree(w);
}
