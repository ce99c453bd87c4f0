/* restarted_ca_lanczos.mexa64 -- [E, V, nres, rnorms, orth_err] =
 *     restarted_ca_lanczos(A, r, max_lanczos, n_wanted_eigs, s, basis, orth, tol)
 *                                          (restarted_ca_lanczos.m:4-198, :6 caps 200) */
#include "cal_mex_common.h"

void mexFunction(int nlhs, mxArray* plhs[], int nrhs, const mxArray* prhs[]) {
    if (nrhs < 3) mexErrMsgIdAndTxt("calanczos:arg", "[E,V,nres,rn,oe] = restarted_ca_lanczos(A,r,max_lanczos,...)");
    cal_ctx* c = cal_mex_ctx_full(prhs[0]);
    const mwSize n = mxGetN(prhs[0]);
    const int ml = (int)mxGetScalar(prhs[2]);
    const int nw = nrhs > 3 ? (int)mxGetScalar(prhs[3]) : 10;          /* :17-33 defaults */
    const int s = nrhs > 4 ? (int)mxGetScalar(prhs[4]) : 6;
    char basis[16] = "newton", orth[16] = "local";
    cal_mex_opt_string(nrhs, prhs, 5, basis, sizeof basis);
    cal_mex_opt_string(nrhs, prhs, 6, orth, sizeof orth);
    const double tol = nrhs > 7 ? mxGetScalar(prhs[7]) : 1.0e-8;
    if (nw < 1) mexErrMsgIdAndTxt("calanczos:arg", "n_wanted_eigs must be positive");
    double* E = (double*)mxMalloc((mwSize)nw * sizeof(double));
    double* V = nlhs > 1 ? (double*)mxMalloc(n * (mwSize)nw * sizeof(double)) : NULL;
    double* rn = (double*)mxMalloc(200 * (mwSize)nw * sizeof(double));
    double oe[200];
    cal_restart_info info;
    cal_mex_check(cal_restarted_ca_lanczos(c, mxGetPr(prhs[1]), ml, nw, s, basis, orth, tol, nlhs > 3, E, V, rn,
                                           oe, &info));
    const int k = info.nconv, nr = info.num_restarts;
    plhs[0] = mxCreateDoubleMatrix(k, 1, mxREAL);
    memcpy(mxGetPr(plhs[0]), E, (size_t)k * sizeof(double));
    if (nlhs > 1) {
        plhs[1] = mxCreateDoubleMatrix(n, k, mxREAL);
        memcpy(mxGetPr(plhs[1]), V, n * (size_t)k * sizeof(double));
    }
    if (nlhs > 2) plhs[2] = mxCreateDoubleScalar(nr);
    if (nlhs > 3) {
        plhs[3] = mxCreateDoubleMatrix(nr, nw, mxREAL);
        for (int j = 0; j < nw; ++j)
            memcpy(mxGetPr(plhs[3]) + (size_t)j * nr, rn + (size_t)j * 200, (size_t)nr * sizeof(double));
    }
    if (nlhs > 4) {
        plhs[4] = mxCreateDoubleMatrix(nr, 1, mxREAL);
        memcpy(mxGetPr(plhs[4]), oe, (size_t)nr * sizeof(double));
    }
    mxFree(rn);
    mxFree(E);
    if (V) mxFree(V);
}
