/* impl_restarted_ca_lanczos.mexa64 -- [conv_eigs, Q_conv, num_restarts] =
 *     impl_restarted_ca_lanczos(A, r, max_lanczos, n_wanted_eigs, s, basis, orth, tol)
 * The implicit restart the reference file sets out to implement (it does
 * not run itself); orth 'full' only.  (impl_restarted_ca_lanczos.m:4-226) */
#include "cal_mex_common.h"

void mexFunction(int nlhs, mxArray* plhs[], int nrhs, const mxArray* prhs[]) {
    if (nrhs < 3) mexErrMsgIdAndTxt("calanczos:arg", "[E,V,nres] = impl_restarted_ca_lanczos(A,r,max_lanczos,...)");
    cal_ctx* c = cal_mex_ctx_full(prhs[0]);
    const mwSize n = mxGetN(prhs[0]);
    const int ml = (int)mxGetScalar(prhs[2]);
    const int nw = nrhs > 3 ? (int)mxGetScalar(prhs[3]) : 10;          /* :13-21 */
    const int s = nrhs > 4 ? (int)mxGetScalar(prhs[4]) : 6;
    char basis[16] = "newton", orth[16] = "full";
    cal_mex_opt_string(nrhs, prhs, 5, basis, sizeof basis);
    cal_mex_opt_string(nrhs, prhs, 6, orth, sizeof orth);
    const double tol = nrhs > 7 ? mxGetScalar(prhs[7]) : 1.0e-6;      /* :37-39 */
    plhs[0] = mxCreateDoubleMatrix(nw, 1, mxREAL);
    double* V = NULL;
    if (nlhs > 1) {
        plhs[1] = mxCreateDoubleMatrix(n, nw, mxREAL);
        V = mxGetPr(plhs[1]);
    }
    cal_restart_info info;
    cal_mex_check(cal_impl_restarted_ca_lanczos(c, mxGetPr(prhs[1]), ml, nw, s, basis, orth, tol, mxGetPr(plhs[0]),
                                                V, NULL, &info));
    if (nlhs > 2) plhs[2] = mxCreateDoubleScalar(info.num_restarts);
    if (!info.converged) mexWarnMsgIdAndTxt("calanczos:warning", "Did not converge.");   /* :225 */
}
