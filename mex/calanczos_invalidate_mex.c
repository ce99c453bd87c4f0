/* calanczos_invalidate.mexa64 -- calanczos_invalidate()
 *
 * Not a reference function: the explicit residency invalidation of the MEX
 * tier (mex/cal_mex_common.h).  After an in-place edit A(i,j) = v of a matrix
 * the shims hold resident, this makes every shim of the MATLAB process
 * re-upload A on its next call (cal_residency_invalidate bumps the
 * library's process-wide generation).  Returns the new generation. */
#include "cal_mex_common.h"

void mexFunction(int nlhs, mxArray* plhs[], int nrhs, const mxArray* prhs[]) {
    (void)prhs;
    if (nrhs != 0) mexErrMsgIdAndTxt("calanczos:arg", "calanczos_invalidate()");
    const long long gen = cal_residency_invalidate();
    if (nlhs > 0) plhs[0] = mxCreateDoubleScalar((double)gen);
}
