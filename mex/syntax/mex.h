/* mex/syntax/mex.h -- DECLARATIONS ONLY, for `make -C mex check`.
 *
 * MATLAB (and its mex.h) is not available in this pipeline.  This header
 * declares the subset of the documented MEX / MX C API that the shims in
 * the mex shims call, with the documented signatures (separate-complex API,
 * `mex -R2017b`), so that `gcc -fsyntax-only` catches drift between the
 * shims and include/calanczos.h.  It defines nothing and is never linked:
 * real builds use MATLAB's own mex.h through the `mex` command
 * (INTEGRATION.md §6). */
#ifndef CAL_MEX_SYNTAX_H
#define CAL_MEX_SYNTAX_H
#include <stddef.h>

typedef struct mxArray_tag mxArray;
typedef size_t mwSize;
typedef size_t mwIndex;
typedef enum { mxREAL, mxCOMPLEX } mxComplexity;

void mexFunction(int nlhs, mxArray* plhs[], int nrhs, const mxArray* prhs[]);
void mexErrMsgIdAndTxt(const char* id, const char* fmt, ...);
void mexWarnMsgIdAndTxt(const char* id, const char* fmt, ...);
int mexPrintf(const char* fmt, ...);
int mexAtExit(void (*fn)(void));

mwSize mxGetM(const mxArray* a);
mwSize mxGetN(const mxArray* a);
mwSize mxGetNumberOfElements(const mxArray* a);
double* mxGetPr(const mxArray* a);
double* mxGetPi(const mxArray* a);
mwIndex* mxGetJc(const mxArray* a);
mwIndex* mxGetIr(const mxArray* a);
double mxGetScalar(const mxArray* a);
int mxGetString(const mxArray* a, char* buf, mwSize buflen);
int mxIsSparse(const mxArray* a);
int mxIsComplex(const mxArray* a);
int mxIsCell(const mxArray* a);
int mxIsChar(const mxArray* a);
int mxIsEmpty(const mxArray* a);
mxArray* mxGetCell(const mxArray* a, mwIndex i);
void mxSetCell(mxArray* a, mwIndex i, mxArray* v);
mxArray* mxCreateDoubleMatrix(mwSize m, mwSize n, mxComplexity c);
mxArray* mxCreateDoubleScalar(double v);
mxArray* mxCreateCellMatrix(mwSize m, mwSize n);
void* mxCalloc(mwSize n, mwSize size);
void* mxMalloc(mwSize n);
void mxFree(void* p);

#endif
