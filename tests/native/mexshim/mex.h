/* mex.h -- the subset of MATLAB's MEX/MX C API that this repository's
 * gateways (the mex directory) use, implemented by mexshim.cpp so the gateways can be
 * compiled and driven from the test suite without MATLAB (which is absent
 * from this image).  TEST INFRASTRUCTURE: MATLAB's own mex.h replaces this
 * when the gateways are built with `mex`.  Arrays are
 * column-major, as in MATLAB. */
#ifndef GQMAP_MEXSHIM_H
#define GQMAP_MEXSHIM_H
#include <stddef.h>
#include <stdint.h>

typedef size_t mwSize;
typedef bool mxLogical;
typedef enum { mxDOUBLE_CLASS, mxUINT8_CLASS, mxLOGICAL_CLASS, mxCHAR_CLASS, mxSTRUCT_CLASS } mxClassID;
typedef enum { mxREAL } mxComplexity;
struct mxArray_tag;
typedef struct mxArray_tag mxArray;

extern "C" {
/* gateway entry, defined by each gateway source */
void mexFunction(int nlhs, mxArray *plhs[], int nrhs, const mxArray *prhs[]);

const mxArray *mxGetField(const mxArray *s, size_t index, const char *name);
double mxGetScalar(const mxArray *a);
bool mxIsChar(const mxArray *a);
bool mxIsStruct(const mxArray *a);
bool mxIsDouble(const mxArray *a);
char *mxArrayToString(const mxArray *a);
void mxFree(void *p);
size_t mxGetM(const mxArray *a);
size_t mxGetN(const mxArray *a);
mwSize mxGetNumberOfDimensions(const mxArray *a);
const mwSize *mxGetDimensions(const mxArray *a);
double *mxGetPr(const mxArray *a);
void *mxGetData(const mxArray *a);
mxLogical *mxGetLogicals(const mxArray *a);
mxArray *mxCreateNumericArray(mwSize ndim, const mwSize *dims, mxClassID cls, mxComplexity c);
mxArray *mxCreateDoubleMatrix(mwSize m, mwSize n, mxComplexity c);
mxArray *mxCreateString(const char *s);
void mxDestroyArray(mxArray *a);
void mexErrMsgIdAndTxt(const char *id, const char *fmt, ...);
int mexPrintf(const char *fmt, ...);
int mexCallMATLAB(int nlhs, mxArray *plhs[], int nrhs, mxArray *prhs[], const char *name);
}
#endif
