/* Declaration-only stand-in for MATLAB's mex.h (TEST INFRASTRUCTURE).
 * Lets tests/test_bindings_cpu.py compile and link the reference MEX sources
 * (matlabWrapper/{write,read}LFMstack.cpp, readLFMheader.cpp) against
 * include/lfm and liblfm.so to prove source/link compatibility of the drop-in
 * boundary; nothing here is ever executed. */
#ifndef LFM_TEST_MEX_SHIM_H
#define LFM_TEST_MEX_SHIM_H
#include <stddef.h>
typedef size_t mwSize;
typedef size_t mwIndex;
typedef struct mxArray_tag mxArray;
typedef enum { mxUNKNOWN_CLASS = 0, mxCELL_CLASS, mxSTRUCT_CLASS, mxLOGICAL_CLASS, mxCHAR_CLASS, mxVOID_CLASS,
               mxDOUBLE_CLASS, mxSINGLE_CLASS, mxINT8_CLASS, mxUINT8_CLASS, mxINT16_CLASS, mxUINT16_CLASS,
               mxINT32_CLASS, mxUINT32_CLASS, mxINT64_CLASS, mxUINT64_CLASS } mxClassID;
typedef enum { mxREAL, mxCOMPLEX } mxComplexity;
extern "C" {
void mexErrMsgTxt(const char*);
char* mxArrayToString(const mxArray*);
mxArray* mxCreateDoubleMatrix(mwSize, mwSize, mxComplexity);
mxArray* mxCreateNumericArray(mwSize, const mwSize*, mxClassID, mxComplexity);
mxArray* mxCreateString(const char*);
mxArray* mxCreateStructMatrix(mwSize, mwSize, int, const char**);
void mxFree(void*);
mxClassID mxGetClassID(const mxArray*);
void* mxGetData(const mxArray*);
const mwSize* mxGetDimensions(const mxArray*);
size_t mxGetN(const mxArray*);
mwSize mxGetNumberOfDimensions(const mxArray*);
size_t mxGetNumberOfElements(const mxArray*);
double* mxGetPr(const mxArray*);
bool mxIsChar(const mxArray*);
bool mxIsEmpty(const mxArray*);
void mxSetFieldByNumber(mxArray*, mwIndex, int, mxArray*);
}
#endif
