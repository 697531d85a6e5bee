// mexshim.cpp -- implementation of tests/native/mexshim/mex.h plus a small C
// API (shim_*) through which tests/test_gpu_mex.py builds MATLAB-style
// arguments, calls a gateway's mexFunction and reads its outputs.  Test
// infrastructure only.
#include "mex.h"

#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <stdexcept>
#include <string>
#include <vector>

struct mxArray_tag {
    mxClassID cls = mxDOUBLE_CLASS;
    std::vector<mwSize> dims;
    std::vector<unsigned char> data;  // element storage
    std::map<std::string, mxArray *> fields;
    size_t numel() const
    {
        size_t n = 1;
        for (mwSize d : dims) n *= d;
        return n;
    }
};

namespace {
std::string g_err, g_log;
std::vector<std::string> g_calls;
size_t esize(mxClassID c) { return c == mxDOUBLE_CLASS ? 8 : 1; }
mxArray *make(mxClassID cls, mwSize ndim, const mwSize *dims)
{
    mxArray *a = new mxArray_tag;
    a->cls = cls;
    a->dims.assign(dims, dims + ndim);
    if (a->dims.size() < 2) a->dims.resize(2, 1);
    a->data.assign(a->numel() * esize(cls), 0);
    return a;
}
struct MexError : std::runtime_error {
    using std::runtime_error::runtime_error;
};
}  // namespace

extern "C" {
const mxArray *mxGetField(const mxArray *s, size_t, const char *name)
{
    auto it = s->fields.find(name);
    return it == s->fields.end() ? nullptr : it->second;
}
double mxGetScalar(const mxArray *a)
{
    if (a->numel() == 0) return 0;
    if (a->cls == mxDOUBLE_CLASS) return *(const double *)a->data.data();
    return (double)a->data[0];
}
bool mxIsChar(const mxArray *a) { return a->cls == mxCHAR_CLASS; }
bool mxIsStruct(const mxArray *a) { return a->cls == mxSTRUCT_CLASS; }
bool mxIsDouble(const mxArray *a) { return a->cls == mxDOUBLE_CLASS; }
char *mxArrayToString(const mxArray *a)
{
    char *s = (char *)std::malloc(a->data.size() + 1);
    std::memcpy(s, a->data.data(), a->data.size());
    s[a->data.size()] = 0;
    return s;
}
void mxFree(void *p) { std::free(p); }
size_t mxGetM(const mxArray *a) { return a->dims[0]; }
size_t mxGetN(const mxArray *a)
{
    size_t n = 1;
    for (size_t k = 1; k < a->dims.size(); ++k) n *= a->dims[k];
    return n;
}
mwSize mxGetNumberOfDimensions(const mxArray *a) { return a->dims.size(); }
const mwSize *mxGetDimensions(const mxArray *a) { return a->dims.data(); }
double *mxGetPr(const mxArray *a) { return (double *)a->data.data(); }
void *mxGetData(const mxArray *a) { return (void *)a->data.data(); }
mxLogical *mxGetLogicals(const mxArray *a) { return (mxLogical *)a->data.data(); }
mxArray *mxCreateNumericArray(mwSize ndim, const mwSize *dims, mxClassID cls, mxComplexity)
{
    return make(cls, ndim, dims);
}
mxArray *mxCreateDoubleMatrix(mwSize m, mwSize n, mxComplexity)
{
    const mwSize d[2] = {m, n};
    return make(mxDOUBLE_CLASS, 2, d);
}
mxArray *mxCreateString(const char *s)
{
    const mwSize d[2] = {1, std::strlen(s)};
    mxArray *a = make(mxCHAR_CLASS, 2, d);
    std::memcpy(a->data.data(), s, std::strlen(s));
    return a;
}
void mxDestroyArray(mxArray *a)
{
    if (!a) return;
    for (auto &f : a->fields) mxDestroyArray(f.second);
    delete a;
}
void mexErrMsgIdAndTxt(const char *id, const char *fmt, ...)
{
    char buf[2048];
    va_list ap;
    va_start(ap, fmt);
    std::vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    throw MexError(std::string(id) + ": " + buf);
}
int mexPrintf(const char *fmt, ...)
{
    char buf[2048];
    va_list ap;
    va_start(ap, fmt);
    const int n = std::vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_log += buf;
    return n;
}
int mexCallMATLAB(int, mxArray **, int nrhs, mxArray **prhs, const char *name)
{
    std::string c = name;
    if (nrhs > 1 && mxIsChar(prhs[nrhs - 1])) {
        char *s = mxArrayToString(prhs[nrhs - 1]);
        c += std::string(" ") + s;
        mxFree(s);
    }
    g_calls.push_back(c);
    return 0;
}

// ---- test-side API --------------------------------------------------------
mxArray *shim_struct() { const mwSize d[2] = {1, 1}; return make(mxSTRUCT_CLASS, 2, d); }
void shim_set_field(mxArray *s, const char *name, mxArray *v)
{
    auto it = s->fields.find(name);
    if (it != s->fields.end()) mxDestroyArray(it->second);
    s->fields[name] = v;
}
mxArray *shim_double(int ndim, const size_t *dims, const double *data)
{
    mxArray *a = make(mxDOUBLE_CLASS, ndim, dims);
    if (data) std::memcpy(a->data.data(), data, a->numel() * 8);
    return a;
}
mxArray *shim_logical(int ndim, const size_t *dims, const unsigned char *data)
{
    mxArray *a = make(mxLOGICAL_CLASS, ndim, dims);
    for (size_t i = 0; i < a->numel(); ++i) a->data[i] = data[i] != 0;
    return a;
}
mxArray *shim_string(const char *s) { return mxCreateString(s); }
int shim_ndims(const mxArray *a) { return (int)a->dims.size(); }
void shim_dims(const mxArray *a, size_t *out) { std::memcpy(out, a->dims.data(), a->dims.size() * sizeof(size_t)); }
const void *shim_data(const mxArray *a) { return a->data.data(); }
void shim_free(mxArray *a) { mxDestroyArray(a); }
// 0 on success; otherwise the gateway raised mexErrMsgIdAndTxt (shim_error())
int shim_call(int nlhs, mxArray **plhs, int nrhs, mxArray **prhs)
{
    g_err.clear();
    try {
        mexFunction(nlhs, plhs, nrhs, (const mxArray **)prhs);
    } catch (const std::exception &e) {
        g_err = e.what();
        return 1;
    }
    return 0;
}
const char *shim_error() { return g_err.c_str(); }
const char *shim_log() { return g_log.c_str(); }
void shim_clear_log() { g_log.clear(); g_calls.clear(); }
int shim_ncalls() { return (int)g_calls.size(); }
const char *shim_call_name(int i) { return g_calls[i].c_str(); }
}
