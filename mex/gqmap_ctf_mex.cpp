// gqmap_ctf_mex.cpp -- MATLAB MEX gateway: drop-in for the coarse-to-fine
// level solver
//   [mu,sigma,rou,AEPE,Energy] = gqmap_ctf(options,I1,I2,GRDT)      (legacy/gqmap_ctf.m:1)
// called per pyramid level by legacy/optical_flow_ctf.m:33, over libgqmap.so
// (include/gqmap.h, GQMAP_ENGINE_CTF).  Built with MATLAB's `mex` (see
// INTEGRATION.md).
//
// Mirrors the reference's outputs: mu, sigma M x N x 2, rou M x N x 2 x 2,
// AEPE its x 1 (every iteration, gqmap_ctf.m:38; 17 after a stop, :13),
// Energy its x 1 (0 after a stop) and the per-iteration console line (:44).
// minu..maxv come from GRDT (:4); GRDT may be larger than I1 (the reference
// passes the full-resolution trueFlow.*scale to every level and indexes its
// top-left block).
#include <mex.h>

#include <cmath>
#include <cstdio>
#include <vector>

#include "gqmap.h"

namespace {

// The context of the running call: mexErrMsgIdAndTxt longjmps out of the
// gateway, so fail() releases it (and its device buffers) first.
gqmap_ctx *g_ctx = nullptr;

void fail(gqmap_status s, const char *what)
{
    if (s == GQMAP_OK) return;
    char msg[512];
    std::snprintf(msg, sizeof msg, "%s: %s", what, gqmap_last_error());
    if (g_ctx) gqmap_destroy(g_ctx);
    g_ctx = nullptr;
    mexErrMsgIdAndTxt("gqmap:error", "%s", msg);
}

double field_d(const mxArray *opt, const char *name, bool required = true, double dflt = 0)
{
    const mxArray *f = mxGetField(opt, 0, name);
    if (!f) {
        if (required) mexErrMsgIdAndTxt("gqmap:options", "options.%s missing", name);
        return dflt;
    }
    return mxGetScalar(f);
}

}  // namespace

void mexFunction(int nlhs, mxArray *plhs[], int nrhs, const mxArray *prhs[])
{
    if (nrhs != 4 || !mxIsStruct(prhs[0]))
        mexErrMsgIdAndTxt("gqmap:usage", "usage: [mu,sigma,rou,AEPE,Energy] = gqmap_ctf(options,I1,I2,GRDT)");
    const mxArray *opt = prhs[0];
    for (int k = 1; k < 4; ++k)
        if (!mxIsDouble(prhs[k])) mexErrMsgIdAndTxt("gqmap:usage", "I1, I2, GRDT must be double arrays");
    const int M = (int)mxGetM(prhs[1]), N = (int)mxGetN(prhs[1]);
    if ((int)mxGetM(prhs[2]) != M || (int)mxGetN(prhs[2]) != N)
        mexErrMsgIdAndTxt("gqmap:usage", "I1 and I2 differ in size");
    const mwSize nd = mxGetNumberOfDimensions(prhs[3]);
    const mwSize *gd = mxGetDimensions(prhs[3]);
    if (nd != 3 || gd[2] != 2 || (int)gd[0] < M || (int)gd[1] < N)
        mexErrMsgIdAndTxt("gqmap:usage", "GRDT must be Mg x Ng x 2 with Mg >= %d, Ng >= %d", M, N);
    const int Mg = (int)gd[0], Ng = (int)gd[1];
    const double *G = mxGetPr(prhs[3]);

    gqmap_options o;
    gqmap_options_default(&o, GQMAP_ENGINE_CTF);
    o.its = (int)field_d(opt, "its");
    o.K = (int)field_d(opt, "K");
    o.epsn = field_d(opt, "epsn");
    o.lambdad = field_d(opt, "lambdad");
    o.lambdas = field_d(opt, "lambdas");
    // minu=min(min(GRDT(:,:,1))) ... (:4): over the whole array passed in
    double mn[2] = {INFINITY, INFINITY}, mx[2] = {-INFINITY, -INFINITY};
    for (int k = 0; k < 2; ++k)
        for (size_t i = 0; i < (size_t)Mg * Ng; ++i) {
            const double v = G[(size_t)Mg * Ng * k + i];
            mn[k] = std::fmin(mn[k], v);
            mx[k] = std::fmax(mx[k], v);
        }
    o.minu = mn[0]; o.maxu = mx[0]; o.minv = mn[1]; o.maxv = mx[1];
    const uint64_t seed = (uint64_t)field_d(opt, "seed", false, 0);

    gqmap_ctx *ctx = nullptr;
    fail(gqmap_create(&ctx, &o, 0), "gqmap_create");
    g_ctx = ctx;
    fail(gqmap_set_images(ctx, mxGetPr(prhs[1]), mxGetPr(prhs[2]), M, N), "gqmap_set_images");
    fail(gqmap_init_state(ctx, seed), "gqmap_init_state");
    fail(gqmap_set_truth(ctx, G, Mg, Ng), "gqmap_set_truth");
    const int its = o.its;
    std::vector<double> trace(3 * (size_t)its), ae(its);
    int done = 0;
    fail(gqmap_run_aepe(ctx, its, &done, trace.data(), ae.data()), "gqmap_run_aepe");
    std::vector<double> AEPE(its, 17.0), Energy(its, 0.0);  // AEPE=ones(its,1)*17 (:13)
    double best = INFINITY;
    int bestat = 1;
    for (int k = 0; k < done; ++k) {
        AEPE[k] = ae[k];
        Energy[k] = trace[3 * (size_t)k];
        if (ae[k] < best) { best = ae[k]; bestat = k + 1; }
        mexPrintf("[%3d], \xce\x94(mu) = %e, \xce\x94(sigma) = %e, AEPE=%e, Energy=%e, best at#%d\n", k + 1,
                  trace[3 * (size_t)k + 1], trace[3 * (size_t)k + 2], ae[k], Energy[k], bestat);
    }
    // mu = cat(3,muu,muv), sigma = cat(3,sigmau,sigmav), rou M x N x 2 x 2
    const size_t MN = (size_t)M * N;
    std::vector<double> st(9 * MN + 2);
    gqmap_state s;
    s.muu = st.data(); s.muv = s.muu + MN; s.sigu = s.muv + MN; s.sigv = s.sigu + MN;
    s.pn = s.sigv + MN; s.rou = s.pn + MN; s.w = s.rou + 4 * MN; s.alpha = s.w + 1;
    fail(gqmap_get_state(ctx, &s), "gqmap_get_state");
    gqmap_destroy(ctx);
    g_ctx = nullptr;
    mwSize d3[3] = {(mwSize)M, (mwSize)N, 2};
    plhs[0] = mxCreateNumericArray(3, d3, mxDOUBLE_CLASS, mxREAL);
    std::copy(s.muu, s.muu + 2 * MN, mxGetPr(plhs[0]));
    if (nlhs > 1) {
        plhs[1] = mxCreateNumericArray(3, d3, mxDOUBLE_CLASS, mxREAL);
        std::copy(s.sigu, s.sigu + 2 * MN, mxGetPr(plhs[1]));
    }
    if (nlhs > 2) {
        mwSize d4[4] = {(mwSize)M, (mwSize)N, 2, 2};
        plhs[2] = mxCreateNumericArray(4, d4, mxDOUBLE_CLASS, mxREAL);
        std::copy(s.rou, s.rou + 4 * MN, mxGetPr(plhs[2]));
    }
    const std::vector<double> *vecs[2] = {&AEPE, &Energy};
    for (int k = 0; k < 2 && nlhs > 3 + k; ++k) {
        plhs[3 + k] = mxCreateDoubleMatrix(its, 1, mxREAL);
        std::copy(vecs[k]->begin(), vecs[k]->end(), mxGetPr(plhs[3 + k]));
    }
}
