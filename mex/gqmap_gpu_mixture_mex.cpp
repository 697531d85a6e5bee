// gqmap_gpu_mixture_mex.cpp -- MATLAB MEX gateway: drop-in for
//   [mu,sigma,alpha,AEPE,Energy,logP] = gqmap_gpu_mixture(options,I1,I2)          (gqmap_gpu_mixture.m:1)
//   [mu,sigma,alpha,AEPE,Energy,logP] = gqmap_gpuSuper_mix_entropy(options,I1,I2) (built with -DGQMAP_SUPER)
// over libgqmap.so (include/gqmap.h).  Built with MATLAB's `mex` (see
// INTEGRATION.md); MATLAB is not part of this repository's build image.
//
// Mirrors the reference's host-side bookkeeping: evaluation every 300
// iterations and at it==1 (MAP, flowToColor, imwrite, AEPE, logP;
// gqmap_gpu_mixture.m:52-68) and the per-iteration console line (:71-72).
#include <mex.h>

#include <cmath>
#include <cstdio>
#include <string>
#include <vector>

#include "gqmap.h"

namespace {

#ifdef GQMAP_SUPER
constexpr int ENGINE = GQMAP_ENGINE_SUPER;
constexpr int CROP = 4;  // repelem(map,4,4), crop 5:end-4 (gqmap_gpuSuper_mix_entropy.m:58-63)
#else
constexpr int ENGINE = GQMAP_ENGINE_MIXTURE;
constexpr int CROP = 1;  // interior M_, N_ (gqmap_gpu_mixture.m:64)
#endif
constexpr int EVAL_EVERY = 300;

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

std::string field_s(const mxArray *opt, const char *name)
{
    const mxArray *f = mxGetField(opt, 0, name);
    if (!f || !mxIsChar(f)) return std::string();
    char *c = mxArrayToString(f);
    std::string s(c);
    mxFree(c);
    return s;
}

}  // namespace

void mexFunction(int nlhs, mxArray *plhs[], int nrhs, const mxArray *prhs[])
{
    if (nrhs != 3 || !mxIsStruct(prhs[0]))
        mexErrMsgIdAndTxt("gqmap:usage", "usage: [mu,sigma,alpha,AEPE,Energy,logP] = f(options,I1,I2)");
    const mxArray *opt = prhs[0];
    if (!mxIsDouble(prhs[1]) || !mxIsDouble(prhs[2]))
        mexErrMsgIdAndTxt("gqmap:usage", "I1, I2 must be double matrices");
    const int Mo = (int)mxGetM(prhs[1]), No = (int)mxGetN(prhs[1]);
    if ((int)mxGetM(prhs[2]) != Mo || (int)mxGetN(prhs[2]) != No)
        mexErrMsgIdAndTxt("gqmap:usage", "I1 and I2 differ in size");

    gqmap_options o;
    gqmap_options_default(&o, ENGINE);
    o.its = (int)field_d(opt, "its");
    o.K = (int)field_d(opt, "K");
    o.L = (int)field_d(opt, "L");
    o.temperature = field_d(opt, "temperature");
    o.drate = field_d(opt, "drate");
    o.epsn = field_d(opt, "epsn");
    o.lambdad = field_d(opt, "lambdad");
    o.lambdas = field_d(opt, "lambdas");
    o.minu = field_d(opt, "minu");
    o.maxu = field_d(opt, "maxu");
    o.minv = field_d(opt, "minv");
    o.maxv = field_d(opt, "maxv");
    // optional (not read by the reference): projsplx alpha update (:49 / super :48, commented there)
    if (mxGetField(opt, 0, "alpha_mode"))
        fail(gqmap_options_alpha_mode(&o, (int)field_d(opt, "alpha_mode")), "options.alpha_mode");
    // optional (not read by the reference): options.arith = 'literal' runs the
    // reference's own operation order (GQMAP_ARITH_LITERAL: bit-identical to a
    // literal fp64 restatement of the MATLAB; fp64 mixture engine)
    if (mxGetField(opt, 0, "arith"))
        o.arith = field_s(opt, "arith") == "literal" ? GQMAP_ARITH_LITERAL : GQMAP_ARITH_FAST;
    const uint64_t seed = (uint64_t)field_d(opt, "seed", false, 0);
    const std::string dir = field_s(opt, "dir");
    const mxArray *tflow = mxGetField(opt, 0, "trueFlow");
    const mxArray *unk = mxGetField(opt, 0, "unknownIdx");

    gqmap_ctx *ctx = nullptr;
    fail(gqmap_create(&ctx, &o, 0), "gqmap_create");
    g_ctx = ctx;
    fail(gqmap_set_images(ctx, mxGetPr(prhs[1]), mxGetPr(prhs[2]), Mo, No), "gqmap_set_images");
    fail(gqmap_init_state(ctx, seed), "gqmap_init_state");
    gqmap_info info;
    fail(gqmap_get_info(ctx, &info), "gqmap_get_info");
    const int M = info.M, N = info.N, L = info.L;
    const size_t MN = (size_t)M * N, MNL = MN * L;

    const int its = o.its;
    std::vector<double> AEPE(its, NAN), Energy(its, 0.0), logP(its, NAN), trace(3 * (size_t)its);
    std::vector<double> map(2 * MN), flow(2 * (size_t)Mo * No);
    std::vector<uint8_t> img, unk_c;
    std::vector<double> flo;
    double best = INFINITY;
    int mark = 0, it = 1;
    while (it <= its) {
        const int next = it == 1 ? 1 : std::min(its, (it / EVAL_EVERY + 1) * EVAL_EVERY);
        const int want = next - it + 1;
        int done = 0;
        fail(gqmap_run(ctx, want, &done, trace.data()), "gqmap_run");
        for (int k = 0; k < done; ++k) {
            Energy[it - 1 + k] = trace[3 * k];
            mexPrintf("[%3d], \xce\x94(mu) = %e, \xce\x94(sigma) = %e, Energy = %e, AEPE=%e,logP=%e \n",
                      it + k, trace[3 * k + 1], trace[3 * k + 2], trace[3 * k], best,
                      mark ? logP[mark - 1] : NAN);
        }
        const int last = it + done - 1;
        if (done == want && (last == 1 || last % EVAL_EVERY == 0)) {
            fail(gqmap_get_map(ctx, map.data()), "gqmap_get_map");
            // flow = map (single scale) or repelem(map,4,4) (super)
            const int f = Mo / M;
            for (int n = 0; n < No; ++n)
                for (int m = 0; m < Mo; ++m)
                    for (int c = 0; c < 2; ++c)
                        flow[m + (size_t)Mo * n + (size_t)Mo * No * c] = map[m / f + (size_t)M * (n / f) + MN * c];
            // colour of the (cropped) flow, written as <dir>/<it>.png
            const int cm = Mo - 2 * (f == 1 ? 0 : CROP), cn = No - 2 * (f == 1 ? 0 : CROP);
            const int off = f == 1 ? 0 : CROP;
            std::vector<double> fc(2 * (size_t)cm * cn);
            for (int c = 0; c < 2; ++c)
                for (int n = 0; n < cn; ++n)
                    for (int m = 0; m < cm; ++m)
                        fc[m + (size_t)cm * n + (size_t)cm * cn * c] =
                            flow[(m + off) + (size_t)Mo * (n + off) + (size_t)Mo * No * c];
            img.assign(3 * (size_t)cm * cn, 0);
            flo.assign(2 * (size_t)cm * cn, 0);
            unk_c.assign((size_t)cm * cn, 0);
            double stats[4];
            fail(gqmap_flow_to_color(fc.data(), cm, cn, 0.0, img.data(), flo.data(), stats,
                                     unk_c.data(), 0), "gqmap_flow_to_color");
            if (!dir.empty()) {
                mwSize dims[3] = {(mwSize)cm, (mwSize)cn, 3};
                mxArray *png = mxCreateNumericArray(3, dims, mxUINT8_CLASS, mxREAL);
                std::copy(img.begin(), img.end(), (uint8_t *)mxGetData(png));
                mxArray *args[2] = {png, mxCreateString((dir + "/" + std::to_string(last) + ".png").c_str())};
                mexCallMATLAB(0, nullptr, 2, args, "imwrite");
                mxDestroyArray(args[0]);
                mxDestroyArray(args[1]);
            }
            if (tflow && unk) {  // flow(unidx)=0; AEPE over the (cropped) interior
                const double *tf = mxGetPr(tflow);
                const mxLogical *u = mxGetLogicals(unk);
                double s = 0;
                for (int n = CROP; n < No - CROP; ++n) {
                    double col = 0;
                    for (int m = CROP; m < Mo - CROP; ++m) {
                        const size_t q = m + (size_t)Mo * n;
                        const double fu = u[q] ? 0 : flow[q], fv = u[q] ? 0 : flow[q + (size_t)Mo * No];
                        const double du = tf[q] - fu, dv = tf[q + (size_t)Mo * No] - fv;
                        col += std::sqrt(du * du + dv * dv);
                    }
                    s += col / (Mo - 2 * CROP);
                }
                AEPE[last - 1] = s / (No - 2 * CROP);
                best = std::min(best, AEPE[last - 1]);
            }
            double lp = 0;
            fail(gqmap_log_p(ctx, map.data(), &lp), "gqmap_log_p");
            logP[last - 1] = lp;
            mark = last;
        }
        it += done;
        if (done < want) break;  // ptdmu < tor (gqmap_gpu_mixture.m:75)
    }

    // outputs: mu = cat(4,muu,muv), sigma = cat(4,sigmau,sigmav), alpha 1x1xL
    std::vector<double> st(MNL * 5 + MNL * 4 + 2 * (size_t)L);
    gqmap_state s;
    s.muu = st.data(); s.muv = s.muu + MNL; s.sigu = s.muv + MNL; s.sigv = s.sigu + MNL;
    s.pn = s.sigv + MNL; s.rou = s.pn + MNL; s.w = s.rou + 4 * MNL; s.alpha = s.w + L;
    fail(gqmap_get_state(ctx, &s), "gqmap_get_state");
    gqmap_destroy(ctx);
    g_ctx = nullptr;
    mwSize d4[4] = {(mwSize)M, (mwSize)N, (mwSize)L, 2};
    plhs[0] = mxCreateNumericArray(4, d4, mxDOUBLE_CLASS, mxREAL);
    std::copy(s.muu, s.muu + 2 * MNL, mxGetPr(plhs[0]));
    if (nlhs > 1) {
        plhs[1] = mxCreateNumericArray(4, d4, mxDOUBLE_CLASS, mxREAL);
        std::copy(s.sigu, s.sigu + 2 * MNL, mxGetPr(plhs[1]));
    }
    if (nlhs > 2) {
        mwSize d3[3] = {1, 1, (mwSize)L};
        plhs[2] = mxCreateNumericArray(3, d3, mxDOUBLE_CLASS, mxREAL);
        std::copy(s.alpha, s.alpha + L, mxGetPr(plhs[2]));
    }
    const std::vector<double> *vecs[3] = {&AEPE, &Energy, &logP};
    for (int k = 0; k < 3 && nlhs > 3 + k; ++k) {
        plhs[3 + k] = mxCreateDoubleMatrix(its, 1, mxREAL);
        std::copy(vecs[k]->begin(), vecs[k]->end(), mxGetPr(plhs[3 + k]));
    }
}
