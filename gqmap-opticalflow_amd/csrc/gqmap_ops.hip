// gqmap_ops.hip -- standalone device ops beside the iteration:
//   projsplx      simplex projection, one thread per column (projsplx.m:15-30,
//                 column form :34-67)
//   mixture MAP   get_map_mex (semantics of legacy/findMixMax.m:39-70 with
//                 MATLAB fminbnd, TolX=1e-4), one thread per pixel
//   flow colour   flowToColor_mex (legacy/flowToColor.m:37-87 +
//                 legacy/computeColor.m:33-115): one reduction pass for the
//                 flow range, one per-pixel colour pass
#include <hip/hip_runtime.h>

#include <cfloat>
#include <cmath>
#include <vector>

#include "gqmap_internal.h"

#pragma clang fp contract(off)
#define GQ_HD __device__ __forceinline__
#define GQ_SQRT(x) sqrt(x)
#define GQ_UNROLL2
#define GQ_PAIR_UNROLL
#define GQ_PAIR_UNROLL_K(n)
#define GQ_NODE_UNROLL
#define GQ_UNROLL_FULL 
#include "gqmap_math.h"

namespace gq {

constexpr int PROJ_NMAX = 64;

__global__ void k_projsplx(const double *__restrict__ Y, double *__restrict__ X, int n, int ncols)
{
    const int col = blockIdx.x * blockDim.x + threadIdx.x;
    if (col >= ncols) return;
    const double *y = Y + (int64_t)col * n;
    double s[PROJ_NMAX];
    for (int i = 0; i < n; ++i) {  // insertion sort, descending
        const double v = y[i];
        int j = i;
        while (j > 0 && s[j - 1] < v) { s[j] = s[j - 1]; --j; }
        s[j] = v;
    }
    double tmpsum = 0, tmax = 0;
    bool bget = false;
    for (int ii = 0; ii < n - 1; ++ii) {
        tmpsum += s[ii];
        tmax = (tmpsum - 1) / (ii + 1);
        if (tmax >= s[ii + 1]) { bget = true; break; }
    }
    if (!bget) tmax = (tmpsum + s[n - 1] - 1) / n;
    for (int i = 0; i < n; ++i) X[(int64_t)col * n + i] = fmax(y[i] - tmax, 0.0);
}

// -- mixture MAP ------------------------------------------------------------
struct Mix {
    double a[GQMAP_LMAX], u[GQMAP_LMAX], o[GQMAP_LMAX];
    int L;
    __device__ double neg(double x) const
    {
        double v = 0;
        for (int l = 0; l < L; ++l) {
            const double z = (x - u[l]) / o[l];
            v += a[l] * (gq_exp(-0.5 * z * z) / (2.5066282746310002 * o[l]));  // normpdf
        }
        return -v;
    }
};

// MATLAB fminbnd (Brent's fmin: golden section + parabolic interpolation).
__device__ double fminbnd(const Mix &f, double ax, double bx, double *fval)
{
    const double tol = 1e-4, seps = 1.4901161193847656e-08, c = 0.3819660112501051;
    double a = ax, b = bx, v = a + c * (b - a), w = v, xf = v, d = 0.0, e = 0.0, x = xf;
    double fx = f.neg(x), fv = fx, fw = fx;
    double xm = 0.5 * (a + b), tol1 = seps * fabs(xf) + tol / 3.0, tol2 = 2.0 * tol1;
    int num = 1;
    while (fabs(xf - xm) > (tol2 - 0.5 * (b - a))) {
        bool gs = true;
        if (fabs(e) > tol1) {
            gs = false;
            double r = (xf - w) * (fx - fv);
            double q = (xf - v) * (fx - fw);
            double p = (xf - v) * q - (xf - w) * r;
            q = 2.0 * (q - r);
            if (q > 0.0) p = -p;
            q = fabs(q);
            r = e;
            e = d;
            if (fabs(p) < fabs(0.5 * q * r) && p > q * (a - xf) && p < q * (b - xf)) {
                d = p / q;
                x = xf + d;
                if ((x - a) < tol2 || (b - x) < tol2) {
                    const double si = (xm - xf > 0) - (xm - xf < 0) + ((xm - xf) == 0);
                    d = tol1 * si;
                }
            } else {
                gs = true;
            }
        }
        if (gs) {
            e = (xf >= xm) ? a - xf : b - xf;
            d = c * e;
        }
        const double si = (d > 0) - (d < 0) + (d == 0);
        x = xf + si * fmax(fabs(d), tol1);
        const double fu = f.neg(x);
        ++num;
        if (fu <= fx) {
            if (x >= xf) a = xf; else b = xf;
            v = w; fv = fw; w = xf; fw = fx; xf = x; fx = fu;
        } else {
            if (x < xf) a = x; else b = x;
            if (fu <= fw || w == xf) { v = w; fv = fw; w = x; fw = fu; }
            else if (fu <= fv || v == xf || v == w) { v = x; fv = fu; }
        }
        xm = 0.5 * (a + b);
        tol1 = seps * fabs(xf) + tol / 3.0;
        tol2 = 2.0 * tol1;
        if (num >= 500) break;  // MaxFunEvals / MaxIter default 500
    }
    *fval = fx;
    return xf;
}

__device__ double map_1d(Mix &f)
{
    double spike = INFINITY, lo = f.u[0], hi = f.u[0];
    int uid = 0;
    for (int l = 0; l < f.L; ++l) {  // [spike, uid] = min(arrayfun(func, u))
        const double v = f.neg(f.u[l]);
        if (v < spike) { spike = v; uid = l; }
        lo = fmin(lo, f.u[l]);
        hi = fmax(hi, f.u[l]);
    }
    double fval;
    const double x = fminbnd(f, lo, hi, &fval);
    return fval < spike ? x : f.u[uid];
}

template <typename R>
__global__ void k_mixture_map(const R *__restrict__ muu, const R *__restrict__ sigu,
                              const R *__restrict__ muv, const R *__restrict__ sigv, int64_t MN,
                              int L, Mix base, double *__restrict__ out)
{
    const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (i >= MN) return;
    Mix f = base;
    for (int l = 0; l < L; ++l) { f.u[l] = muu[i + MN * l]; f.o[l] = sigu[i + MN * l]; }
    out[i] = map_1d(f);
    for (int l = 0; l < L; ++l) { f.u[l] = muv[i + MN * l]; f.o[l] = sigv[i + MN * l]; }
    out[MN + i] = map_1d(f);
}

hipError_t mixture_map_device(const double *alpha, const void *st, bool fp32, int64_t MNL, int M,
                              int N, int L, double *out, hipStream_t s)
{
    Mix base{};
    base.L = L;
    for (int l = 0; l < L; ++l) base.a[l] = alpha[l];
    const int64_t MN = (int64_t)M * N;
    const int blocks = (int)((MN + 255) / 256);
    if (fp32) {
        const float *p = (const float *)st;
        k_mixture_map<float><<<blocks, 256, 0, s>>>(p, p + 2 * MNL, p + MNL, p + 3 * MNL, MN, L, base, out);
    } else {
        const double *p = (const double *)st;
        k_mixture_map<double><<<blocks, 256, 0, s>>>(p, p + 2 * MNL, p + MNL, p + 3 * MNL, MN, L, base, out);
    }
    return hipGetLastError();
}

// -- flow colour ------------------------------------------------------------
struct Range {
    double maxu, minu, maxv, minv, maxrad;
};

__device__ __forceinline__ double nanmax(double a, double b) { return isnan(b) ? a : fmax(a, b); }
__device__ __forceinline__ double nanmin(double a, double b) { return isnan(b) ? a : fmin(a, b); }

__global__ void k_flow_range(const double *__restrict__ flow, int64_t MN, Range *partials)
{
    Range r{-999.0, 999.0, -999.0, 999.0, -1.0};
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < MN;
         i += (int64_t)gridDim.x * blockDim.x) {
        double u = flow[i], v = flow[MN + i];
        if (fabs(u) > 1e9 || fabs(v) > 1e9) u = v = 0.0;  // UNKNOWN_FLOW_THRESH
        r.maxu = nanmax(r.maxu, u); r.minu = nanmin(r.minu, u);
        r.maxv = nanmax(r.maxv, v); r.minv = nanmin(r.minv, v);
        r.maxrad = nanmax(r.maxrad, sqrt(u * u + v * v));
    }
    __shared__ Range sh[256];
    sh[threadIdx.x] = r;
    __syncthreads();
    for (int s = blockDim.x / 2; s > 0; s >>= 1) {
        if ((int)threadIdx.x < s) {
            Range &a = sh[threadIdx.x];
            const Range &b = sh[threadIdx.x + s];
            a.maxu = fmax(a.maxu, b.maxu); a.minu = fmin(a.minu, b.minu);
            a.maxv = fmax(a.maxv, b.maxv); a.minv = fmin(a.minv, b.minv);
            a.maxrad = fmax(a.maxrad, b.maxrad);
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) partials[blockIdx.x] = sh[0];
}

__constant__ unsigned char c_wheel[55][3];

__global__ void k_flow_color(const double *__restrict__ flow, int64_t MN, double scale,
                             uint8_t *__restrict__ img, double *__restrict__ flo,
                             uint8_t *__restrict__ unknown)
{
    const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (i >= MN) return;
    double u = flow[i], v = flow[MN + i];
    const bool unk = fabs(u) > 1e9 || fabs(v) > 1e9;
    if (unk) u = v = 0.0;
    flo[i] = u;
    flo[MN + i] = v;
    unknown[i] = unk;
    u = u / scale;  // u/(maxrad+eps)
    v = v / scale;
    const bool nan_ = isnan(u) || isnan(v);
    if (nan_) u = v = 0.0;
    const int ncols = 55;
    const double rad = sqrt(u * u + v * v);
    const double a = atan2(-v, -u) / M_PI;
    const double fk = (a + 1) / 2 * (ncols - 1) + 1;
    const int k0 = (int)floor(fk);
    int k1 = k0 + 1;
    if (k1 == ncols + 1) k1 = 1;
    const double f = fk - k0;
    for (int ch = 0; ch < 3; ++ch) {
        const double col0 = c_wheel[k0 - 1][ch] / 255.0, col1 = c_wheel[k1 - 1][ch] / 255.0;
        double col = (1 - f) * col0 + f * col1;
        if (rad <= 1) col = 1 - rad * (1 - col);
        else col = col * 0.75;
        double q = floor(255 * col * (1 - (double)nan_));
        q = fmin(fmax(q, 0.0), 255.0);
        img[i + MN * ch] = unk ? 0 : (uint8_t)q;
    }
}

// makeColorwheel (legacy/computeColor.m:76-115)
static void make_wheel(unsigned char w[55][3])
{
    const int RY = 15, YG = 6, GC = 4, CB = 11, BM = 13, MR = 6;
    for (int i = 0; i < 55; ++i) w[i][0] = w[i][1] = w[i][2] = 0;
    int col = 0;
    for (int i = 0; i < RY; ++i) { w[col + i][0] = 255; w[col + i][1] = (unsigned char)std::floor(255.0 * i / RY); }
    col += RY;
    for (int i = 0; i < YG; ++i) { w[col + i][0] = (unsigned char)(255 - std::floor(255.0 * i / YG)); w[col + i][1] = 255; }
    col += YG;
    for (int i = 0; i < GC; ++i) { w[col + i][1] = 255; w[col + i][2] = (unsigned char)std::floor(255.0 * i / GC); }
    col += GC;
    for (int i = 0; i < CB; ++i) { w[col + i][1] = (unsigned char)(255 - std::floor(255.0 * i / CB)); w[col + i][2] = 255; }
    col += CB;
    for (int i = 0; i < BM; ++i) { w[col + i][2] = 255; w[col + i][0] = (unsigned char)std::floor(255.0 * i / BM); }
    col += BM;
    for (int i = 0; i < MR; ++i) { w[col + i][2] = (unsigned char)(255 - std::floor(255.0 * i / MR)); w[col + i][0] = 255; }
}

}  // namespace gq

using namespace gq;

namespace {
struct DevBuf {
    void *p = nullptr;
    ~DevBuf()
    {
        if (p) (void)hipFree(p);
    }
};
}  // namespace

extern "C" {

gqmap_status gqmap_projsplx(const double *Y, double *X, int n, int ncols, int device)
{
    clear_error();
    GQ_CHECK(Y && X, GQMAP_ERR_INVALID_ARG, "null argument");
    GQ_CHECK(n >= 1 && n <= PROJ_NMAX, GQMAP_ERR_INVALID_ARG, "projsplx: n=%d outside [1,%d]", n, PROJ_NMAX);
    GQ_CHECK(ncols >= 0, GQMAP_ERR_INVALID_ARG, "ncols < 0");
    if (ncols == 0) return GQMAP_OK;
    GQ_CHECK(gqmap_device_count() > device && device >= 0, GQMAP_ERR_NO_DEVICE, "no HIP device %d", device);
    DeviceGuard dg(device);
    const size_t bytes = sizeof(double) * (size_t)n * ncols;
    DevBuf dy, dx;
    GQ_HIP(hipMalloc(&dy.p, bytes));
    GQ_HIP(hipMalloc(&dx.p, bytes));
    GQ_HIP(hipMemcpy(dy.p, Y, bytes, hipMemcpyHostToDevice));
    k_projsplx<<<(ncols + 255) / 256, 256>>>((const double *)dy.p, (double *)dx.p, n, ncols);
    GQ_HIP(hipGetLastError());
    GQ_HIP(hipMemcpy(X, dx.p, bytes, hipMemcpyDeviceToHost));
    return GQMAP_OK;
}

gqmap_status gqmap_mixture_map(const double *alpha, const double *muu, const double *sigu,
                               const double *muv, const double *sigv, int M, int N, int L,
                               double *out, int device)
{
    clear_error();
    GQ_CHECK(alpha && muu && sigu && muv && sigv && out, GQMAP_ERR_INVALID_ARG, "null argument");
    GQ_CHECK(L >= 1 && L <= GQMAP_LMAX, GQMAP_ERR_INVALID_ARG, "L=%d outside [1,%d]", L, GQMAP_LMAX);
    GQ_CHECK(M >= 1 && N >= 1, GQMAP_ERR_INVALID_ARG, "empty grid");
    GQ_CHECK(gqmap_device_count() > device && device >= 0, GQMAP_ERR_NO_DEVICE, "no HIP device %d", device);
    DeviceGuard dg(device);
    const int64_t MNL = (int64_t)M * N * L;
    // pack as the engine's state planes: muu, muv, sigu, sigv
    std::vector<double> st((size_t)MNL * 4);
    std::copy(muu, muu + MNL, st.begin());
    std::copy(muv, muv + MNL, st.begin() + MNL);
    std::copy(sigu, sigu + MNL, st.begin() + 2 * MNL);
    std::copy(sigv, sigv + MNL, st.begin() + 3 * MNL);
    DevBuf dst, dout;
    GQ_HIP(hipMalloc(&dst.p, st.size() * sizeof(double)));
    GQ_HIP(hipMalloc(&dout.p, sizeof(double) * 2 * M * (size_t)N));
    GQ_HIP(hipMemcpy(dst.p, st.data(), st.size() * sizeof(double), hipMemcpyHostToDevice));
    GQ_HIP(mixture_map_device(alpha, dst.p, false, MNL, M, N, L, (double *)dout.p, 0));
    GQ_HIP(hipMemcpy(out, dout.p, sizeof(double) * 2 * M * (size_t)N, hipMemcpyDeviceToHost));
    return GQMAP_OK;
}

gqmap_status gqmap_flow_to_color(const double *flow, int M, int N, double max_flow, uint8_t *img,
                                 double *flo, double *stats, uint8_t *unknown, int device)
{
    clear_error();
    GQ_CHECK(flow && img && flo && stats && unknown, GQMAP_ERR_INVALID_ARG, "null argument");
    GQ_CHECK(M >= 1 && N >= 1, GQMAP_ERR_INVALID_ARG, "empty flow");
    GQ_CHECK(gqmap_device_count() > device && device >= 0, GQMAP_ERR_NO_DEVICE, "no HIP device %d", device);
    DeviceGuard dg(device);
    static bool wheel_ready[64] = {false};
    if (device < 64 && !wheel_ready[device]) {
        unsigned char w[55][3];
        make_wheel(w);
        GQ_HIP(hipMemcpyToSymbol(HIP_SYMBOL(c_wheel), w, sizeof w));
        wheel_ready[device] = true;
    }
    const int64_t MN = (int64_t)M * N;
    const int rblocks = 128;
    DevBuf dflow, dimg, dflo, dunk, dpart;
    GQ_HIP(hipMalloc(&dflow.p, sizeof(double) * 2 * MN));
    GQ_HIP(hipMalloc(&dflo.p, sizeof(double) * 2 * MN));
    GQ_HIP(hipMalloc(&dimg.p, 3 * MN));
    GQ_HIP(hipMalloc(&dunk.p, MN));
    GQ_HIP(hipMalloc(&dpart.p, sizeof(Range) * rblocks));
    GQ_HIP(hipMemcpy(dflow.p, flow, sizeof(double) * 2 * MN, hipMemcpyHostToDevice));
    k_flow_range<<<rblocks, 256>>>((const double *)dflow.p, MN, (Range *)dpart.p);
    GQ_HIP(hipGetLastError());
    std::vector<Range> part(rblocks);
    GQ_HIP(hipMemcpy(part.data(), dpart.p, sizeof(Range) * rblocks, hipMemcpyDeviceToHost));
    Range r = part[0];
    for (int b = 1; b < rblocks; ++b) {
        r.maxu = std::fmax(r.maxu, part[b].maxu); r.minu = std::fmin(r.minu, part[b].minu);
        r.maxv = std::fmax(r.maxv, part[b].maxv); r.minv = std::fmin(r.minv, part[b].minv);
        r.maxrad = std::fmax(r.maxrad, part[b].maxrad);
    }
    double maxrad = r.maxrad;
    if (max_flow > 0) maxrad = max_flow;
    stats[0] = r.minu; stats[1] = r.maxu; stats[2] = r.minv; stats[3] = r.maxv;
    k_flow_color<<<(int)((MN + 255) / 256), 256>>>((const double *)dflow.p, MN, maxrad + DBL_EPSILON,
                                                   (uint8_t *)dimg.p, (double *)dflo.p, (uint8_t *)dunk.p);
    GQ_HIP(hipGetLastError());
    GQ_HIP(hipMemcpy(img, dimg.p, 3 * MN, hipMemcpyDeviceToHost));
    GQ_HIP(hipMemcpy(flo, dflo.p, sizeof(double) * 2 * MN, hipMemcpyDeviceToHost));
    GQ_HIP(hipMemcpy(unknown, dunk.p, MN, hipMemcpyDeviceToHost));
    return GQMAP_OK;
}

}  // extern "C"
