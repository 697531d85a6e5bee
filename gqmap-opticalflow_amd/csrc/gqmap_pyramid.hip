// gqmap_pyramid.hip -- coarse-to-fine driver of legacy/optical_flow_ctf.m:21-35
// on the device.
//
// Per level (scale s, each level twice the previous):
//   I1 = imresize(img_1, s); I2 = imresize(img_2, s)          :26-27  (at set_images)
//   warp = imresize(warp, 2) .* 2                              :29     k_resize_dim1/2
//   I1_w = interp2(I1, x - warp(:,:,1), y - warp(:,:,2))       :30-31  k_warp
//   I1_w = fillmissing(fillmissing(I1_w,'nearest',1),'nearest',2)  :32 k_fill
//   flow = gqmap_ctf(options, I1_w, I2, trueFlow .* s)         :33     level engine (k_iter<ENG=2>)
//   warp = warp + flow                                         :34     k_add_flow
//
// Everything stays resident in HBM; the host only sequences levels.  These
// resampling kernels move a few MB per level and are launch-latency bound:
// thread-per-output, m-fastest (coalesced column-major stores), the tap
// tables of a dim-2 pass are wave-uniform (scalar loads).
//
// Arithmetic is plain IEEE fp64 with contraction off, in the order of the
// restatement in oracle/gqmap_pyramid_oracle.c, so the device matches it bit
// for bit.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cmath>
#include <cstring>
#include <vector>

#include "gqmap_internal.h"

#pragma clang fp contract(off)

namespace gq {
namespace {

constexpr int TPB = 256;

inline int grid_for(int64_t n) { return (int)((n + TPB - 1) / TPB); }

// getVV (gqmap_gpu_mixture.m:191-208), same expressions as build_padded():
// pass 1 writes the interior columns with their top/bottom pads, pass 2 the
// first/last columns (corners included) from the padded columns 1..3.
__global__ void k_pad_interior(const double *__restrict__ I2, int M, int N, double *__restrict__ VV)
{
    const int M2 = M + 2;
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= (int64_t)M2 * N) return;
    const int r = (int)(t % M2), n = (int)(t / M2);
    const double *c = I2 + (size_t)M * n;
    double v;
    if (r == 0) v = (3.0 * c[0] - 3.0 * c[1]) + c[2];
    else if (r == M2 - 1) v = (3.0 * c[M - 1] - 3.0 * c[M - 2]) + c[M - 3];
    else v = c[r - 1];
    VV[r + (size_t)M2 * (n + 1)] = v;
}

__global__ void k_pad_sides(int M, int N, double *__restrict__ VV)
{
    const int M2 = M + 2, N2 = N + 2;
    const int r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= M2) return;
    double *first = VV, *last = VV + (size_t)M2 * (N2 - 1);
    first[r] = (3.0 * first[r + M2] - 3.0 * first[r + 2 * M2]) + first[r + 3 * M2];
    last[r] = (3.0 * last[r - M2] - 3.0 * last[r - 2 * M2]) + last[r - 3 * M2];
}

__global__ void k_f32_exact(const double *__restrict__ d, int64_t n, int *flag)
{
    int bad = 0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        bad |= (double)(float)d[i] != d[i];
    if (bad) atomicOr(flag, 1);
}

template <typename T>
__global__ void k_convert(const double *__restrict__ s, T *__restrict__ d, int64_t n)
{
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        d[i] = T(s[i]);
}

// imresize along dim 1: out(i, rest) = sum_k w(i,k) * in(idx(i,k), rest)
__global__ void k_resize_dim1(const double *__restrict__ in, int M, int64_t rest,
                              const double *__restrict__ w, const int *__restrict__ idx, int P, int oM,
                              double *__restrict__ out)
{
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= (int64_t)oM * rest) return;
    const int i = (int)(t % oM);
    const int64_t r = t / oM;
    const double *col = in + (size_t)M * r;
    const double *wi = w + (size_t)i * P;
    const int *ji = idx + (size_t)i * P;
    double s = 0.0;
    for (int k = 0; k < P; ++k) s += wi[k] * col[ji[k]];
    out[t] = s;
}

// imresize along dim 2 (+ the driver's scalar factor, e.g. .*2 of the prolong)
__global__ void k_resize_dim2(const double *__restrict__ in, int oM, int N, int C,
                              const double *__restrict__ w, const int *__restrict__ idx, int P, int oN,
                              double post, double *__restrict__ out)
{
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= (int64_t)oM * oN * C) return;
    const int i = (int)(t % oM);
    const int j = (int)((t / oM) % oN);
    const int c = (int)(t / ((int64_t)oM * oN));
    const double *plane = in + (size_t)oM * N * c + i;
    const double *wj = w + (size_t)j * P;
    const int *jj = idx + (size_t)j * P;
    double s = 0.0;
    for (int k = 0; k < P; ++k) s += wj[k] * plane[(size_t)oM * jj[k]];
    out[t] = post == 1.0 ? s : s * post;
}

// interp2(V, x - wu, y - wv), 'linear', NaN outside [1,N] x [1,M]
__global__ void k_warp(const double *__restrict__ V, int M, int N, const double *__restrict__ warp,
                       double *__restrict__ out)
{
    const int64_t MN = (int64_t)M * N;
    const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= MN) return;
    const int m = (int)(q % M), n = (int)(q / M);
    const double xq = (double)(n + 1) - warp[q], yq = (double)(m + 1) - warp[q + MN];
    if (!(xq >= 1.0 && xq <= (double)N && yq >= 1.0 && yq <= (double)M)) {
        out[q] = __builtin_nan("");
        return;
    }
    const int ix = min((int)floor(xq), N - 1), iy = min((int)floor(yq), M - 1);
    const double s = xq - ix, t = yq - iy;
    const double *c0 = V + (size_t)M * (ix - 1) + (iy - 1), *c1 = c0 + M;
    const double top = (1.0 - s) * c0[0] + s * c1[0];
    const double bot = (1.0 - s) * c0[1] + s * c1[1];
    out[q] = (1.0 - t) * top + t * bot;
}

// fillmissing(A,'nearest',dim): nearest non-NaN along the line, tie -> later
__global__ void k_fill(const double *__restrict__ in, int M, int N, int dim, double *__restrict__ out)
{
    const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= (int64_t)M * N) return;
    const double v = in[q];
    if (!isnan(v)) {
        out[q] = v;
        return;
    }
    const int m = (int)(q % M), n = (int)(q / M);
    const int k = dim == 1 ? m : n, len = dim == 1 ? M : N;
    const int64_t stride = dim == 1 ? 1 : M;
    const double *line = in + (dim == 1 ? (int64_t)M * n : (int64_t)m);
    int lo = k - 1, hi = k + 1;
    while (lo >= 0 && isnan(line[stride * lo])) --lo;
    while (hi < len && isnan(line[stride * hi])) ++hi;
    double r = v;
    if (lo >= 0 && hi < len) r = (k - lo < hi - k) ? line[stride * lo] : line[stride * hi];
    else if (lo >= 0) r = line[stride * lo];
    else if (hi < len) r = line[stride * hi];
    out[q] = r;
}

// warp = warp + flow (optical_flow_ctf.m:34); also keeps the level flow
template <typename R>
__global__ void k_add_flow(double *__restrict__ warp, const R *__restrict__ muu, const R *__restrict__ muv,
                           double *__restrict__ flow, int64_t MN)
{
    const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= MN) return;
    const double u = double(muu[q]), v = double(muv[q]);
    flow[q] = u;
    flow[q + MN] = v;
    warp[q] = warp[q] + u;
    warp[q + MN] = warp[q + MN] + v;
}

// Tap tables of one separable imresize (dim 1 and dim 2) on the device.
struct Resampler {
    int in_len[2] = {0, 0}, out_len[2] = {0, 0}, P[2] = {0, 0};
    double *w[2] = {nullptr, nullptr};
    int *idx[2] = {nullptr, nullptr};

    // the tables are uploaded on stream s, the stream apply() will run on
    // (the pyramid's stream is non-blocking: null-stream copies would not be
    // ordered with it)
    gqmap_status build(int M, int N, double scale, int antialias, hipStream_t s)
    {
        release();
        const int len[2] = {M, N};
        for (int d = 0; d < 2; ++d) {
            std::vector<double> hw;
            std::vector<int> hi;
            in_len[d] = len[d];
            out_len[d] = resize_len(len[d], scale);
            GQ_CHECK(out_len[d] >= 1, GQMAP_ERR_INVALID_ARG, "imresize: empty output (len %d, scale %g)",
                     len[d], scale);
            P[d] = resize_contrib(len[d], out_len[d], scale, antialias, hw, hi);
            GQ_HIP(hipMalloc(&w[d], hw.size() * sizeof(double)));
            GQ_HIP(hipMalloc(&idx[d], hi.size() * sizeof(int)));
            GQ_HIP(hipMemcpyAsync(w[d], hw.data(), hw.size() * sizeof(double), hipMemcpyHostToDevice, s));
            GQ_HIP(hipMemcpyAsync(idx[d], hi.data(), hi.size() * sizeof(int), hipMemcpyHostToDevice, s));
            GQ_HIP(hipStreamSynchronize(s));  // hw / hi are host temporaries
        }
        return GQMAP_OK;
    }
    // in: in_len[0] x in_len[1] x C; tmp: out_len[0] x in_len[1] x C
    hipError_t apply(const double *in, int C, double post, double *tmp, double *out, hipStream_t s) const
    {
        const int64_t n1 = (int64_t)out_len[0] * in_len[1] * C;
        k_resize_dim1<<<grid_for(n1), TPB, 0, s>>>(in, in_len[0], (int64_t)in_len[1] * C, w[0], idx[0], P[0],
                                                   out_len[0], tmp);
        const int64_t n2 = (int64_t)out_len[0] * out_len[1] * C;
        k_resize_dim2<<<grid_for(n2), TPB, 0, s>>>(tmp, out_len[0], in_len[1], C, w[1], idx[1], P[1],
                                                   out_len[1], post, out);
        return hipGetLastError();
    }
    void release()
    {
        for (int d = 0; d < 2; ++d) {
            if (w[d]) (void)hipFree(w[d]);
            if (idx[d]) (void)hipFree(idx[d]);
            w[d] = nullptr;
            idx[d] = nullptr;
        }
    }
};

hipError_t warp_fill(const double *V, int M, int N, const double *warp, bool fill, double *tmp, double *out,
                     hipStream_t s)
{
    const int64_t MN = (int64_t)M * N;
    if (!fill) {
        k_warp<<<grid_for(MN), TPB, 0, s>>>(V, M, N, warp, out);
        return hipGetLastError();
    }
    k_warp<<<grid_for(MN), TPB, 0, s>>>(V, M, N, warp, out);
    k_fill<<<grid_for(MN), TPB, 0, s>>>(out, M, N, 1, tmp);
    k_fill<<<grid_for(MN), TPB, 0, s>>>(tmp, M, N, 2, out);
    return hipGetLastError();
}

// RAII device buffer for the standalone entry points
struct DBuf {
    void *p = nullptr;
    ~DBuf()
    {
        if (p) (void)hipFree(p);
    }
};

}  // namespace

hipError_t pad_vv_device(const double *dI2, int M, int N, double *dVV, hipStream_t s)
{
    k_pad_interior<<<grid_for((int64_t)(M + 2) * N), TPB, 0, s>>>(dI2, M, N, dVV);
    k_pad_sides<<<grid_for(M + 2), TPB, 0, s>>>(M, N, dVV);
    return hipGetLastError();
}

hipError_t f32_exact_device(const double *d, size_t n, int *d_flag, bool *exact, hipStream_t s)
{
    hipError_t e = hipMemsetAsync(d_flag, 0, sizeof(int), s);
    if (e != hipSuccess) return e;
    k_f32_exact<<<std::min(grid_for((int64_t)n), 1024), TPB, 0, s>>>(d, (int64_t)n, d_flag);
    int h = 0;
    if ((e = hipMemcpyAsync(&h, d_flag, sizeof(int), hipMemcpyDeviceToHost, s)) != hipSuccess) return e;
    if ((e = hipStreamSynchronize(s)) != hipSuccess) return e;
    *exact = h == 0;
    return hipSuccess;
}

hipError_t convert_device(const double *src, void *dst, size_t n, bool to_f32, hipStream_t s)
{
    const int g = std::min(grid_for((int64_t)n), 4096);
    if (to_f32) k_convert<float><<<g, TPB, 0, s>>>(src, (float *)dst, (int64_t)n);
    else k_convert<double><<<g, TPB, 0, s>>>(src, (double *)dst, (int64_t)n);
    return hipGetLastError();
}

}  // namespace gq

using namespace gq;

struct gqmap_pyramid {
    struct Level {
        int M = 0, N = 0;
        double scale = 1;
        double *I1 = nullptr, *I2 = nullptr, *I1w = nullptr, *warp = nullptr, *flow = nullptr;
        Resampler img, pro;  // full-res -> level (frames); previous warp -> level (x2)
        gqmap_ctx *ctx = nullptr;
        int its_done = 0;
        std::vector<double> energy, aepe;  // per iteration of the last run (gqmap_ctf's Energy, AEPE)
        bool has_truth = false;
    };
    gqmap_options opt;
    int device = 0, nlev = 0;
    double scales[GQMAP_CTF_MAX_LEVELS];
    int M = 0, N = 0;
    hipStream_t stream = nullptr;
    double *img[2] = {nullptr, nullptr};
    double *warp0 = nullptr;  // imresize(zeros(M,N,2), scales(1)/2)  (:24)
    int M0 = 0, N0 = 0;
    double *scratch = nullptr, *vv = nullptr, *tmp = nullptr;
    int *flag = nullptr;
    Level lev[GQMAP_CTF_MAX_LEVELS];
    bool ran = false;
    std::vector<double> truth;  // gqmap_ctf_set_truth: full-resolution trueFlow, M x N x 2 (host)

    void release_levels()
    {
        for (int l = 0; l < nlev; ++l) {
            Level &L = lev[l];
            if (L.ctx) gqmap_destroy(L.ctx);
            L.ctx = nullptr;
            L.img.release();
            L.pro.release();
            for (double **b : {&L.I1, &L.I2, &L.I1w, &L.warp, &L.flow}) {
                if (*b) (void)hipFree(*b);
                *b = nullptr;
            }
        }
        for (double **b : {&img[0], &img[1], &warp0, &scratch, &vv, &tmp}) {
            if (*b) (void)hipFree(*b);
            *b = nullptr;
        }
        if (flag) (void)hipFree(flag);
        flag = nullptr;
    }
};

namespace {

gqmap_status download_d(double *dst, const double *src, size_t n, hipStream_t s)
{
    if (!dst) return GQMAP_OK;
    GQ_HIP(hipMemcpyAsync(dst, src, n * sizeof(double), hipMemcpyDeviceToHost, s));
    GQ_HIP(hipStreamSynchronize(s));
    return GQMAP_OK;
}

}  // namespace

extern "C" {

int gqmap_resize_len(int len, double scale) { return resize_len(len, scale); }

gqmap_status gqmap_imresize(const double *in, int M, int N, int C, double scale, int antialias,
                            double *out, int device)
{
    clear_error();
    GQ_CHECK(in && out, GQMAP_ERR_INVALID_ARG, "gqmap_imresize: null argument");
    GQ_CHECK(M >= 1 && N >= 1 && C >= 1, GQMAP_ERR_INVALID_ARG, "gqmap_imresize: empty input");
    GQ_CHECK(scale > 0 && std::isfinite(scale), GQMAP_ERR_INVALID_ARG, "gqmap_imresize: scale %g", scale);
    DeviceGuard dg(device);
    Resampler r;
    gqmap_status st = r.build(M, N, scale, antialias, nullptr);
    if (st != GQMAP_OK) {
        r.release();
        return st;
    }
    const int oM = r.out_len[0], oN = r.out_len[1];
    DBuf din, dtmp, dout;
    hipError_t e = hipMalloc(&din.p, (size_t)M * N * C * sizeof(double));
    if (e == hipSuccess) e = hipMalloc(&dtmp.p, (size_t)oM * N * C * sizeof(double));
    if (e == hipSuccess) e = hipMalloc(&dout.p, (size_t)oM * oN * C * sizeof(double));
    if (e == hipSuccess) e = hipMemcpy(din.p, in, (size_t)M * N * C * sizeof(double), hipMemcpyHostToDevice);
    if (e == hipSuccess) e = r.apply((const double *)din.p, C, 1.0, (double *)dtmp.p, (double *)dout.p, nullptr);
    if (e == hipSuccess) e = hipMemcpy(out, dout.p, (size_t)oM * oN * C * sizeof(double), hipMemcpyDeviceToHost);
    r.release();
    GQ_HIP(e);
    return GQMAP_OK;
}

gqmap_status gqmap_warp_image(const double *V, int M, int N, const double *warp, int fill, double *out,
                              int device)
{
    clear_error();
    GQ_CHECK(V && warp && out, GQMAP_ERR_INVALID_ARG, "gqmap_warp_image: null argument");
    GQ_CHECK(M >= 2 && N >= 2, GQMAP_ERR_INVALID_ARG, "gqmap_warp_image: %dx%d", M, N);
    DeviceGuard dg(device);
    const size_t MN = (size_t)M * N;
    DBuf dv, dw, dt, dout;
    GQ_HIP(hipMalloc(&dv.p, MN * sizeof(double)));
    GQ_HIP(hipMalloc(&dw.p, 2 * MN * sizeof(double)));
    GQ_HIP(hipMalloc(&dt.p, MN * sizeof(double)));
    GQ_HIP(hipMalloc(&dout.p, MN * sizeof(double)));
    GQ_HIP(hipMemcpy(dv.p, V, MN * sizeof(double), hipMemcpyHostToDevice));
    GQ_HIP(hipMemcpy(dw.p, warp, 2 * MN * sizeof(double), hipMemcpyHostToDevice));
    GQ_HIP(warp_fill((const double *)dv.p, M, N, (const double *)dw.p, fill != 0, (double *)dt.p,
                     (double *)dout.p, nullptr));
    GQ_HIP(hipMemcpy(out, dout.p, MN * sizeof(double), hipMemcpyDeviceToHost));
    return GQMAP_OK;
}

gqmap_status gqmap_ctf_create(gqmap_pyramid **out, const gqmap_options *level_opt, const double *scales,
                              int n_levels, int device)
{
    clear_error();
    GQ_CHECK(out && level_opt && scales, GQMAP_ERR_INVALID_ARG, "gqmap_ctf_create: null argument");
    *out = nullptr;
    GQ_CHECK(level_opt->engine == GQMAP_ENGINE_CTF, GQMAP_ERR_INVALID_ARG,
             "gqmap_ctf_create: level options must use GQMAP_ENGINE_CTF");
    GQ_CHECK(n_levels >= 1 && n_levels <= GQMAP_CTF_MAX_LEVELS, GQMAP_ERR_INVALID_ARG,
             "n_levels=%d outside [1,%d]", n_levels, GQMAP_CTF_MAX_LEVELS);
    GQ_CHECK(scales[n_levels - 1] == 1.0, GQMAP_ERR_INVALID_ARG, "the last level must have scale 1");
    for (int l = 0; l < n_levels; ++l)
        GQ_CHECK(scales[l] > 0 && scales[l] <= 1.0 && (l == 0 || scales[l] > scales[l - 1]),
                 GQMAP_ERR_INVALID_ARG, "scales must ascend in (0,1] (scale[%d]=%g)", l, scales[l]);
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
        set_error("no HIP device available");
        return GQMAP_ERR_NO_DEVICE;
    }
    GQ_CHECK(device >= 0 && device < ndev, GQMAP_ERR_INVALID_ARG, "device %d of %d", device, ndev);
    DeviceGuard dg(device);
    gqmap_pyramid *p = new gqmap_pyramid();
    p->opt = *level_opt;
    p->device = device;
    p->nlev = n_levels;
    for (int l = 0; l < n_levels; ++l) p->scales[l] = scales[l];
    if (hipStreamCreateWithFlags(&p->stream, hipStreamNonBlocking) != hipSuccess) {
        delete p;
        set_error("hipStreamCreate failed");
        return GQMAP_ERR_HIP;
    }
    *out = p;
    return GQMAP_OK;
}

gqmap_status gqmap_ctf_set_images(gqmap_pyramid *p, const double *img1, const double *img2, int M, int N)
{
    clear_error();
    GQ_CHECK(p && img1 && img2, GQMAP_ERR_INVALID_ARG, "gqmap_ctf_set_images: null argument");
    GQ_CHECK(M >= 4 && N >= 4, GQMAP_ERR_INVALID_ARG, "image %dx%d too small", M, N);
    DeviceGuard dg(p->device);
    // level geometry first (all checks before any allocation)
    int Ml[GQMAP_CTF_MAX_LEVELS], Nl[GQMAP_CTF_MAX_LEVELS];
    const int M0 = resize_len(M, p->scales[0] / 2), N0 = resize_len(N, p->scales[0] / 2);
    for (int l = 0; l < p->nlev; ++l) {
        Ml[l] = resize_len(M, p->scales[l]);
        Nl[l] = resize_len(N, p->scales[l]);
        const int pm = l ? Ml[l - 1] : M0, pn = l ? Nl[l - 1] : N0;
        GQ_CHECK(resize_len(pm, 2.0) == Ml[l] && resize_len(pn, 2.0) == Nl[l], GQMAP_ERR_INVALID_ARG,
                 "level %d: imresize(warp,2) of %dx%d is not the level size %dx%d "
                 "(optical_flow_ctf.m:29-31 needs each level twice the previous)",
                 l, pm, pn, Ml[l], Nl[l]);
        GQ_CHECK(Ml[l] >= 4 && Nl[l] >= 4, GQMAP_ERR_INVALID_ARG, "level %d is %dx%d (< 4)", l, Ml[l], Nl[l]);
    }
    (void)hipStreamSynchronize(p->stream);
    p->release_levels();
    p->ran = false;
    p->M = M;
    p->N = N;
    p->M0 = M0;
    p->N0 = N0;
    const size_t MN = (size_t)M * N;
    GQ_HIP(hipMalloc(&p->img[0], MN * sizeof(double)));
    GQ_HIP(hipMalloc(&p->img[1], MN * sizeof(double)));
    GQ_HIP(hipMalloc(&p->scratch, 2 * MN * sizeof(double)));
    GQ_HIP(hipMalloc(&p->tmp, MN * sizeof(double)));
    GQ_HIP(hipMalloc(&p->vv, (size_t)(M + 2) * (N + 2) * sizeof(double)));
    GQ_HIP(hipMalloc(&p->flag, sizeof(int)));
    GQ_HIP(hipMalloc(&p->warp0, (size_t)M0 * N0 * 2 * sizeof(double)));
    GQ_HIP(hipMemsetAsync(p->warp0, 0, (size_t)M0 * N0 * 2 * sizeof(double), p->stream));
    GQ_HIP(hipMemcpyAsync(p->img[0], img1, MN * sizeof(double), hipMemcpyHostToDevice, p->stream));
    GQ_HIP(hipMemcpyAsync(p->img[1], img2, MN * sizeof(double), hipMemcpyHostToDevice, p->stream));
    for (int l = 0; l < p->nlev; ++l) {
        gqmap_pyramid::Level &L = p->lev[l];
        L.M = Ml[l];
        L.N = Nl[l];
        L.scale = p->scales[l];
        const size_t mn = (size_t)L.M * L.N;
        GQ_HIP(hipMalloc(&L.I1, mn * sizeof(double)));
        GQ_HIP(hipMalloc(&L.I2, mn * sizeof(double)));
        GQ_HIP(hipMalloc(&L.I1w, mn * sizeof(double)));
        GQ_HIP(hipMalloc(&L.warp, 2 * mn * sizeof(double)));
        GQ_HIP(hipMalloc(&L.flow, 2 * mn * sizeof(double)));
        gqmap_status s = L.img.build(M, N, L.scale, 1, p->stream);
        if (s != GQMAP_OK) return s;
        s = L.pro.build(l ? Ml[l - 1] : M0, l ? Nl[l - 1] : N0, 2.0, 1, p->stream);
        if (s != GQMAP_OK) return s;
        // I1 = imresize(img_1, scale); I2 = imresize(img_2, scale)  (:26-27)
        GQ_HIP(L.img.apply(p->img[0], 1, 1.0, p->scratch, L.I1, p->stream));
        GQ_HIP(L.img.apply(p->img[1], 1, 1.0, p->scratch, L.I2, p->stream));
        // level engine: gqmap_ctf(options, I1_w, I2, trueFlow.*scale)
        gqmap_options o = p->opt;
        o.minu *= L.scale;
        o.maxu *= L.scale;
        o.minv *= L.scale;
        o.maxv *= L.scale;
        s = gqmap_create(&L.ctx, &o, p->device);
        L.has_truth = false;
        if (s != GQMAP_OK) return s;
        ctx_adopt_stream(L.ctx, p->stream);
    }
    GQ_HIP(hipStreamSynchronize(p->stream));
    return GQMAP_OK;
}

gqmap_status gqmap_ctf_run(gqmap_pyramid *p, uint64_t seed, double *flow, int *its_done, double *elapsed_ms)
{
    clear_error();
    GQ_CHECK(p, GQMAP_ERR_INVALID_ARG, "null pyramid");
    GQ_CHECK(p->lev[0].ctx, GQMAP_ERR_STATE, "gqmap_ctf_run before gqmap_ctf_set_images");
    DeviceGuard dg(p->device);
    GQ_HIP(hipStreamSynchronize(p->stream));
    const auto t0 = std::chrono::steady_clock::now();
    for (int l = 0; l < p->nlev; ++l) {
        gqmap_pyramid::Level &L = p->lev[l];
        const double *prev = l ? p->lev[l - 1].warp : p->warp0;
        // warp = imresize(warp,2).*2 (:29)
        GQ_HIP(L.pro.apply(prev, 2, 2.0, p->scratch, L.warp, p->stream));
        // I1_w = fillmissing(fillmissing(interp2(I1, x-wu, y-wv),'nearest',1),'nearest',2) (:30-32)
        GQ_HIP(warp_fill(L.I1, L.M, L.N, L.warp, true, p->tmp, L.I1w, p->stream));
        gqmap_status s = ctx_set_images_device(L.ctx, L.I1w, L.I2, L.M, L.N, p->vv, p->flag);
        if (s != GQMAP_OK) return s;
        if ((s = gqmap_init_state(L.ctx, seed + (uint64_t)l)) != GQMAP_OK) return s;
        // gqmap_ctf(options,I1_w,I2,trueFlow.*scale) (:33): GRDT is the full
        // resolution GT times the level scale; the level reads its top-left block
        if (!p->truth.empty()) {
            const size_t MN = (size_t)p->M * p->N;
            std::vector<double> blk(2 * (size_t)L.M * L.N);
            for (int k = 0; k < 2; ++k)
                for (int n = 0; n < L.N; ++n)
                    for (int m = 0; m < L.M; ++m)
                        blk[(size_t)L.M * L.N * k + (size_t)L.M * n + m] = p->truth[MN * k + (size_t)p->M * n + m] * L.scale;
            if ((s = gqmap_set_truth(L.ctx, blk.data(), L.M, L.N)) != GQMAP_OK) return s;
            L.has_truth = true;
        } else if (L.has_truth) {
            if ((s = gqmap_set_truth(L.ctx, nullptr, 0, 0)) != GQMAP_OK) return s;
            L.has_truth = false;
        }
        int done = 0;
        std::vector<double> tr(3 * (size_t)std::max(p->opt.its, 1));
        L.aepe.assign((size_t)std::max(p->opt.its, 1), 0.0);
        if ((s = gqmap_run_aepe(L.ctx, p->opt.its, &done, tr.data(), L.aepe.data())) != GQMAP_OK) return s;
        L.its_done = done;
        L.aepe.resize(done);
        L.energy.resize(done);
        for (int i = 0; i < done; ++i) L.energy[i] = tr[3 * (size_t)i];
        const void *muu, *muv;
        bool f32;
        if ((s = ctx_flow_device(L.ctx, &muu, &muv, &f32)) != GQMAP_OK) return s;
        const int64_t mn = (int64_t)L.M * L.N;
        // warp = warp + flow (:34)
        if (f32)
            k_add_flow<float><<<grid_for(mn), TPB, 0, p->stream>>>(L.warp, (const float *)muu, (const float *)muv,
                                                                   L.flow, mn);
        else
            k_add_flow<double><<<grid_for(mn), TPB, 0, p->stream>>>(L.warp, (const double *)muu,
                                                                    (const double *)muv, L.flow, mn);
        GQ_HIP(hipGetLastError());
    }
    GQ_HIP(hipStreamSynchronize(p->stream));
    const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    p->ran = true;
    if (elapsed_ms) *elapsed_ms = ms;
    if (its_done)
        for (int l = 0; l < p->nlev; ++l) its_done[l] = p->lev[l].its_done;
    const gqmap_pyramid::Level &F = p->lev[p->nlev - 1];
    return download_d(flow, F.warp, (size_t)F.M * F.N * 2, p->stream);
}

gqmap_status gqmap_ctf_get_level(gqmap_pyramid *p, int level, int *Ml, int *Nl, double *I1w, double *I2,
                                 double *flow, double *warp)
{
    clear_error();
    GQ_CHECK(p, GQMAP_ERR_INVALID_ARG, "null pyramid");
    GQ_CHECK(level >= 0 && level < p->nlev, GQMAP_ERR_INVALID_ARG, "level %d of %d", level, p->nlev);
    const gqmap_pyramid::Level &L = p->lev[level];
    GQ_CHECK(L.ctx, GQMAP_ERR_STATE, "gqmap_ctf_get_level before gqmap_ctf_set_images");
    GQ_CHECK(p->ran || !(I1w || flow || warp), GQMAP_ERR_STATE, "gqmap_ctf_get_level before gqmap_ctf_run");
    DeviceGuard dg(p->device);
    if (Ml) *Ml = L.M;
    if (Nl) *Nl = L.N;
    const size_t mn = (size_t)L.M * L.N;
    gqmap_status s;
    if ((s = download_d(I1w, L.I1w, mn, p->stream)) != GQMAP_OK) return s;
    if ((s = download_d(I2, L.I2, mn, p->stream)) != GQMAP_OK) return s;
    if ((s = download_d(flow, L.flow, 2 * mn, p->stream)) != GQMAP_OK) return s;
    return download_d(warp, L.warp, 2 * mn, p->stream);
}

gqmap_status gqmap_ctf_set_truth(gqmap_pyramid *p, const double *flow, int M, int N)
{
    clear_error();
    GQ_CHECK(p, GQMAP_ERR_INVALID_ARG, "null pyramid");
    if (!flow) {
        p->truth.clear();
        return GQMAP_OK;
    }
    GQ_CHECK(p->lev[0].ctx, GQMAP_ERR_STATE, "gqmap_ctf_set_truth before gqmap_ctf_set_images");
    GQ_CHECK(M == p->M && N == p->N, GQMAP_ERR_INVALID_ARG, "truth %dx%d, frames %dx%d", M, N, p->M, p->N);
    p->truth.assign(flow, flow + 2 * (size_t)M * N);
    return GQMAP_OK;
}

gqmap_status gqmap_ctf_get_trace(gqmap_pyramid *p, int level, int *n, double *energy, double *aepe)
{
    clear_error();
    GQ_CHECK(p, GQMAP_ERR_INVALID_ARG, "null pyramid");
    GQ_CHECK(level >= 0 && level < p->nlev, GQMAP_ERR_INVALID_ARG, "level %d of %d", level, p->nlev);
    GQ_CHECK(p->ran, GQMAP_ERR_STATE, "gqmap_ctf_get_trace before gqmap_ctf_run");
    const gqmap_pyramid::Level &L = p->lev[level];
    if (n) *n = L.its_done;
    if (energy) std::copy(L.energy.begin(), L.energy.end(), energy);
    if (aepe) std::copy(L.aepe.begin(), L.aepe.end(), aepe);
    return GQMAP_OK;
}

// Not in the public header: level `level`'s padded frame as its engine reads
// it (gqmap_debug_read_vv of the level context).
gqmap_status gqmap_debug_read_vv(gqmap_ctx *c, double *out, size_t n, int *stored_f32);
gqmap_status gqmap_ctf_debug_read_vv(gqmap_pyramid *p, int level, double *out, size_t n, int *stored_f32)
{
    clear_error();
    GQ_CHECK(p, GQMAP_ERR_INVALID_ARG, "null pyramid");
    GQ_CHECK(level >= 0 && level < p->nlev, GQMAP_ERR_INVALID_ARG, "level %d of %d", level, p->nlev);
    GQ_CHECK(p->ran, GQMAP_ERR_STATE, "gqmap_ctf_debug_read_vv before gqmap_ctf_run");
    return gqmap_debug_read_vv(p->lev[level].ctx, out, n, stored_f32);
}

void gqmap_ctf_destroy(gqmap_pyramid *p)
{
    if (!p) return;
    DeviceGuard dg(p->device);
    if (p->stream) (void)hipStreamSynchronize(p->stream);
    p->release_levels();
    if (p->stream) (void)hipStreamDestroy(p->stream);
    delete p;
}

}  // extern "C"
