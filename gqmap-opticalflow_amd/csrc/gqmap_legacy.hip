// gqmap_legacy.hip -- device drop-in for legacy/gqmap_cpu.m, the legacy
// flow-denoising QGMAP ([mu,sigma,rou] = gqmap_cpu(options, flow)): a
// Gaussian observation of a given flow field (node, :20-26), truncated
// quadratic pairwise terms (edges, :28-54), the reference's own neighbour
// shift in the gradient sum (:58-60), plain gradient ascent with
// sigma = |sigma + dsigma*step| and rou clamped to +-0.97 (:62-65).
//
// Per iteration: k_legacy_grad (one thread per node m < M-1, n < N-1: the
// K-point node rule and the four K x K edge rules, written to dnode/dedge in
// the reference's M x N x 2 x 2 / M x N x 2 x 5 x 2 layout), k_legacy_update
// (one thread per node and layer: sums, step, clamps, exact running maxima
// via atomicMax on the bit patterns of |x|), k_legacy_ctl (trace, stop rule).
// No host round trip inside the loop.  Plain fp64 with contraction off in the
// order of the MATLAB expressions, so the device matches the C restatement
// (oracle/gqmap_legacy_oracle.c) bit for bit.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstring>
#include <vector>

#include "gqmap_internal.h"

#pragma clang fp contract(off)

namespace gq {
namespace {

constexpr int LG_KMAX = GQMAP_KMAX;

struct LgParams {
    const double *flow;
    double *mu, *sigma, *rou, *dnode, *dedge;
    unsigned long long *maxbits;  // [its][3]
    int *ctl;                     // it, stop, done
    double *trace;
    int M, N, K, its, min_its;
    double var, gama, dta, step0, step_decay, corr, tor;
    double X[LG_KMAX], W[LG_KMAX];
};

__device__ __forceinline__ size_t i3(int M, int N, int m, int n, int l) { return m + (size_t)M * (n + (size_t)N * l); }
__device__ __forceinline__ size_t i4(int M, int N, int m, int n, int a, int b)
{
    return m + (size_t)M * (n + (size_t)N * (a + 2 * (size_t)b));
}
__device__ __forceinline__ size_t i5(int M, int N, int m, int n, int j, int q, int l)
{
    return m + (size_t)M * (n + (size_t)N * (j + 2 * (q + 5 * (size_t)l)));
}

// GAMA1 / VAR1: gama == 1 / var == 1, where x / 1 == x exactly (no division)
template <bool GAMA1, bool VAR1>
__global__ void k_legacy_grad(LgParams P)
{
    if (P.ctl[1]) return;
    const int M = P.M, N = P.N, K = P.K;
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= (int64_t)(M - 1) * (N - 1)) return;
    const int m = (int)(t % (M - 1)), n = (int)(t / (M - 1));
    const double sq2 = sqrt(2.0), PI = 3.14159265358979323846;
    for (int l = 0; l < 2; ++l) {  // (:20-26)
        const double o = P.sigma[i3(M, N, m, n, l)], u = P.mu[i3(M, N, m, n, l)], f = P.flow[i3(M, N, m, n, l)];
        double du = 0, dsum = 0;
        for (int k = 0; k < K; ++k) {
            const double x = sq2 * o * P.X[k] + u;
            const double dval = VAR1 ? P.W[k] * (f - x) : P.W[k] * (f - x) / P.var;
            du += dval;
            dsum += dval * P.X[k];
        }
        P.dnode[i4(M, N, m, n, 0, l)] = du / sqrt(PI);
        P.dnode[i4(M, N, m, n, 1, l)] = dsum * sqrt(2.0 / PI);
    }
    for (int j = 0; j < 2; ++j) {  // (:28-54)
        const int m2 = m + (j == 0), n2 = n + (j == 1);
        for (int l = 0; l < 2; ++l) {
            const double p = P.rou[i4(M, N, m, n, j, l)];
            const double o1 = P.sigma[i3(M, N, m, n, l)], o2 = P.sigma[i3(M, N, m2, n2, l)];
            const double u1 = P.mu[i3(M, N, m, n, l)], u2 = P.mu[i3(M, N, m2, n2, l)];
            const double q = sqrt(1 + p), r = sqrt(1 - p);
            const double s = (q + r) / 2, tt = (q - r) / 2;
            const double ds = (1 / q - 1 / r) / 4, dt = (1 / q + 1 / r) / 4;
            double s1 = 0, s2 = 0, so1 = 0, so2 = 0, sp = 0;
            for (int c = 0; c < K; ++c) {  // sum(sum(A)): column sums first
                double c1 = 0, c2 = 0, co1 = 0, co2 = 0, cp = 0;
                const double xi = P.X[c];
                for (int rr = 0; rr < K; ++rr) {
                    const double xj = P.X[rr], ww = P.W[c] * P.W[rr];
                    const double ZI = s * xi + tt * xj, ZJ = tt * xi + s * xj;
                    const double x1 = sq2 * o1 * ZI + u1, x2 = sq2 * o2 * ZJ + u2;
                    double diff = x2 - x1;
                    if (fabs(diff) > P.dta) diff = 0;  // (:44)
                    const double df1 = GAMA1 ? ww * diff : ww * diff / P.gama, df2 = -df1;
                    c1 += df1;
                    c2 += df2;
                    co1 += df1 * ZI;
                    co2 += df2 * ZJ;
                    cp += o1 * df1 * (ds * xi + dt * xj) + o2 * df2 * (dt * xi + ds * xj);
                }
                s1 += c1; s2 += c2; so1 += co1; so2 += co2; sp += cp;
            }
            P.dedge[i5(M, N, m, n, j, 0, l)] = 1 / PI * s1;
            P.dedge[i5(M, N, m, n, j, 1, l)] = 1 / PI * s2;
            P.dedge[i5(M, N, m, n, j, 2, l)] = 1 / PI * sq2 * so1;
            P.dedge[i5(M, N, m, n, j, 3, l)] = 1 / PI * sq2 * so2;
            P.dedge[i5(M, N, m, n, j, 4, l)] = 1 / PI * sq2 * sp;
        }
    }
}

// |v| as its bit pattern: for |v| >= 0 (and NaN above +inf) the unsigned
// order of the bits is the order of the values, so max is exact in any order
__device__ __forceinline__ unsigned long long abits(double v)
{
    return (unsigned long long)__double_as_longlong(fabs(v));
}

// Block maximum of three bit patterns, then one atomicMax per slot and block
// (one atomic per thread on three addresses serialised in L2: 240 us/launch).
__device__ void block_amax3(unsigned long long *slot, unsigned long long a, unsigned long long b,
                            unsigned long long c)
{
    __shared__ unsigned long long red[3][4];
    for (int o = 32; o > 0; o >>= 1) {
        a = max(a, __shfl_xor(a, o));
        b = max(b, __shfl_xor(b, o));
        c = max(c, __shfl_xor(c, o));
    }
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    if (lane == 0) { red[0][wave] = a; red[1][wave] = b; red[2][wave] = c; }
    __syncthreads();
    if (threadIdx.x < 3) {
        const int q = threadIdx.x;
        const unsigned long long v = max(max(red[q][0], red[q][1]), max(red[q][2], red[q][3]));
        if (v) atomicMax(slot + q, v);
    }
}

__global__ void k_legacy_update(LgParams P)
{
    if (P.ctl[1]) return;
    const int M = P.M, N = P.N;
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int it = P.ctl[0];
    unsigned long long *slot = P.maxbits + 3 * (size_t)(it - 1);
    // Threads past the last node contribute zeros: every thread reaches the
    // single block_amax3 call below (its barrier is never on a divergent path).
    double a = 0, b = 0, mp = 0;
    if (t < (int64_t)M * N * 2) {
        const int m = (int)(t % M), n = (int)((t / M) % N), l = (int)(t / ((int64_t)M * N));
        const double *de = P.dedge;
        // (:58-59) dmu = dnode + sum_j dedge(:,:,j,1) + (dedge(m+1,n,1,2) + dedge(m,n+1,2,2))
        a = P.dnode[i4(M, N, m, n, 0, l)] + (de[i5(M, N, m, n, 0, 0, l)] + de[i5(M, N, m, n, 1, 0, l)]);
        b = P.dnode[i4(M, N, m, n, 1, l)] + (de[i5(M, N, m, n, 0, 2, l)] + de[i5(M, N, m, n, 1, 2, l)]);
        const double nu = m + 1 < M ? de[i5(M, N, m + 1, n, 0, 1, l)] : 0.0;
        const double nl = n + 1 < N ? de[i5(M, N, m, n + 1, 1, 1, l)] : 0.0;
        const double su = m + 1 < M ? de[i5(M, N, m + 1, n, 0, 3, l)] : 0.0;
        const double sl = n + 1 < N ? de[i5(M, N, m, n + 1, 1, 3, l)] : 0.0;
        a = a + (nu + nl);
        b = b + (su + sl);
        const double step = P.step0 / (1 + it / P.step_decay);  // (:62)
        const size_t q = i3(M, N, m, n, l);
        P.mu[q] = P.mu[q] + a * step;               // (:63)
        P.sigma[q] = fabs(P.sigma[q] + b * step);   // (:64)
        for (int j = 0; j < 2; ++j) {               // (:65)
            const double d = de[i5(M, N, m, n, j, 4, l)];
            mp = fmax(mp, fabs(d));
            const size_t r = i4(M, N, m, n, j, l);
            P.rou[r] = fmax(fmin(P.rou[r] + d * step, P.corr), -P.corr);
        }
    }
    block_amax3(slot, abits(a), abits(b), abits(mp));
}

// sigma = rand(M,N,2) + 2 (:10) from the library RNG stream 3: the host
// formula, evaluated on the device
__global__ void k_legacy_sigma0(double *sigma, int64_t n, uint64_t base)
{
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) sigma[i] = u01(base, (uint64_t)i) + 2;
}

__global__ void k_legacy_ctl(LgParams P)
{
    if (P.ctl[1]) return;
    const int it = P.ctl[0];
    const unsigned long long *slot = P.maxbits + 3 * (size_t)(it - 1);
    double mx[3];
    for (int q = 0; q < 3; ++q) {
        mx[q] = __longlong_as_double((long long)slot[q]);
        P.trace[3 * (it - 1) + q] = mx[q];
    }
    P.ctl[0] = it + 1;
    P.ctl[2] = it;
    if (it + 1 > P.its || (it + 1 > P.min_its && mx[0] < P.tor)) P.ctl[1] = 1;  // (:70)
}

// One device arena per host thread and device, kept across calls: the nine
// buffers (~300 B per pixel) of gqmap_cpu_run are carved from it, so a
// repeated call pays no hipMalloc/hipFree (they dominated a 50-iteration
// call's wall clock).  gqmap_cpu_release() frees the calling thread's arenas.
struct Arena {
    void *p = nullptr;
    size_t cap = 0;
    hipError_t release()
    {
        void *q = p;
        p = nullptr;  // cleared before the result is checked: never a dangling pointer
        cap = 0;
        return q ? hipFree(q) : hipSuccess;
    }
    ~Arena() { (void)release(); }
};
constexpr int kArenaDev = 64;
thread_local Arena g_arenas[kArenaDev];

}  // namespace
}  // namespace gq

using namespace gq;

extern "C" {

void gqmap_cpu_options_default(gqmap_cpu_options *o)
{
    std::memset(o, 0, sizeof(*o));
    o->its = 50;
    o->K = 9;
    o->var = 1.0;
    o->gama = 1.0;
    o->dta = INFINITY;
    o->step0 = 0.1;          // step = 0.1/(1+it/1000) (:62)
    o->step_decay = 1000.0;
    o->corr_tor = 0.97;      // (:65)
    o->tor = 1e-3;           // (:12)
    o->min_its = 100;        // (:70)
}

gqmap_status gqmap_cpu_release(void)
{
    clear_error();
    int cur = -1;
    (void)hipGetDevice(&cur);
    hipError_t first = hipSuccess;
    for (int d = 0; d < kArenaDev; ++d) {
        if (!g_arenas[d].p) continue;
        if (hipSetDevice(d) != hipSuccess) continue;
        const hipError_t e = g_arenas[d].release();
        if (first == hipSuccess) first = e;
    }
    if (cur >= 0) (void)hipSetDevice(cur);
    GQ_HIP(first);
    return GQMAP_OK;
}

gqmap_status gqmap_cpu_run(const gqmap_cpu_options *o, const double *flow, int M, int N, const double *sigma0,
                           uint64_t seed, double *mu, double *sigma, double *rou, double *trace, int *its_done,
                           int device)
{
    clear_error();
    GQ_CHECK(o && flow && mu && sigma && rou, GQMAP_ERR_INVALID_ARG, "gqmap_cpu_run: null argument");
    GQ_CHECK(M >= 2 && N >= 2, GQMAP_ERR_INVALID_ARG, "gqmap_cpu_run: flow %dx%d too small", M, N);
    GQ_CHECK(o->K >= 1 && o->K <= GQMAP_KMAX, GQMAP_ERR_INVALID_ARG, "K=%d outside [1,%d]", o->K, GQMAP_KMAX);
    GQ_CHECK(o->its >= 1, GQMAP_ERR_INVALID_ARG, "its=%d", o->its);
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
        set_error("no HIP device available");
        return GQMAP_ERR_NO_DEVICE;
    }
    GQ_CHECK(device >= 0 && device < ndev, GQMAP_ERR_INVALID_ARG, "device %d of %d", device, ndev);
    DeviceGuard dg(device);
    LgParams P{};
    P.M = M; P.N = N; P.K = o->K; P.its = o->its; P.min_its = o->min_its;
    P.var = o->var; P.gama = o->gama; P.dta = o->dta; P.step0 = o->step0; P.step_decay = o->step_decay;
    P.corr = o->corr_tor; P.tor = o->tor;
    if (gauss_hermite(o->K, P.X, P.W) != 0) {
        set_error("Gauss-Hermite did not converge for K=%d", o->K);
        return GQMAP_ERR_INVALID_ARG;
    }
    const size_t MN = (size_t)M * N;
    // mu = flow (:9); sigma = rand(M,N,2) + 2 (:10, library RNG stream 3,
    // drawn on the device) unless given; rou = 0 (:11)
    // One device arena per host thread and device, kept across calls: the
    // nine buffers (~300 B per pixel) are carved from it, so a repeated call
    // pays no hipMalloc/hipFree (they dominated a 50-iteration call's wall clock).
    struct Buf { void *p = nullptr; };
    Buf bflow, bmu, bsg, brou, bdn, bde, bmax, bctl, btr;
    GQ_CHECK(device < kArenaDev, GQMAP_ERR_INVALID_ARG, "device %d >= %d", device, kArenaDev);
    const size_t sizes[9] = {sizeof(double) * 2 * MN, sizeof(double) * 2 * MN, sizeof(double) * 2 * MN,
                             sizeof(double) * 4 * MN, sizeof(double) * 4 * MN, sizeof(double) * 20 * MN,
                             sizeof(unsigned long long) * 3 * (size_t)o->its, sizeof(int) * 4,
                             sizeof(double) * 3 * (size_t)o->its};
    Buf *bufs[9] = {&bflow, &bmu, &bsg, &brou, &bdn, &bde, &bmax, &bctl, &btr};
    size_t need = 0;
    for (size_t sz : sizes) need += (sz + 255) & ~(size_t)255;
    Arena &A = g_arenas[device];
    // Regrow when too small, shrink when a call needs under a quarter of it
    // (a large call does not pin its footprint for the thread's lifetime).
    if (A.cap < need || need < A.cap / 4) {
        GQ_HIP(A.release());
        const size_t cap = need + need / 8;  // headroom: a longer run reuses it
        GQ_HIP(hipMalloc(&A.p, cap));
        A.cap = cap;
    }
    size_t off = 0;
    for (int i = 0; i < 9; ++i) {
        bufs[i]->p = (char *)A.p + off;
        off += (sizes[i] + 255) & ~(size_t)255;
    }
    GQ_HIP(hipMemcpy(bflow.p, flow, sizeof(double) * 2 * MN, hipMemcpyHostToDevice));
    GQ_HIP(hipMemcpy(bmu.p, bflow.p, sizeof(double) * 2 * MN, hipMemcpyDeviceToDevice));
    if (sigma0)
        GQ_HIP(hipMemcpy(bsg.p, sigma0, sizeof(double) * 2 * MN, hipMemcpyHostToDevice));
    else
        k_legacy_sigma0<<<(int)((2 * MN + 255) / 256), 256>>>((double *)bsg.p, (int64_t)(2 * MN), stream_base(seed, 3));
    GQ_HIP(hipMemset(brou.p, 0, sizeof(double) * 4 * MN));
    GQ_HIP(hipMemset(bdn.p, 0, sizeof(double) * 4 * MN));   // dnode = zeros (:14): last row/col stay 0
    GQ_HIP(hipMemset(bde.p, 0, sizeof(double) * 20 * MN));  // dedge = zeros (:15)
    GQ_HIP(hipMemset(bmax.p, 0, sizeof(unsigned long long) * 3 * (size_t)o->its));
    const int ctl0[4] = {1, 0, 0, 0};
    GQ_HIP(hipMemcpy(bctl.p, ctl0, sizeof(ctl0), hipMemcpyHostToDevice));
    P.flow = (const double *)bflow.p; P.mu = (double *)bmu.p; P.sigma = (double *)bsg.p; P.rou = (double *)brou.p;
    P.dnode = (double *)bdn.p; P.dedge = (double *)bde.p; P.maxbits = (unsigned long long *)bmax.p;
    P.ctl = (int *)bctl.p; P.trace = (double *)btr.p;
    const int g1 = (int)(((int64_t)(M - 1) * (N - 1) + 255) / 256), g2 = (int)((2 * (int64_t)MN + 255) / 256);
    auto grad = P.gama == 1.0 ? (P.var == 1.0 ? k_legacy_grad<true, true> : k_legacy_grad<true, false>)
                              : (P.var == 1.0 ? k_legacy_grad<false, true> : k_legacy_grad<false, false>);
    for (int it = 0; it < o->its; ++it) {
        grad<<<g1, 256>>>(P);
        k_legacy_update<<<g2, 256>>>(P);
        k_legacy_ctl<<<1, 1>>>(P);
    }
    GQ_HIP(hipGetLastError());
    GQ_HIP(hipDeviceSynchronize());
    int ctl[4];
    GQ_HIP(hipMemcpy(ctl, bctl.p, sizeof(ctl), hipMemcpyDeviceToHost));
    GQ_HIP(hipMemcpy(mu, bmu.p, sizeof(double) * 2 * MN, hipMemcpyDeviceToHost));
    GQ_HIP(hipMemcpy(sigma, bsg.p, sizeof(double) * 2 * MN, hipMemcpyDeviceToHost));
    GQ_HIP(hipMemcpy(rou, brou.p, sizeof(double) * 4 * MN, hipMemcpyDeviceToHost));
    if (trace) GQ_HIP(hipMemcpy(trace, btr.p, sizeof(double) * 3 * (size_t)ctl[2], hipMemcpyDeviceToHost));
    if (its_done) *its_done = ctl[2];
    return GQMAP_OK;
}

}  // extern "C"
