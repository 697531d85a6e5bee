// gqmap_legacy.hip -- device drop-in for legacy/gqmap_cpu.m, the legacy
// flow-denoising QGMAP ([mu,sigma,rou] = gqmap_cpu(options, flow)): a
// Gaussian observation of a given flow field (node, :20-26), truncated
// quadratic pairwise terms (edges, :28-54), the reference's own neighbour
// shift in the gradient sum (:58-60), plain gradient ascent with
// sigma = |sigma + dsigma*step| and rou clamped to +-0.97 (:62-65).
//
// Per iteration: k_legacy_grad (one thread per node m < M-1, n < N-1, edge
// and layer: one K x K edge rule, plus the K-point node rule on the j = 0
// threads, written to dnode/dedge in the reference's M x N x 2 x 2 /
// M x N x 2 x 5 x 2 layout), k_legacy_update (one thread per node and layer:
// sums, step, clamps, per-workgroup maxima on the bit patterns of |x|),
// k_legacy_ctl (their maxima -> trace, stop rule).
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
    unsigned long long *blkmax;   // [update workgroups][3]: |dmu|, |dsigma|, |drou| maxima as bits
    int *ctl;                     // it, stop, done
    double *trace;
    int M, N, K, its, min_its, nblk;
    double var, gama, dta, step0, step_decay, corr, tor;
    double X[LG_KMAX], W[LG_KMAX];
    double WW[LG_KMAX * LG_KMAX];  // W[c] * W[r] at r + K*c (WIWJ, :5-6), the host's product
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

// One thread per node m < M-1, n < N-1, edge j and layer l ((j, l) slowest:
// a wave stays on one edge of one layer): the edge rule (j, l) of the node,
// and on the j = 0 threads the node rule of layer l too (9 of ~170 points).
// Every expression keeps the reference's operand order; what is hoisted is a
// whole subexpression of it, computed once with the same operands:
//   s*XI, t*XI, ds*XI, dt*XI per column c and t*XJ, s*XJ, dt*XJ, ds*XJ per
//   row r (when K is a template constant: held in registers), sq2*o1 and
//   sq2*o2, WIWJ from the host table.
// c2 (the sum of df2 = -df1) is 0 - c1 exactly: both start at +0, IEEE
// addition is symmetric under negation, and an exact-zero sum is +0 in both
// chains -- so column and total sums of df2 are not formed (s2 = 0 - s1).
// KT: K as a template constant (0: P.K at run time); GAMA1 / VAR1: gama == 1
// / var == 1, where x / 1 == x exactly; DTA_INF: dta == inf, where
// fabs(diff) > dta is false for every diff (NaN included).
template <int KT, bool GAMA1, bool VAR1, bool DTA_INF>
__global__ __launch_bounds__(256) void k_legacy_grad(LgParams P)
{
    if (P.ctl[1]) return;
    const int M = P.M, N = P.N, K = KT ? KT : P.K;
    constexpr int UNR = KT ? KT : 1;  // full unroll for a constant K
    const int64_t MN1 = (int64_t)(M - 1) * (N - 1);
    int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= 4 * MN1) return;
    const int jl = (int)(t / MN1), j = jl & 1, l = jl >> 1;
    t -= jl * MN1;
    const int m = (int)(t % (M - 1)), n = (int)(t / (M - 1));
    const double sq2 = sqrt(2.0), PI = 3.14159265358979323846;
    const double o1 = P.sigma[i3(M, N, m, n, l)], u1 = P.mu[i3(M, N, m, n, l)];
    const double so1 = sq2 * o1;
    if (j == 0) {  // (:20-26)
        const double f = P.flow[i3(M, N, m, n, l)];
        double du = 0, dsum = 0;
#pragma unroll UNR
        for (int k = 0; k < K; ++k) {
            const double x = so1 * P.X[k] + u1;
            const double dval = VAR1 ? P.W[k] * (f - x) : P.W[k] * (f - x) / P.var;
            du += dval;
            dsum += dval * P.X[k];
        }
        P.dnode[i4(M, N, m, n, 0, l)] = du / sqrt(PI);
        P.dnode[i4(M, N, m, n, 1, l)] = dsum * sqrt(2.0 / PI);
    }
    {  // (:28-54)
        const int m2 = m + (j == 0), n2 = n + (j == 1);
        const double p = P.rou[i4(M, N, m, n, j, l)];
        const double o2 = P.sigma[i3(M, N, m2, n2, l)], u2 = P.mu[i3(M, N, m2, n2, l)];
        const double so2 = sq2 * o2;
        const double q = sqrt(1 + p), r = sqrt(1 - p);
        const double s = (q + r) / 2, tt = (q - r) / 2;
        const double ds = (1 / q - 1 / r) / 4, dt = (1 / q + 1 / r) / 4;
        double txj[UNR], sxj[UNR], dtxj[UNR], dsxj[UNR];
        if (KT) {
#pragma unroll UNR
            for (int rr = 0; rr < UNR; ++rr) {
                txj[rr] = tt * P.X[rr];
                sxj[rr] = s * P.X[rr];
                dtxj[rr] = dt * P.X[rr];
                dsxj[rr] = ds * P.X[rr];
            }
        }
        double s1 = 0, so1s = 0, so2s = 0, sp = 0;
#pragma unroll UNR
        for (int c = 0; c < K; ++c) {  // sum(sum(A)): column sums first
            const double xi = P.X[c];
            const double sxi = s * xi, txi = tt * xi, dsxi = ds * xi, dtxi = dt * xi;
            double c1 = 0, co1 = 0, co2 = 0, cp = 0;
#pragma unroll UNR
            for (int rr = 0; rr < K; ++rr) {
                const double xj = P.X[rr];
                const double tx = KT ? txj[rr] : tt * xj, sx = KT ? sxj[rr] : s * xj;
                const double dtx = KT ? dtxj[rr] : dt * xj, dsx = KT ? dsxj[rr] : ds * xj;
                const double ZI = sxi + tx, ZJ = txi + sx;
                const double x1 = so1 * ZI + u1, x2 = so2 * ZJ + u2;
                double diff = x2 - x1;
                if (!DTA_INF && fabs(diff) > P.dta) diff = 0;  // (:44)
                const double ww = P.WW[rr + K * c];
                const double df1 = GAMA1 ? ww * diff : ww * diff / P.gama, df2 = -df1;
                c1 += df1;
                co1 += df1 * ZI;
                co2 += df2 * ZJ;
                cp += o1 * df1 * (dsxi + dtx) + o2 * df2 * (dtxi + dsx);
            }
            s1 += c1; so1s += co1; so2s += co2; sp += cp;
        }
        const double s2 = 0.0 - s1;
        P.dedge[i5(M, N, m, n, j, 0, l)] = 1 / PI * s1;
        P.dedge[i5(M, N, m, n, j, 1, l)] = 1 / PI * s2;
        P.dedge[i5(M, N, m, n, j, 2, l)] = 1 / PI * sq2 * so1s;
        P.dedge[i5(M, N, m, n, j, 3, l)] = 1 / PI * sq2 * so2s;
        P.dedge[i5(M, N, m, n, j, 4, l)] = 1 / PI * sq2 * sp;
    }
}

// |v| as its bit pattern: for |v| >= 0 (and NaN above +inf) the unsigned
// order of the bits is the order of the values, so max is exact in any order
__device__ __forceinline__ unsigned long long abits(double v)
{
    return (unsigned long long)__double_as_longlong(fabs(v));
}

// Maximum over the block of three bit patterns (thread 0 holds the result).
__device__ void block_max3(unsigned long long &a, unsigned long long &b, unsigned long long &c)
{
    __shared__ unsigned long long red[3][16];
    for (int o = 32; o > 0; o >>= 1) {
        a = max(a, __shfl_xor(a, o));
        b = max(b, __shfl_xor(b, o));
        c = max(c, __shfl_xor(c, o));
    }
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, nw = (int)(blockDim.x + 63) >> 6;
    if (lane == 0) { red[0][wave] = a; red[1][wave] = b; red[2][wave] = c; }
    __syncthreads();
    if (threadIdx.x == 0)
        for (int w = 1; w < nw; ++w) {
            a = max(a, red[0][w]);
            b = max(b, red[1][w]);
            c = max(c, red[2][w]);
        }
}

// One thread per node and layer: sums, step, clamps; the workgroup's maxima
// of |dmu|, |dsigma|, |drou| go to its own blkmax row (plain stores: one
// atomicMax per workgroup on three shared addresses serialises in L2, and a
// last-workgroup reduction needs a device-scope release per workgroup, an L2
// writeback each -- 70 us per launch) and k_legacy_ctl reduces the rows.
__global__ __launch_bounds__(256) void k_legacy_update(LgParams P)
{
    if (P.ctl[1]) return;
    const int M = P.M, N = P.N;
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int it = P.ctl[0];
    // Threads past the last node contribute zeros: every thread reaches the
    // single block_max3 call below (its barrier is never on a divergent path).
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
    unsigned long long ba = abits(a), bb = abits(b), bm = abits(mp);
    block_max3(ba, bb, bm);
    if (threadIdx.x == 0) {
        unsigned long long *row = P.blkmax + 3 * (size_t)blockIdx.x;
        row[0] = ba;
        row[1] = bb;
        row[2] = bm;
    }
}

// sigma = rand(M,N,2) + 2 (:10) from the library RNG stream 3: the host
// formula, evaluated on the device
__global__ void k_legacy_sigma0(double *sigma, int64_t n, uint64_t base)
{
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) sigma[i] = u01(base, (uint64_t)i) + 2;
}

// One workgroup: the maxima over the update's blkmax rows -> trace, then
// the iteration counter and the stop rule.
__global__ __launch_bounds__(1024) void k_legacy_ctl(LgParams P)
{
    if (P.ctl[1]) return;
    unsigned long long a = 0, b = 0, c = 0;
    for (int i = threadIdx.x; i < P.nblk; i += blockDim.x) {
        const unsigned long long *row = P.blkmax + 3 * (size_t)i;
        a = max(a, row[0]);
        b = max(b, row[1]);
        c = max(c, row[2]);
    }
    block_max3(a, b, c);
    if (threadIdx.x != 0) return;
    const int it = P.ctl[0];
    const unsigned long long bits[3] = {a, b, c};
    double mx[3];
    for (int q = 0; q < 3; ++q) {
        mx[q] = __longlong_as_double((long long)bits[q]);
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

}  // extern "C"

namespace {

// Does p point into device memory of `device` (or managed memory)?  Memory
// of another GPU would be read through peer access, or fault.
bool on_device(const void *p, int device)
{
    hipPointerAttribute_t at{};
    if (hipPointerGetAttributes(&at, p) != hipSuccess) {
        (void)hipGetLastError();  // a plain host pointer: clear the sticky error
        return false;
    }
    if (at.type == hipMemoryTypeManaged) return true;
    return at.type == hipMemoryTypeDevice && at.device == device;
}

// Do the byte ranges [a, a + na) and [b, b + nb) overlap?
bool overlap(const void *a, size_t na, const void *b, size_t nb)
{
    const uintptr_t x = (uintptr_t)a, y = (uintptr_t)b;
    return na && nb && x < y + nb && y < x + na;
}

// gqmap_cpu_run (DEV = false: host arrays, copied in and out) and
// gqmap_cpu_run_device (DEV = true: flow / sigma0 / mu / sigma / rou / trace
// are device arrays; the iteration runs on mu / sigma / rou in place).
gqmap_status cpu_run(const gqmap_cpu_options *o, const double *flow, int M, int N, const double *sigma0, uint64_t seed,
                     double *mu, double *sigma, double *rou, double *trace, int *its_done, int device, bool DEV)
{
    const char *fn = DEV ? "gqmap_cpu_run_device" : "gqmap_cpu_run";
    GQ_CHECK(o && flow && mu && sigma && rou, GQMAP_ERR_INVALID_ARG, "%s: null argument", fn);
    GQ_CHECK(M >= 2 && N >= 2, GQMAP_ERR_INVALID_ARG, "%s: flow %dx%d too small", fn, M, N);
    GQ_CHECK(o->K >= 1 && o->K <= GQMAP_KMAX, GQMAP_ERR_INVALID_ARG, "K=%d outside [1,%d]", o->K, GQMAP_KMAX);
    GQ_CHECK(o->its >= 1, GQMAP_ERR_INVALID_ARG, "its=%d", o->its);
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
        set_error("no HIP device available");
        return GQMAP_ERR_NO_DEVICE;
    }
    GQ_CHECK(device >= 0 && device < ndev, GQMAP_ERR_INVALID_ARG, "device %d of %d", device, ndev);
    GQ_CHECK(device < kArenaDev, GQMAP_ERR_INVALID_ARG, "device %d >= %d", device, kArenaDev);
    DeviceGuard dg(device);
    const size_t MN = (size_t)M * N;
    if (DEV) {
        GQ_CHECK(on_device(flow, device) && on_device(mu, device) && on_device(sigma, device) &&
                     on_device(rou, device) && (!sigma0 || on_device(sigma0, device)) &&
                     (!trace || on_device(trace, device)),
                 GQMAP_ERR_INVALID_ARG, "%s: every array must be device memory of device %d", fn, device);
        // the outputs (written in place during the run) must not overlap each
        // other or an input
        const size_t b2 = sizeof(double) * 2 * MN;
        const struct { const void *p; size_t n; } out[4] = {
            {mu, b2}, {sigma, b2}, {rou, 2 * b2}, {trace, trace ? sizeof(double) * 3 * (size_t)o->its : 0}};
        const struct { const void *p; size_t n; } in[2] = {{flow, b2}, {sigma0, sigma0 ? b2 : 0}};
        for (int i = 0; i < 4; ++i) {
            for (int j = i + 1; j < 4; ++j)
                GQ_CHECK(!overlap(out[i].p, out[i].n, out[j].p, out[j].n), GQMAP_ERR_INVALID_ARG,
                         "%s: output arrays %d and %d overlap (mu, sigma, rou, trace)", fn, i, j);
            for (int j = 0; j < 2; ++j)
                GQ_CHECK(!overlap(out[i].p, out[i].n, in[j].p, in[j].n), GQMAP_ERR_INVALID_ARG,
                         "%s: output array %d (mu, sigma, rou, trace) overlaps %s", fn, i, j ? "sigma0" : "flow");
        }
    }
    LgParams P{};
    P.M = M; P.N = N; P.K = o->K; P.its = o->its; P.min_its = o->min_its;
    P.var = o->var; P.gama = o->gama; P.dta = o->dta; P.step0 = o->step0; P.step_decay = o->step_decay;
    P.corr = o->corr_tor; P.tor = o->tor;
    if (gauss_hermite(o->K, P.X, P.W) != 0) {
        set_error("Gauss-Hermite did not converge for K=%d", o->K);
        return GQMAP_ERR_INVALID_ARG;
    }
    for (int c = 0; c < o->K; ++c)
        for (int r = 0; r < o->K; ++r) P.WW[r + o->K * c] = P.W[c] * P.W[r];  // WIWJ (:5-6)
    const int g1 = (int)((4 * (int64_t)(M - 1) * (N - 1) + 255) / 256), nblk = (int)((2 * (int64_t)MN + 255) / 256);
    P.nblk = nblk;
    // One device arena per host thread and device, kept across calls: the
    // buffers (~300 B per pixel with host arrays, ~200 with device arrays)
    // are carved from it, so a repeated call pays no hipMalloc/hipFree (they
    // dominated a 50-iteration call's wall clock).
    struct Buf { void *p = nullptr; };
    Buf bflow, bmu, bsg, brou, bdn, bde, bmax, bctl, btr;
    const size_t io = DEV ? 0 : 1, tr = DEV && trace ? 0 : 1;
    const size_t sizes[9] = {io * sizeof(double) * 2 * MN, io * sizeof(double) * 2 * MN, io * sizeof(double) * 2 * MN,
                             io * sizeof(double) * 4 * MN, sizeof(double) * 4 * MN, sizeof(double) * 20 * MN,
                             sizeof(unsigned long long) * 3 * (size_t)nblk, sizeof(int) * 4,
                             tr * sizeof(double) * 3 * (size_t)o->its};
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
    if (DEV) {
        bflow.p = const_cast<double *>(flow);
        bmu.p = mu;
        bsg.p = sigma;
        brou.p = rou;
        if (trace) btr.p = trace;
    } else {
        GQ_HIP(hipMemcpy(bflow.p, flow, sizeof(double) * 2 * MN, hipMemcpyHostToDevice));
    }
    // mu = flow (:9); sigma = rand(M,N,2) + 2 (:10, library RNG stream 3,
    // drawn on the device) unless given; rou = 0 (:11)
    GQ_HIP(hipMemcpy(bmu.p, bflow.p, sizeof(double) * 2 * MN, hipMemcpyDeviceToDevice));
    if (sigma0)
        GQ_HIP(hipMemcpy(bsg.p, sigma0, sizeof(double) * 2 * MN, DEV ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice));
    else
        k_legacy_sigma0<<<(int)((2 * MN + 255) / 256), 256>>>((double *)bsg.p, (int64_t)(2 * MN), stream_base(seed, 3));
    GQ_HIP(hipMemset(brou.p, 0, sizeof(double) * 4 * MN));
    GQ_HIP(hipMemset(bdn.p, 0, sizeof(double) * 4 * MN));   // dnode = zeros (:14): last row/col stay 0
    GQ_HIP(hipMemset(bde.p, 0, sizeof(double) * 20 * MN));  // dedge = zeros (:15)
    const int ctl0[4] = {1, 0, 0, 0};
    GQ_HIP(hipMemcpy(bctl.p, ctl0, sizeof(ctl0), hipMemcpyHostToDevice));
    P.flow = (const double *)bflow.p; P.mu = (double *)bmu.p; P.sigma = (double *)bsg.p; P.rou = (double *)brou.p;
    P.dnode = (double *)bdn.p; P.dedge = (double *)bde.p; P.blkmax = (unsigned long long *)bmax.p;
    P.ctl = (int *)bctl.p; P.trace = (double *)btr.p;
    // the grad kernel's compile-time variants: K = 9 (the reference's) or any
    // K; gama / var == 1; dta == inf (the defaults)
    using Grad = void (*)(LgParams);
    static constexpr Grad kGrad[2][2][2][2] = {
        {{{k_legacy_grad<0, false, false, false>, k_legacy_grad<0, false, false, true>},
          {k_legacy_grad<0, false, true, false>, k_legacy_grad<0, false, true, true>}},
         {{k_legacy_grad<0, true, false, false>, k_legacy_grad<0, true, false, true>},
          {k_legacy_grad<0, true, true, false>, k_legacy_grad<0, true, true, true>}}},
        {{{k_legacy_grad<9, false, false, false>, k_legacy_grad<9, false, false, true>},
          {k_legacy_grad<9, false, true, false>, k_legacy_grad<9, false, true, true>}},
         {{k_legacy_grad<9, true, false, false>, k_legacy_grad<9, true, false, true>},
          {k_legacy_grad<9, true, true, false>, k_legacy_grad<9, true, true, true>}}}};
    const Grad grad = kGrad[P.K == 9][P.gama == 1.0][P.var == 1.0][P.dta == INFINITY];
    for (int it = 0; it < o->its; ++it) {
        grad<<<g1, 256>>>(P);
        k_legacy_update<<<nblk, 256>>>(P);
        k_legacy_ctl<<<1, 1024>>>(P);
    }
    GQ_HIP(hipGetLastError());
    GQ_HIP(hipDeviceSynchronize());
    int ctl[4];
    GQ_HIP(hipMemcpy(ctl, bctl.p, sizeof(ctl), hipMemcpyDeviceToHost));
    if (!DEV) {
        GQ_HIP(hipMemcpy(mu, bmu.p, sizeof(double) * 2 * MN, hipMemcpyDeviceToHost));
        GQ_HIP(hipMemcpy(sigma, bsg.p, sizeof(double) * 2 * MN, hipMemcpyDeviceToHost));
        GQ_HIP(hipMemcpy(rou, brou.p, sizeof(double) * 4 * MN, hipMemcpyDeviceToHost));
        if (trace)
            GQ_HIP(hipMemcpy(trace, btr.p, sizeof(double) * 3 * (size_t)ctl[2], hipMemcpyDeviceToHost));
    }
    if (its_done) *its_done = ctl[2];
    return GQMAP_OK;
}

}  // namespace

extern "C" {

gqmap_status gqmap_cpu_run(const gqmap_cpu_options *o, const double *flow, int M, int N, const double *sigma0,
                           uint64_t seed, double *mu, double *sigma, double *rou, double *trace, int *its_done,
                           int device)
{
    clear_error();
    return cpu_run(o, flow, M, N, sigma0, seed, mu, sigma, rou, trace, its_done, device, false);
}

gqmap_status gqmap_cpu_run_device(const gqmap_cpu_options *o, const double *flow, int M, int N,
                                  const double *sigma0, uint64_t seed, double *mu, double *sigma, double *rou,
                                  double *trace, int *its_done, int device)
{
    clear_error();
    return cpu_run(o, flow, M, N, sigma0, seed, mu, sigma, rou, trace, its_done, device, true);
}

}  // extern "C"
