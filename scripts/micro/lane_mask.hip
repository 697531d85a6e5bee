// Does a wave64 with part of its lanes masked off cost less VALU time on
// gfx950 (SIMD-32: two passes of 32 lanes)?  Times f64 / f32 FMA chains with
// `active` lanes enabled (a contiguous low block, or every other lane), and
// v_pk_fma_f32 against two v_fma_f32.  Grid: 256 CUs x 4 SIMDs x W waves.
#include <hip/hip_runtime.h>
#include <cstdio>

template <typename T, int MODE>
__global__ __launch_bounds__(256) void k(T *out, int iters, T a, T b, int active)
{
    const int lane = threadIdx.x & 63;
    const bool on = MODE == 0 ? lane < active : (lane & 1) == 0;
    T x[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) x[c] = T(threadIdx.x + c) * T(1e-3);
    if (on) {
        for (int i = 0; i < iters; ++i) {
#pragma unroll
            for (int c = 0; c < 8; ++c) x[c] = fma(x[c], a, b);
        }
    }
    T s = 0;
#pragma unroll
    for (int c = 0; c < 8; ++c) s += x[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

typedef float f2 __attribute__((ext_vector_type(2)));
__global__ __launch_bounds__(256) void kpk(float *out, int iters, float a, float b)
{
    f2 x[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) x[c] = f2{float(threadIdx.x + c), float(c)} * 1e-3f;
    const f2 av = {a, a}, bv = {b, b};
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int c = 0; c < 8; ++c) x[c] = __builtin_elementwise_fma(x[c], av, bv);
    }
    float s = 0;
#pragma unroll
    for (int c = 0; c < 8; ++c) s += x[c].x + x[c].y;
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <typename F>
double time_ms(F launch)
{
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    launch(16);
    hipEventRecord(e0);
    launch(4096);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    return ms;
}

int main()
{
    int dev; hipGetDevice(&dev);
    hipDeviceProp_t p; hipGetDeviceProperties(&p, dev);
    const int cus = p.multiProcessorCount;
    const int W = 4;
    const int blocks = cus * W;
    void *out; hipMalloc(&out, sizeof(double) * blocks * 256);
    const double winstr = (double)W * 4096 * 8;  // wave-instructions per SIMD
    for (int active : {64, 48, 33, 32, 16, 1}) {
        double md = time_ms([&](int it) { k<double, 0><<<blocks, 256>>>((double *)out, it, 0.999, 1e-3, active); });
        double mf = time_ms([&](int it) { k<float, 0><<<blocks, 256>>>((float *)out, it, 0.999f, 1e-3f, active); });
        printf("active lanes %2d (low block): f64 fma %.2f cyc/instr, f32 fma %.2f cyc/instr\n", active,
               md * 1e-3 * 2.4e9 / winstr, mf * 1e-3 * 2.4e9 / winstr);
    }
    double md = time_ms([&](int it) { k<double, 1><<<blocks, 256>>>((double *)out, it, 0.999, 1e-3, 0); });
    double mf = time_ms([&](int it) { k<float, 1><<<blocks, 256>>>((float *)out, it, 0.999f, 1e-3f, 0); });
    printf("even lanes only: f64 fma %.2f cyc/instr, f32 fma %.2f cyc/instr\n", md * 1e-3 * 2.4e9 / winstr,
           mf * 1e-3 * 2.4e9 / winstr);
    double mp = time_ms([&](int it) { kpk<<<blocks, 256>>>((float *)out, it, 0.999f, 1e-3f); });
    printf("v_pk_fma_f32 (2 fma each): %.2f cyc/instr = %.2f cyc per f32 fma-pair\n", mp * 1e-3 * 2.4e9 / winstr,
           mp * 1e-3 * 2.4e9 / winstr);
    hipFree(out);
    return 0;
}
