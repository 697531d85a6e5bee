// Calibrates VALU issue cost on gfx950: cycles per wave-instruction per SIMD
// for f64/f32 FMA, f64 rsq, f64<->i32 cvt, with CHAINS independent chains per
// lane and W waves per SIMD (grid = 256 CUs * 4 SIMDs * W waves).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

template <int OP, int CHAINS, typename T>
__global__ __launch_bounds__(256) void k(T *out, int iters, T a, T b)
{
    T x[CHAINS];
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) x[c] = T(threadIdx.x + c) * T(1e-3);
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int c = 0; c < CHAINS; ++c) {
            if constexpr (OP == 0) x[c] = fma(x[c], a, b);                    // fma
            else if constexpr (OP == 1) x[c] = __builtin_amdgcn_rsq(x[c] + b);  // rsq f64
            else if constexpr (OP == 2) x[c] = T((int)x[c]) + a;              // cvt round trip + add
            else if constexpr (OP == 3) x[c] = x[c] * a + b;                  // mul + add (no contract)
        }
    }
    T s = 0;
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) s += x[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int OP, int CHAINS, typename T>
void run(const char *name, int ops_per_chain_iter)
{
    int dev; hipGetDevice(&dev);
    hipDeviceProp_t p; hipGetDeviceProperties(&p, dev);
    const int cus = p.multiProcessorCount;
    T *out; hipMalloc(&out, sizeof(T) * cus * 4 * 8 * 64 * 4);
    const int iters = 4096;
    for (int w = 1; w <= 8; w *= 2) {
        const int blocks = cus * w;  // 256-thread blocks = 4 waves = 1 per SIMD
        hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
        k<OP, CHAINS, T><<<blocks, 256>>>(out, 16, T(0.999), T(1e-3));
        hipEventRecord(e0);
        k<OP, CHAINS, T><<<blocks, 256>>>(out, iters, T(0.999), T(1e-3));
        hipEventRecord(e1); hipEventSynchronize(e1);
        float ms; hipEventElapsedTime(&ms, e0, e1);
        const double winstr_per_simd = (double)w * iters * CHAINS * ops_per_chain_iter;  // per SIMD
        const double cyc = ms * 1e-3 * 2.4e9;  // at nominal 2.4 GHz
        printf("%-22s chains=%d waves/SIMD=%d : %.2f cycles per wave-instr per SIMD (%.3f ms)\n",
               name, CHAINS, w, cyc / winstr_per_simd, ms);
    }
    hipFree(out);
}

int main()
{
    run<0, 1, double>("f64 fma dep", 1);
    run<0, 8, double>("f64 fma", 1);
    run<3, 8, double>("f64 mul+add", 2);
    run<1, 8, double>("f64 add+rsq", 2);
    run<2, 8, double>("f64 cvt_i32+cvt_f64+add", 3);
    run<0, 1, float>("f32 fma dep", 1);
    run<0, 8, float>("f32 fma", 1);
    return 0;
}
