// Checks raw buffer b128 loads at 4-byte-aligned (not 16-byte-aligned)
// offsets against plain loads.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__global__ void k(const float *p, int n, int M2, const int *offs, float *out_buf, float *out_glb)
{
    const int t = threadIdx.x + blockIdx.x * blockDim.x;
    const int off = offs[t];
    __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void *)p, (short)0, n * 4, 0x00020000);
    for (int j = 0; j < 4; ++j) {
        unsigned v[4];
        for (int i = 0; i < 4; ++i) v[i] = __builtin_amdgcn_raw_buffer_load_b32(r, off * 4 + 4 * i, j * M2 * 4, 0);
        for (int i = 0; i < 4; ++i) {
            out_buf[t * 16 + j * 4 + i] = __builtin_bit_cast(float, v[i]);
            out_glb[t * 16 + j * 4 + i] = p[off + j * M2 + i];
        }
    }
}

int main()
{
    const int M2 = 390, n = 390 * 586, T = 256;
    std::vector<float> h(n);
    for (int i = 0; i < n; ++i) h[i] = (float)i;
    std::vector<int> offs(T);
    for (int t = 0; t < T; ++t) offs[t] = (t * 7919) % (n - 4 * M2 - 8);
    float *d, *ob, *og;
    int *dofs;
    hipMalloc(&d, n * 4); hipMalloc(&ob, T * 64); hipMalloc(&og, T * 64); hipMalloc(&dofs, T * 4);
    hipMemcpy(d, h.data(), n * 4, hipMemcpyHostToDevice);
    hipMemcpy(dofs, offs.data(), T * 4, hipMemcpyHostToDevice);
    k<<<1, T>>>(d, n, M2, dofs, ob, og);
    std::vector<float> b(T * 16), g(T * 16);
    hipMemcpy(b.data(), ob, T * 64, hipMemcpyDeviceToHost);
    hipMemcpy(g.data(), og, T * 64, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int i = 0; i < T * 16; ++i)
        if (b[i] != g[i]) {
            if (bad < 8) printf("t %d j %d i %d off %d: buffer %g global %g\n", i / 16, (i % 16) / 4, i % 4, offs[i / 16], b[i], g[i]);
            ++bad;
        }
    printf("mismatches: %d of %d\n", bad, T * 16);
    return 0;
}
