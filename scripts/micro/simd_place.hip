// Which SIMD does wave w of a workgroup land on?  Records HW_ID per wave for a
// k_iter-like launch (925 blocks x 256 threads, 3 resident per CU) and counts,
// per CU, how many wave-0s each SIMD hosts (k_iter gives wave 0 the halo edge
// jobs of its tile: 5 edge jobs against 4).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <map>
#include <vector>

__global__ void __launch_bounds__(256) k(unsigned *out, int spin)
{
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
        unsigned hw = __builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11));   // HW_REG_HW_ID
        unsigned xcc = __builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (15 << 11)); // HW_REG_XCC_ID
        out[8 * blockIdx.x + 2 * w] = hw;
        out[8 * blockIdx.x + 2 * w + 1] = xcc;
    }
    volatile double x = threadIdx.x;
    for (int i = 0; i < spin; ++i) x = x * 1.0000001 + 1e-9;
}

int main()
{
    const int nb = 925;
    unsigned *d;
    if (hipMalloc(&d, nb * 32) != hipSuccess) return 1;
    for (int rep = 0; rep < 2; ++rep) {
        k<<<nb, 256, 48 * 1024>>>(d, rep ? 200000 : 20000);
        std::vector<unsigned> h(8 * nb);
        if (hipMemcpy(h.data(), d, nb * 32, hipMemcpyDeviceToHost) != hipSuccess) return 1;
        // hist[w][s]: wave w of its block on SIMD s; per CU: wave-0 count per SIMD
        int hist[4][4] = {};
        std::map<unsigned, std::vector<int>> w0_per_cu;
        for (int b = 0; b < nb; ++b)
            for (int w = 0; w < 4; ++w) {
                const unsigned hw = h[8 * b + 2 * w], xcc = h[8 * b + 2 * w + 1] & 0xf;
                const unsigned simd = (hw >> 4) & 3, cu = (hw >> 8) & 0xf, sh = (hw >> 12) & 1, se = (hw >> 13) & 7;
                hist[w][simd]++;
                if (w == 0) {
                    const unsigned key = (xcc << 16) | (se << 8) | (sh << 4) | cu;
                    auto &v = w0_per_cu[key];
                    if (v.empty()) v.assign(4, 0);
                    v[simd]++;
                }
            }
        printf("spin %d: wave -> SIMD histogram (rows wave 0..3, cols SIMD 0..3)\n", rep ? 200000 : 20000);
        for (int w = 0; w < 4; ++w) printf("  wave %d: %4d %4d %4d %4d\n", w, hist[w][0], hist[w][1], hist[w][2], hist[w][3]);
        std::map<int, int> maxw0;  // max wave-0s on one SIMD of a CU -> number of CUs
        for (auto &kv : w0_per_cu) {
            int mx = 0;
            for (int s = 0; s < 4; ++s) mx = kv.second[s] > mx ? kv.second[s] : mx;
            maxw0[mx]++;
        }
        printf("  CUs by the max number of wave-0s on one of their SIMDs:");
        for (auto &kv : maxw0) printf(" %d:%d", kv.first, kv.second);
        printf(" (of %zu CUs)\n", w0_per_cu.size());
        int shown = 0;
        for (auto &kv : w0_per_cu)
            if (shown++ < 6)
                printf("  cu key %06x wave-0s per SIMD %d %d %d %d\n", kv.first, kv.second[0], kv.second[1],
                       kv.second[2], kv.second[3]);
    }
    return 0;
}
