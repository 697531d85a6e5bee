// Where do workgroups land?  Records XCC id and HW_ID (CU/SH/SE) per block for a
// k_iter-like launch (925 blocks x 256 threads, ~3 resident per CU).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <map>

__global__ void __launch_bounds__(256) k(unsigned *out, int spin)
{
    if (threadIdx.x == 0) {
        unsigned hw = __builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11));   // HW_REG_HW_ID
        unsigned xcc = __builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (15 << 11)); // HW_REG_XCC_ID
        out[2 * blockIdx.x] = hw;
        out[2 * blockIdx.x + 1] = xcc;
    }
    // keep the block busy so placement reflects co-residency
    volatile double x = threadIdx.x;
    for (int i = 0; i < spin; ++i) x = x * 1.0000001 + 1e-9;
}

int main()
{
    const int nb = 925;
    unsigned *d;
    hipMalloc(&d, nb * 8);
    k<<<nb, 256, 48 * 1024>>>(d, 200000);  // 48 KB LDS -> at most 3 blocks per CU
    std::vector<unsigned> h(2 * nb);
    hipMemcpy(h.data(), d, nb * 8, hipMemcpyDeviceToHost);
    std::map<unsigned, std::vector<int>> per_cu;
    for (int b = 0; b < nb; ++b) {
        unsigned hw = h[2 * b], xcc = h[2 * b + 1] & 0xf;
        unsigned cu = (hw >> 8) & 0xf, sh = (hw >> 12) & 1, se = (hw >> 13) & 0x7;
        unsigned key = (xcc << 16) | (se << 8) | (sh << 4) | cu;
        per_cu[key].push_back(b);
        if (b < 24) printf("block %3d -> xcc %u se %u sh %u cu %u\n", b, xcc, se, sh, cu);
    }
    int shown = 0;
    for (auto &kv : per_cu) {
        if (shown++ < 12) {
            printf("xcc %u se %u sh %u cu %2u:", kv.first >> 16, (kv.first >> 8) & 0xff, (kv.first >> 4) & 0xf, kv.first & 0xf);
            for (int b : kv.second) printf(" %d", b);
            printf("\n");
        }
    }
    printf("distinct CUs: %zu\n", per_cu.size());
    return 0;
}
