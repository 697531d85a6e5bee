// FETCH_SIZE / WRITE_SIZE calibration for the access widths the QGMAP
// kernels use (MI355X_MICROARCH.md: "calibrate on a known byte count in
// your own access pattern"): coalesced 8-B and 4-B per-lane streaming reads
// of a 1 GiB buffer (past the 256 MiB Infinity Cache) and 8-B / 4-B stores.
#include <hip/hip_runtime.h>

#include <cstdio>

template <typename T>
__global__ void k_read(const T *__restrict__ a, size_t n, T *out)
{
    T s = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        s += a[i];
    if (s == T(12345)) out[0] = s;  // never true: keeps the loads
}

template <typename T>
__global__ void k_write(T *__restrict__ a, size_t n)
{
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        a[i] = T(i & 7);
}

int main()
{
    const size_t bytes = (size_t)1 << 30;
    void *buf, *out;
    if (hipMalloc(&buf, bytes) != hipSuccess || hipMalloc(&out, 64) != hipSuccess) return 1;
    (void)hipMemset(buf, 0, bytes);
    for (int r = 0; r < 3; ++r) {
        k_read<double><<<4096, 256>>>((const double *)buf, bytes / 8, (double *)out);
        k_read<float><<<4096, 256>>>((const float *)buf, bytes / 4, (float *)out);
        k_write<double><<<4096, 256>>>((double *)buf, bytes / 8);
        k_write<float><<<4096, 256>>>((float *)buf, bytes / 4);
    }
    if (hipDeviceSynchronize() != hipSuccess) return 2;
    printf("calibration kernels done: %zu bytes each\n", bytes);
    return 0;
}
