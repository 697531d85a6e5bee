// Internal helpers shared by the HIP translation units of libgqmap.so.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <vector>

#include "../../include/gqmap.h"

namespace gq {

void set_error(const char *fmt, ...);
void clear_error();

#define GQ_HIP(call)                                                                        \
    do {                                                                                    \
        hipError_t e_ = (call);                                                             \
        if (e_ != hipSuccess) {                                                             \
            gq::set_error("%s:%d %s failed: %s", __FILE__, __LINE__, #call,                \
                          hipGetErrorString(e_));                                           \
            return GQMAP_ERR_HIP;                                                           \
        }                                                                                   \
    } while (0)

#define GQ_CHECK(cond, code, ...)                                                           \
    do {                                                                                    \
        if (!(cond)) {                                                                      \
            gq::set_error(__VA_ARGS__);                                                     \
            return code;                                                                    \
        }                                                                                   \
    } while (0)

// SplitMix64 finaliser; counter-based U(0,1) used for the seeded initial state.
__host__ __device__ inline uint64_t mix64(uint64_t z)
{
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}
__host__ __device__ inline uint64_t stream_base(uint64_t seed, uint32_t stream)
{
    return mix64(seed + 0xD1B54A32D192ED03ULL * (uint64_t)(stream + 1));
}
__host__ __device__ inline double u01(uint64_t base, uint64_t idx)
{
    return (double)(mix64(base + (idx + 1) * 0x9E3779B97F4A7C15ULL) >> 11) * 0x1.0p-53;
}

// Device selection guard: restores the caller's device on scope exit.
struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(int dev)
    {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (dev >= 0) (void)hipSetDevice(dev);
    }
    ~DeviceGuard()
    {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
};

// Host fp64 getVV (gqmap_gpu_mixture.m:191-208), independent of the oracle.
void build_padded(const double *I2, int M, int N, double *VV);
// Gauss-Hermite by Newton iteration on the orthonormal Hermite recurrence.
int gauss_hermite(int K, double *x, double *w);

// ---- coarse-to-fine plumbing (legacy/optical_flow_ctf.m:21-35) -------------
// MATLAB imresize contributions(): Keys kernel widened by 1/scale when
// antialiasing a reduction, symmetric edge mirroring, all-zero tap columns
// removed.  w/idx: [out_len][P] row-major, idx 0-based; returns P.
int resize_contrib(int in_len, int out_len, double scale, int antialias, std::vector<double> &w,
                   std::vector<int> &idx);
// imresize output length: ceil(scale * len)
int resize_len(int len, double scale);

// device helpers (gqmap_pyramid.hip), all asynchronous on s unless noted
hipError_t pad_vv_device(const double *dI2, int M, int N, double *dVV, hipStream_t s);
// *exact = every value representable in float (synchronises s)
hipError_t f32_exact_device(const double *d, size_t n, int *d_flag, bool *exact, hipStream_t s);
hipError_t convert_device(const double *src, void *dst, size_t n, bool to_f32, hipStream_t s);

}  // namespace gq

// ---- engine context, internal API used by the coarse-to-fine driver -------
struct gqmap_ctx;
namespace gq {
// images already on the device (fp64 M x N each); d_scratch holds
// (Mo+2)*(No+2) doubles, d_flag one int
gqmap_status ctx_set_images_device(gqmap_ctx *c, const double *dI1, const double *dI2, int Mo, int No,
                                   double *d_scratch, int *d_flag);
// current muu / muv planes (fp64 or fp32 per *fp32); synchronises the stream
gqmap_status ctx_flow_device(gqmap_ctx *c, const void **muu, const void **muv, bool *fp32);
// run the context on a caller-owned stream
void ctx_adopt_stream(gqmap_ctx *c, hipStream_t s);
}  // namespace gq
