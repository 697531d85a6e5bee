// gqmap_host.cpp -- host-side helpers of libgqmap.so (no device code).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <string>

#include "gqmap_internal.h"

namespace gq {

static thread_local std::string g_err;

void set_error(const char *fmt, ...)
{
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    std::vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
}

void clear_error() { g_err.clear(); }

// getVV (gqmap_gpu_mixture.m:191-208): copy I2 into the interior of an
// (M+2)x(N+2) array, then extrapolate the first/last row of every column and
// afterwards the first/last column of every row with 3*f1 - 3*f2 + f3 -- the
// boundary rule of MATLAB interp2(...,'cubic').  Column-major throughout.
void build_padded(const double *I2, int M, int N, double *VV)
{
    const int M2 = M + 2, N2 = N + 2;
    std::fill(VV, VV + (size_t)M2 * N2, 0.0);
    for (int n = 0; n < N; ++n)
        std::memcpy(VV + (size_t)M2 * (n + 1) + 1, I2 + (size_t)M * n, sizeof(double) * M);
    for (int col = 0; col < N2; ++col) {
        double *c = VV + (size_t)M2 * col;
        c[0] = (3.0 * c[1] - 3.0 * c[2]) + c[3];
        c[M2 - 1] = (3.0 * c[M2 - 2] - 3.0 * c[M2 - 3]) + c[M2 - 4];
    }
    double *first = VV, *last = VV + (size_t)M2 * (N2 - 1);
    for (int r = 0; r < M2; ++r) {
        first[r] = (3.0 * first[r + M2] - 3.0 * first[r + 2 * M2]) + first[r + 3 * M2];
        last[r] = (3.0 * last[r - M2] - 3.0 * last[r - 2 * M2]) + last[r - 3 * M2];
    }
}

// imresize 'bicubic' kernel (Keys, a = -0.5) in its unscaled form
static double keys_cubic(double x)
{
    const double ax = std::fabs(x), ax2 = ax * ax, ax3 = ax2 * ax;
    return ax <= 1.0 ? 1.5 * ax3 - 2.5 * ax2 + 1.0
         : ax <= 2.0 ? -0.5 * ax3 + 2.5 * ax2 - 4.0 * ax + 2.0
                     : 0.0;
}

int resize_len(int len, double scale) { return (int)std::ceil(scale * (double)len); }

// MATLAB imresize contributions(): output sample x (1-based) sits at
// u = x/scale + (1 - 1/scale)/2 in input coordinates; taps left..left+P-1
// with left = floor(u - width/2); a reduction widens the kernel to 4/scale
// and scales it by `scale` (antialiasing); rows are normalised to sum 1;
// out-of-range taps mirror symmetrically; tap columns that are zero for
// every output are dropped (so scale 1 is an exact copy).
int resize_contrib(int in_len, int out_len, double scale, int antialias, std::vector<double> &w,
                   std::vector<int> &idx)
{
    const bool aa = antialias && scale < 1.0;
    const double width = aa ? 4.0 / scale : 4.0;
    const int P = (int)std::ceil(width) + 2;
    std::vector<double> wf((size_t)out_len * P);
    std::vector<int> jf((size_t)out_len * P);
    const long period = 2L * in_len;
    for (int i = 0; i < out_len; ++i) {
        const double u = (double)(i + 1) / scale + 0.5 * (1.0 - 1.0 / scale);
        const double left = std::floor(u - width / 2.0);
        double *wr = &wf[(size_t)i * P];
        double sum = 0.0;
        for (int k = 0; k < P; ++k) {
            const double d = u - (left + (double)k);
            wr[k] = aa ? scale * keys_cubic(scale * d) : keys_cubic(d);
            sum += wr[k];
        }
        for (int k = 0; k < P; ++k) {
            wr[k] /= sum;
            long j = ((long)left + k - 1) % period;
            if (j < 0) j += period;
            jf[(size_t)i * P + k] = (int)(j < in_len ? j : period - 1 - j);
        }
    }
    std::vector<int> keep;
    for (int k = 0; k < P; ++k)
        for (int i = 0; i < out_len; ++i)
            if (wf[(size_t)i * P + k] != 0.0) { keep.push_back(k); break; }
    const int Pk = (int)keep.size();
    w.assign((size_t)out_len * Pk, 0.0);
    idx.assign((size_t)out_len * Pk, 0);
    for (int i = 0; i < out_len; ++i)
        for (int k = 0; k < Pk; ++k) {
            w[(size_t)i * Pk + k] = wf[(size_t)i * P + keep[k]];
            idx[(size_t)i * Pk + k] = jf[(size_t)i * P + keep[k]];
        }
    return Pk;
}

// Gauss-Hermite nodes/weights for int exp(-x^2) f(x): Newton iteration on the
// orthonormal Hermite recurrence with asymptotic starting guesses.  The
// reference (GaussHermite_2.m) takes the eigen-decomposition of the Jacobi
// matrix instead; both give the same rule (tests compare with numpy.hermgauss).
int gauss_hermite(int n, double *x, double *w)
{
    if (n < 1 || n > GQMAP_KMAX) return 1;
    const double pim4 = 0.7511255444649425;  // pi^(-1/4)
    const int half = (n + 1) / 2;
    double z = 0, pp = 1;
    double xd[GQMAP_KMAX], wd[GQMAP_KMAX];  // descending
    for (int i = 0; i < half; ++i) {
        if (i == 0) z = std::sqrt(2.0 * n + 1) - 1.85575 * std::pow(2.0 * n + 1, -1.0 / 6.0);
        else if (i == 1) z -= 1.14 * std::pow((double)n, 0.426) / z;
        else if (i == 2) z = 1.86 * z - 0.86 * xd[0];
        else if (i == 3) z = 1.91 * z - 0.91 * xd[1];
        else z = 2.0 * z - xd[i - 2];
        int iter = 0;
        for (; iter < 200; ++iter) {
            double p1 = pim4, p2 = 0.0;
            for (int j = 1; j <= n; ++j) {
                const double p3 = p2;
                p2 = p1;
                p1 = z * std::sqrt(2.0 / j) * p2 - std::sqrt((j - 1.0) / j) * p3;
            }
            pp = std::sqrt(2.0 * n) * p2;
            const double z1 = z;
            z = z1 - p1 / pp;
            if (std::fabs(z - z1) <= 1e-15 * std::max(1.0, std::fabs(z))) break;
        }
        if (iter == 200) return 2;
        xd[i] = z;
        xd[n - 1 - i] = -z;
        wd[i] = wd[n - 1 - i] = 2.0 / (pp * pp);
    }
    if (n % 2 == 1) xd[half - 1] = 0.0;  // exact symmetric middle node
    for (int i = 0; i < n; ++i) {
        x[i] = xd[n - 1 - i];
        w[i] = wd[n - 1 - i];
    }
    return 0;
}

}  // namespace gq

extern "C" {

const char *gqmap_last_error(void) { return gq::g_err.c_str(); }

gqmap_status gqmap_gauss_hermite(int K, double *x, double *w)
{
    gq::clear_error();
    GQ_CHECK(x && w, GQMAP_ERR_INVALID_ARG, "null argument");
    GQ_CHECK(K >= 1 && K <= GQMAP_KMAX, GQMAP_ERR_INVALID_ARG, "K=%d outside [1,%d]", K, GQMAP_KMAX);
    GQ_CHECK(gq::gauss_hermite(K, x, w) == 0, GQMAP_ERR_INVALID_ARG, "Gauss-Hermite did not converge");
    return GQMAP_OK;
}

void gqmap_rand_uniform(uint64_t seed, uint32_t stream, uint64_t first, size_t n, double *out)
{
    const uint64_t base = gq::stream_base(seed, stream);
    for (size_t i = 0; i < n; ++i) out[i] = gq::u01(base, first + i);
}

int gqmap_device_count(void)
{
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

}  // extern "C"

// ---------------------------------------------------------------------------
// Middlebury .flo I/O and AEPE, host-side library calls
// ---------------------------------------------------------------------------
extern "C" {

// readFlowFile.m:33-84: "PIEH" tag (float 202021.25), int32 width, int32
// height, then rows of interleaved (u, v) float32; flow is M x N x 2 doubles
// (column-major).  flow == NULL: only the size is returned.
gqmap_status gqmap_read_flo(const char *path, int *M, int *N, double *flow)
{
    gq::clear_error();
    GQ_CHECK(path && M && N, GQMAP_ERR_INVALID_ARG, "gqmap_read_flo: null argument");
    const size_t len = std::strlen(path);
    GQ_CHECK(len > 4 && std::strcmp(path + len - 4, ".flo") == 0, GQMAP_ERR_INVALID_ARG,
             "readFlowFile: filename %s should have extension '.flo'", path);
    FILE *f = std::fopen(path, "rb");
    GQ_CHECK(f, GQMAP_ERR_INVALID_ARG, "readFlowFile: could not open %s", path);
    float tag = 0;
    int32_t wh[2] = {0, 0};
    const bool hdr = std::fread(&tag, 4, 1, f) == 1 && std::fread(wh, 4, 2, f) == 2;
    if (!hdr || tag != 202021.25f || wh[0] < 1 || wh[0] > 99999 || wh[1] < 1 || wh[1] > 99999) {
        std::fclose(f);
        gq::set_error("readFlowFile(%s): wrong tag or illegal size", path);
        return GQMAP_ERR_INVALID_ARG;
    }
    const int W = wh[0], H = wh[1];
    *M = H;
    *N = W;
    if (!flow) {
        std::fclose(f);
        return GQMAP_OK;
    }
    std::vector<float> row((size_t)2 * W);
    for (int m = 0; m < H; ++m) {
        if (std::fread(row.data(), sizeof(float), row.size(), f) != row.size()) {
            std::fclose(f);
            gq::set_error("readFlowFile(%s): truncated data", path);
            return GQMAP_ERR_INVALID_ARG;
        }
        for (int n = 0; n < W; ++n) {
            flow[m + (size_t)H * n] = row[2 * (size_t)n];
            flow[m + (size_t)H * n + (size_t)H * W] = row[2 * (size_t)n + 1];
        }
    }
    std::fclose(f);
    return GQMAP_OK;
}

// legacy/writeFlowFile.m:33-76
gqmap_status gqmap_write_flo(const char *path, const double *flow, int M, int N)
{
    gq::clear_error();
    GQ_CHECK(path && flow && M > 0 && N > 0, GQMAP_ERR_INVALID_ARG, "gqmap_write_flo: bad argument");
    const size_t len = std::strlen(path);
    GQ_CHECK(len > 4 && std::strcmp(path + len - 4, ".flo") == 0, GQMAP_ERR_INVALID_ARG,
             "writeFlowFile: filename %s should have extension '.flo'", path);
    FILE *f = std::fopen(path, "wb");
    GQ_CHECK(f, GQMAP_ERR_INVALID_ARG, "writeFlowFile: could not open %s", path);
    const int32_t wh[2] = {N, M};
    bool ok = std::fwrite("PIEH", 1, 4, f) == 4 && std::fwrite(wh, 4, 2, f) == 2;
    std::vector<float> row((size_t)2 * N);
    for (int m = 0; m < M && ok; ++m) {
        for (int n = 0; n < N; ++n) {
            row[2 * (size_t)n] = (float)flow[m + (size_t)M * n];
            row[2 * (size_t)n + 1] = (float)flow[m + (size_t)M * n + (size_t)M * N];
        }
        ok = std::fwrite(row.data(), sizeof(float), row.size(), f) == row.size();
    }
    ok = (std::fclose(f) == 0) && ok;
    GQ_CHECK(ok, GQMAP_ERR_INVALID_ARG, "writeFlowFile: write to %s failed", path);
    return GQMAP_OK;
}

// gqmap_gpu_mixture.m:63-64: flow(unknown) = 0, then
// mean(mean(sqrt(sum((tflow - flow).^2, 3)))) over rows/cols crop..end-crop
// (column means first).  unknown may be NULL.
gqmap_status gqmap_aepe(const double *tflow, const double *flow, const uint8_t *unknown, int M, int N, int crop,
                        double *out)
{
    gq::clear_error();
    GQ_CHECK(tflow && flow && out, GQMAP_ERR_INVALID_ARG, "gqmap_aepe: null argument");
    GQ_CHECK(crop >= 0 && M > 2 * crop && N > 2 * crop, GQMAP_ERR_INVALID_ARG, "gqmap_aepe: crop %d of %dx%d",
             crop, M, N);
    const size_t MN = (size_t)M * N;
    double total = 0;
    for (int n = crop; n < N - crop; ++n) {
        double col = 0;
        for (int m = crop; m < M - crop; ++m) {
            const size_t q = m + (size_t)M * n;
            const bool unk = unknown && unknown[q];
            const double du = tflow[q] - (unk ? 0.0 : flow[q]);
            const double dv = tflow[q + MN] - (unk ? 0.0 : flow[q + MN]);
            col += std::sqrt(du * du + dv * dv);
        }
        total += col / (M - 2 * crop);
    }
    *out = total / (N - 2 * crop);
    return GQMAP_OK;
}

}  // extern "C"
