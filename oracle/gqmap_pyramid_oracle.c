/*
 * gqmap_pyramid_oracle.c -- CPU restatement of the coarse-to-fine plumbing of
 * legacy/optical_flow_ctf.m:21-35 (fp64).
 *
 * TEST INFRASTRUCTURE ONLY (see gqmap_oracle.h).
 *
 * The reference calls three MATLAB R2018b builtins here; none is vendored, so
 * their published algorithms are restated and parity at this boundary is
 * "parity unpinned" (no reference output exists to compare with):
 *   imresize(A, s)          default 'bicubic', Antialiasing=true: separable
 *                           resampling with the Keys (a=-0.5) kernel, widened
 *                           by 1/s when s<1; contributions() with symmetric
 *                           (mirror) edge handling and all-zero tap columns
 *                           removed; dimensions in sort(scale) order (rows
 *                           first for a uniform scale); output ceil(s*size).
 *                           Call sites optical_flow_ctf.m:23,26,27,29.
 *   interp2(V, Xq, Yq)      default 'linear': bilinear on the unit grid, NaN
 *                           outside [1,N]x[1,M] (optical_flow_ctf.m:31).
 *   fillmissing(A,'nearest',dim)  every NaN takes the nearest non-NaN along
 *                           dim; a tie takes the later sample (interp1
 *                           'nearest' rounds half up); an all-NaN line stays
 *                           NaN (optical_flow_ctf.m:32).
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "gqmap_oracle.h"

/* imresize.m cubic(): Keys a=-0.5 kernel in the standard (not x2) form */
static double cubic(double x)
{
    const double ax = fabs(x), ax2 = ax * ax, ax3 = ax2 * ax;
    if (ax <= 1.0) return 1.5 * ax3 - 2.5 * ax2 + 1.0;
    if (ax <= 2.0) return -0.5 * ax3 + 2.5 * ax2 - 4.0 * ax + 2.0;
    return 0.0;
}

int orc_resize_taps(double scale, int antialias)
{
    const double kw = (scale < 1.0 && antialias) ? 4.0 / scale : 4.0;
    return (int)ceil(kw) + 2;
}

/* imresize.m contributions(): w/idx are [out_len][P] row-major, idx 0-based.
 * Returns the number of tap columns kept (all-zero columns removed). */
int orc_resize_contrib(int in_len, int out_len, double scale, int antialias, double *w, int *idx)
{
    const int aa = scale < 1.0 && antialias;
    const double kw = aa ? 4.0 / scale : 4.0;
    const int P = (int)ceil(kw) + 2;
    for (int i = 0; i < out_len; ++i) {
        const double x = (double)(i + 1);
        const double u = x / scale + 0.5 * (1.0 - 1.0 / scale);
        const double left = floor(u - kw / 2.0);
        double sum = 0.0;
        for (int k = 0; k < P; ++k) {
            const double d = u - (left + (double)k);
            const double h = aa ? scale * cubic(scale * d) : cubic(d);
            w[(size_t)i * P + k] = h;
            sum += h;
        }
        for (int k = 0; k < P; ++k) {
            w[(size_t)i * P + k] /= sum;
            /* aux = [1:in, in:-1:1]; idx = aux(mod(idx-1, 2*in) + 1) */
            long j = (long)left + k - 1;  /* 0-based position before mirroring */
            const long n2 = 2L * in_len;
            j = ((j % n2) + n2) % n2;
            idx[(size_t)i * P + k] = (int)(j < in_len ? j : n2 - 1 - j);
        }
    }
    /* kill = find(~any(weights,1)) */
    int keep = 0;
    for (int k = 0; k < P; ++k) {
        int any = 0;
        for (int i = 0; i < out_len && !any; ++i) any = w[(size_t)i * P + k] != 0.0;
        if (!any) continue;
        for (int i = 0; i < out_len; ++i) {
            w[(size_t)i * P + keep] = w[(size_t)i * P + k];
            idx[(size_t)i * P + keep] = idx[(size_t)i * P + k];
        }
        ++keep;
    }
    /* compact rows to stride `keep` */
    for (int i = 0; i < out_len; ++i)
        for (int k = 0; k < keep; ++k) {
            w[(size_t)i * keep + k] = w[(size_t)i * P + k];
            idx[(size_t)i * keep + k] = idx[(size_t)i * P + k];
        }
    return keep;
}

int orc_resize_len(int len, double scale) { return (int)ceil(scale * (double)len); }

/* imresize(A, scale): A is M x N x C column-major, out ceil(sM) x ceil(sN) x C. */
void orc_imresize(const double *in, int M, int N, int C, double scale, int antialias, double *out)
{
    const int oM = orc_resize_len(M, scale), oN = orc_resize_len(N, scale);
    const int P = orc_resize_taps(scale, antialias);
    double *wm = malloc(sizeof(double) * (size_t)oM * P), *wn = malloc(sizeof(double) * (size_t)oN * P);
    int *im = malloc(sizeof(int) * (size_t)oM * P), *in_ = malloc(sizeof(int) * (size_t)oN * P);
    const int Pm = orc_resize_contrib(M, oM, scale, antialias, wm, im);
    const int Pn = orc_resize_contrib(N, oN, scale, antialias, wn, in_);
    double *tmp = malloc(sizeof(double) * (size_t)oM * N);
    for (int c = 0; c < C; ++c) {
        const double *A = in + (size_t)M * N * c;
        /* dim 1 (rows) first */
        for (int n = 0; n < N; ++n)
            for (int i = 0; i < oM; ++i) {
                double s = 0.0;
                for (int k = 0; k < Pm; ++k) s += wm[(size_t)i * Pm + k] * A[im[(size_t)i * Pm + k] + (size_t)M * n];
                tmp[i + (size_t)oM * n] = s;
            }
        double *B = out + (size_t)oM * oN * c;
        for (int j = 0; j < oN; ++j)
            for (int i = 0; i < oM; ++i) {
                double s = 0.0;
                for (int k = 0; k < Pn; ++k) s += wn[(size_t)j * Pn + k] * tmp[i + (size_t)oM * in_[(size_t)j * Pn + k]];
                B[i + (size_t)oM * j] = s;
            }
    }
    free(tmp); free(wm); free(wn); free(im); free(in_);
}

/* interp2(V, x - wu, y - wv), 'linear', NaN outside (optical_flow_ctf.m:30-31) */
void orc_warp_image(const double *V, int M, int N, const double *warp, double *out)
{
    const size_t MN = (size_t)M * N;
    for (int n = 0; n < N; ++n)
        for (int m = 0; m < M; ++m) {
            const size_t q = m + (size_t)M * n;
            const double xq = (double)(n + 1) - warp[q], yq = (double)(m + 1) - warp[q + MN];
            if (!(xq >= 1.0 && xq <= (double)N && yq >= 1.0 && yq <= (double)M)) {
                out[q] = NAN;
                continue;
            }
            int ix = (int)floor(xq), iy = (int)floor(yq);
            if (ix > N - 1) ix = N - 1;
            if (iy > M - 1) iy = M - 1;
            const double s = xq - ix, t = yq - iy;
            const double *c0 = V + (size_t)M * (ix - 1) + (iy - 1), *c1 = c0 + M;
            const double top = (1.0 - s) * c0[0] + s * c1[0];
            const double bot = (1.0 - s) * c0[1] + s * c1[1];
            out[q] = (1.0 - t) * top + t * bot;
        }
}

/* fillmissing(A, 'nearest', dim) in place, dim 1 (down columns) or 2 (along rows) */
void orc_fillmissing_nearest(double *A, int M, int N, int dim)
{
    const int len = dim == 1 ? M : N, lines = dim == 1 ? N : M;
    const size_t stride = dim == 1 ? 1 : (size_t)M, lstride = dim == 1 ? (size_t)M : 1;
    double *src = malloc(sizeof(double) * (size_t)len);
    for (int l = 0; l < lines; ++l) {
        double *a = A + lstride * l;
        for (int k = 0; k < len; ++k) src[k] = a[stride * k];
        for (int k = 0; k < len; ++k) {
            if (!isnan(src[k])) continue;
            int lo = k - 1, hi = k + 1;
            while (lo >= 0 && isnan(src[lo])) --lo;
            while (hi < len && isnan(src[hi])) ++hi;
            if (lo < 0 && hi >= len) continue;              /* all missing */
            if (lo < 0) a[stride * k] = src[hi];
            else if (hi >= len) a[stride * k] = src[lo];
            else a[stride * k] = (k - lo < hi - k) ? src[lo] : src[hi];  /* tie -> later */
        }
    }
    free(src);
}
