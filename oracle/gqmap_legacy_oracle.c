/*
 * gqmap_legacy_oracle.c -- CPU restatement of legacy/gqmap_cpu.m (fp64), the
 * legacy flow-denoising QGMAP: Gaussian observation of a given flow field,
 * truncated-quadratic pairwise terms, Gauss-Hermite quadrature.
 *
 * TEST INFRASTRUCTURE ONLY (see gqmap_oracle.h).  Literal order of the MATLAB
 * expressions; every line cites legacy/gqmap_cpu.m.  options.var / gama / dta
 * are never set anywhere in the reference: they are inputs
 * here, so results for a particular choice are "parity unpinned".
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "gqmap_oracle.h"

#define PI 3.14159265358979323846

/* index helpers, MATLAB column-major */
#define I3(m, n, l) ((m) + (size_t)M * ((n) + (size_t)N * (l)))                      /* M x N x 2      */
#define I4(m, n, a, b) ((m) + (size_t)M * ((n) + (size_t)N * ((a) + 2 * (size_t)(b)))) /* M x N x 2 x 2  */
#define I5(m, n, j, q, l) ((m) + (size_t)M * ((n) + (size_t)N * ((j) + 2 * ((q) + 5 * (size_t)(l)))))

int orc_cpu_run(const orc_cpu_params *P, const double *X, const double *W, const double *flow, int M, int N,
                double *mu, double *sigma, double *rou, double *trace, int nthreads)
{
    if (nthreads <= 0) nthreads = 1;
    const int K = P->K, K2 = K * K;
    const double sq2 = sqrt(2.0);
    /* [XI,XJ] = meshgrid(X); WIWJ = WI.*WJ  (:5-6), k = r + K*c */
    double *XI = malloc(sizeof(double) * K2), *XJ = malloc(sizeof(double) * K2), *WW = malloc(sizeof(double) * K2);
    for (int c = 0; c < K; ++c)
        for (int r = 0; r < K; ++r) {
            XI[r + K * c] = X[c];
            XJ[r + K * c] = X[r];
            WW[r + K * c] = W[c] * W[r];
        }
    double *dnode = calloc((size_t)M * N * 4, sizeof(double));      /* (:14) */
    double *dedge = calloc((size_t)M * N * 20, sizeof(double));     /* (:15) */
    double *dmu = malloc(sizeof(double) * (size_t)M * N * 2), *dsg = malloc(sizeof(double) * (size_t)M * N * 2);
    int it = 1, done = 0;
    for (;;) {
        /* parfor m=1:M-1 (:17): rows are independent (each writes its own
         * dnode/dedge entries), so any thread count gives the same bits */
#pragma omp parallel for num_threads(nthreads) schedule(static)
        for (int m = 0; m < M - 1; ++m)
            for (int n = 0; n < N - 1; ++n) {     /* for n=1:N-1   (:18)  */
                for (int l = 0; l < 2; ++l) {     /* (:20-26) */
                    double du = 0, dsum = 0;
                    for (int k = 0; k < K; ++k) {
                        const double x = sq2 * sigma[I3(m, n, l)] * X[k] + mu[I3(m, n, l)];
                        const double dval = W[k] * (flow[I3(m, n, l)] - x) / P->var;
                        du += dval;
                        dsum += dval * X[k];
                    }
                    dnode[I4(m, n, 0, l)] = du / sqrt(PI);
                    dnode[I4(m, n, 1, l)] = dsum * sqrt(2.0 / PI);
                }
                for (int j = 0; j < 2; ++j) {     /* (:28-54) */
                    const int m2 = m + (j == 0), n2 = n + (j == 1);
                    for (int l = 0; l < 2; ++l) {
                        const double p = rou[I4(m, n, j, l)];
                        const double o1 = sigma[I3(m, n, l)], o2 = sigma[I3(m2, n2, l)];
                        const double u1 = mu[I3(m, n, l)], u2 = mu[I3(m2, n2, l)];
                        const double q = sqrt(1 + p), r = sqrt(1 - p);
                        const double s = (q + r) / 2, t = (q - r) / 2;
                        const double ds = (1 / q - 1 / r) / 4, dt = (1 / q + 1 / r) / 4;
                        /* sum(sum(A)): column sums (over r) first, then their sum */
                        double s1 = 0, s2 = 0, so1 = 0, so2 = 0, sp = 0;
                        for (int c = 0; c < K; ++c) {
                            double c1 = 0, c2 = 0, co1 = 0, co2 = 0, cp = 0;
                            for (int rr = 0; rr < K; ++rr) {
                                const int k = rr + K * c;
                                const double ZI = s * XI[k] + t * XJ[k], ZJ = t * XI[k] + s * XJ[k];
                                const double x1 = sq2 * o1 * ZI + u1, x2 = sq2 * o2 * ZJ + u2;
                                double diff = x2 - x1;
                                if (fabs(diff) > P->dta) diff = 0;        /* (:44) */
                                const double df1 = WW[k] * diff / P->gama, df2 = -df1;
                                c1 += df1;
                                c2 += df2;
                                co1 += df1 * ZI;
                                co2 += df2 * ZJ;
                                cp += o1 * df1 * (ds * XI[k] + dt * XJ[k]) + o2 * df2 * (dt * XI[k] + ds * XJ[k]);
                            }
                            s1 += c1; s2 += c2; so1 += co1; so2 += co2; sp += cp;
                        }
                        dedge[I5(m, n, j, 0, l)] = 1 / PI * s1;
                        dedge[I5(m, n, j, 1, l)] = 1 / PI * s2;
                        dedge[I5(m, n, j, 2, l)] = 1 / PI * sq2 * so1;
                        dedge[I5(m, n, j, 3, l)] = 1 / PI * sq2 * so2;
                        dedge[I5(m, n, j, 4, l)] = 1 / PI * sq2 * sp;
                    }
                }
            }
        /* sum up (:58-60): the neighbour terms come from row m+1 / column n+1
         * (cat(1,dedge(2:M,..),zeros) -- the reference's own shift) */
        double mx_mu = 0, mx_sg = 0, mx_p = 0;
        for (int l = 0; l < 2; ++l)
            for (int n = 0; n < N; ++n)
                for (int m = 0; m < M; ++m) {
                    double a = dnode[I4(m, n, 0, l)] + (dedge[I5(m, n, 0, 0, l)] + dedge[I5(m, n, 1, 0, l)]);
                    double b = dnode[I4(m, n, 1, l)] + (dedge[I5(m, n, 0, 2, l)] + dedge[I5(m, n, 1, 2, l)]);
                    const double nu = m + 1 < M ? dedge[I5(m + 1, n, 0, 1, l)] : 0.0;
                    const double nl = n + 1 < N ? dedge[I5(m, n + 1, 1, 1, l)] : 0.0;
                    const double su = m + 1 < M ? dedge[I5(m + 1, n, 0, 3, l)] : 0.0;
                    const double sl = n + 1 < N ? dedge[I5(m, n + 1, 1, 3, l)] : 0.0;
                    a = a + (nu + nl);
                    b = b + (su + sl);
                    dmu[I3(m, n, l)] = a;
                    dsg[I3(m, n, l)] = b;
                    if (fabs(a) > mx_mu) mx_mu = fabs(a);
                    if (fabs(b) > mx_sg) mx_sg = fabs(b);
                }
        const double step = P->step0 / (1 + it / P->step_decay);   /* 0.1/(1+it/1000) (:62) */
        for (size_t i = 0; i < (size_t)M * N * 2; ++i) {
            mu[i] = mu[i] + dmu[i] * step;                 /* (:63) */
            sigma[i] = fabs(sigma[i] + dsg[i] * step);     /* (:64) */
        }
        for (int l = 0; l < 2; ++l)
            for (int j = 0; j < 2; ++j)
                for (int n = 0; n < N; ++n)
                    for (int m = 0; m < M; ++m) {
                        const double d = dedge[I5(m, n, j, 4, l)];
                        if (fabs(d) > mx_p) mx_p = fabs(d);
                        double v = rou[I4(m, n, j, l)] + d * step;
                        rou[I4(m, n, j, l)] = fmax(fmin(v, P->corr_tor), -P->corr_tor);  /* (:65) */
                    }
        trace[3 * done + 0] = mx_mu;
        trace[3 * done + 1] = mx_sg;
        trace[3 * done + 2] = mx_p;
        ++done;
        it = it + 1;
        if (it > P->its || (it > P->min_its && mx_mu < P->tor)) break;   /* (:70) */
    }
    free(XI); free(XJ); free(WW); free(dnode); free(dedge); free(dmu); free(dsg);
    return done;
}
