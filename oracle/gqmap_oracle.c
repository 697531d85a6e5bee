/*
 * gqmap_oracle.c -- CPU fp64 restatement of the QGMAP hot path.
 *
 * TEST INFRASTRUCTURE ONLY (see gqmap_oracle.h).  Deliberately written as a
 * literal restatement of the MATLAB element functions and array algebra --
 * no algebraic refactoring -- so that it can serve as the parity checker for
 * the HIP kernels.  Compiled with -ffp-contract=off (no FMA contraction).
 *
 * Reference lines restated (paths relative to the reference repo):
 *   GaussHermite_2.m:21-32              orc_gauss_hermite
 *   gqmap_gpu_mixture.m:191-208         orc_get_vv (getVV)
 *   gqmap_gpu_mixture.m:156-182         node_pot / edge_pot
 *   gqmap_gpu_mixture.m:87-146          node_grad / edge_grad (spectral)
 *   gqmap_gpuSuper_mix_entropy.m:87-122 super node_grad (4x4 block sum)
 *   gqmap_gpu_mixture.m:26-76, 78-86    iteration loop + updateAlpha
 *   gqmap_gpuSuper_mix_entropy.m:25-75  super iteration loop + T decay
 *   projsplx.m:15-30                    orc_projsplx
 *   legacy/flowToColor.m:37-87, legacy/computeColor.m:33-115  orc_flow_to_color
 *   legacy/findMixMax.m:39-70 (+ MATLAB fminbnd)              orc_get_map
 */
#include "gqmap_oracle.h"

#include <float.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define KMAX 32
static const double SQRT2 = 1.4142135623730951;

/* ------------------------------------------------------------------ */
/* GaussHermite_2.m:21-32: CM = diag(sqrt(i/2),+-1); [V,L]=eig(CM);   */
/* x = sort(diag(L)); w = sqrt(pi)*V(1,:).^2                           */
/* ------------------------------------------------------------------ */
void orc_gauss_hermite(int K, double *x, double *w)
{
    double A[KMAX][KMAX], V[KMAX][KMAX];
    memset(A, 0, sizeof A);
    memset(V, 0, sizeof V);
    for (int i = 0; i < K; ++i) V[i][i] = 1.0;
    for (int i = 0; i + 1 < K; ++i) A[i][i + 1] = A[i + 1][i] = sqrt((i + 1) / 2.0);
    /* cyclic Jacobi rotations until the off-diagonal mass vanishes */
    for (int sweep = 0; sweep < 100; ++sweep) {
        double off = 0.0;
        for (int p = 0; p < K; ++p)
            for (int q = p + 1; q < K; ++q) off += A[p][q] * A[p][q];
        if (off < 1e-300) break;
        for (int p = 0; p < K; ++p) {
            for (int q = p + 1; q < K; ++q) {
                if (fabs(A[p][q]) < 1e-300) continue;
                double theta = (A[q][q] - A[p][p]) / (2.0 * A[p][q]);
                double t = (theta >= 0 ? 1.0 : -1.0) / (fabs(theta) + sqrt(theta * theta + 1.0));
                double c = 1.0 / sqrt(t * t + 1.0), s = t * c;
                for (int k = 0; k < K; ++k) {
                    double akp = A[k][p], akq = A[k][q];
                    A[k][p] = c * akp - s * akq;
                    A[k][q] = s * akp + c * akq;
                }
                for (int k = 0; k < K; ++k) {
                    double apk = A[p][k], aqk = A[q][k];
                    A[p][k] = c * apk - s * aqk;
                    A[q][k] = s * apk + c * aqk;
                }
                for (int k = 0; k < K; ++k) {
                    double vkp = V[k][p], vkq = V[k][q];
                    V[k][p] = c * vkp - s * vkq;
                    V[k][q] = s * vkp + c * vkq;
                }
            }
        }
    }
    int idx[KMAX];
    for (int i = 0; i < K; ++i) idx[i] = i;
    for (int i = 1; i < K; ++i) { /* insertion sort by eigenvalue */
        int j = i, v = idx[i];
        while (j > 0 && A[idx[j - 1]][idx[j - 1]] > A[v][v]) { idx[j] = idx[j - 1]; --j; }
        idx[j] = v;
    }
    const double sqpi = sqrt(M_PI);
    for (int i = 0; i < K; ++i) {
        x[i] = A[idx[i]][idx[i]];
        double v0 = V[0][idx[i]];
        w[i] = sqpi * v0 * v0;
    }
}

/* getVV: gqmap_gpu_mixture.m:191-208 (column loop first, then row loop). */
void orc_get_vv(const double *V, int M, int N, double *VV)
{
    const int M2 = M + 2, N2 = N + 2, M2N2 = M2 * N2;
    memset(VV, 0, sizeof(double) * (size_t)M2N2);
    for (int n = 0; n < N; ++n)
        for (int m = 0; m < M; ++m) VV[(m + 1) + (size_t)M2 * (n + 1)] = V[m + (size_t)M * n];
    /* MATLAB 1-based linear indices rewritten 0-based */
    for (int i = 0; i < N2; ++i) {
        int ix = M2 * i, iy = ix + M2 - 1;
        VV[ix] = (3.0 * VV[ix + 1] - 3.0 * VV[ix + 2]) + VV[ix + 3];
        VV[iy] = (3.0 * VV[iy - 1] - 3.0 * VV[iy - 2]) + VV[iy - 3];
    }
    for (int i = 0; i < M2; ++i) {
        VV[i] = (3.0 * VV[M2 + i] - 3.0 * VV[M2 * 2 + i]) + VV[M2 * 3 + i];
        VV[M2N2 - M2 + i] = (3.0 * VV[M2N2 - M2 * 2 + i] - 3.0 * VV[M2N2 - M2 * 3 + i]) +
                            VV[M2N2 - M2 * 4 + i];
    }
}

/* Bicubic (Keys, a=-1/2, x2 form) on the padded VV, exactly as node_pot
 * (gqmap_gpu_mixture.m:157-176).  Xq, Yq are 1-based positions, clamped. */
double orc_interp_cubic(const double *VV, int M, int N, double Xq, double Yq)
{
    const int M2 = M + 2;
    Xq = fmin(fmax(Xq, 1.0), (double)N);
    Yq = fmin(fmax(Yq, 1.0), (double)M);
    int ix, iy;
    if (Xq <= 1.0) ix = 1; else if (Xq <= N - 1) ix = (int)floor(Xq); else ix = N - 1;
    if (Yq <= 1.0) iy = 1; else if (Yq <= M - 1) iy = (int)floor(Yq); else iy = M - 1;
    const double so = Xq - ix, to = Yq - iy;
    const double t0 = ((2.0 - to) * to - 1.0) * to;
    const double t1 = (3.0 * to - 5.0) * to * to + 2.0;
    const double t2 = ((4.0 - 3.0 * to) * to + 1.0) * to;
    const double t3 = (to - 1.0) * to * to;
    /* MATLAB 1-based iy1 = iy + M2*(ix-1) -> 0-based iy1-1 */
    const double *c1 = VV + (iy - 1) + (size_t)M2 * (ix - 1);
    const double *c2 = c1 + M2, *c3 = c2 + M2, *c4 = c3 + M2;
    double ss = ((2.0 - so) * so - 1.0) * so;
    double Vq = ((c1[0] * ss * t0 + c1[1] * ss * t1) + c1[2] * ss * t2) + c1[3] * ss * t3;
    ss = (3.0 * so - 5.0) * so * so + 2.0;
    Vq = Vq + c2[0] * ss * t0 + c2[1] * ss * t1 + c2[2] * ss * t2 + c2[3] * ss * t3;
    ss = ((4.0 - 3.0 * so) * so + 1.0) * so;
    Vq = Vq + c3[0] * ss * t0 + c3[1] * ss * t1 + c3[2] * ss * t2 + c3[3] * ss * t3;
    ss = (so - 1.0) * so * so;
    Vq = Vq + c4[0] * ss * t0 + c4[1] * ss * t1 + c4[2] * ss * t2 + c4[3] * ss * t3;
    return Vq / 4;
}

/* ------------------------------------------------------------------ */
typedef struct {
    const orc_params *p;
    const double *I1, *VV;
    int K2;
    double XI[KMAX * KMAX], XJ[KMAX * KMAX], WIWJ[KMAX * KMAX], XIXJ[KMAX * KMAX];
    double XI2aXJ2[KMAX * KMAX], XI2mXJ2[KMAX * KMAX];
} orc_ctx;

static void ctx_init(orc_ctx *c, const orc_params *p, const double *I1, const double *VV)
{
    double X[KMAX], W[KMAX];
    c->p = p; c->I1 = I1; c->VV = VV;
    if (p->gh_x && p->gh_w) {
        memcpy(X, p->gh_x, sizeof(double) * (size_t)p->K);
        memcpy(W, p->gh_w, sizeof(double) * (size_t)p->K);
    } else {
        orc_gauss_hermite(p->K, X, W);
    }
    c->K2 = p->K * p->K;
    /* [XI,XJ] = meshgrid(X): XI(r,c)=X(c), XJ(r,c)=X(r); linear k = r + K*c */
    for (int cc = 0; cc < p->K; ++cc)
        for (int r = 0; r < p->K; ++r) {
            int k = r + p->K * cc;
            c->XI[k] = X[cc]; c->XJ[k] = X[r];
            c->WIWJ[k] = W[cc] * W[r];
            c->XIXJ[k] = X[cc] * X[r];
            c->XI2aXJ2[k] = X[cc] * X[cc] + X[r] * X[r];
            c->XI2mXJ2[k] = X[cc] * X[cc] - X[r] * X[r];
        }
}

/* node_pot, gqmap_gpu_mixture.m:156-179 (1-based i,j on the image grid) */
static inline double node_pot(const orc_ctx *c, double x1, double x2, int i, int j)
{
    const int Mo = c->p->Mo, No = c->p->No;
    double Vq = orc_interp_cubic(c->VV, Mo, No, j + x1, i + x2);
    double d = c->I1[(i - 1) + (size_t)Mo * (j - 1)] - Vq;
    return -c->p->lambdad * sqrt(c->p->epsn + d * d);
}

/* legacy/gqmap_ctf.m:96: I2_cont(clamp(round((m+x2-1)*rfc2+1),1,MM), clamp(round((n+x1-1)*rfc2+1),1,NN))
 * with I2_cont = interp2(I2,6,'cubic'); entry (r,c) of the 64x-refined table is
 * the cubic interpolation at (1+(c-1)/64, 1+(r-1)/64), evaluated here directly. */
static inline double ctf_lookup(const orc_ctx *c, double x1, double x2, int m, int n)
{
    const int Mo = c->p->Mo, No = c->p->No;
    const double rfc2 = 64.0, MM = 64.0 * (Mo - 1) + 1, NN = 64.0 * (No - 1) + 1;
    const double r = fmin(fmax(round((m + x2 - 1) * rfc2 + 1), 1.0), MM);
    const double cc = fmin(fmax(round((n + x1 - 1) * rfc2 + 1), 1.0), NN);
    return orc_interp_cubic(c->VV, Mo, No, (cc - 1) / rfc2 + 1, (r - 1) / rfc2 + 1);
}

/* node_grad_spectral of legacy/gqmap_ctf.m:79-110 (no mixture weight, no entropy) */
static void ctf_node_grad(const orc_ctx *c, double u1, double u2, double o1, double o2, double p,
                          int m, int n, double *out)
{
    const orc_params *P = c->p;
    double du1 = 0, du2 = 0, do1 = 0, do2 = 0, dp = 0, nener = 0;
    const double s = (sqrt(1 + p) + sqrt(1 - p)) / 2;
    const double t = (sqrt(1 + p) - sqrt(1 - p)) / 2;
    const double pr = 1 - p * p, sqrtpr = sqrt(pr);
    const double o1pr = SQRT2 / (o1 * pr), o2pr = SQRT2 / (o2 * pr);
    const double I = c->I1[(m - 1) + (size_t)P->Mo * (n - 1)];
    for (int k = 0; k < c->K2; ++k) {
        const double zi = s * c->XI[k] + t * c->XJ[k], zj = t * c->XI[k] + s * c->XJ[k];
        const double x1 = SQRT2 * o1 * zi + u1, x2 = SQRT2 * o2 * zj + u2;
        const double d = I - ctf_lookup(c, x1, x2, m, n);
        const double fval = c->WIWJ[k] * sqrt(P->epsn + d * d);
        dp = dp + fval * (p - p * c->XI2aXJ2[k] + 2 * c->XIXJ[k]);
        du1 = du1 + fval * (zi - p * zj);
        du2 = du2 + fval * (zj - p * zi);
        do1 = do1 + fval * (c->XI2aXJ2[k] - 1 + c->XI2mXJ2[k] / sqrtpr);
        do2 = do2 + fval * (c->XI2aXJ2[k] - 1 - c->XI2mXJ2[k] / sqrtpr);
        nener = nener + fval;
    }
    const double lam = P->lambdad;
    out[0] = 0;
    out[1] = -lam * du1 * o1pr / M_PI;
    out[2] = -lam * du2 * o2pr / M_PI;
    out[3] = -lam * do1 / M_PI / o1;
    out[4] = -lam * do2 / M_PI / o2;
    out[5] = -lam * dp / M_PI / pr;
    out[6] = -lam * nener;
}

/* edge_grad_spectral of legacy/gqmap_ctf.m:128-150 */
static void ctf_edge_grad(const orc_ctx *c, double u1, double u2, double o1, double o2, double p,
                          double *out)
{
    const orc_params *P = c->p;
    double du1 = 0, du2 = 0, do1 = 0, do2 = 0, dp = 0, eener = 0;
    const double s = (sqrt(1 + p) + sqrt(1 - p)) / 2;
    const double t = (sqrt(1 + p) - sqrt(1 - p)) / 2;
    const double pr = 1 - p * p, sqrtpr = sqrt(pr);
    const double o1pr = SQRT2 / (o1 * pr), o2pr = SQRT2 / (o2 * pr);
    for (int k = 0; k < c->K2; ++k) {
        const double zi = s * c->XI[k] + t * c->XJ[k], zj = t * c->XI[k] + s * c->XJ[k];
        const double d = SQRT2 * o1 * zi + u1 - SQRT2 * o2 * zj - u2;
        const double fval = c->WIWJ[k] * sqrt(P->epsn + d * d);
        dp = dp + fval * (p - p * c->XI2aXJ2[k] + 2 * c->XIXJ[k]);
        du1 = du1 + fval * (zi - p * zj);
        du2 = du2 + fval * (zj - p * zi);
        do1 = do1 + fval * (c->XI2aXJ2[k] - 1 + c->XI2mXJ2[k] / sqrtpr);
        do2 = do2 + fval * (c->XI2aXJ2[k] - 1 - c->XI2mXJ2[k] / sqrtpr);
        eener = eener + fval;
    }
    const double lam = P->lambdas;
    out[0] = 0;
    out[1] = -lam * du1 * o1pr / M_PI;
    out[2] = -lam * du2 * o2pr / M_PI;
    out[3] = -lam * do1 / M_PI / o1;
    out[4] = -lam * do2 / M_PI / o2;
    out[5] = -lam * dp / M_PI / pr;
    out[6] = -lam * eener;
}

/* edge_pot, gqmap_gpu_mixture.m:180-182 */
static inline double edge_pot(const orc_ctx *c, double x1, double x2)
{
    double d = x1 - x2;
    return -c->p->lambdas * sqrt(c->p->epsn + d * d);
}

/* log of the entropy terms (:111, :141): libm by default; orc_set_ent_log()
 * swaps in another implementation (the device's deterministic gq_log, from
 * the emulator) so that T != 0 runs can be compared bit for bit with the
 * literal-order engine.  MATLAB's own log is unpinned. */
static double (*ent_log)(double) = log;
void orc_set_ent_log(double (*f)(double)) { ent_log = f ? f : log; }

/* node_grad_spectral: gqmap_gpu_mixture.m:87-116 (super: gqmap_gpuSuper_mix_entropy.m:87-122).
 * m, n are 1-based node indices.  out = {da,du1,du2,do1,do2,dp,Ei}. */
static void node_grad(const orc_ctx *c, double T, double a, double u1, double u2, double o1,
                      double o2, double p, int m, int n, double *out)
{
    const orc_params *P = c->p;
    double du1 = 0, du2 = 0, do1 = 0, do2 = 0, dp = 0, Ei = 0;
    const double s = (sqrt(1 + p) + sqrt(1 - p)) / 2;
    const double t = (sqrt(1 + p) - sqrt(1 - p)) / 2;
    const double pr = 1 - p * p, sqrtpr = sqrt(pr);
    const double o1pr = SQRT2 / (o1 * pr), o2pr = SQRT2 / (o2 * pr);
    const double const1 = 1 + ent_log(2 * M_PI);
    for (int k = 0; k < c->K2; ++k) {
        const double zi = s * c->XI[k] + t * c->XJ[k], zj = t * c->XI[k] + s * c->XJ[k];
        const double x1 = SQRT2 * o1 * zi + u1, x2 = SQRT2 * o2 * zj + u2;
        double pot;
        if (P->super_) {
            const int bottom = 4 * m, top = bottom - 3, right = 4 * n, left = right - 3;
            double sup = 0;
            for (int i = top; i <= bottom; ++i)
                for (int j = left; j <= right; ++j) sup = sup + node_pot(c, x1, x2, i, j);
            pot = sup;
        } else {
            pot = node_pot(c, x1, x2, m, n);
        }
        const double fval = c->WIWJ[k] * pot;
        if (!P->guard_a || a != 0) {
            dp = dp + fval * (p - p * c->XI2aXJ2[k] + 2 * c->XIXJ[k]);
            du1 = du1 + fval * (zi - p * zj);
            du2 = du2 + fval * (zj - p * zi);
            do1 = do1 + fval * (c->XI2aXJ2[k] - 1 + c->XI2mXJ2[k] / sqrtpr);
            do2 = do2 + fval * (c->XI2aXJ2[k] - 1 - c->XI2mXJ2[k] / sqrtpr);
        }
        Ei = Ei + fval;
    }
    du1 = a * du1 * o1pr / M_PI;
    du2 = a * du2 * o2pr / M_PI;
    const double da = Ei / M_PI - 3 * T * (const1 + ent_log(sqrtpr * o1 * o2));
    do1 = a * (do1 / M_PI - 3 * T) / o1;
    do2 = a * (do2 / M_PI - 3 * T) / o2;
    dp = a * (dp / M_PI + 3 * T * p) / pr;
    out[0] = da; out[1] = du1; out[2] = du2; out[3] = do1; out[4] = do2; out[5] = dp;
    out[6] = a * da;
}

/* edge_grad_spectral: gqmap_gpu_mixture.m:118-146 */
static void edge_grad(const orc_ctx *c, double T, double a, double u1, double u2, double o1,
                      double o2, double p, double *out)
{
    const orc_params *P = c->p;
    double du1 = 0, du2 = 0, do1 = 0, do2 = 0, dp = 0, Ei = 0;
    const double s = (sqrt(1 + p) + sqrt(1 - p)) / 2;
    const double t = (sqrt(1 + p) - sqrt(1 - p)) / 2;
    const double pr = 1 - p * p, sqrtpr = sqrt(pr);
    const double o1pr = SQRT2 / (o1 * pr), o2pr = SQRT2 / (o2 * pr);
    const double const1 = 1 + ent_log(2 * M_PI);
    for (int k = 0; k < c->K2; ++k) {
        const double zi = s * c->XI[k] + t * c->XJ[k], zj = t * c->XI[k] + s * c->XJ[k];
        const double x1 = SQRT2 * o1 * zi + u1, x2 = SQRT2 * o2 * zj + u2;
        const double fval = c->WIWJ[k] * edge_pot(c, x1, x2);
        if (!P->guard_a || a != 0) {
            dp = dp + fval * (p - p * c->XI2aXJ2[k] + 2 * c->XIXJ[k]);
            du1 = du1 + fval * (zi - p * zj);
            du2 = du2 + fval * (zj - p * zi);
            do1 = do1 + fval * (c->XI2aXJ2[k] - 1 + c->XI2mXJ2[k] / sqrtpr);
            do2 = do2 + fval * (c->XI2aXJ2[k] - 1 - c->XI2mXJ2[k] / sqrtpr);
        }
        Ei = Ei + fval;
    }
    du1 = a * du1 * o1pr / M_PI;
    du2 = a * du2 * o2pr / M_PI;
    const double da = Ei / M_PI + T * (const1 + ent_log(sqrtpr * o1 * o2));
    do1 = a * (do1 / M_PI + T) / o1;
    do2 = a * (do2 / M_PI + T) / o2;
    dp = a * (dp / M_PI - T * p) / pr;
    out[0] = da; out[1] = du1; out[2] = du2; out[3] = do1; out[4] = do2; out[5] = dp;
    out[6] = a * da;
}

/* Evaluate both arrayfun kernels over the whole grid (gqmap_gpu_mixture.m:29-34).
 * node: [7][MNL]; edge: [7][MNL*4] in MATLAB order (m,n,l,dir,uv). */
static void eval_grads(const orc_ctx *c, const orc_state *st, double T, double *node,
                       double *edge)
{
    const orc_params *P = c->p;
    const int M = P->M, N = P->N, L = P->L;
    const size_t MN = (size_t)M * N, MNL = MN * L;
#pragma omp parallel for schedule(dynamic, 1)
    for (int n = 0; n < N; ++n) {
        double o[7];
        for (int l = 0; l < L; ++l)
            for (int m = 0; m < M; ++m) {
                const size_t i = m + (size_t)M * n + MN * l;
                if (P->ctf)
                    ctf_node_grad(c, st->muu[i], st->muv[i], st->sigu[i], st->sigv[i], st->pn[i],
                                  m + 1, n + 1, o);
                else
                    node_grad(c, T, st->alpha[l], st->muu[i], st->muv[i], st->sigu[i], st->sigv[i],
                              st->pn[i], m + 1, n + 1, o);
                for (int q = 0; q < 7; ++q) node[q * MNL + i] = o[q];
                for (int dir = 0; dir < 2; ++dir) {
                    /* circshift(X,-1): row m+1 (wrap); circshift(X,-1,2): col n+1 (wrap) */
                    const int m2 = dir == 0 ? (m + 1) % M : m;
                    const int n2 = dir == 1 ? (n + 1) % N : n;
                    const size_t j = m2 + (size_t)M * n2 + MN * l;
                    for (int uv = 0; uv < 2; ++uv) {
                        const double *mu = uv == 0 ? st->muu : st->muv;
                        const double *sg = uv == 0 ? st->sigu : st->sigv;
                        const size_t e = i + MNL * (dir + 2 * uv);
                        if (P->ctf) ctf_edge_grad(c, mu[i], mu[j], sg[i], sg[j], st->rou[e], o);
                        else edge_grad(c, T, st->alpha[l], mu[i], mu[j], sg[i], sg[j], st->rou[e], o);
                        for (int q = 0; q < 7; ++q) edge[q * MNL * 4 + e] = o[q];
                    }
                }
            }
    }
}

void orc_gradients(const orc_params *p, const double *I1, const double *VV,
                   const orc_state *st, double T, double *node_out, double *edge_out,
                   int nthreads)
{
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#endif
    orc_ctx *c = (orc_ctx *)malloc(sizeof(orc_ctx));
    ctx_init(c, p, I1, VV);
    eval_grads(c, st, T, node_out, edge_out);
    free(c);
}

static inline double clampd(double x, double lo, double hi) { return fmin(fmax(x, lo), hi); }

int orc_run(const orc_params *P, const double *I1, const double *VV, orc_state *st,
            double *T_io, int it_first, int n_iter, double *trace, int nthreads)
{
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#endif
    const int M = P->M, N = P->N, L = P->L;
    const size_t MN = (size_t)M * N, MNL = MN * L;
    orc_ctx *c = (orc_ctx *)malloc(sizeof(orc_ctx));
    ctx_init(c, P, I1, VV);
    double *node = (double *)malloc(sizeof(double) * 7 * MNL);
    double *edge = (double *)malloc(sizeof(double) * 7 * MNL * 4);
    double *g[4]; /* assembled dmuu, dmuv, dsigmau, dsigmav */
    for (int q = 0; q < 4; ++q) g[q] = (double *)malloc(sizeof(double) * MNL);
    double T = *T_io;
    int done = 0;
    for (int it = it_first; it < it_first + n_iter; ++it) {
        const double step = P->step0 / (1 + it / P->step_decay);
        eval_grads(c, st, T, node, edge);
        const double *dan = node, *nE = node + 6 * MNL;
        const double *dae = edge, *dmu1 = edge + 1 * 4 * MNL, *dmu2 = edge + 2 * 4 * MNL;
        const double *dsg1 = edge + 3 * 4 * MNL, *dsg2 = edge + 4 * 4 * MNL;
        const double *drou = edge + 5 * 4 * MNL, *eE = edge + 6 * 4 * MNL;
        /* dalpha (:36): interior sums, m fastest then n */
        double dalpha[64];
        for (int l = 0; l < L; ++l) {
            double sn = 0, se = 0;
            for (int n = 1; n < N - 1; ++n) {
                double col = 0;
                for (int m = 1; m < M - 1; ++m) col += dan[m + (size_t)M * n + MN * l];
                sn += col;
            }
            for (int uv = 0; uv < 2; ++uv)
                for (int dir = 0; dir < 2; ++dir) {
                    double sd = 0;
                    for (int n = 1; n < N - 1; ++n) {
                        double col = 0;
                        for (int m = 1; m < M - 1; ++m)
                            col += dae[m + (size_t)M * n + MN * l + MNL * (dir + 2 * uv)];
                        sd += col;
                    }
                    se += sd;
                }
            dalpha[l] = sn + se;
        }
        /* gradient assembly (:37-40) with circshift(+1) neighbour scatter */
#pragma omp parallel for
        for (int n = 0; n < N; ++n)
            for (int l = 0; l < L; ++l)
                for (int m = 0; m < M; ++m) {
                    const size_t i = m + (size_t)M * n + MN * l;
                    const size_t iu = (size_t)((m + M - 1) % M) + (size_t)M * n + MN * l;
                    const size_t il = m + (size_t)M * ((n + N - 1) % N) + MN * l;
                    for (int uv = 0; uv < 2; ++uv) {
                        const size_t o0 = MNL * (0 + 2 * uv), o1 = MNL * (1 + 2 * uv);
                        g[uv][i] = node[(1 + uv) * MNL + i] + (dmu1[o0 + i] + dmu1[o1 + i]) +
                                   dmu2[o0 + iu] + dmu2[o1 + il];
                        g[2 + uv][i] = node[(3 + uv) * MNL + i] + (dsg1[o0 + i] + dsg1[o1 + i]) +
                                       dsg2[o0 + iu] + dsg2[o1 + il];
                    }
                }
        /* clamped ascent on the interior (:41-46) */
#pragma omp parallel for
        for (int n = 1; n < N - 1; ++n)
            for (int l = 0; l < L; ++l)
                for (int m = 1; m < M - 1; ++m) {
                    const size_t i = m + (size_t)M * n + MN * l;
                    st->muu[i] = clampd(st->muu[i] + g[0][i] * step, P->minu, P->maxu);
                    st->muv[i] = clampd(st->muv[i] + g[1][i] * step, P->minv, P->maxv);
                    if (P->ctf) { /* gqmap_ctf.m:34-35: dsigmau*step*0.3 */
                        st->sigu[i] = clampd(st->sigu[i] + g[2][i] * step * P->sig_step, P->sig_lo, P->sig_hi);
                        st->sigv[i] = clampd(st->sigv[i] + g[3][i] * step * P->sig_step, P->sig_lo, P->sig_hi);
                    } else {
                        st->sigu[i] = clampd(st->sigu[i] + g[2][i] * step, P->sig_lo, P->sig_hi);
                        st->sigv[i] = clampd(st->sigv[i] + g[3][i] * step, P->sig_lo, P->sig_hi);
                    }
                    for (int e = 0; e < 4; ++e)
                        st->rou[i + MNL * e] = clampd(st->rou[i + MNL * e] + drou[i + MNL * e] * step,
                                                      -P->corr_tor, P->corr_tor);
                    st->pn[i] = clampd(st->pn[i] + node[5 * MNL + i] * step, -P->corr_tor, P->corr_tor);
                }
        /* Energy (:48) */
        double En = 0, Ee = 0;
        for (int l = 0; l < L; ++l)
            for (int n = 1; n < N - 1; ++n)
                for (int m = 1; m < M - 1; ++m) En += nE[m + (size_t)M * n + MN * l];
        for (int e = 0; e < 4; ++e)
            for (int l = 0; l < L; ++l)
                for (int n = 1; n < N - 1; ++n)
                    for (int m = 1; m < M - 1; ++m) Ee += eE[m + (size_t)M * n + MN * l + MNL * e];
        const double energy = En + Ee;
        /* alpha update (:50, :78-86) or projsplx (:49, commented in the reference) */
        if (it > P->alpha_start && L != 1) {
            if (P->alpha_mode == 0) {
                double sda = 0;
                for (int l = 0; l < L; ++l) sda += dalpha[l] * st->alpha[l];
                double se = 0, ew[64];
                for (int l = 0; l < L; ++l) {
                    const double dw = st->alpha[l] * (dalpha[l] - sda);
                    st->w[l] = clampd(st->w[l] + dw * step * P->alpha_lr, -300, 300);
                    ew[l] = exp(st->w[l]);
                    se += ew[l];
                }
                for (int l = 0; l < L; ++l) st->alpha[l] = ew[l] / se;
            } else {
                double y[64];
                for (int l = 0; l < L; ++l) y[l] = st->alpha[l] + dalpha[l] * step * P->alpha_lr;
                orc_projsplx(y, st->alpha, L);
            }
        }
        /* ptdmu / ptdsigma (:69-70) */
        double smu = 0, ssg = 0;
        for (int l = 0; l < L; ++l)
            for (int n = 1; n < N - 1; ++n)
                for (int m = 1; m < M - 1; ++m) {
                    const size_t i = m + (size_t)M * n + MN * l;
                    smu += fabs(g[0][i]);
                    ssg += fabs(g[2][i]);
                }
        const double cnt = (double)(M - 2) * (N - 2) * L;
        const double ptdmu = smu / cnt, ptdsig = ssg / cnt;
        trace[3 * done + 0] = energy;
        trace[3 * done + 1] = ptdmu;
        trace[3 * done + 2] = ptdsig;
        /* temperature decay (gqmap_gpuSuper_mix_entropy.m:72) */
        if (P->t_decay_every > 0 && it % P->t_decay_every == 0) T = fmax(T * P->drate, P->t_min);
        ++done;
        if (ptdmu < P->tor) break;
    }
    *T_io = T;
    for (int q = 0; q < 4; ++q) free(g[q]);
    free(node); free(edge); free(c);
    return done;
}

/* projsplx.m:15-30 */
static int cmp_desc(const void *a, const void *b)
{
    double x = *(const double *)a, y = *(const double *)b;
    return (x < y) - (x > y);
}
void orc_projsplx(const double *y, double *x, int m)
{
    double s[256];
    memcpy(s, y, sizeof(double) * m);
    qsort(s, m, sizeof(double), cmp_desc);
    double tmpsum = 0, tmax = 0;
    int bget = 0;
    for (int ii = 0; ii < m - 1; ++ii) {
        tmpsum = tmpsum + s[ii];
        tmax = (tmpsum - 1) / (ii + 1);
        if (tmax >= s[ii + 1]) { bget = 1; break; }
    }
    if (!bget) tmax = (tmpsum + s[m - 1] - 1) / m;
    for (int i = 0; i < m; ++i) x[i] = fmax(y[i] - tmax, 0);
}

/* ------------------------------------------------------------------ */
/* flowToColor.m / computeColor.m                                      */
/* ------------------------------------------------------------------ */
static void make_colorwheel(double cw[55][3])
{
    const int RY = 15, YG = 6, GC = 4, CB = 11, BM = 13, MR = 6;
    memset(cw, 0, sizeof(double) * 55 * 3);
    int col = 0;
    for (int i = 0; i < RY; ++i) { cw[i][0] = 255; cw[i][1] = floor(255.0 * i / RY); }
    col += RY;
    for (int i = 0; i < YG; ++i) { cw[col + i][0] = 255 - floor(255.0 * i / YG); cw[col + i][1] = 255; }
    col += YG;
    for (int i = 0; i < GC; ++i) { cw[col + i][1] = 255; cw[col + i][2] = floor(255.0 * i / GC); }
    col += GC;
    for (int i = 0; i < CB; ++i) { cw[col + i][1] = 255 - floor(255.0 * i / CB); cw[col + i][2] = 255; }
    col += CB;
    for (int i = 0; i < BM; ++i) { cw[col + i][2] = 255; cw[col + i][0] = floor(255.0 * i / BM); }
    col += BM;
    for (int i = 0; i < MR; ++i) { cw[col + i][2] = 255 - floor(255.0 * i / MR); cw[col + i][0] = 255; }
}

void orc_flow_to_color(const double *flow, int M, int N, double max_flow, unsigned char *img,
                       double *flo, double *stats, unsigned char *unknown)
{
    const size_t MN = (size_t)M * N;
    double maxu = -999, maxv = -999, minu = 999, minv = 999, maxrad = -1;
    double *u = (double *)malloc(sizeof(double) * MN), *v = (double *)malloc(sizeof(double) * MN);
    for (size_t i = 0; i < MN; ++i) {
        u[i] = flow[i]; v[i] = flow[MN + i];
        unknown[i] = (fabs(u[i]) > 1e9) || (fabs(v[i]) > 1e9);
        if (unknown[i]) { u[i] = 0; v[i] = 0; }
        flo[i] = u[i]; flo[MN + i] = v[i];
    }
    /* MATLAB max/min ignore NaN */
    for (size_t i = 0; i < MN; ++i) {
        if (!isnan(u[i])) { maxu = fmax(maxu, u[i]); minu = fmin(minu, u[i]); }
        if (!isnan(v[i])) { maxv = fmax(maxv, v[i]); minv = fmin(minv, v[i]); }
        const double rad = sqrt(u[i] * u[i] + v[i] * v[i]);
        if (!isnan(rad)) maxrad = fmax(maxrad, rad);
    }
    if (max_flow > 0) maxrad = max_flow;
    stats[0] = minu; stats[1] = maxu; stats[2] = minv; stats[3] = maxv;
    double cw[55][3];
    make_colorwheel(cw);
    const int ncols = 55;
    for (size_t i = 0; i < MN; ++i) {
        double uu = u[i] / (maxrad + DBL_EPSILON), vv = v[i] / (maxrad + DBL_EPSILON);
        const int nan_ = isnan(uu) || isnan(vv);
        if (nan_) { uu = 0; vv = 0; }
        const double rad = sqrt(uu * uu + vv * vv);
        const double a = atan2(-vv, -uu) / M_PI;
        const double fk = (a + 1) / 2 * (ncols - 1) + 1;
        const int k0 = (int)floor(fk);
        int k1 = k0 + 1;
        if (k1 == ncols + 1) k1 = 1;
        const double f = fk - k0;
        for (int ch = 0; ch < 3; ++ch) {
            const double col0 = cw[k0 - 1][ch] / 255, col1 = cw[k1 - 1][ch] / 255;
            double col = (1 - f) * col0 + f * col1;
            if (rad <= 1) col = 1 - rad * (1 - col);
            else col = col * 0.75;
            double q = floor(255 * col * (1 - nan_));
            if (q < 0) q = 0;
            if (q > 255) q = 255;
            img[i + MN * ch] = unknown[i] ? 0 : (unsigned char)q;
        }
    }
    free(u); free(v);
}

double orc_aepe(const double *tflow, const double *flow, const unsigned char *unknown, int M,
                int N, int r0)
{
    const size_t MN = (size_t)M * N;
    double s = 0;
    for (int n = r0; n < N - r0; ++n) {
        double col = 0;
        for (int m = r0; m < M - r0; ++m) {
            const size_t i = m + (size_t)M * n;
            const double fu = unknown[i] ? 0 : flow[i], fv = unknown[i] ? 0 : flow[MN + i];
            const double du = tflow[i] - fu, dv = tflow[MN + i] - fv;
            col += sqrt(du * du + dv * dv);
        }
        s += col / (M - 2 * r0);
    }
    return s / (N - 2 * r0);
}

/* profile_logP (gqmap_gpu_mixture.m:148-154; super gqmap_gpuSuper_mix_entropy.m:
 * 152-169).  map is the M x N x 2 MAP flow on the node grid.
 *   np = arrayfun(@node_pot, us, vs, ms, ns)    (super: node_lp, the 4x4 block
 *                                                sum of node_pot, :160-169)
 *   ep = arrayfun(@edge_pot, cat(4,uv,uv), cat(4,circshift(uv,-1),circshift(uv,-1,2)))
 *   lp = sum(sum(np(M_,N_))) + sum(sum(sum(sum(ep(M_,N_,:,:)))))
 * with M_ = 2:M-1, N_ = 2:N-1.  MATLAB's sum order: down each column, then
 * across the columns (ep: then over the uv and direction planes). */
double orc_log_p(const orc_params *p, const double *I1, const double *VV, const double *map)
{
    orc_ctx c;
    ctx_init(&c, p, I1, VV);
    const int M = p->M, N = p->N;
    const size_t MN = (size_t)M * N;
    double snp = 0;
    for (int n = 2; n <= N - 1; ++n) {  /* 1-based node columns */
        double col = 0;
        for (int m = 2; m <= M - 1; ++m) {
            const size_t i = (m - 1) + (size_t)M * (n - 1);
            const double x1 = map[i], x2 = map[MN + i];
            double v;
            if (p->super_) {
                const int bottom = 4 * m, top = bottom - 3, right = 4 * n, left = right - 3;
                v = 0;
                for (int ii = top; ii <= bottom; ++ii)
                    for (int jj = left; jj <= right; ++jj) v = v + node_pot(&c, x1, x2, ii, jj);
            } else {
                v = node_pot(&c, x1, x2, m, n);
            }
            col += v;
        }
        snp += col;
    }
    /* ep(:,:,uv,dir): dir 1 pairs (m,n) with circshift(uv,-1) = (m+1,n), dir 2
     * with circshift(uv,-1,2) = (m,n+1) (wrapping, as circshift does) */
    double sep = 0;
    for (int dir = 0; dir < 2; ++dir) {
        double sdir = 0;
        for (int uv = 0; uv < 2; ++uv) {
            double suv = 0;
            for (int n = 1; n <= N - 2; ++n) {
                double col = 0;
                for (int m = 1; m <= M - 2; ++m) {
                    const int m2 = dir == 0 ? (m + 1) % M : m, n2 = dir == 1 ? (n + 1) % N : n;
                    col += edge_pot(&c, map[MN * uv + m + (size_t)M * n], map[MN * uv + m2 + (size_t)M * n2]);
                }
                suv += col;
            }
            sdir += suv;
        }
        sep += sdir;
    }
    return snp + sep;
}

/* ------------------------------------------------------------------ */
/* Mixture MAP (findMixMax.m:39-70) with MATLAB fminbnd (Brent)         */
/* ------------------------------------------------------------------ */
/* exp used by the mixture density: libm by default; orc_set_map_exp()
 * swaps in another implementation (the device's deterministic gq_exp from
 * the emulator) so the MAP restatement can be compared bit for bit.  The
 * reference's get_map_mex uses its own runtime's exp (parity unpinned). */
static double (*map_exp)(double) = exp;
void orc_set_map_exp(double (*f)(double)) { map_exp = f ? f : exp; }

static double neg_mix(double x, const double *a, const double *u, const double *o, int L)
{
    double v = 0;
    for (int l = 0; l < L; ++l) {
        const double z = (x - u[l]) / o[l];
        v += a[l] * (map_exp(-0.5 * z * z) / (sqrt(2 * M_PI) * o[l]));
    }
    return -v;
}

static double fminbnd(const double *al, const double *u, const double *o, int L, double ax,
                      double bx, double *fval)
{
    const double tol = 1e-4, seps = sqrt(DBL_EPSILON), c = 0.5 * (3.0 - sqrt(5.0));
    double a = ax, b = bx, v = a + c * (b - a), w = v, xf = v, d = 0.0, e = 0.0, x = xf;
    double fx = neg_mix(x, al, u, o, L), fv = fx, fw = fx;
    double xm = 0.5 * (a + b), tol1 = seps * fabs(xf) + tol / 3.0, tol2 = 2.0 * tol1;
    int num = 1, iter = 0;
    while (fabs(xf - xm) > (tol2 - 0.5 * (b - a))) {
        int gs = 1;
        if (fabs(e) > tol1) {
            gs = 0;
            double r = (xf - w) * (fx - fv);
            double q = (xf - v) * (fx - fw);
            double p = (xf - v) * q - (xf - w) * r;
            q = 2.0 * (q - r);
            if (q > 0.0) p = -p;
            q = fabs(q);
            r = e; e = d;
            if ((fabs(p) < fabs(0.5 * q * r)) && (p > q * (a - xf)) && (p < q * (b - xf))) {
                d = p / q;
                x = xf + d;
                if (((x - a) < tol2) || ((b - x) < tol2)) {
                    const double si = (xm - xf > 0) - (xm - xf < 0) + ((xm - xf) == 0);
                    d = tol1 * si;
                }
            } else {
                gs = 1;
            }
        }
        if (gs) {
            e = (xf >= xm) ? a - xf : b - xf;
            d = c * e;
        }
        const double si = (d > 0) - (d < 0) + (d == 0);
        x = xf + si * fmax(fabs(d), tol1);
        const double fu = neg_mix(x, al, u, o, L);
        ++num; ++iter;
        if (fu <= fx) {
            if (x >= xf) a = xf; else b = xf;
            v = w; fv = fw; w = xf; fw = fx; xf = x; fx = fu;
        } else {
            if (x < xf) a = x; else b = x;
            if ((fu <= fw) || (w == xf)) { v = w; fv = fw; w = x; fw = fu; }
            else if ((fu <= fv) || (v == xf) || (v == w)) { v = x; fv = fu; }
        }
        xm = 0.5 * (a + b);
        tol1 = seps * fabs(xf) + tol / 3.0;
        tol2 = 2.0 * tol1;
        if (num >= 500 || iter >= 500) break;
    }
    *fval = fx;
    return xf;
}

static double find_max_1d(const double *al, const double *u, const double *o, int L)
{
    double spike = INFINITY;
    int uid = 0;
    double lo = u[0], hi = u[0];
    for (int l = 0; l < L; ++l) {
        const double f = neg_mix(u[l], al, u, o, L);
        if (f < spike) { spike = f; uid = l; }
        lo = fmin(lo, u[l]); hi = fmax(hi, u[l]);
    }
    double fval;
    const double x = fminbnd(al, u, o, L, lo, hi, &fval);
    return fval < spike ? x : u[uid];
}

void orc_get_map(const double *alpha, const double *muu, const double *sigu, const double *muv,
                 const double *sigv, int M, int N, int L, double *out, int nthreads)
{
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#endif
    const size_t MN = (size_t)M * N;
#pragma omp parallel for
    for (int n = 0; n < N; ++n)
        for (int m = 0; m < M; ++m) {
            double u1[64], o1[64], u2[64], o2[64];
            const size_t i = m + (size_t)M * n;
            for (int l = 0; l < L; ++l) {
                u1[l] = muu[i + MN * l]; o1[l] = sigu[i + MN * l];
                u2[l] = muv[i + MN * l]; o2[l] = sigv[i + MN * l];
            }
            out[i] = find_max_1d(alpha, u1, o1, L);
            out[MN + i] = find_max_1d(alpha, u2, o2, L);
        }
}
