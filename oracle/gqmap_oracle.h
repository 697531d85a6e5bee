/*
 * gqmap_oracle.h -- CPU restatement of the QGMAP hot path (fp64).
 *
 * TEST INFRASTRUCTURE ONLY.  This library is the parity checker and the timed
 * CPU baseline.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load it.  The product path (libgqmap.so) never links,
 * loads or calls anything under oracle/.
 *
 * Parity status: the reference is MATLAB (no MATLAB/Octave here, MEX binaries
 * are Windows-only), so the solver loop is pinned by (i) known-answer tests
 * (Gauss-Hermite == numpy.hermgauss, Keys cubic reproduces quadratics, colour
 * wheel table, .flo GT round trip) and (ii) agreement with an independent
 * numpy restatement of the same MATLAB lines (oracle/gqmap_np.py, committed
 * goldens under tests/golden/).  No output of the reference itself exists, so
 * end-to-end solver parity against MATLAB is "parity unpinned".
 *
 * Every array is MATLAB column-major (row index m fastest).
 */
#ifndef GQMAP_ORACLE_H
#define GQMAP_ORACLE_H
#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
    int M, N;            /* node grid; super: Mo/4 x No/4                      */
    int Mo, No;          /* image size (rows, cols)                            */
    int L, K;            /* mixture components, quadrature order               */
    int super_;          /* 0: gqmap_gpu_mixture.m, 1: gqmap_gpuSuper_mix_entropy.m */
    int guard_a;         /* `if a~=0` guard (gqmap_gpu_mixture.m:98)           */
    double T, drate, t_min; int t_decay_every;   /* gqmap_gpuSuper_mix_entropy.m:72 */
    double epsn, lambdad, lambdas;
    double minu, maxu, minv, maxv;
    double step0, step_decay;                    /* step = step0/(1+it/step_decay) */
    double sig_lo, sig_hi, corr_tor;
    int alpha_mode;      /* 0 softmax (gqmap_gpu_mixture.m:78-86), 1 projsplx (:49) */
    int alpha_start;     /* alpha update when it > alpha_start (:50)           */
    double alpha_lr;     /* 1e-7                                               */
    double tor;          /* stop when ptdmu < tor (:75)                        */
    int ctf;             /* 1: legacy/gqmap_ctf.m level solver (rounded I2_cont lookup) */
    double sig_step;     /* sigma step scale (ctf: 0.3, gqmap_ctf.m:34-35)     */
    /* Gauss-Hermite rule (K nodes ascending, weights): NULL = this library's
     * restatement of GaussHermite_2.m (orc_gauss_hermite); otherwise the
     * caller's rule, so the iteration arithmetic can be compared bit for bit
     * with an engine that uses another (equally accurate) rule. */
    const double *gh_x, *gh_w;
} orc_params;

typedef struct {
    double *muu, *muv, *sigu, *sigv, *pn;   /* [M*N*L]          */
    double *rou;                            /* [M*N*L*2*2]      */
    double *w, *alpha;                      /* [L]              */
} orc_state;

/* GaussHermite_2.m:21-32 -- eig of the symmetric Jacobi matrix (cyclic Jacobi). */
void orc_gauss_hermite(int K, double *x, double *w);
/* getVV (gqmap_gpu_mixture.m:191-208): (M+2)x(N+2) cubic-convolution pad. */
void orc_get_vv(const double *I2, int M, int N, double *VV);
/* node_pot (gqmap_gpu_mixture.m:156-179), 1-based (i,j), for KATs. */
double orc_interp_cubic(const double *VV, int M, int N, double Xq, double Yq);

/* Run iterations it_first .. it_first+n_iter-1 of the engine loop
 * (gqmap_gpu_mixture.m:26-76 / gqmap_gpuSuper_mix_entropy.m:25-75).
 * trace[3*i] = Energy, ptdmu, ptdsigma.  *T_io carries the temperature.
 * Returns the number of iterations executed (stops early when ptdmu < tor). */
int orc_run(const orc_params *p, const double *I1, const double *VV, orc_state *st,
            double *T_io, int it_first, int n_iter, double *trace, int nthreads);

/* One-iteration gradient dump for fine-grained parity: all node/edge outputs
 * before the update.  node_out [7][M*N*L]: da,du1,du2,do1,do2,dp,E ;
 * edge_out [7][M*N*L*4] in MATLAB order (m,n,l,dir,uv). */
void orc_gradients(const orc_params *p, const double *I1, const double *VV,
                   const orc_state *st, double T, double *node_out, double *edge_out,
                   int nthreads);

/* The log of the entropy terms: NULL = libm log (default), else f. */
void orc_set_ent_log(double (*f)(double));

/* projsplx.m:15-30 */
void orc_projsplx(const double *y, double *x, int n);

/* flowToColor.m:37-87 + computeColor.m:33-115.  flow [M*N*2].
 * img [M*N*3] uint8, flo [M*N*2], stats = {minu,maxu,minv,maxv}, unknown [M*N]. */
void orc_flow_to_color(const double *flow, int M, int N, double max_flow,
                       unsigned char *img, double *flo, double *stats,
                       unsigned char *unknown);

/* AEPE over the interior window rows r0..M-1-r0, cols r0..N-1-r0 (0-based),
 * flow(unknown)=0 first (gqmap_gpu_mixture.m:63-64). */
double orc_aepe(const double *tflow, const double *flow, const unsigned char *unknown,
                int M, int N, int r0);

/* profile_logP (gqmap_gpu_mixture.m:148-154; super node_lp,
 * gqmap_gpuSuper_mix_entropy.m:152-169) of the M x N x 2 MAP flow `map`. */
double orc_log_p(const orc_params *p, const double *I1, const double *VV, const double *map);

/* findMixMax.m:39-70 semantics: per pixel, best of component means vs
 * fminbnd (Brent, TolX=1e-4) on [min mu, max mu].  out [M*N*2]. */
void orc_get_map(const double *alpha, const double *muu, const double *sigu,
                 const double *muv, const double *sigv, int M, int N, int L,
                 double *out, int nthreads);

/* ---- coarse-to-fine plumbing (gqmap_pyramid_oracle.c) ----------------- */
/* imresize.m contributions(): taps before/after removing all-zero columns */
int orc_resize_taps(double scale, int antialias);
int orc_resize_contrib(int in_len, int out_len, double scale, int antialias, double *w, int *idx);
int orc_resize_len(int len, double scale);
/* imresize(A, scale) bicubic (+antialias for scale<1), A M x N x C */
void orc_imresize(const double *in, int M, int N, int C, double scale, int antialias, double *out);
/* interp2(V, x-warp(:,:,1), y-warp(:,:,2)) linear, NaN outside */
void orc_warp_image(const double *V, int M, int N, const double *warp, double *out);
/* fillmissing(A,'nearest',dim) in place */
void orc_fillmissing_nearest(double *A, int M, int N, int dim);

/* ---- legacy flow-denoising engine legacy/gqmap_cpu.m (gqmap_legacy_oracle.c) */
typedef struct {
    int its, K;
    double var, gama, dta;          /* options.var / gama / dta (never set in the reference) */
    double step0, step_decay;       /* step = 0.1/(1+it/1000) (:62)                          */
    double corr_tor;                /* rou clamp 0.97 (:65)                                  */
    double tor;                     /* stop: it > min_its && max|dmu| < tor (:70)            */
    int min_its;                    /* 100                                                   */
} orc_cpu_params;
/* flow M x N x 2; mu/sigma (M x N x 2) and rou (M x N x 2 x 2) hold the initial
 * state on entry (mu = flow, sigma = rand + 2, rou = 0 in the reference) and
 * the result on exit; trace[3*i] = max|dmu|, max|dsigma|, max|drou| of
 * iteration i+1.  Returns the number of iterations run. */
/* exp of the mixture density in orc_get_map (NULL: libm exp). */
void orc_set_map_exp(double (*f)(double));
int orc_cpu_run(const orc_cpu_params *P, const double *X, const double *W, const double *flow, int M, int N,
                double *mu, double *sigma, double *rou, double *trace, int nthreads);

#ifdef __cplusplus
}
#endif
#endif
