/*
 * gqmap.h -- C ABI of the MI355X-native QGMAP optical-flow hot path.
 *
 * This is the drop-in boundary.  The reference's engines are MATLAB
 * functions called from the driver scripts:
 *
 *   [mu,sigma,alpha,AEPE,Energy,logP] = gqmap_gpu_mixture(options,I1,I2)
 *        -- gqmap_gpu_mixture.m:1          (called from optical_flow.m:27)
 *   [mu,sigma,alpha,AEPE,Energy,logP] = gqmap_gpuSuper_mix_entropy(options,I1,I2)
 *        -- gqmap_gpuSuper_mix_entropy.m:1 (called from optical_flowSuper.m:34)
 *   [mu,sigma,rou,AEPE,Energy]        = gqmap_ctf(options,I1,I2,GRDT)
 *        -- legacy/gqmap_ctf.m:1           (called from legacy/optical_flow_ctf.m:33)
 *
 * A MEX gateway (mex/gqmap_gpu_mixture_mex.cpp) shadows
 * the .m files on the MATLAB path and forwards to these entry points.  The
 * host-side bookkeeping that stays in MATLAB (AEPE every 300 its, PNG
 * snapshots, fprintf) is reproduced by the Python mirror in
 * gqmap_opticalflow_amd/engine.py.
 *
 * Conventions: plain C types only; every array is caller-owned host memory in
 * MATLAB column-major order (row index m fastest); every call returns a
 * gqmap_status and gqmap_last_error() gives a message for the calling thread.
 * One context per host thread; a context owns one HIP stream on one device.
 */
#ifndef GQMAP_H
#define GQMAP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GQMAP_ABI_VERSION 2  /* 2: gqmap_options.arith */
#define GQMAP_LMAX 8   /* mixture components supported (reference uses L<=3) */
#define GQMAP_KMAX 16  /* quadrature order supported (reference uses K=9, 11) */

typedef enum gqmap_status {
    GQMAP_OK = 0,
    GQMAP_ERR_INVALID_ARG = 1,
    GQMAP_ERR_HIP = 2,
    GQMAP_ERR_OUT_OF_MEMORY = 3,
    GQMAP_ERR_NO_DEVICE = 4,
    GQMAP_ERR_STATE = 5,       /* e.g. run before set_images / set_state       */
    GQMAP_ERR_UNSUPPORTED = 6
} gqmap_status;

typedef enum gqmap_engine_kind {
    GQMAP_ENGINE_MIXTURE = 0,  /* gqmap_gpu_mixture.m: one node per pixel          */
    GQMAP_ENGINE_SUPER = 1,    /* gqmap_gpuSuper_mix_entropy.m: one node per 4x4   */
    GQMAP_ENGINE_CTF = 2       /* legacy/gqmap_ctf.m: one pyramid level, L=1       */
} gqmap_engine_kind;

typedef enum gqmap_precision { GQMAP_FP64 = 0, GQMAP_FP32 = 1 } gqmap_precision;
/* gqmap_options.split: Q = 1 arithmetic, node and edge phases on separate waves */
#define GQMAP_SPLIT_ROLE (-1)
/* gqmap_options.arith: the order of the per-node arithmetic.
 *  FAST    the kernel's specification (gqmap_math.h: basis sums, fma, 1/pi
 *          folded into a scale) -- within a rounding or two per gradient of
 *          the reference's expressions, the fastest form.
 *  LITERAL every expression of node_grad_spectral / edge_grad_spectral /
 *          node_pot / edge_pot (gqmap_gpu_mixture.m:87-182) in MATLAB's
 *          expression order under non-fused IEEE semantics (left to right,
 *          every operation correctly rounded).  That is how the .m source
 *          reads; the reference itself ran arrayfun JIT-compiled for the
 *          GPU, which may contract to FMA, so this is a restatement of the
 *          source's order, not a replay of what MATLAB executed.  Bit-identical to the
 *          literal restatement oracle/gqmap_oracle.c while the alpha update
 *          is off (L = 1, or it <= alpha_start).  fp64 mixture engine only,
 *          one lane per node (split 0 or 1). */
typedef enum gqmap_arith { GQMAP_ARITH_FAST = 0, GQMAP_ARITH_LITERAL = 1 } gqmap_arith;
typedef enum gqmap_alpha_mode {
    GQMAP_ALPHA_SOFTMAX = 0,   /* updateAlpha, gqmap_gpu_mixture.m:78-86 (live path)   */
    GQMAP_ALPHA_PROJSPLX = 1   /* projsplx(alpha+dalpha*step*lr), :49 (commented out)   */
} gqmap_alpha_mode;

/* Options.  The first block mirrors the MATLAB `options` fields read by the
 * engines (gqmap_gpu_mixture.m:3-6); the second block holds constants that
 * are hard-coded in the reference source -- gqmap_options_default() fills
 * them with the reference values for the chosen engine. */
typedef struct gqmap_options {
    int its, K, L;
    double temperature, drate, epsn, lambdad, lambdas;
    double minu, maxu, minv, maxv;
    /* --- engine knobs (reference constants) --- */
    int engine;          /* gqmap_engine_kind                                    */
    int precision;       /* gqmap_precision                                      */
    int alpha_mode;      /* gqmap_alpha_mode                                     */
    int alpha_start;     /* alpha update when it > alpha_start        (500, :50) */
    double alpha_lr;     /* 1e-7                                        (:83)     */
    int guard_a;         /* `if a~=0` guard: 1 mixture (:98), 0 super             */
    int t_decay_every;   /* 0 mixture (:73 commented), 500 super (super:72)       */
    double t_min;        /* 0.001 (super:72)                                     */
    double step0;        /* 0.1 mixture (:27), 0.001 super (super:26)            */
    double step_decay;   /* 8000 mixture, 4000 super                             */
    double sig_lo, sig_hi;  /* 0.01 / 23 mixture (:43-44), 0.01 / 25 super       */
    double corr_tor;     /* 1-1e-5 (:7)                                          */
    double tor;          /* 1e-4 stop threshold on ptdmu (:25,75)                */
    int split;           /* lanes per node Q (1/2/4/8/16/64), 0 = auto from the grid
                            size; part of the arithmetic (partial quadrature sums);
                            GQMAP_SPLIT_ROLE: Q = 1 arithmetic with the node and
                            edge phases on separate waves (mid-size grids)       */
    double sig_step;     /* sigma step scale: 1, ctf 0.3 (gqmap_ctf.m:34-35)     */
    double sig_init;     /* init sigma = U + sig_init; < 0: U + (max - min)      */
    int arith;           /* gqmap_arith (ABI 2)                                  */
} gqmap_options;

/* Engine state, MATLAB layout (M x N x L [x 2 x 2]).  M,N = node grid
 * (image size for MIXTURE, image size / 4 for SUPER).  `it` is the index of
 * the next iteration (1-based, as in the reference loop); T the temperature.
 * The reference returns mu/sigma/alpha only (gqmap_gpu_mixture.m:183-185);
 * this ABI also carries pn, rou, w so a run can be checkpointed/resumed. */
typedef struct gqmap_state {
    double *muu, *muv, *sigu, *sigv, *pn;  /* [M*N*L]        */
    double *rou;                           /* [M*N*L*2*2]    */
    double *w, *alpha;                     /* [L]            */
    int it;
    double T;
} gqmap_state;

typedef struct gqmap_info {
    int Mo, No;          /* image size         */
    int M, N, L, K;      /* node grid          */
    int it;              /* next iteration     */
    int stopped;         /* ptdmu < tor reached */
    double T;
    int device;
    int split;           /* lanes per node Q in use                             */
    int n_tiles, tile;   /* column-strip tiling (1, 0 for a whole-grid context) */
    int col0, col1;      /* node columns [col0, col1) owned by this context     */
} gqmap_info;

typedef struct gqmap_ctx gqmap_ctx;

/* ---- engine (gqmap_gpu_mixture.m / gqmap_gpuSuper_mix_entropy.m) ---- */
void gqmap_options_default(gqmap_options *opt, int engine);
/* Select the alpha update and set alpha_start / alpha_lr to the reference
 * constants of that mode for opt->engine: softmax (updateAlpha) it>500,
 * 1e-7 (gqmap_gpu_mixture.m:50,83; gqmap_gpuSuper_mix_entropy.m:49,82);
 * projsplx: mixture it>500, 1e-7 (gqmap_gpu_mixture.m:49), super it>200,
 * 1e-6 (gqmap_gpuSuper_mix_entropy.m:48).  Call after gqmap_options_default. */
gqmap_status gqmap_options_alpha_mode(gqmap_options *opt, int mode);
gqmap_status gqmap_create(gqmap_ctx **out, const gqmap_options *opt, int device);
/* I1,I2: Mo x No doubles (greyscale 0..255).  SUPER needs Mo,No divisible by 4.
 * Builds the cubic-convolution padded copy of I2 (getVV, gqmap_gpu_mixture.m:191). */
gqmap_status gqmap_set_images(gqmap_ctx *ctx, const double *I1, const double *I2, int Mo, int No);
/* Initial state exactly as gqmap_gpu_mixture.m:18-24 with this library's
 * counter-based RNG (SplitMix64; gqmap_rand_uniform) in place of MATLAB's
 * rand(...,'gpuArray'), generated on the device. */
gqmap_status gqmap_init_state(gqmap_ctx *ctx, uint64_t seed);
gqmap_status gqmap_set_state(gqmap_ctx *ctx, const gqmap_state *st);
gqmap_status gqmap_get_state(gqmap_ctx *ctx, gqmap_state *st);
/* Run up to n_iter iterations (one iteration = gqmap_gpu_mixture.m:27-75
 * minus the host evaluation block).  Stops early when ptdmu < tor.
 * trace (optional, n_iter*3): Energy, ptdmu, ptdsigma per executed iteration. */
gqmap_status gqmap_run(gqmap_ctx *ctx, int n_iter, int *n_done, double *trace);
/* Same as gqmap_run with n_iter iterations, timed on the context's stream
 * with HIP events: total_ms over all launches, iter_kernel_ms = sum of the
 * fused iteration kernel's durations (event pair around each launch). */
/* Ground truth of the ctf level engine: GRDT Mg x Ng x 2 (Mg >= M, Ng >= N;
 * its top-left M x N block is used, as gqmap_ctf.m:38 indexes GRDT(M_,N_,:)
 * of whatever it is passed).  NULL clears it.  With a truth set every
 * iteration also reduces the AEPE of the updated mean on the device. */
gqmap_status gqmap_set_truth(gqmap_ctx *ctx, const double *grdt, int Mg, int Ng);
/* gqmap_run plus aepe[n_done] (optional): the per-iteration AEPE of
 * gqmap_ctf.m:38 (NaN when no truth is set) -- the reference's AEPE output. */
gqmap_status gqmap_run_aepe(gqmap_ctx *ctx, int n_iter, int *n_done, double *trace, double *aepe);
gqmap_status gqmap_run_timed(gqmap_ctx *ctx, int n_iter, int *n_done, double *total_ms,
                             double *iter_kernel_ms);
/* Capture and upload the replayed iteration graph now (gqmap_run otherwise
 * builds it on its first call of >= 50 iterations): no iteration runs. */
gqmap_status gqmap_prepare(gqmap_ctx *ctx);
gqmap_status gqmap_get_info(gqmap_ctx *ctx, gqmap_info *info);
/* Current mean |mu| flow (L==1) or mixture MAP (L>1, device get_map) as an
 * M x N x 2 field -- the `map` of gqmap_gpu_mixture.m:53-58. */
gqmap_status gqmap_get_map(gqmap_ctx *ctx, double *map);
/* profile_logP (gqmap_gpu_mixture.m:148-154) of a given M x N x 2 map. */
gqmap_status gqmap_log_p(gqmap_ctx *ctx, const double *map, double *logp);
gqmap_status gqmap_synchronize(gqmap_ctx *ctx);
void gqmap_destroy(gqmap_ctx *ctx);

/* ---- multi-GPU: column-strip tiles with ghost-column (halo) exchange ----
 * The node grid is split into n_tiles strips of whole columns (contiguous in
 * the column-major layout); tile t owns node columns
 * [floor(Ng*t/n), floor(Ng*(t+1)/n)) and keeps one ghost column per
 * neighbour.  Every iteration the tiles exchange their boundary columns (the
 * state planes the neighbour reads) and the per-tile exact fixed-point totals (Energy, sums of
 * |dmu|, |dsigma|, dalpha), so a tiled solve is bit-identical to the whole-
 * grid solve (§8(e) of SURVEY.md: gqmap_gpu_mixture.m:29-46 is Jacobi).
 * A tile context takes the FULL frames in gqmap_set_images (replicated: the
 * bicubic samples reach far outside the strip), and FULL-grid state arrays
 * in gqmap_set_state / gqmap_get_state / gqmap_get_map (set reads the tile's
 * columns, get writes the owned columns only).  gqmap_log_p is whole-grid. */
gqmap_status gqmap_create_tile(gqmap_ctx **ctx, const gqmap_options *opt, int device, int n_tiles,
                               int tile);
/* RCCL transport (one process per GPU): rank 0 draws the id, the caller
 * broadcasts it (e.g. torch.distributed), every tile attaches with rank ==
 * tile.  Collective: blocks until all n_tiles ranks have attached.  After it,
 * gqmap_run / gqmap_run_timed exchange over RCCL on the context's stream. */
gqmap_status gqmap_comm_unique_id(uint8_t id[128]);
gqmap_status gqmap_tile_attach_rccl(gqmap_ctx *ctx, const uint8_t id[128]);
/* In-process transport: tiles[0..n_tiles-1] (tile index order, one device)
 * run n_iter iterations in lockstep, exchanging through device copies.
 * trace as gqmap_run (tile 0's copy; every tile computes the same). */
gqmap_status gqmap_tile_group_run(gqmap_ctx **tiles, int n_tiles, int n_iter, int *n_done,
                                  double *trace);
/* Host-staged transport, for callers that move the boundary data themselves
 * (MPI between nodes, sockets, torch.distributed gloo; one process per tile,
 * any device).  One iteration is
 *   gqmap_tile_exchange_begin: the iteration kernel, this tile's exact totals
 *       and its boundary columns, copied out to host buffers;
 *   the caller sends send_left to tile-1 (its recv_right) and send_right to
 *       tile+1 (its recv_left), and all-gathers the totals in tile order;
 *   gqmap_tile_exchange_end: the received columns into the ghost columns, the
 *       finalize over all tiles' totals; trace3 (optional) = Energy, ptdmu,
 *       ptdsigma of the iteration (NaN once the run has stopped).
 * The boundary messages carry only what the neighbour reads: 4 planes (mu,
 * sigma) leftwards, 6 (mu, sigma, rou of the right edges) rightwards.
 * gqmap_tile_exchange_sizes: bytes of send_left, send_right, recv_left,
 * recv_right (0 at the strip ends), one tile's totals, all tiles' totals.  The RCCL path above is the
 * same exchange on the device (gqmap_gpu_mixture.m:29-46, 69-75). */
gqmap_status gqmap_tile_attach_host(gqmap_ctx *ctx);
gqmap_status gqmap_tile_exchange_sizes(gqmap_ctx *ctx, size_t sizes[6]);
gqmap_status gqmap_tile_exchange_begin(gqmap_ctx *ctx, void *send_left, void *send_right, void *totals);
gqmap_status gqmap_tile_exchange_end(gqmap_ctx *ctx, const void *recv_left, const void *recv_right,
                                     const void *totals_all, double *trace3);

/* ---- standalone device ops (host pointers in/out) ---- */
/* projsplx.m:15-30, applied independently to each of `ncols` columns of Y
 * (n x ncols, column-major) -- the commented column-wise form projsplx.m:34-67. */
gqmap_status gqmap_projsplx(const double *Y, double *X, int n, int ncols, int device);
/* get_map_mex / findMixMax.m:39-70: mixture MAP per pixel (fminbnd, TolX 1e-4). */
gqmap_status gqmap_mixture_map(const double *alpha, const double *muu, const double *sigu,
                               const double *muv, const double *sigv, int M, int N, int L,
                               double *out, int device);
/* flowToColor_mex / legacy/flowToColor.m + computeColor.m: img M x N x 3 uint8,
 * flo M x N x 2 (unknown zeroed), stats {minu,maxu,minv,maxv}, unknown M x N. */
gqmap_status gqmap_flow_to_color(const double *flow, int M, int N, double max_flow,
                                 uint8_t *img, double *flo, double *stats, uint8_t *unknown,
                                 int device);

/* imresize(A, scale) (MATLAB default 'bicubic', Antialiasing on for scale<1)
 * of an M x N x C array -> ceil(scale*M) x ceil(scale*N) x C, resampled on the
 * device (legacy/optical_flow_ctf.m:26-27, 29). */
gqmap_status gqmap_imresize(const double *in, int M, int N, int C, double scale, int antialias,
                            double *out, int device);
/* interp2(V, x - warp(:,:,1), y - warp(:,:,2)) bilinear, NaN outside
 * (optical_flow_ctf.m:30-31); fill != 0 then applies fillmissing 'nearest'
 * along dim 1 and then dim 2 (:32).  V M x N, warp M x N x 2. */
gqmap_status gqmap_warp_image(const double *V, int M, int N, const double *warp, int fill,
                              double *out, int device);

/* ---- coarse-to-fine driver: legacy/optical_flow_ctf.m:21-35 ---- */
#define GQMAP_CTF_MAX_LEVELS 8
typedef struct gqmap_pyramid gqmap_pyramid;
/* level_opt: options of every level (engine GQMAP_ENGINE_CTF, its = iterations
 * per level); minu..maxv = range of the FULL-RESOLUTION ground truth: level s
 * uses them times s, as gqmap_ctf(options,I1_w,I2,trueFlow.*scale) does
 * (optical_flow_ctf.m:33, gqmap_ctf.m:4).  scales: n_levels ascending factors,
 * e.g. {1/16,1/8,1/4,1/2,1}; each level must be exactly twice the previous. */
gqmap_status gqmap_ctf_create(gqmap_pyramid **out, const gqmap_options *level_opt,
                              const double *scales, int n_levels, int device);
/* Full-resolution frames img1/img2 (M x N double): each level's frames are
 * resampled on the device (imresize, :26-27). */
gqmap_status gqmap_ctf_set_images(gqmap_pyramid *p, const double *img1, const double *img2, int M,
                                  int N);
/* The whole pyramid on the device: per level prolong (imresize(warp,2).*2,
 * :29), warp I1 (interp2 + fillmissing, :30-32), seeded init (seed + level),
 * the level solver (gqmap_ctf) and warp += flow (:34).  flow: M x N x 2 final
 * warp; its_done[n_levels]; elapsed_ms: wall time of the pyramid (all may be
 * NULL). */
gqmap_status gqmap_ctf_run(gqmap_pyramid *p, uint64_t seed, double *flow, int *its_done,
                           double *elapsed_ms);
/* Intermediates of level `level` after a run (each output may be NULL): the
 * warped I1 and resampled I2 (Ml x Nl), the level's flow and the warp after
 * the level (Ml x Nl x 2). */
gqmap_status gqmap_ctf_get_level(gqmap_pyramid *p, int level, int *Ml, int *Nl, double *I1w,
                                 double *I2, double *flow, double *warp);
/* trueFlow (M x N x 2, the full-resolution GT as flowToColor returns it):
 * every level then records gqmap_ctf's per-iteration AEPE against
 * trueFlow.*scale (optical_flow_ctf.m:33, gqmap_ctf.m:38).  NULL clears it. */
gqmap_status gqmap_ctf_set_truth(gqmap_pyramid *p, const double *flow, int M, int N);
/* Per-iteration Energy and AEPE (NaN without a truth) of level `level` in the
 * last gqmap_ctf_run; *n = its_done of the level (each array may be NULL). */
gqmap_status gqmap_ctf_get_trace(gqmap_pyramid *p, int level, int *n, double *energy, double *aepe);
void gqmap_ctf_destroy(gqmap_pyramid *p);

/* ---- legacy flow-denoising engine: legacy/gqmap_cpu.m ----
 * [mu,sigma,rou] = gqmap_cpu(options, flow) (legacy/gqmap_cpu.m:1): the
 * legacy model that smooths a GIVEN flow field (Gaussian observation +
 * truncated-quadratic pairwise terms), run on the device.  options.var /
 * gama / dta are never set in the reference; defaults here: 1, 1, inf. */
typedef struct gqmap_cpu_options {
    int its, K;
    double var, gama, dta;
    double step0, step_decay;   /* step = step0/(1+it/step_decay): 0.1, 1000 (:62) */
    double corr_tor;            /* rou clamp 0.97 (:65)                             */
    double tor;                 /* stop: it > min_its && max|dmu| < tor (:70)       */
    int min_its;                /* 100                                              */
} gqmap_cpu_options;
void gqmap_cpu_options_default(gqmap_cpu_options *o);
/* flow M x N x 2 (column-major).  mu = flow; sigma = sigma0 (M x N x 2) or,
 * when sigma0 is NULL, U(0,1) + 2 from the library RNG (seed, stream 3);
 * rou = 0.  Outputs mu, sigma (M x N x 2), rou (M x N x 2 x 2); trace[3*i] =
 * max|dmu|, max|dsigma|, max|drou| of iteration i+1 (its x 3, may be NULL). */
gqmap_status gqmap_cpu_run(const gqmap_cpu_options *o, const double *flow, int M, int N,
                           const double *sigma0, uint64_t seed, double *mu, double *sigma, double *rou,
                           double *trace, int *its_done, int device);
/* gqmap_cpu_run with device arrays (inputs already resident in HBM, no host
 * copies): flow, sigma0 (or NULL), mu, sigma, rou and trace (or NULL) point
 * to memory of `device`, in the layouts above; the iteration runs on mu /
 * sigma / rou in place; *its_done is a host int.  Same results as
 * gqmap_cpu_run bit for bit.  GQMAP_ERR_INVALID_ARG for a host array or mu
 * aliasing flow.  (Reference counterpart: the same gqmap_cpu.m call on
 * gpuArray inputs.) */
gqmap_status gqmap_cpu_run_device(const gqmap_cpu_options *o, const double *flow, int M, int N,
                                  const double *sigma0, uint64_t seed, double *mu, double *sigma, double *rou,
                                  double *trace, int *its_done, int device);
/* gqmap_cpu_run keeps its device buffers in a per-thread, per-device arena
 * across calls (a call needing under a quarter of it shrinks it); this frees
 * the calling thread's arenas now.  Replaces nothing in the reference (the
 * MATLAB runtime owns its gpuArray pool). */
gqmap_status gqmap_cpu_release(void);

/* ---- host helpers (no device needed) ---- */
/* readFlowFile.m: M x N x 2 (flow == NULL: size query). */
gqmap_status gqmap_read_flo(const char *path, int *M, int *N, double *flow);
/* legacy/writeFlowFile.m. */
gqmap_status gqmap_write_flo(const char *path, const double *flow, int M, int N);
/* AEPE of gqmap_gpu_mixture.m:63-64 (unknown pixels of flow zeroed, column
 * means over the crop..end-crop interior, then their mean); unknown may be NULL. */
gqmap_status gqmap_aepe(const double *tflow, const double *flow, const uint8_t *unknown, int M, int N,
                        int crop, double *out);
/* imresize output length for a scale factor: ceil(scale*len). */
int gqmap_resize_len(int len, double scale);
/* GaussHermite_2(K) (GaussHermite_2.m): nodes ascending + weights. */
gqmap_status gqmap_gauss_hermite(int K, double *x, double *w);
/* U(0,1) doubles of stream `stream`, indices [first, first+n): the RNG used by
 * gqmap_init_state (stream 0 = w, 1 = muu, 2 = muv, 3 = sigmau, 4 = sigmav). */
void gqmap_rand_uniform(uint64_t seed, uint32_t stream, uint64_t first, size_t n, double *out);
const char *gqmap_last_error(void);
int gqmap_abi_version(void);
int gqmap_device_count(void);

#ifdef __cplusplus
}
#endif
#endif /* GQMAP_H */
