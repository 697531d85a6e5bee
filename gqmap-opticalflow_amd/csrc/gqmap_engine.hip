// gqmap_engine.hip -- the QGMAP iteration on CDNA4 (gfx950).
//
// One iteration of gqmap_gpu_mixture.m:27-75 (and gqmap_gpuSuper_mix_entropy.m:26-75)
// is two launches:
//
//   k_iter      fused stencil kernel: node potentials + node gradient
//               (node_grad_spectral, :87-116), the four owned edges
//               (edge_grad_spectral, :118-146), the 1-px halo edges recomputed
//               into LDS, the neighbour gradient scatter (:37-40), the clamped
//               ascent (:41-46) and per-workgroup partial sums of Energy,
//               dalpha, |dmu|, |dsigma| (:36, :48, :69-70).  Jacobi update:
//               reads state buffer A, writes buffer B (ping-pong).
//   k_finalize  one workgroup: deterministic reduction of the partials, the
//               alpha update (softmax :78-86 or projsplx :49), the temperature
//               decay (super :72), the stop test (:75), the trace record.
//
// All loop control lives on the device (Ctl), so a chunk of iterations is
// captured once into a hipGraph and replayed; a stopped run turns the
// remaining launches into no-ops.  (Normally the finalize is fused into the
// last k_iter workgroup.  The smallest coarse-to-fine levels run a whole
// chunk in one k_iter_persist launch; column-strip tiles over RCCL add the
// ghost-column exchange and, for L = 1, all-gather and finalize the exact
// totals once per 50-iteration sequence.)
//
// Layout: every field is a MATLAB column-major plane (m fastest).  A state
// buffer is 9 planes of M*N*L: muu, muv, sigu, sigv, pn, rou(dir=1,u),
// rou(dir=2,u), rou(dir=1,v), rou(dir=2,v) -- i.e. rou(m,n,l,dir,uv) exactly as
// the reference's 5-D array.  Tiles of 16x16 nodes map to 256-thread
// workgroups (4 wave64s); lane order is m-fastest so state loads coalesce.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cstdlib>
#include <cmath>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "gqmap_internal.h"

#pragma clang fp contract(off)

namespace gq {
// correctly rounded sqrt without the denormal rescaling: every argument is
// eps + d^2 (eps > 0), 1 +- p (|p| < 1) or 1 - p^2, all far above 2^-767,
// where LLVM's f64 sqrt sequence applies no scaling -- same bits as sqrt().
__device__ __forceinline__ double gq_sqrt_dev(double x)
{
    const double y = __builtin_amdgcn_rsq(x);
    double g = x * y, h = 0.5 * y;
    const double r = fma(-h, g, 0.5);
    g = fma(g, r, g);
    h = fma(h, r, h);
    double d = fma(-g, g, x);
    g = fma(d, h, g);
    d = fma(-g, g, x);
    return fma(d, h, g);
}
// correctly rounded f32 sqrt for normal x >= 2^-96 (every argument is eps + d^2
// with eps >= 2^-96 -- gqmap_create checks that for fp32 -- 1 +- p or 1 - p^2):
// v_sqrt_f32 is within 1 ulp, the neighbour whose residual brackets x wins
// (LLVM's f32 sequence without its denormal rescaling and inf/zero fix-up:
// 9 instructions instead of 17, same bits as sqrtf).
__device__ __forceinline__ float gq_sqrt_dev(float x)
{
    const float s = __builtin_amdgcn_sqrtf(x);
    const int si = __float_as_int(s);
    const float sm = __int_as_float(si - 1), sp = __int_as_float(si + 1);
    const float rm = fmaf(-sm, s, x), rp = fmaf(-sp, s, x);
    const float r = rm <= 0.f ? sm : s;
    return rp > 0.f ? sp : r;
}
}  // namespace gq

#define GQ_HD __device__ __forceinline__
#define GQ_SQRT(x) gq::gq_sqrt_dev(x)
#include "gqmap_tuning.h"
#define GQ_STR2(x) #x
#define GQ_PRAGMA_UNROLL(n) _Pragma(GQ_STR2(unroll n))
#define GQ_UNROLL2 GQ_PRAGMA_UNROLL(GQ_EDGE_UNROLL_N)
#define GQ_PAIR_UNROLL GQ_PRAGMA_UNROLL(GQ_PAIR_UNROLL_N)
#define GQ_PAIR_UNROLL_K(n) GQ_PRAGMA_UNROLL(n)
#define GQ_NODE_UNROLL GQ_PRAGMA_UNROLL(GQ_NODE_UNROLL_N)
#define GQ_UNROLL_FULL _Pragma("unroll")
#define GQ_UMUL24(a, b) __umul24((uint32_t)(a), (uint32_t)(b))
#define GQ_FRACT(x) __builtin_amdgcn_fract(x)  // v_fract_f64
#include "gqmap_math.h"

namespace gq {

// VV storage of the fp64 engine for integer-valued frames (exact).  binary16
// (exact too: C2's values lie in [-510, 765]) halves the tap-gather bytes but
// needs two conversions per tap: C2 fast 141.7 -> 179.7 us/it, literal
// 250.4 -> 267.7 (profiles/r06_vvh_ab.txt); double storage (policy
// vv_float=0) drops the conversion but doubles the bytes and the tap
// registers: literal 255 -> 296 (profiles/r06_lit_vv_ab.txt).
typedef float vvs_t;

constexpr int TILE = 16;
constexpr int BLOCK = TILE * TILE;
constexpr int TS = TAB_STRIDE;
constexpr int NPLANES = 9;
constexpr int TRACE_CAP = 8192;
constexpr int GRAPH_CHUNK = 50;
constexpr int NFIX = 5;        // fixed slots per block: Energy, sum|dmu_u|, sum|dsig_u|, #nonfinite, AEPE sum
constexpr int ACC_SLICES = 8;
constexpr int TRACE_W = 4;     // trace ring columns: Energy, ptdmu, ptdsigma, AEPE (NaN without a truth)

struct Ctl {
    int it;    // next iteration (1-based)
    int done;  // completed iterations since the state was set (ping-pong parity)
    int stop;  // ptdmu < tor reached
    int arrive;  // fused finalize: workgroups done with this iteration
    double T;
    double alpha[GQMAP_LMAX];
    double w[GQMAP_LMAX];
    // fused finalize: the iteration's exact sums as four 32-bit limbs each
    // (acc[x][q][k] = sum over the blocks b with b % ACC_SLICES == x of limb
    // k of the block's fix128), added with 64-bit integer atomics --
    // order-independent -- and cleared by the last workgroup after it reads
    // them.  One slice per XCD (blocks go round-robin to the 8 XCDs): fewer
    // atomics on one address when a small grid's workgroups end together.
    unsigned long long acc[ACC_SLICES][NFIX + GQMAP_LMAX][4];
    // deferred-totals RCCL tiles (L = 1, launch_seq_deferred): the iteration
    // the kernels run next -- advanced by the ghost unpack every iteration,
    // ahead of it / done / T, which the sequence's finalize advances when it
    // has judged the stop rule on the all-gathered totals.  A cache line of
    // their own.  ovr: 1 + the sequence row whose totals met the stop rule
    // when later iterations of the sequence had already run (the host then
    // restores the sequence's snapshot and re-runs it exactly, ovr_recover);
    // also 1 + the launch-local stop iteration of a dataflow launch whose
    // items ran two or more iterations past it (GQ_FLOW_LAG > 2).
    alignas(128) int it_i;
    int done_i;
    double T_i;
    int ovr;
};

struct FinParams {
    const fix128 *partials;  // q-major block partials, row stride nblocks (part_word)
    int nblocks, L;
    const fix128 *gathered;  // nranks > 0: per-tile totals [nranks][NFIX+L] (exact, any order)
    int nranks;
    Ctl *ctl;
    double *trace;     // TRACE_CAP x TRACE_W
    int aepe;          // 1: tot[4] is the AEPE sum of gqmap_ctf.m:38 (a truth is set)
    double count;      // interior nodes * L
    double step0, step_decay;
    int alpha_mode, alpha_start;
    double alpha_lr;
    int t_decay_every;
    double drate, t_min, tor;
};

template <typename R, typename VT = R>
struct IterParams {
    const VT *__restrict__ VV;  // (Mo+2) x (No+2) cubic-convolution padded I2 (VT: storage type)
    const R *__restrict__ I1;   // Mo x No
    R *st0;
    R *st1;
    const R *__restrict__ tab;  // TS x NTAB, point-major (tab_at)
    Ctl *ctl;
    fix128 *partials;           // (NFIX + L) x nblocks, q-major (part_word)
    int M, N, Mo, No, M2, L, K2;
    // column-strip tiling (multi-GPU): local node column n is global column
    // n + n_off of Ng; only local columns [own_lo, own_hi) are updated, the
    // others are ghost copies of the neighbours' boundary columns.  A single
    // context has n_off = 0, [0, N), Ng = N.
    int n_off, own_lo, own_hi, Ng;
    int tiles_m, tiles_n;
    // the tiles of this launch: up to two runs of column-major tile indices
    // [seg_lo[s], seg_lo[s] + seg_n[s]) (a tile context launches its boundary
    // tile columns and its interior separately, to overlap the ghost-column
    // exchange); block b writes partial row part_off + b
    int seg_lo[2], seg_n[2], part_off;
    // fused finalize: the last workgroup to finish (arrival ticket in Ctl)
    // reduces the partials and runs the k_finalize step in the same launch
    int fused;
    // RCCL tile (not fused): the blocks of the iteration's launches (boundary
    // + interior, ticket_total in all) add their sums into Ctl::acc like a
    // fused launch, and the last one writes the tile's exact totals to
    // tile_totals (this rank's row of the all-gathered table)
    int tile_acc, ticket_total;
    fix128 *tile_totals;
    int lpar;                // 1: a block runs all components of its tile; L: one component per block
    // lpar > 1, whole-grid fused launch: block b runs component (b >> 3) % L
    // of the tile of virtual block ((b >> 3) / L) << 3 | (b & 7) -- a tile's
    // L components on one XCD, back to back (they share its I1 block and
    // nearby gather windows in that L2); 8 L ceil(tiles / 8) blocks, those
    // past the last tile idle
    int lpar_xcd;
    int cu_group, cu_slots;  // co-resident workgroups per CU, CUs per XCD (tile order only)
    // whole-grid launch on a frame beyond the L2s: each XCD walks its band of
    // tile columns row by row (tile_of_block; tile order only)
    int band_rows;
    FinParams fin;
    R epsn, lamd, lams;
    R minu, maxu, minv, maxv, sig_lo, sig_hi, corr, sig_step;
    R gh_xmax;  // max |Gauss-Hermite node| (node_unclamped)
    const double *truth;  // ctf engine: M x N x 2 top-left block of GRDT, or null (gqmap_set_truth)
    double step0, step_decay;
    int guard;
    int64_t MNL;
    unsigned *bar;  // k_iter_persist: barrier counters (BAR_WORDS, zero between launches)
    int spec;       // deferred-totals RCCL tile: run iteration Ctl::it_i / done_i / T_i
};

// Quadrature tables are read with wave-uniform indices; routing them through
// the constant address space turns every access into a scalar (SMEM) load.
template <typename R>
using ctab_t = const __attribute__((address_space(4))) R *;
template <typename R>
__device__ __forceinline__ ctab_t<R> as_const(const R *p)
{
    return (ctab_t<R>)p;
}

__device__ __forceinline__ fix128 shfl_xor_fix(fix128 v, int o)
{
    const int64_t hi = (int64_t)(v >> 64);
    const uint64_t lo = (uint64_t)v;
    const int64_t h2 = __shfl_xor(hi, o, 64);
    const uint64_t l2 = (uint64_t)__shfl_xor((int64_t)lo, o, 64);
    return ((fix128)h2 << 64) | (fix128)l2;
}
__device__ __forceinline__ fix128 wave_sum_fix(fix128 v)
{
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += shfl_xor_fix(v, o);
    return v;
}
__device__ __forceinline__ bool finite_d(double x) { return (bits_of(x) & 0x7ff0000000000000ULL) != 0x7ff0000000000000ULL; }

__device__ __forceinline__ double shfl_xor_r(double v, int o) { return __shfl_xor(v, o, 64); }
__device__ __forceinline__ float shfl_xor_r(float v, int o) { return __shfl_xor(v, o, 64); }

// ---------------------------------------------------------------------------
// fp32 edge sums on packed registers.  A mirror pair's two potentials (d =
// C +- p) travel as one float2 through v_pk_add_f32 / v_pk_fma_f32, and the
// six accumulators as three float2 against adjacent table rows (W, WA),
// (WXI, WXJ), (WM, WX).  Every lane of a packed op is the scalar op of
// gqmap_math.h edge_sums in the same order: bit-identical to it (and to the
// CPU model, which runs the scalar form).
// ---------------------------------------------------------------------------
typedef float f2v __attribute__((ext_vector_type(2)));

__device__ __forceinline__ f2v pk_fma(f2v a, f2v b, f2v c) { return __builtin_elementwise_fma(a, b, c); }

// gq_sqrt_dev(float) of both lanes: v_sqrt_f32 each, the neighbour residuals packed
__device__ __forceinline__ f2v sqrt2_pk(f2v x)
{
    const f2v s = {__builtin_amdgcn_sqrtf(x.x), __builtin_amdgcn_sqrtf(x.y)};
    const f2v sm = {__int_as_float(__float_as_int(s.x) - 1), __int_as_float(__float_as_int(s.y) - 1)};
    const f2v sp = {__int_as_float(__float_as_int(s.x) + 1), __int_as_float(__float_as_int(s.y) + 1)};
    const f2v rm = pk_fma(-sm, s, x), rp = pk_fma(-sp, s, x);
    f2v r;
    r.x = rp.x > 0.f ? sp.x : (rm.x <= 0.f ? sm.x : s.x);
    r.y = rp.y > 0.f ? sp.y : (rm.y <= 0.f ? sm.y : s.y);
    return r;
}

template <int PU, typename TP>
__device__ __forceinline__ Sums<float> edge_sums_pk(TP tab, int k0, int K2, int dk, float eps, const EdgeCoef<float> &c)
{
    f2v s0a = {0.f, 0.f}, sij = {0.f, 0.f}, smx = {0.f, 0.f};  // (s0, sa), (sxi, sxj), (sm, sx)
    const int np = K2 >> 1;
    constexpr int U = PU ? PU : GQ_PAIR_UNROLL_N;
    GQ_PRAGMA_UNROLL(U)
    for (int k = k0; k < np; k += dk) {
        const float p = fma(c.A, tab[tab_at(T_XI, k)], c.B * tab[tab_at(T_XJ, k)]);
        const f2v d = f2v{c.C, c.C} + f2v{p, -p};  // C + p, C - p
        const f2v f = sqrt2_pk(pk_fma(d, d, f2v{eps, eps}));
        const f2v fs = f2v{f.x, f.x} + f2v{f.y, f.y}, fd = f2v{f.x, f.x} - f2v{f.y, f.y};
        s0a = pk_fma(f2v{tab[tab_at(T_W, k)], tab[tab_at(T_WA, k)]}, fs, s0a);
        sij = pk_fma(f2v{tab[tab_at(T_WXI, k)], tab[tab_at(T_WXJ, k)]}, fd, sij);
        smx = pk_fma(f2v{tab[tab_at(T_WM, k)], tab[tab_at(T_WX, k)]}, fs, smx);
    }
    Sums<float> S;
    S.s0 = s0a.x; S.sa = s0a.y; S.sxi = sij.x; S.sxj = sij.y; S.sm = smx.x; S.sx = smx.y;
    if ((K2 & 1) && np >= k0 && (np - k0) % dk == 0) {  // the centre point (xi = xj = 0)
        const int k = np;
        const float d = fma(c.A, tab[tab_at(T_XI, k)], fma(c.B, tab[tab_at(T_XJ, k)], c.C));
        S.add(tab, k, gq_sqrt_dev(fma(d, d, eps)));
    }
    return S;
}

// PU: mirror pairs per loop trip (0: GQ_PAIR_UNROLL_N)
template <int PU = 0, typename R, typename TP>
__device__ __forceinline__ Sums<R> edge_sums_dev(TP tab, int k0, int K2, int dk, R eps, const EdgeCoef<R> &c)
{
    if constexpr (sizeof(R) == 4 && GQ_EDGE_PK)
        return edge_sums_pk<PU>(tab, k0, K2, dk, eps, c);
    else
        return edge_sums<PU>(tab, k0, K2, dk, eps, c);
}

// Combine the Q partial quadrature sums of a node's lane group (adjacent
// lanes): the xor butterfly of gqmap_math.h's butterfly(), every lane ends
// with the same total.
template <int Q, typename R>
__device__ __forceinline__ Sums<R> lane_combine(Sums<R> S)
{
#pragma unroll
    for (int o = Q / 2; o > 0; o >>= 1) {
        S.s0 = S.s0 + shfl_xor_r(S.s0, o);
        S.sxi = S.sxi + shfl_xor_r(S.sxi, o);
        S.sxj = S.sxj + shfl_xor_r(S.sxj, o);
        S.sa = S.sa + shfl_xor_r(S.sa, o);
        S.sm = S.sm + shfl_xor_r(S.sm, o);
        S.sx = S.sx + shfl_xor_r(S.sx, o);
    }
    return S;
}

// Block partials, q-major: the low / high 64-bit halves of row r's quantity q
// are words (2q) * PS + r and (2q + 1) * PS + r, PS = rows allocated (the
// context's nblocks).  The finalize's loads of consecutive rows are then
// contiguous: with row-major rows every lane's load touched its own cache
// line (C2: ~10k line requests, 4 us of an 8 us reduction).
__device__ __forceinline__ int64_t part_word(int PS, int r, int q, int half)
{
    return (int64_t)(2 * q + half) * PS + r;
}
// Device-coherent stores/loads of a partial (agent-scope relaxed 64-bit
// atomics: they bypass the non-coherent per-XCD L2s).
__device__ __forceinline__ void store_part_agent(fix128 *parts, int PS, int r, int q, fix128 v)
{
    uint64_t *w = reinterpret_cast<uint64_t *>(parts);
    __hip_atomic_store(w + part_word(PS, r, q, 0), (uint64_t)v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(w + part_word(PS, r, q, 1), (uint64_t)(v >> 64), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ fix128 load_part_agent(const fix128 *parts, int PS, int r, int q)
{
    const uint64_t *w = reinterpret_cast<const uint64_t *>(parts);
    const uint64_t lo = __hip_atomic_load(w + part_word(PS, r, q, 0), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint64_t hi = __hip_atomic_load(w + part_word(PS, r, q, 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return (fix128)(((unsigned __int128)hi << 64) | lo);
}

// Fused finalize transport: a block adds its fix128 partial q into Ctl::acc
// as limbs 0-2 (unsigned 32-bit) and 3 (signed): sum_k limb_k 2^(32k) = v.
// The limb sums stay far inside int64 (925 blocks x 2^32), and integer adds
// commute, so the totals do not depend on the arrival order.  Zero limbs are
// skipped.  (Reading rows of partials instead cost the last workgroup a
// 256-thread reduction: 2.9 us at 80 rows, 4.0 us at 925.)
__device__ __forceinline__ void acc_add_agent(unsigned long long *acc4, fix128 v)
{
    const unsigned __int128 u = (unsigned __int128)v;
    const long long limb[4] = {(long long)(uint32_t)u, (long long)(uint32_t)(u >> 32),
                               (long long)(uint32_t)(u >> 64), (long long)(int32_t)(uint32_t)(u >> 96)};
#pragma unroll
    for (int k = 0; k < 4; ++k)
        if (limb[k] != 0)
            __hip_atomic_fetch_add(acc4 + k, (unsigned long long)limb[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// The last workgroup: Ctl::acc -> tot[] (LDS), then clear acc for the next
// iteration.  All 256 threads call it.
// acc_src: the accumulators to reduce (default Ctl::acc; the dataflow
// kernel's per-iteration slots, k_iter_flow).
__device__ void fin_reduce_acc(const FinParams &F, double *tot, unsigned long long *sh,
                               unsigned long long *acc_src = nullptr)
{
    const int NPR = F.L > 1 ? NFIX + F.L : NFIX;
    const int tid = threadIdx.x;
    constexpr int SL = (NFIX + GQMAP_LMAX) * 4;  // words per slice
    if (tid < 4 * NPR) {
        // all slices' loads in flight together, then the clears (one memory
        // round trip instead of eight: finalize 2.9 -> ~1 us)
        unsigned long long *a = (acc_src ? acc_src : &F.ctl->acc[0][0][0]) + tid;
        unsigned long long v[ACC_SLICES];
#pragma unroll
        for (int x = 0; x < ACC_SLICES; ++x) v[x] = __hip_atomic_load(a + x * SL, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        unsigned long long t = 0;
#pragma unroll
        for (int x = 0; x < ACC_SLICES; ++x) t += v[x];
#pragma unroll
        for (int x = 0; x < ACC_SLICES; ++x) __hip_atomic_store(a + x * SL, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        sh[tid] = t;
    }
    __syncthreads();
    if (tid < NPR) {
        fix128 v = 0;
#pragma unroll
        for (int k = 3; k >= 0; --k) v = (v << 32) + (fix128)(long long)sh[4 * tid + k];
        tot[tid] = from_fix(v);
    }
    __syncthreads();
}

// Exact reduction of the per-block (or per-tile) fixed-point partials into
// tot[] (LDS), all 256 threads of one workgroup.
__device__ void fin_reduce(const FinParams &F, double *tot, fix128 *sh)
{
    // the NFIX fixed sums together, the dalpha sums one at a time (few live
    // registers: this code shares the k_iter register budget when fused)
    // (L = 1: no dalpha sum, fin_apply reads it only when L > 1)
    const int NP = NFIX + F.L, NPR = F.L > 1 ? NP : NFIX;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int rows = F.nranks > 0 ? F.nranks : F.nblocks;
    const bool gathered = F.nranks > 0;
    auto row_val = [&](int r, int q) -> fix128 {
        return gathered ? F.gathered[(int64_t)r * NP + q] : load_part_agent(F.partials, F.nblocks, r, q);
    };
#if GQ_FIN_GROUP
    {   // the NFIX fixed quantities of FIN_ROWS rows per thread together: all
        // their (device-coherent, high-latency) loads in flight at once
        constexpr int FIN_ROWS = 4;
        fix128 v[NFIX] = {};
        for (int r0 = tid; r0 < rows; r0 += FIN_ROWS * 256) {
            fix128 x[FIN_ROWS][NFIX];
#pragma unroll
            for (int u = 0; u < FIN_ROWS; ++u)
#pragma unroll
                for (int q = 0; q < NFIX; ++q) x[u][q] = r0 + u * 256 < rows ? row_val(r0 + u * 256, q) : (fix128)0;
#pragma unroll
            for (int u = 0; u < FIN_ROWS; ++u)
#pragma unroll
                for (int q = 0; q < NFIX; ++q) v[q] += x[u][q];
        }
#pragma unroll
        for (int q = 0; q < NFIX; ++q) {
            const fix128 w = wave_sum_fix(v[q]);
            if (lane == 0) sh[q * 4 + wave] = w;
        }
    }
    for (int q = NFIX; q < NPR; ++q) {
#else
    for (int q = 0; q < NPR; ++q) {
#endif
        fix128 v = 0;
        for (int r0 = tid; r0 < rows; r0 += 4 * 256) {
            fix128 x[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) x[u] = r0 + u * 256 < rows ? row_val(r0 + u * 256, q) : (fix128)0;
            v += (x[0] + x[1]) + (x[2] + x[3]);
        }
        v = wave_sum_fix(v);
        if (lane == 0) sh[q * 4 + wave] = v;
    }
    __syncthreads();
    if (tid < NPR) tot[tid] = from_fix((sh[tid * 4] + sh[tid * 4 + 1]) + (sh[tid * 4 + 2] + sh[tid * 4 + 3]));
    __syncthreads();
}

// The rest of the iteration's host loop (gqmap_gpu_mixture.m:48-50, 69-75;
// super :72): one thread.
__device__ void fin_apply(const FinParams &F, const double *tot)
{
    Ctl *ctl = F.ctl;
    const int it = ctl->it;
    const double step = F.step0 / (1.0 + it / F.step_decay);
    const bool bad = tot[3] != 0.0;  // a NaN/Inf contribution poisons the sums
    const double nan = __builtin_nan("");
    const double energy = bad ? nan : tot[0];
    const double ptdmu = bad ? nan : tot[1] / F.count, ptdsig = bad ? nan : tot[2] / F.count;
    const int L = F.L;
    if (it > F.alpha_start && L != 1) {
        double dal[GQMAP_LMAX];
        for (int l = 0; l < L; ++l) dal[l] = bad ? nan : tot[NFIX + l];
        if (F.alpha_mode == GQMAP_ALPHA_SOFTMAX) {  // updateAlpha, gqmap_gpu_mixture.m:78-86
            double sda = 0;
            for (int l = 0; l < L; ++l) sda = sda + dal[l] * ctl->alpha[l];
            double se = 0, ew[GQMAP_LMAX];
            for (int l = 0; l < L; ++l) {
                const double dw = ctl->alpha[l] * (dal[l] - sda);
                ctl->w[l] = fmin(fmax(ctl->w[l] + dw * step * F.alpha_lr, -300.0), 300.0);
                ew[l] = gq_exp(ctl->w[l]);
                se = se + ew[l];
            }
            for (int l = 0; l < L; ++l) ctl->alpha[l] = ew[l] / se;
        } else {  // projsplx(alpha + dalpha*step*lr), projsplx.m:15-30
            double y[GQMAP_LMAX], s[GQMAP_LMAX];
            for (int l = 0; l < L; ++l) s[l] = y[l] = ctl->alpha[l] + dal[l] * step * F.alpha_lr;
            for (int i = 1; i < L; ++i) {
                double v = s[i];
                int j = i;
                while (j > 0 && s[j - 1] < v) { s[j] = s[j - 1]; --j; }
                s[j] = v;
            }
            double tmpsum = 0, tmax = 0;
            bool bget = false;
            for (int ii = 0; ii < L - 1; ++ii) {
                tmpsum = tmpsum + s[ii];
                tmax = (tmpsum - 1) / (ii + 1);
                if (tmax >= s[ii + 1]) { bget = true; break; }
            }
            if (!bget) tmax = (tmpsum + s[L - 1] - 1) / L;
            for (int l = 0; l < L; ++l) ctl->alpha[l] = fmax(y[l] - tmax, 0.0);
        }
    }
    const int slot = (it - 1) % TRACE_CAP;
    F.trace[TRACE_W * slot + 0] = energy;
    F.trace[TRACE_W * slot + 1] = ptdmu;
    F.trace[TRACE_W * slot + 2] = ptdsig;
    // gqmap_ctf.m:38: mean(mean(sqrt((GRDT-mu)^2...))) over the interior after
    // the update -- equal-length columns, so the exact total / count
    F.trace[TRACE_W * slot + 3] = F.aepe ? (bad ? nan : tot[4] / F.count) : nan;
    if (F.t_decay_every > 0 && it % F.t_decay_every == 0) ctl->T = fmax(ctl->T * F.drate, F.t_min);
    ctl->it = it + 1;
    ctl->done = ctl->done + 1;
    if (ptdmu < F.tor) ctl->stop = 1;
}


// ---------------------------------------------------------------------------
// fused iteration kernel
//
// A workgroup owns a TM x TM tile of nodes; each node is served by Q adjacent
// lanes (Q = 1 for full-resolution grids; 4 or 16 for the small node grids of
// the super engine and coarse pyramid levels, so they still fill 256 CUs).
// Lane j of a node sums the quadrature points k = j, j+Q, ... and the lanes
// combine with an xor butterfly (the spec's butterfly()).
// ---------------------------------------------------------------------------
// Waves per SIMD the register allocation must allow (MI355X: 136-168 VGPRs
// -> 3, 176-256 -> 2, more -> 1).  Left to the allocator: forcing 3 waves on
// the single-scale engine moved arrays to scratch (C2 +24%); bounding the
// super engine to 2 made its block sum 25% slower than the allocator's own
// 2-wave (<= 256 VGPR) schedule.  GQ_MIN_WAVES / GQ_SUPER_WAVES: experiments.
// smallest lanes-per-node split whose edge jobs prefetch the next job's
// operands / run fully unrolled (experiments: GQ_PREFETCH_MIN_Q, GQ_UNROLL_MIN_Q)
constexpr int min_waves(int eng, int q)
{
    return GQ_MIN_WAVES > 1 ? GQ_MIN_WAVES
         : eng == 1        ? GQ_SUPER_WAVES
         : (q >= 2 && q <= 8) ? GQ_MIDQ_WAVES : 1;
}

// Tile index of block b: XCD-aware order.  Blocks b and b+8 share an XCD
// (round-robin dispatch), so each XCD gets a contiguous band of tiles (L2
// locality of the VV gathers).  Speed only; results never depend on placement.
// Position i of the row-by-row walk over the tiles [s, e) (column-major
// numbering, TM tile rows): the range covers column cf from row rf down,
// the full columns cf+1 .. cl-1, and column cl down to row re; row tm holds
// inner + (tm >= rf) + (tm <= re) of them.  Consecutive tiles of the walk
// then share the frame lines their samples read -- a band's gather window
// stays in its XCD's L2 while the state streams through it (down a column,
// the frame lines are reused only a column of tiles later, ~3.6 MB of state
// per column on C5 against a 4 MB L2).
__device__ __forceinline__ int band_row_tile(int i, int s, int e, int TM)
{
    const int cf = s / TM, rf = s - cf * TM, cl = (e - 1) / TM, re = (e - 1) - cl * TM;
    if (cf == cl) return s + i;
    const int inner = cl - cf - 1;
    // tiles in rows < tm: tm inner + max(0, tm - rf) + min(tm, re + 1); the
    // largest tm with that count <= i
    int lo = 0, hi = TM - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        const int before = mid * inner + max(0, mid - rf) + min(mid, re + 1);
        if (before <= i) lo = mid;
        else hi = mid - 1;
    }
    const int tm = lo;
    const int j = i - (tm * inner + max(0, tm - rf) + min(tm, re + 1));
    const int col = tm >= rf ? cf + j : cf + 1 + j;
    return col * TM + tm;
}

__device__ __forceinline__ int tile_of_block(int b, int nb, int cu_group, int S, int band_tm = 0)
{
    int tile = b >> 3;
    // Within an XCD, local blocks j, j+S, j+2S, ... (S = CUs per XCD) start on
    // the same CU (scripts/micro/placement.hip): give those co-resident blocks
    // vertically adjacent tiles of the band (shared L1 lines of the gathers).
    if (cu_group > 1) {
        const int band = (nb - (b & 7) + 7) >> 3;
        if (cu_group >= 100) {  // whole band: slot s takes a contiguous run
            const int Rn = (band + S - 1) / S, X = band - (Rn - 1) * S;  // X slots get Rn tiles
            const int s = tile % S, r = tile / S;
            tile = s * (Rn - 1) + min(s, X) + r;
        } else {
            const int g = min(cu_group, band / S);
            if (g > 1 && tile < S * g) tile = (tile % S) * g + tile / S;
        }
    }
    const int xcd = b & 7;
    int s = 0;
    for (int y = 0; y < xcd; ++y) s += (nb - y + 7) >> 3;
    if (band_tm > 0) return band_row_tile(tile, s, s + ((nb - xcd + 7) >> 3), band_tm);
    return s + tile;
}

// Node rows of a tile with Q lanes per node (256 / Q nodes): 16 x 16, 16 x 8
// (two 16-row columns per wave), 8 x 8, 4 x 4; lanes are m-fastest.
// Q = 64 (k_iter_wn): one wave per node, WN_TM waves per workgroup, tiles of
// WN_TM x 1 nodes.
// Q = 0 (kernel shape only): the role split -- Q = 1 arithmetic on 16 x 8
// tiles, lanes 0-127 (waves 0-1) run the node phase, lanes 128-255 (waves
// 2-3) the edge phase of the same nodes, side by side (iter_tile).
constexpr int WN_TM = 5;
constexpr int tile_pix(int q) { return q == 0 ? BLOCK / 2 : q == 64 ? WN_TM : BLOCK / q; }
constexpr int tile_rows(int q) { return q <= 2 ? 16 : q <= 8 ? 8 : q == 64 ? WN_TM : 4; }
constexpr int tile_cols(int q) { return q == 64 ? 1 : tile_pix(q) / tile_rows(q); }
constexpr int arith_q(int q) { return q == 0 ? 1 : q; }  // lanes per node of the arithmetic

// LDS of one tile: in_up[uv][q][pix]: du2/do2 of the edge from (m-1,n);
// in_left: from (m,n-1); red: per-wave partial sums.  Declared by the kernels
// (one copy whatever the number of iter_tile instantiations).
template <typename R, int TPIX, bool TAB, bool RS>
struct TileLds {
    R in_up[2][2][TPIX];
    R in_left[2][2][TPIX];
    fix128 red[GQMAP_LMAX + NFIX][4];
    // Q > 1: the quadrature table, so lane-varying table reads are LDS reads
    // (with Q lanes per node the index k differs across a wave's lanes)
    R tab[TAB ? NTAB * TS : 1];
    // role split: the node phase's gradient (du1, du2, do1, do2, dp, E, da)
    R nd[RS ? 7 : 1][RS ? TPIX : 1];
};
template <typename R, int Q>
using TileLdsQ = TileLds<R, tile_pix(Q), (Q > 1 && GQ_TAB_LDS), Q == 0>;

#if GQ_TIMELINE
// debug builds: per-block stamps (s_memrealtime, 100 MHz) of k_iter
// iterations GQ_TIMELINE and GQ_TIMELINE + 1 (gqmap_debug_timeline), 16 words
// per block and iteration: 0 start, 1 wave 0 done with phase 0, 2 both
// phases done (all waves), 3 components done, 4 partials stored, 5 HW_ID,
// 6 XCC_ID, 7 finalize done; last block only: 8 ticket taken, 9 partials
// reduced
__device__ unsigned long long g_timeline[8192 * 32];
#define TL_STAMP(s, v)                                                                        \
    do {                                                                                      \
        const int d_ = ctl->it - GQ_TIMELINE;                                                 \
        if (threadIdx.x == 0 && (d_ == 0 || d_ == 1) && blockIdx.x < 8192)                    \
            g_timeline[32 * blockIdx.x + 16 * d_ + (s)] = (v);                                 \
    } while (0)
#else
#define TL_STAMP(s, v) do {} while (0)
#endif

// Interior node (updated by this context): rows 1..M-2, owned local columns,
// global columns 1..Ng-2.
template <typename R, typename VT>
__device__ __forceinline__ bool node_interior(const IterParams<R, VT> &P, int mm, int nn)
{
    return mm >= 1 && mm <= P.M - 2 && nn >= P.own_lo && nn < P.own_hi && nn + P.n_off >= 1 &&
           nn + P.n_off <= P.Ng - 2;
}

// State-buffer access.  COH (the persistent small-grid kernel, whose
// workgroups hand state to each other inside one launch): device-coherent
// (agent-scope relaxed) loads and stores -- write-through on the producer,
// L1 bypassed on the consumer -- so no L2 write-back / invalidate is needed
// between its iterations.  Otherwise plain accesses (kernel boundaries order
// them).
template <bool COH, typename R>
__device__ __forceinline__ R ld_state(const R *p)
{
    if constexpr (COH) return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else return *p;
}
// NT: a non-temporal store -- the state of a frame larger than the L2s is
// streamed once per iteration; kept out of the L2 it does not evict the
// padded frame's gather lines (C5: fetch bytes -16%, profiles/r04_c5_nt_store.txt).
// A compile-time choice: a run-time one lets the compiler merge the two
// stores into one plain store.
template <bool COH, typename R, bool NT = false>
__device__ __forceinline__ void st_state(R *p, R v)
{
    if constexpr (COH) __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else if constexpr (NT) __builtin_nontemporal_store(v, p);
    else *p = v;
}

// Edge job e of a lane: e = dir + 2*uv (< 4) is the node's own down / right
// edge, e = 4 the halo edge entering the tile (top row / left column) that
// the lane group tid / Q computes; with its operands loaded (rou plane 5+e of
// the head node, the tail node's mean / sigma).
template <typename R>
struct EdgeJob {
    int dir, uv, hr;
    bool need;
    R u1, o1, p, o2, u2;
};
template <typename R, typename VT, int Q, int TM, int TN, bool COH>
__device__ __forceinline__ EdgeJob<R> edge_job(const IterParams<R, VT> &P, const R *__restrict__ src, int e,
                                               int tid, int m, int n, int m0, int n0, int64_t loff, bool inner,
                                               bool valid, R mu_u, R mu_v, R sg_u, R sg_v)
{
    EdgeJob<R> jb{};
    int hm, hn, rm, rn;
    const bool own_edge = e < 4;
    if (own_edge) {
        jb.dir = e & 1; jb.uv = e >> 1;
        hm = m; hn = n;
        rm = jb.dir == 0 ? m + 1 : m; rn = jb.dir == 1 ? n + 1 : n;
    } else {
        const int h = tid / Q;  // halo edge index
        const bool top = h < 2 * TN;
        const int hh = top ? h : h - 2 * TN, span = top ? TN : TM;
        jb.uv = hh / span;
        jb.hr = hh % span;
        jb.dir = top ? 0 : 1;
        hm = top ? m0 - 1 : m0 + jb.hr; hn = top ? n0 + jb.hr : n0 - 1;
        rm = top ? m0 : hm;             rn = top ? hn : n0;
    }
    const int M = P.M, N = P.N;
    const int64_t MNL = P.MNL;
    const bool r_inner = rm < M && rn < N && node_interior(P, rm, rn);
    jb.need = own_edge ? (inner || (valid && r_inner)) : (hm >= 0 && hn >= 0 && r_inner);
    if (jb.need) {
        const int uv = jb.uv;
        const int64_t h = hm + (int64_t)M * hn + loff;
        const int64_t r = rm + (int64_t)M * rn + loff;
        jb.u1 = own_edge ? (uv ? mu_v : mu_u) : ld_state<COH>(src + h + MNL * uv);
        jb.o1 = own_edge ? (uv ? sg_v : sg_u) : ld_state<COH>(src + h + MNL * (2 + uv));
        jb.p = ld_state<COH>(src + h + MNL * (5 + jb.dir + 2 * uv));  // rou plane 5+e
        jb.o2 = ld_state<COH>(src + r + MNL * (2 + uv));
        jb.u2 = ld_state<COH>(src + r + MNL * uv);
    }
    return jb;
}

// The clamped ascent of one interior node from its assembled gradients
// (gqmap_gpu_mixture.m:41-45; gqmap_ctf.m:34-35), the updated state into dst
// and the node's exact contributions to the block sums; returns its dalpha.
template <int ENG, bool COH, bool NT = false, typename R, typename VT>
__device__ __forceinline__ fix128 node_apply(const IterParams<R, VT> &P, R *__restrict__ dst, int64_t i, int m,
                                             int n, R step, R mu_u, R mu_v, R sg_u, R sg_v, R pn, const Grad<R> &nd,
                                             R gmu_u, R gmu_v, R gsg_u, R gsg_v, R eE, R eda, fix128 &fE,
                                             fix128 &fmu, fix128 &fsg, fix128 &fae, int &nonfinite)
{
    const int M = P.M;
    const int64_t MNL = P.MNL, MN = (int64_t)M * P.N;
    auto cl = [](R x, R lo, R hi) { return fmin(fmax(x, lo), hi); };
    const R nu = cl(mu_u + gmu_u * step, P.minu, P.maxu), nv = cl(mu_v + gmu_v * step, P.minv, P.maxv);
    st_state<COH, R, NT>(dst + i + MNL * 0, nu);
    st_state<COH, R, NT>(dst + i + MNL * 1, nv);
    if constexpr (ENG == 2) {  // AEPE of gqmap_ctf.m:38 against the updated mean
        if (P.truth) {
            const double du = P.truth[m + (int64_t)M * n] - (double)nu;
            const double dv = P.truth[m + (int64_t)M * n + MN] - (double)nv;
            fae += to_fix(gq_sqrt_dev(du * du + dv * dv));
        }
    }
    // sigma step: gqmap_ctf.m:34-35 scales it by 0.3 ((dsigma*step)*0.3)
    const R su = ENG == 2 ? (gsg_u * step) * P.sig_step : gsg_u * step;
    const R sv = ENG == 2 ? (gsg_v * step) * P.sig_step : gsg_v * step;
    st_state<COH, R, NT>(dst + i + MNL * 2, cl(sg_u + su, P.sig_lo, P.sig_hi));
    st_state<COH, R, NT>(dst + i + MNL * 3, cl(sg_v + sv, P.sig_lo, P.sig_hi));
    st_state<COH, R, NT>(dst + i + MNL * 4, cl(pn + nd.dp * step, -P.corr, P.corr));
    // per-node contributions to the global sums (exact fixed point)
    const double cE = (double)nd.E + (double)eE, cda = (double)nd.da + (double)eda;
    const double cmu = fabs((double)gmu_u), csg = fabs((double)gsg_u);
    nonfinite += !finite_d(cE) + !finite_d(cda) + !finite_d(cmu) + !finite_d(csg);
    fE += to_fix(cE);
    fmu += to_fix(cmu);
    fsg += to_fix(csg);
    return to_fix(cda);
}

// Last workgroup of a fused launch (arrival ticket) runs the finalize step;
// all threads of every workgroup call it after storing their partials.
__device__ __forceinline__ void fused_finalize_tail(const FinParams &F)
{
    Ctl *ctl = F.ctl;
    __shared__ int last;
    if (threadIdx.x == 0) {
        __builtin_amdgcn_s_waitcnt(0);
        last = atomicAdd(&ctl->arrive, 1) == (int)gridDim.x - 1;
    }
    __syncthreads();
    if (!last) return;
    TL_STAMP(8, __builtin_amdgcn_s_memrealtime());
    __shared__ double tot[NFIX + GQMAP_LMAX];
    __shared__ unsigned long long sh_acc[4 * (NFIX + GQMAP_LMAX)];
    fin_reduce_acc(F, tot, sh_acc);
    TL_STAMP(9, __builtin_amdgcn_s_memrealtime());
#if GQ_TIMELINE
    const int tl_it = ctl->it;
#endif
    if (threadIdx.x == 0) {
        fin_apply(F, tot);
        ctl->arrive = 0;
#if GQ_TIMELINE
        const int d_ = tl_it - GQ_TIMELINE;
        if ((d_ == 0 || d_ == 1) && blockIdx.x < 8192) g_timeline[32 * blockIdx.x + 16 * d_ + 7] = __builtin_amdgcn_s_memrealtime();
#endif
    }
}

// RCCL tile: the last of the iteration's ticket_total workgroups (the
// strip's launch) turns Ctl::acc into the tile's exact
// totals (fix128, this rank's row of the table the all-gather shares) and
// clears acc and the ticket.  All threads of every workgroup call it.
__device__ __forceinline__ void tile_totals_tail(const FinParams &F, int total, fix128 *out)
{
    Ctl *ctl = F.ctl;
    __shared__ int last;
    if (threadIdx.x == 0) {
        __builtin_amdgcn_s_waitcnt(0);
        last = atomicAdd(&ctl->arrive, 1) == total - 1;
    }
    __syncthreads();
    if (!last) return;
    const int NP = NFIX + F.L, tid = threadIdx.x;
    constexpr int SL = (NFIX + GQMAP_LMAX) * 4;
    __shared__ unsigned long long sh[4 * (NFIX + GQMAP_LMAX)];
    if (tid < 4 * NP) {
        unsigned long long *a = &ctl->acc[0][0][0] + tid;
        unsigned long long v[ACC_SLICES];
#pragma unroll
        for (int x = 0; x < ACC_SLICES; ++x) v[x] = __hip_atomic_load(a + x * SL, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        unsigned long long t = 0;
#pragma unroll
        for (int x = 0; x < ACC_SLICES; ++x) t += v[x];
#pragma unroll
        for (int x = 0; x < ACC_SLICES; ++x) __hip_atomic_store(a + x * SL, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        sh[tid] = t;
    }
    __syncthreads();
    if (tid < NP) {
        fix128 v = 0;
#pragma unroll
        for (int k = 3; k >= 0; --k) v = (v << 32) + (fix128)(long long)sh[4 * tid + k];
        out[tid] = v;
    }
    if (tid == 0) ctl->arrive = 0;
}

// One tile of one iteration (absolute iteration `it`, reading state buffer
// `parity`): node and edge gradients, neighbour scatter, clamped ascent into
// the other buffer, and the tile's exact partial sums into partial row part_r.
// Tcur: the temperature of this iteration (Ctl::T; the persistent kernel keeps
// its own copy).  tab_ready: the LDS table is already loaded (persistent).
// LIT: the literal-order arithmetic of gqmap_math.h (lit_node_grad /
// lit_edge_grad; fp64 single-scale mixture engine, Q = 1) in place of the fast
// specification's node_sums / edge_sums; everything around it is shared.
template <typename R, typename VT, int ENG, int Q, bool EDGE_FIRST, bool COH = false, bool NT = false,
          bool LIT = false>
__device__ __forceinline__ void iter_tile(const IterParams<R, VT> P, int tile, int it, int parity,
                                          int part_r, TileLdsQ<R, Q> &lds, int l0, int l1, double Tcur,
                                          bool tab_ready, unsigned long long *acc_ring = nullptr)
{
    static_assert(!LIT || (ENG == 0 && Q == 1 && sizeof(R) == 8), "literal order: fp64 mixture, Q = 1");
    constexpr bool RS = Q == 0;                       // role split (node / edge waves)
    constexpr int QA = arith_q(Q);                    // lanes per node of the arithmetic
    constexpr int TPIX = tile_pix(Q);                 // nodes per tile
    constexpr int TM = tile_rows(Q), TN = TPIX / TM;  // tile rows x columns
    static_assert(TM * TN == TPIX, "tile");
    Ctl *ctl = P.ctl;
    const R *__restrict__ src = parity ? P.st1 : P.st0;
    R *__restrict__ dst = parity ? P.st0 : P.st1;
    const R T = R(Tcur);
    const R step = R(P.step0 / (1.0 + it / P.step_decay));

    const int tm = tile % P.tiles_m, tn = tile / P.tiles_m;
    const int tid = threadIdx.x;
    // role split: lanes [0, TPIX) the node phase, [TPIX, 2 TPIX) the edge phase
    // of the same TPIX nodes (wave-uniform roles)
    const int rtid = RS ? tid % TPIX : tid;
    const bool do_node = !RS || tid < TPIX, do_edge = !RS || tid >= TPIX;
    const int pix = rtid / QA, kj = rtid % QA;  // node within the tile, lane within the node
    const int lm = pix % TM, ln = pix / TM;
    const int m0 = tm * TM, n0 = tn * TN;
    const int m = m0 + lm, n = n0 + ln;
    const int M = P.M, N = P.N;
    const int64_t MNL = P.MNL, MN = (int64_t)M * N;
    const bool valid = m < M && n < N;
    const bool inner = valid && node_interior(P, m, n);
    const bool lead = kj == 0;  // the lane that owns the node's outputs
    const int K2 = P.K2;
    constexpr bool TAB_LDS = QA > 1 && GQ_TAB_LDS;
    using tab_t = std::conditional_t<TAB_LDS, const R *, ctab_t<R>>;
    tab_t tab;
    if constexpr (TAB_LDS) {
        if (!tab_ready) {
            for (int e = threadIdx.x; e < NTAB * K2; e += BLOCK) lds.tab[e] = P.tab[e];
            __syncthreads();
        }
        tab = lds.tab;
    } else {
        tab = as_const(P.tab);
    }

    auto &in_up = lds.in_up;
    auto &in_left = lds.in_left;
    auto &red = lds.red;

    fix128 fE = 0, fmu = 0, fsg = 0, fae = 0;
    int nonfinite = 0;
    const int wave = tid >> 6, lane = tid & 63;
    // halo: 2*(TN+TM) edges (top row and left column, u and v) x Q lanes
    constexpr int HALO_LANES = 2 * (TN + TM) * QA;
    const bool halo_lane = rtid < HALO_LANES;

    for (int l = l0; l < l1; ++l) {
        // (COH: the dataflow kernel, whose alpha a finalize on another XCD
        // may just have updated)
        const R a = R(COH ? __hip_atomic_load(&ctl->alpha[l], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : ctl->alpha[l]);
        const int64_t i = m + (int64_t)M * n + MN * l;
        // mu_u, mu_v, sigma_u, sigma_v, pn of the node; the four rou planes
        // are read and updated by their edge jobs.  (Named scalars, not an
        // array: a select between two array elements by the run-time uv
        // below would put the array in scratch.)
        const R mu_u = valid ? ld_state<COH>(src + i) : R(0);
        const R mu_v = valid ? ld_state<COH>(src + i + MNL) : R(0);
        const R sg_u = valid ? ld_state<COH>(src + i + MNL * 2) : R(0);
        const R sg_v = valid ? ld_state<COH>(src + i + MNL * 3) : R(0);
        const R pn = valid ? ld_state<COH>(src + i + MNL * 4) : R(0);
        Grad<R> nd{};
        R sum_mu0 = 0, sum_mu1 = 0, sum_sg0 = 0, sum_sg1 = 0;  // sum over dir of du1 / do1
        R eE = 0, eda = 0;                                     // sum over the 4 edges
        // Node phase then edge phase, or (EDGE_FIRST) the reverse: the node
        // phase is gather-heavy, the edge phase pure VALU; mixing the orders
        // among the workgroups that share a CU overlaps the two.  Both orders
        // are compile-time straight-line code (the loop below is unrolled; no
        // lambdas: captured locals ended up in scratch).
#pragma unroll
        for (int ph = 0; ph < 2; ++ph) {
        if ((ph == 0) != EDGE_FIRST) {
        if (do_node && LIT) {
            if constexpr (LIT)
                if (inner)
                    nd = lit_node_grad(tab, K2, P.VV, P.M2, P.I1, P.Mo, P.No, P.epsn, P.lamd, P.guard != 0, T, a,
                                       mu_u, mu_v, sg_u, sg_v, pn, m, n + P.n_off);
        } else if (do_node) {
        NodeCoef<R> c{};
        if (inner) c = node_coef(sg_u, sg_v, pn);
        // single-scale engine: when no sample of any node of the wave can be
        // clamped (wave vote), run the quadrature without the clamps
        // (not for ctf: its clamp-free form measured slower on C3, 0.71 vs
        // 0.76 Gpix-it/s -- a second node loop in an already large kernel)
        const bool fast = ENG == 0 && __all(!inner || node_unclamped(c, mu_u, mu_v, m, n + P.n_off, P.Mo, P.No,
                                                                     P.gh_xmax, R(ENG == 2 ? CTF_MARGIN : 0.0)));
        if (inner) {
            const auto fv = frame_view(P.VV, P.M2);
            // (at one lane per node only with float taps: the fp64-tap Q = 1
            // kernels would cross 168 VGPRs, 3 -> 2 waves per SIMD)
            constexpr bool PF = QA >= GQ_NODE_PF_MIN_Q && (QA > 1 || sizeof(VT) == 4);
            Sums<R> S = fast ? node_sums<ENG, false, PF>(tab, kj, K2, QA, fv, P.I1, P.Mo, P.No, P.epsn, c, mu_u,
                                                         mu_v, m, n + P.n_off)
                             : node_sums<ENG, true, PF>(tab, kj, K2, QA, fv, P.I1, P.Mo, P.No, P.epsn, c, mu_u,
                                                        mu_v, m, n + P.n_off);
            if (QA > 1) S = lane_combine<QA>(S);
            nd = node_epi(S, c, P.lamd, P.guard != 0, T, a, sg_u, sg_v, pn, ENG == 2);
            if constexpr (RS) {  // to the edge lane of the same node
                lds.nd[0][pix] = nd.du1; lds.nd[1][pix] = nd.du2; lds.nd[2][pix] = nd.do1;
                lds.nd[3][pix] = nd.do2; lds.nd[4][pix] = nd.dp; lds.nd[5][pix] = nd.E; lds.nd[6][pix] = nd.da;
            }
        }
        }
        } else if (do_edge) {
        // Edge jobs e = dir + 2*uv (rou plane 5+e) for the owned down/right
        // edges, then job 4 on the halo lanes: the edges entering the tile from
        // the row above / the column to the left.  One edge body, streamed into
        // accumulators and LDS, keeps VGPRs low.
        // Wave-uniform for Q = 1, 4, 8, 16 (HALO_LANES = 64, 128, 192, 256); for Q = 2
        // it is 96, so wave 1 diverges on the halo job.  That is safe because
        // nothing wave-wide runs inside a job: the only cross-lane op is
        // lane_combine<Q>, an xor butterfly inside one node's Q adjacent
        // lanes, and a node's lanes are all halo lanes or none (asserted).
        static_assert(HALO_LANES % QA == 0, "a node's lanes share their job count");
        const int njobs = halo_lane ? 5 : 4;
        // Q >= 4 (small grids, about one wave per SIMD: latency-bound) loads
        // job e+1's operands before computing job e
        constexpr bool PREFETCH = QA >= GQ_PREFETCH_MIN_Q;
        auto job_at = [&](int e) {
            return edge_job<R, VT, QA, TM, TN, COH>(P, src, e, rtid, m, n, m0, n0, MN * l, inner, valid, mu_u, mu_v,
                                                sg_u, sg_v);
        };
        EdgeJob<R> next{};
        if (PREFETCH) next = job_at(0);
        // Q >= 4 single-pixel engines: a constant trip count, fully unrolled
        // (independent jobs overlap; ctf 30x40 30.0 -> 28.8 us/it; not the
        // super engine, which it would push past 256 VGPRs: C4 355 -> 407)
        constexpr bool JOBS_UNROLLED = QA >= GQ_UNROLL_MIN_Q && ENG != 1;
        constexpr int JOB_UNROLL = JOBS_UNROLLED ? 5 : 1;
#pragma unroll JOB_UNROLL
        for (int e = 0; e < (JOBS_UNROLLED ? 5 : njobs); ++e) {
            if (JOBS_UNROLLED && e >= njobs) continue;
            EdgeJob<R> jb;
            if (PREFETCH) {
                jb = next;
                if (e + 1 < njobs) next = job_at(e + 1);
            } else {
                jb = job_at(e);
            }
            const int dir = jb.dir, uv = jb.uv, hr = jb.hr;
            const bool own_edge = e < 4;
            Grad<R> g{};
            if (jb.need) {
                if constexpr (LIT) {
                    g = lit_edge_grad(tab, K2, P.epsn, P.lams, P.guard != 0, T, a, jb.u1, jb.u2, jb.o1, jb.o2, jb.p);
                } else {
                    const EdgeCoef<R> c = edge_coef(jb.u1, jb.u2, jb.o1, jb.o2, jb.p);
                    // 4 mirror pairs per trip at Q = 1 for the fp32 mixture, the
                    // fp64 ctf levels and the non-temporal (large-frame, C5)
                    // kernels with float taps (profiles/r05_unroll_knobs.txt,
                    // r05_c5_variants.txt), else 2 (fp32 ctf: 130 VGPRs and the
                    // double-tap mixture NT kernel 170: 3 -> 2 waves per SIMD)
                    constexpr int PU =
                        QA == 1 && ((sizeof(R) == 4 && ENG == 0) ||
                                    (sizeof(R) == 8 && (ENG == 2 || (NT && sizeof(VT) == 4))))
                            ? GQ_PAIR_UNROLL_Q1 : 0;
                    Sums<R> S = edge_sums_dev<PU>(tab, kj, K2, QA, P.epsn, c);
                    if (QA > 1) S = lane_combine<QA>(S);
                    g = edge_epi(S, c, P.lams, P.guard != 0, T, a, jb.o1, jb.o2, jb.p, ENG == 2);
                }
                // the edge owns its correlation: clamped ascent right here
                // (gqmap_gpu_mixture.m:46), nothing else reads drou
                if (own_edge && inner && lead)
                    st_state<COH, R, NT>(dst + i + MNL * (5 + e), fmin(fmax(jb.p + g.dp * step, -P.corr), P.corr));
            }
            if (own_edge) {
                if (uv == 0) { sum_mu0 = sum_mu0 + g.du1; sum_sg0 = sum_sg0 + g.do1; }
                else         { sum_mu1 = sum_mu1 + g.du1; sum_sg1 = sum_sg1 + g.do1; }
                eE = eE + g.E;
                eda = eda + g.da;
                // neighbour share: (m+1,n) reads in_up, (m,n+1) reads in_left
                if (lead && dir == 0 && lm + 1 < TM) { in_up[uv][0][pix + 1] = g.du2; in_up[uv][1][pix + 1] = g.do2; }
                if (lead && dir == 1 && ln + 1 < TN) { in_left[uv][0][pix + TM] = g.du2; in_left[uv][1][pix + TM] = g.do2; }
            } else if (rtid % QA == 0) {
                if (dir == 0) { in_up[uv][0][hr * TM] = g.du2; in_up[uv][1][hr * TM] = g.do2; }
                else          { in_left[uv][0][hr] = g.du2; in_left[uv][1][hr] = g.do2; }
            }
        }
        }
        if (ph == 0) TL_STAMP(1, __builtin_amdgcn_s_memrealtime());
        }
        __syncthreads();
        TL_STAMP(2, __builtin_amdgcn_s_memrealtime());
        fix128 fda = 0;
        if (inner && lead && do_edge) {
            if constexpr (RS) {
                nd.du1 = lds.nd[0][pix]; nd.du2 = lds.nd[1][pix]; nd.do1 = lds.nd[2][pix];
                nd.do2 = lds.nd[3][pix]; nd.dp = lds.nd[4][pix]; nd.E = lds.nd[5][pix]; nd.da = lds.nd[6][pix];
            }
            // dmuu = dmuu + sum(dmu1(:,:,:,:,1),4) + circshift(dmu2(..1,1),1) + circshift(dmu2(..2,1),1,2)
            const R gmu_u = ((nd.du1 + sum_mu0) + in_up[0][0][pix]) + in_left[0][0][pix];
            const R gmu_v = ((nd.du2 + sum_mu1) + in_up[1][0][pix]) + in_left[1][0][pix];
            const R gsg_u = ((nd.do1 + sum_sg0) + in_up[0][1][pix]) + in_left[0][1][pix];
            const R gsg_v = ((nd.do2 + sum_sg1) + in_up[1][1][pix]) + in_left[1][1][pix];
            fda = node_apply<ENG, COH, NT>(P, dst, i, m, n, step, mu_u, mu_v, sg_u, sg_v, pn, nd, gmu_u, gmu_v, gsg_u, gsg_v,
                                  eE, eda, fE, fmu, fsg, fae, nonfinite);
        }
        if (P.L > 1) {  // dalpha(l): only consumed by the alpha update
            fda = wave_sum_fix(fda);
            if (lane == 0) red[NFIX + l][wave] = fda;
        }
        __syncthreads();  // LDS reuse by the next component
    }

    TL_STAMP(3, __builtin_amdgcn_s_memrealtime());
    // block partials: Energy, sum|dmu_u|, sum|dsigma_u|, #nonfinite, dalpha[0..L-1]
    fE = wave_sum_fix(fE);
    fmu = wave_sum_fix(fmu);
    fsg = wave_sum_fix(fsg);
    fix128 fnf = wave_sum_fix((fix128)nonfinite);
    if (ENG == 2) fae = wave_sum_fix(fae);
    if (lane == 0) {
        red[0][wave] = fE;
        red[1][wave] = fmu;
        red[2][wave] = fsg;
        red[3][wave] = fnf;
        red[4][wave] = fae;
    }
    __syncthreads();
    const int NP = NFIX + P.L;
    if (tid < NP) {  // NP <= 12: all in wave 0
        fix128 v = 0;
        const int lq = tid - NFIX;  // dalpha of the components this block ran
        if (tid < NFIX || (P.L > 1 && lq >= l0 && lq < l1))
            v = (red[tid][0] + red[tid][1]) + (red[tid][2] + red[tid][3]);
        if (acc_ring) {  // the dataflow kernel's slot of this iteration (k_iter_flow)
            if (v != 0) acc_add_agent(acc_ring + ((blockIdx.x % ACC_SLICES) * (NFIX + GQMAP_LMAX) + tid) * 4, v);
        } else if (P.fused || P.tile_acc) {
            if (v != 0) acc_add_agent(&ctl->acc[blockIdx.x % ACC_SLICES][tid][0], v);
        } else {
            store_part_agent(P.partials, P.fin.nblocks, part_r, tid, v);
        }
    }
}


template <typename R, typename VT, int ENG, int Q, bool NT = false, bool LIT = false>
__device__ __forceinline__ void k_iter_body(const IterParams<R, VT> &P)
{
    Ctl *ctl = P.ctl;
    if (ctl->stop) return;
#if GQ_TIMELINE
    const unsigned long long tl0 = __builtin_amdgcn_s_memrealtime();
#endif
    const int nb = P.seg_n[0] + P.seg_n[1];  // tiles in this launch
    const int b = blockIdx.x;
    // lpar > 1: one block per (tile, component), component-major
    int bt = P.lpar > 1 ? b % nb : b;
    int l0 = P.lpar > 1 ? b / nb : 0;
    if (P.lpar_xcd) {
        const int j = b >> 3, jt = j / P.lpar;
        l0 = j - jt * P.lpar;
        bt = (jt << 3) | (b & 7);
    }
    const int l1 = P.lpar > 1 ? l0 + 1 : P.L;
    const bool idle = bt >= nb;  // lpar_xcd padding
    const int tl = idle ? 0 : tile_of_block(bt, nb, P.cu_group, P.cu_slots, P.band_rows ? P.tiles_m : 0);
    const int tile = tl < P.seg_n[0] ? P.seg_lo[0] + tl : P.seg_lo[1] + (tl - P.seg_n[0]);
    // workgroups that start on one CU are local blocks j, j+S, j+2S of the
    // XCD (see tile_of_block): alternate the phase order among them (node,
    // edge, node first; the ctf levels at Q = 1 edge, node, edge: 480x640
    // -2.7%, against +4.6% on C2 and +34% on C2 fp32, profiles/r05_phase_mix_inv.txt).
    // Not for the super engine, whose node phase dominates (C4: 850 vs 680 us/it).
    constexpr int INV = ENG == 2 && Q == 1 ? GQ_PHASE_MIX_CTF_Q1_INV : GQ_PHASE_MIX_OTHER_INV;
    const bool edge_first = GQ_PHASE_MIX && ENG != 1 && ((((b >> 3) / P.cu_slots) & 1) != INV);
    __shared__ TileLdsQ<R, Q> lds;
    const int part_r = P.part_off + b;
    if (idle) {
        // nothing to compute or add; still takes its arrival ticket below
    } else if (edge_first)
        iter_tile<R, VT, ENG, Q, true, false, NT, LIT>(P, tile, P.spec ? ctl->it_i : ctl->it,
                                                       (P.spec ? ctl->done_i : ctl->done) & 1, part_r, lds, l0, l1,
                                                       P.spec ? ctl->T_i : ctl->T, false);
    else
        iter_tile<R, VT, ENG, Q, false, false, NT, LIT>(P, tile, P.spec ? ctl->it_i : ctl->it,
                                                        (P.spec ? ctl->done_i : ctl->done) & 1, part_r, lds, l0, l1,
                                                        P.spec ? ctl->T_i : ctl->T, false);
#if GQ_TIMELINE
    __syncthreads();
    TL_STAMP(0, tl0);
    TL_STAMP(4, __builtin_amdgcn_s_memrealtime());
    TL_STAMP(5, (unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 4));
    TL_STAMP(6, (unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 20));
    const int tl_it = ctl->it;
#endif
    if (!P.fused) {
        if (P.tile_acc) tile_totals_tail(P.fin, P.ticket_total, P.tile_totals);
        return;
    }
    const int tid = threadIdx.x;
    // Last workgroup in runs the finalize step: release the partials at
    // device scope (the XCDs' L2s are not coherent), take an arrival ticket,
    // and the final arriver acquires them all.
    // The partials went out as device-coherent (agent-scope) stores, which
    // write through this XCD's L2; once wave 0 has seen them complete it
    // takes the arrival ticket.  No L2 write-back or invalidate: a fence here
    // costs every workgroup (measured +20..70 us per iteration on C2).
    __shared__ int last;
    if (tid == 0) {
        __builtin_amdgcn_s_waitcnt(0);
        last = atomicAdd(&ctl->arrive, 1) == (int)gridDim.x - 1;
    }
    __syncthreads();
    if (!last) return;
#if GQ_TIMELINE
    const bool tl_on = (tl_it == GQ_TIMELINE || tl_it == GQ_TIMELINE + 1) && b < 8192 && tid == 0;
    unsigned long long *tl_row = g_timeline + 32 * b + 16 * (tl_it - GQ_TIMELINE);
    if (tl_on) tl_row[8] = __builtin_amdgcn_s_memrealtime();
#endif
    __shared__ double tot[NFIX + GQMAP_LMAX];
    __shared__ unsigned long long sh_acc[4 * (NFIX + GQMAP_LMAX)];
    fin_reduce_acc(P.fin, tot, sh_acc);
#if GQ_TIMELINE
    if (tl_on) tl_row[9] = __builtin_amdgcn_s_memrealtime();
#endif
    if (tid == 0) {
        fin_apply(P.fin, tot);
        ctl->arrive = 0;
#if GQ_TIMELINE
        if (tl_on) tl_row[7] = __builtin_amdgcn_s_memrealtime();
#endif
    }
}

template <typename R, typename VT, int ENG, int Q, bool NT = false>
__global__ __launch_bounds__(BLOCK, min_waves(ENG, Q)) void k_iter(IterParams<R, VT> P)
{
    k_iter_body<R, VT, ENG, Q, NT>(P);
}

// The literal-order arithmetic (gqmap_options.arith = GQMAP_ARITH_LITERAL):
// the same tiles, halo, update and finalize with lit_node_grad / lit_edge_grad.
#ifndef GQ_LIT_WAVES  // waves per SIMD the literal kernel's allocation must allow (1: the allocator's choice)
#define GQ_LIT_WAVES 3
#endif
template <typename VT, bool NT = false>
__global__ __launch_bounds__(BLOCK, GQ_LIT_WAVES) void k_iter_lit(IterParams<double, VT> P)
{
    k_iter_body<double, VT, 0, 1, NT, true>(P);
}


// ---------------------------------------------------------------------------
// Smallest grids (below 2^13 nodes: the coarse pyramid levels): one wave per
// node (Q = 64).  A workgroup's four waves take four nodes of one column
// (tile = 4 x 1 nodes).  Per node and component:
//   node   the K^2 points over the wave's 64 lanes + a 6-level butterfly;
//   round 1  its four own edges (down/right x u/v), one per 16-lane group
//          (the Q = 16 edge order, edge_parts), the edge owner's clamped rou
//          update;
//   round 2  the four edges entering it (from the node above / to the left),
//          again one per group -- the neighbour recomputes nothing for it and
//          no LDS or grid exchange is needed;
// then the update of the node.  The work of the round-2 edges is done twice
// (by the owner for its rou and du1/do1, by the tail node for du2/do2), which
// costs nothing here: each wave's dependent chain is one node's 2 points +
// two edge jobs instead of 8 points + five jobs at Q = 16 (the lanes are
// idle otherwise at this size).  Same bits as the CPU model with split 64.
// Five waves per workgroup: the 30 x 40 level's 1200 nodes make 240
// workgroups, one per CU (with four, 300 workgroups put two on 44 CUs and
// those set the end of the launch).
// ---------------------------------------------------------------------------
constexpr int WN_THREADS = 64 * WN_TM;

template <typename R>
struct WnLds {
    fix128 red[GQMAP_LMAX + NFIX][WN_TM];
    R tab[NTAB * TS];
};

// One tile (WN_TM x 1 nodes) of one iteration; block b's partial row part_r.
// copy_tab: load the quadrature table into LDS first (the persistent kernel
// loads it once).
template <typename R, typename VT, int ENG, bool COH>
__device__ __forceinline__ void wn_tile(const IterParams<R, VT> &P, int tile, int it, int parity, double Tcur,
                                        int part_r, WnLds<R> &lds, bool copy_tab)
{
    Ctl *ctl = P.ctl;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int grp = lane >> 4, gl = lane & 15;  // 16-lane group of the edge jobs
    const int K2 = P.K2;
    const R *__restrict__ src = parity ? P.st1 : P.st0;
    R *__restrict__ dst = parity ? P.st0 : P.st1;
    const R T = R(Tcur);
    const R step = R(P.step0 / (1.0 + it / P.step_decay));
    const int tm = tile % P.tiles_m, tn = tile / P.tiles_m;
    const int m = tm * WN_TM + wave, n = tn;
    const int M = P.M, N = P.N;
    const int64_t MNL = P.MNL, MN = (int64_t)M * N;
    const bool inner = m < M && n < N && node_interior(P, m, n);  // wave-uniform
    fix128 fE = 0, fmu = 0, fsg = 0, fae = 0;
    int nonfinite = 0;
    auto &red = lds.red;
    const R *tab = lds.tab;

    for (int l = 0; l < P.L; ++l) {
        fix128 fda = 0;
        const int64_t i = m + (int64_t)M * n + MN * l;
        const int dir = grp & 1, uv = grp >> 1;
        const int64_t r = dir == 0 ? i + 1 : i + M;  // own edge: tail node (m+1,n) / (m,n+1)
        const int64_t h = dir == 0 ? i - 1 : i - M;  // entering edge: head node (m-1,n) / (m,n-1)
        // this node's state and the operands of the lane group's two edge
        // jobs, loaded before the table copy's barrier
        R mu_u = 0, mu_v = 0, sg_u = 0, sg_v = 0, pn = 0, p1 = 0, u2 = 0, o2 = 0, p2 = 0, hu = 0, ho = 0;
        if (inner) {
            mu_u = ld_state<COH>(src + i); mu_v = ld_state<COH>(src + i + MNL);
            sg_u = ld_state<COH>(src + i + MNL * 2); sg_v = ld_state<COH>(src + i + MNL * 3);
            pn = ld_state<COH>(src + i + MNL * 4);
            p1 = ld_state<COH>(src + i + MNL * (5 + grp)); u2 = ld_state<COH>(src + r + MNL * uv);
            o2 = ld_state<COH>(src + r + MNL * (2 + uv));
            p2 = ld_state<COH>(src + h + MNL * (5 + grp)); hu = ld_state<COH>(src + h + MNL * uv);
            ho = ld_state<COH>(src + h + MNL * (2 + uv));
        }
        if (l == 0 && copy_tab) {
            for (int e = tid; e < NTAB * K2; e += WN_THREADS) lds.tab[e] = P.tab[e];
            __syncthreads();
            TL_STAMP(1, __builtin_amdgcn_s_memrealtime());
        }
        if (inner) {
            const R a = R(ctl->alpha[l]);
            const R own_u = uv ? mu_v : mu_u, own_o = uv ? sg_v : sg_u;
            // node: 64 lanes
            const NodeCoef<R> c = node_coef(sg_u, sg_v, pn);
            Sums<R> S = node_sums<ENG, true>(tab, lane, K2, 64, frame_view(P.VV, P.M2), P.I1, P.Mo, P.No, P.epsn, c, mu_u,
                                             mu_v, m, n + P.n_off);
            S = lane_combine<64>(S);
            const Grad<R> nd = node_epi(S, c, P.lamd, P.guard != 0, T, a, sg_u, sg_v, pn, ENG == 2);
            // round 1: own edge e = grp (dir + 2 uv), Q = 16 in the group
            const EdgeCoef<R> c1 = edge_coef(own_u, u2, own_o, o2, p1);
            Sums<R> S1 = edge_sums_dev(tab, gl, K2, 16, P.epsn, c1);
            S1 = lane_combine<16>(S1);
            const Grad<R> g1 = edge_epi(S1, c1, P.lams, P.guard != 0, T, a, own_o, o2, p1, ENG == 2);
            if (gl == 0) st_state<COH, R>(dst + i + MNL * (5 + grp), fmin(fmax(p1 + g1.dp * step, -P.corr), P.corr));
            // round 2: the edge entering from the head node h (its edge grp)
            const EdgeCoef<R> c2 = edge_coef(hu, own_u, ho, own_o, p2);
            Sums<R> S2 = edge_sums_dev(tab, gl, K2, 16, P.epsn, c2);
            S2 = lane_combine<16>(S2);
            const Grad<R> g2 = edge_epi(S2, c2, P.lams, P.guard != 0, T, a, ho, own_o, p2, ENG == 2);
            // the four groups' results to every lane (group e's values from lane 16 e)
            auto from = [&](R v, int e) { return __shfl(v, 16 * e, 64); };
            R sum_mu0 = 0, sum_mu1 = 0, sum_sg0 = 0, sum_sg1 = 0, eE = 0, eda = 0;
            // iter_tile's order: edge jobs e = 0..3 accumulated in turn
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const R du1 = from(g1.du1, e), do1 = from(g1.do1, e);
                if ((e >> 1) == 0) { sum_mu0 = sum_mu0 + du1; sum_sg0 = sum_sg0 + do1; }
                else               { sum_mu1 = sum_mu1 + du1; sum_sg1 = sum_sg1 + do1; }
                eE = eE + from(g1.E, e);
                eda = eda + from(g1.da, e);
            }
            // the neighbours' shares: in_up[uv] from group 2 uv (dir 0), in_left[uv] from 2 uv + 1
            R up[2][2], left[2][2];
#pragma unroll
            for (int v = 0; v < 2; ++v) {
                up[v][0] = from(g2.du2, 2 * v); up[v][1] = from(g2.do2, 2 * v);
                left[v][0] = from(g2.du2, 2 * v + 1); left[v][1] = from(g2.do2, 2 * v + 1);
            }
            if (lane == 0) {
                const R gmu_u = ((nd.du1 + sum_mu0) + up[0][0]) + left[0][0];
                const R gmu_v = ((nd.du2 + sum_mu1) + up[1][0]) + left[1][0];
                const R gsg_u = ((nd.do1 + sum_sg0) + up[0][1]) + left[0][1];
                const R gsg_v = ((nd.do2 + sum_sg1) + up[1][1]) + left[1][1];
                fda = node_apply<ENG, COH>(P, dst, i, m, n, step, mu_u, mu_v, sg_u, sg_v, pn, nd, gmu_u, gmu_v, gsg_u,
                                      gsg_v, eE, eda, fE, fmu, fsg, fae, nonfinite);
            }
        }
        if (P.L > 1 && lane == 0) red[NFIX + l][wave] = fda;
        TL_STAMP(2, __builtin_amdgcn_s_memrealtime());
    }
    TL_STAMP(3, __builtin_amdgcn_s_memrealtime());
    // block partials: only lane 0 of each wave holds a node's contributions
    if (lane == 0) {
        red[0][wave] = fE;
        red[1][wave] = fmu;
        red[2][wave] = fsg;
        red[3][wave] = (fix128)nonfinite;
        red[4][wave] = fae;
    }
    __syncthreads();
    const int NP = NFIX + P.L;
    if (tid < NP) {
        fix128 v = 0;
#pragma unroll
        for (int w = 0; w < WN_TM; ++w) v += red[tid][w];
        if (P.fused || P.tile_acc) {
            if (v != 0) acc_add_agent(&ctl->acc[blockIdx.x % ACC_SLICES][tid][0], v);
        } else {
            store_part_agent(P.partials, P.fin.nblocks, part_r, tid, v);
        }
    }
}

template <typename R, typename VT, int ENG>
__global__ __launch_bounds__(WN_THREADS, 1) void k_iter_wn(IterParams<R, VT> P)
{
    Ctl *ctl = P.ctl;
    if (ctl->stop) return;
#if GQ_TIMELINE
    const unsigned long long tl0 = __builtin_amdgcn_s_memrealtime();
#endif
    const int nb = P.seg_n[0] + P.seg_n[1];
    const int b = blockIdx.x;
    const int tl = tile_of_block(b, nb, 1, P.cu_slots);
    const int tile = tl < P.seg_n[0] ? P.seg_lo[0] + tl : P.seg_lo[1] + (tl - P.seg_n[0]);
    __shared__ WnLds<R> lds;
    wn_tile<R, VT, ENG, false>(P, tile, P.spec ? ctl->it_i : ctl->it, (P.spec ? ctl->done_i : ctl->done) & 1,
                               P.spec ? ctl->T_i : ctl->T, P.part_off + b, lds, true);
    TL_STAMP(0, tl0);
    TL_STAMP(4, __builtin_amdgcn_s_memrealtime());
    if (P.fused) fused_finalize_tail(P.fin);
    else if (P.tile_acc) tile_totals_tail(P.fin, P.ticket_total, P.tile_totals);
}

// ---------------------------------------------------------------------------
// Persistent small-grid kernel (ctf engine, L = 1, every workgroup
// co-resident): one launch runs a chunk of iterations.  Workgroups 0..G-1 own
// one tile each (the k_iter / k_iter_wn tiles, same arithmetic, same bits);
// workgroup G is the finalizer.  Iteration j's state goes from one workgroup
// to its neighbours through device-coherent stores and loads (ld_state /
// st_state), its exact partial sums through partial rows (j & 1) * G + b,
// and a grid barrier (per-XCD-slot arrival counters, polled together by one
// wave) separates iteration j from j + 1.
//
// Nothing of the next iteration depends on the finalize step when L = 1
// except the stop rule: alpha is constant, the step size and the temperature
// decay depend only on the iteration number (each workgroup keeps its own T,
// updated as fin_apply updates Ctl::T).  So the finalizer reduces iteration
// j - 1 while the tiles compute iteration j; iteration j is speculative until
// finalize(j - 1) has run.  Before iteration j + 1 (after barrier j, by which
// the finalizer has finished finalize(j - 1)) every workgroup reads the stop
// flag: if iteration j - 1 met the stop rule, iteration j is discarded (it
// wrote the buffer that held state j - 2; state j - 1 is untouched and
// Ctl::done still points at it) and everyone exits.  This replaces per
// iteration: the launch gap, the LDS table copy and the serial fused finalize
// of the last workgroup.
// ---------------------------------------------------------------------------
constexpr int BAR_LINE = 32;  // unsigned words per 128-byte line: one counter per line
// BAR_STOP: 1 + the launch-local index of the iteration that met the stop
// rule (0: none).  Per iteration, not a flag: the finalizer may already be
// writing finalize(j - 1)'s verdict while a slow workgroup still reads
// finalize(j - 2)'s after barrier j - 1.
// BAR_INJECT (tests only, gqmap_debug_persist_fault): j + 1 makes barrier j
// of the next persistent launch fail as a timed-out one does.
constexpr int BAR_EXIT = 8 * BAR_LINE, BAR_FAIL = 9 * BAR_LINE, BAR_STOP = 10 * BAR_LINE, BAR_INJECT = 11 * BAR_LINE,
              BAR_WORDS = 12 * BAR_LINE;
constexpr unsigned BAR_SPIN_LIMIT = 1u << 21;  // polls (~1 us each) before a barrier gives up

// Arrival: every wave's stores (state, partial row) have completed, then one
// lane adds to the counter of its slot (blockIdx & 7: blocks of one XCD).
__device__ __forceinline__ void pbar_arrive(unsigned *bar)
{
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0)
        __hip_atomic_fetch_add(bar + (blockIdx.x & 7) * BAR_LINE, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Wait for barrier phase j (0-based) over nblk workgroups: wave 0 polls the 8
// slot counters (slot x receives (nblk - x + 7) / 8 arrivals per phase) and
// the failure word together.  Then the stop word: iteration j + 1 runs only
// if no iteration up to j - 1 met the stop rule (the finalizer judged those
// before its arrival at barrier j).  Returns true when the caller should go
// on: the barrier completed and no stop.  A spin that exceeds BAR_SPIN_LIMIT (the
// grid was not co-resident) raises the failure word and returns false; the
// host reports it.
__device__ __forceinline__ bool pbar_wait(unsigned *bar, int j, int nblk, int *sh_flag)
{
    if (threadIdx.x < 64) {
        const int x = threadIdx.x;
        const unsigned need = x < 8 ? (unsigned)((nblk - x + 7) >> 3) * (unsigned)(j + 1) : 0u;
        unsigned spins = 0;
        int go = 1;
        while (true) {
            unsigned v = 0xffffffffu, f = 0;
            if (x < 8) v = __hip_atomic_load(bar + x * BAR_LINE, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            else if (x == 8) f = __hip_atomic_load(bar + BAR_FAIL, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            else if (x == 9)  // injected failure of barrier j (tests): as a timeout below
                f = __hip_atomic_load(bar + BAR_INJECT, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (unsigned)(j + 1);
            if (__any(f != 0)) {
                if (x == 9 && f) __hip_atomic_store(bar + BAR_FAIL, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                go = 0;
                break;
            }
            if (__all(v >= need)) break;
            if (++spins > BAR_SPIN_LIMIT) {
                if (x == 0) __hip_atomic_store(bar + BAR_FAIL, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                go = 0;
                break;
            }
            __builtin_amdgcn_s_sleep(GQ_PERSIST_SLEEP);
        }
        if (x == 0) {
            if (go) {
                const unsigned st = __hip_atomic_load(bar + BAR_STOP, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (st != 0 && (int)st <= j) go = 0;  // iteration st - 1 <= j - 1 stopped the run
            }
            *sh_flag = go;
        }
    }
    __syncthreads();
    return *sh_flag != 0;
}

// Exit: the last workgroup out (all others are past their last poll) clears
// the counters for the next launch (the failure word stays for the host).
__device__ __forceinline__ void pbar_exit(unsigned *bar, int nblk)
{
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned old = __hip_atomic_fetch_add(bar + BAR_EXIT, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (old == (unsigned)nblk - 1) {
            for (int x = 0; x < 8; ++x)
                __hip_atomic_store(bar + x * BAR_LINE, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(bar + BAR_STOP, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(bar + BAR_EXIT, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

// Finalizer: exact reduction of partial rows [row0, row0 + rows) (L = 1: the
// NFIX fixed sums; integer adds, any order) into tot[].
__device__ void pfin_reduce(const FinParams &F, int row0, int rows, double *tot, fix128 (*sh)[8])
{
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, nw = blockDim.x >> 6;
    fix128 v[NFIX] = {};
    for (int r = tid; r < rows; r += blockDim.x)
#pragma unroll
        for (int q = 0; q < NFIX; ++q) v[q] += load_part_agent(F.partials, F.nblocks, row0 + r, q);
#pragma unroll
    for (int q = 0; q < NFIX; ++q) {
        const fix128 w = wave_sum_fix(v[q]);
        if (lane == 0) sh[q][wave] = w;
    }
    __syncthreads();
    if (tid < NFIX) {
        fix128 t = 0;
        for (int w = 0; w < nw; ++w) t += sh[tid][w];
        tot[tid] = from_fix(t);
    }
    __syncthreads();
}

template <typename R, typename VT, int ENG, int Q>
__global__ __launch_bounds__(Q == 64 ? WN_THREADS : BLOCK, Q == 64 ? 1 : min_waves(ENG, Q))
void k_iter_persist(IterParams<R, VT> P, int n_iter)
{
    Ctl *ctl = P.ctl;
    // nothing writes Ctl before the first barrier, which every workgroup
    // reaches only after these reads: all workgroups see the same values
    if (ctl->stop) return;
    unsigned *bar = P.bar;
    // a failed launch (this one, or an earlier one of the same replay): do
    // nothing -- the host restores the chunk's snapshot (k_persist_snap) and
    // re-runs it with one launch per iteration
    if (__hip_atomic_load(bar + BAR_FAIL, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) return;
    const int nblk = gridDim.x, G = nblk - 1, b = blockIdx.x;
    const int it0 = ctl->it, done0 = ctl->done;
    double T = ctl->T;
    __shared__ int sh_flag;
    if (b == G) {  // finalizer: finalize(j - 1) during iteration j
        __shared__ fix128 fsh[NFIX][8];
        __shared__ double tot[NFIX];
        for (int j = 0; j <= n_iter; ++j) {
            if (j > 0) {
                if (!pbar_wait(bar, j - 1, nblk, &sh_flag)) break;
                pfin_reduce(P.fin, ((j - 1) & 1) * G, G, tot, fsh);
                if (threadIdx.x == 0) {
                    fin_apply(P.fin, tot);
                    // the verdict travels device-coherent (read by pbar_wait)
                    if (ctl->stop)
                        __hip_atomic_store(bar + BAR_STOP, (unsigned)j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
            }
            if (j < n_iter) pbar_arrive(bar);
        }
        pbar_exit(bar, nblk);
        return;
    }
    const int tile = tile_of_block(b, G, Q == 64 ? 1 : P.cu_group, P.cu_slots);
    const bool edge_first = GQ_PHASE_MIX && Q != 64 && (((b >> 3) / P.cu_slots) & 1);
    for (int j = 0; j < n_iter; ++j) {
        if (j > 0 && !pbar_wait(bar, j - 1, nblk, &sh_flag)) break;
        const int it = it0 + j, parity = (done0 + j) & 1, part_r = ((j & 1) * G) + b;
        if constexpr (Q == 64) {
            __shared__ WnLds<R> lds_wn;
            wn_tile<R, VT, ENG, true>(P, tile, it, parity, T, part_r, lds_wn, j == 0);
        } else {
            __shared__ TileLdsQ<R, Q> lds;
            if (edge_first)
                iter_tile<R, VT, ENG, Q, true, true>(P, tile, it, parity, part_r, lds, 0, P.L, T, j > 0);
            else
                iter_tile<R, VT, ENG, Q, false, true>(P, tile, it, parity, part_r, lds, 0, P.L, T, j > 0);
        }
        pbar_arrive(bar);
        // fin_apply's temperature decay after iteration it (gqmap_gpuSuper_mix_entropy.m:72)
        if (P.fin.t_decay_every > 0 && it % P.fin.t_decay_every == 0) T = fmax(T * P.fin.drate, P.fin.t_min);
    }
    pbar_exit(bar, nblk);
}

// Before every persistent / dataflow launch: the state it starts from (the
// current ping-pong buffer and Ctl), unless a launch has already failed or
// the run has stopped -- then the snapshot of the failed (or stopping)
// launch's start is kept for the host to restore (persist_recover,
// ovr_recover).
template <typename R>
__global__ __launch_bounds__(256) void k_persist_snap(const Ctl *ctl, const unsigned *bar, const R *st0, const R *st1,
                                                      R *snap, Ctl *snap_ctl, int64_t n)
{
    if (__hip_atomic_load(bar + BAR_FAIL, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0 || ctl->stop) return;
    const R *cur = (ctl->done & 1) ? st1 : st0;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        snap[i] = cur[i];
    if (blockIdx.x == 0) {
        constexpr int W = (int)(sizeof(Ctl) / sizeof(uint32_t));
        static_assert(sizeof(Ctl) % sizeof(uint32_t) == 0, "Ctl words");
        const uint32_t *a = reinterpret_cast<const uint32_t *>(ctl);
        uint32_t *d = reinterpret_cast<uint32_t *>(snap_ctl);
        for (int w = threadIdx.x; w < W; w += blockDim.x) d[w] = a[w];
    }
}

// ---------------------------------------------------------------------------
// Dataflow launch of the single-scale engine (policy `flow`, opt-in; fp64/fp32
// mixture, L = 1, one lane per node, whole grid).  One launch runs a chunk of
// iterations without a grid barrier: resident workgroups claim (iteration,
// tile) items in order from the queue of their XCD (blockIdx & 7; each XCD's
// queue walks its band of tiles, iteration-major) and run one tile of one
// iteration each -- iter_tile, the same arithmetic and bits as k_iter.  Item
// (j, t) starts when tile t and its four neighbours have finished iteration
// j - 1 (Jacobi: it reads their state j - 1; and the buffer it writes held
// state j - 2, which they read during j - 1), and when iterations up to j - 2
// are finalized.  So the tiles of iteration j + 1 fill the CUs that the tail
// of iteration j leaves idle: a launch per iteration pays for its busiest
// CU's tile count (C2: 925 tiles on 768 resident slots).
//
// Deadlock-free without co-residency: an item is claimed only by a running
// workgroup, which holds it until done, and waits only for items earlier in
// its own queue's order or of the previous iteration in a neighbouring band;
// the earliest unfinished item therefore always has its inputs.  Spins are
// still bounded: a timeout raises the persistent path's failure word
// (BAR_FAIL), every workgroup leaves, and the host restores the chunk's
// snapshot and goes on with one launch per iteration (persist_recover).
//
// Totals: each tile adds its exact sums into the accumulator slot of its
// iteration (j % GQ_FLOW_LAG); the tile arriving last for iteration j waits for
// finalize(j - 1), then reduces the slot and runs fin_apply (acquire and
// release fences around it: the previous finalizer may have run on another
// XCD) and publishes the finalized count.  The stop rule: finalize(s) stores
// 1 + s in the stop word before it publishes; items of iteration >= s + 1
// that see it leave, and those of iteration >= s + 2 see it (they wait for
// finalize(s)); iteration s + 1 may already
// have run -- it wrote the buffer of state s - 1 -- and its finalize is
// skipped, so Ctl and the buffer holding state s stay as the whole-grid run
// leaves them.  State moves between workgroups through device-coherent
// (agent-scope) loads and stores (ld_state / st_state).
// ---------------------------------------------------------------------------
// GQ_FLOW_LAG: iterations an item may run ahead of the finalize -- item j
// starts once iterations up to j - GQ_FLOW_LAG are finalized.  2 (kept): the
// buffer an item writes never holds a state that may have met the stop
// rule.  Deeper (a diagnostic): an item of iteration s + 2 may overwrite the
// buffer of a state s that met it; the launch then records the overshoot
// (Ctl::ovr) and the host restores the chunk's snapshot and re-runs up to s
// with one launch per iteration (ovr_recover).  The timeline of the lag-2
// form shows items waiting 24% of their time; lags 4, 6 and 8 left both the
// wait (lag 6: 24%) and C2 / the C3 levels unchanged within 1%
// (profiles/r06_flow_lag_ab.txt, r06_flow_timeline_lag{2,6}.txt): the wait
// is the neighbour dependencies -- a band of 116 tiles per XCD against 96
// resident slots leaves about 1.2 item-times between an item's claim and
// its neighbours' claims of the previous iteration -- not the finalize.
#ifndef GQ_FLOW_LAG
#define GQ_FLOW_LAG 2
#endif
constexpr int FL_SLOTS = GQ_FLOW_LAG;              // accumulator / ticket slots (iteration j: j % FL_SLOTS)
constexpr int FL_LINE = 32;                        // 32-bit words per 128-byte line
constexpr int FL_Q = 0;                            // 8 per-XCD claim counters, a line each
constexpr int FL_FIN = 8 * FL_LINE;                // iterations finalized (launch-local)
constexpr int FL_STOP = 9 * FL_LINE;               // 1 + the launch-local iteration that stopped the run
constexpr int FL_EXIT = 10 * FL_LINE;              // workgroups that have left
constexpr int FL_MAXJ = 11 * FL_LINE;              // 1 + the largest iteration an item started
constexpr int FL_ARR = 12 * FL_LINE;               // arrival tickets of the slots (a line each)
constexpr int FL_ACC = FL_ARR + FL_SLOTS * FL_LINE;  // the slots' ACC_SLICES x (NFIX + LMAX) x 4 u64 limbs
constexpr int FL_ACC_SLOT = ACC_SLICES * (NFIX + GQMAP_LMAX) * 4;  // u64 per slot
constexpr int FL_DONE = FL_ACC + 2 * FL_SLOTS * FL_ACC_SLOT;       // per tile: iterations done (launch-local)
constexpr int flow_words(int ntiles) { return FL_DONE + ntiles; }
static_assert(FL_SLOTS >= 2, "the finalize lag is at least 2");
static_assert((FL_ACC & 1) == 0, "u64 alignment of the accumulator slots");

// Wait (wave 0 polls, the workgroup follows) until item (j, tile) may run.
// Returns 1: run it; 0: leave (the run stopped before iteration j - 1, or a
// failure -- injected, another workgroup's, or this spin's own timeout).
// Per-tile counters are per (tile, component) item: index tile * L + l (the
// super engine's mixture components are separate items, L > 1).  fin_need:
// the finalized count item j needs -- j - 1 normally (iterations up to
// j - 2), j when finalize(j - 1) updated alpha (L > 1 past alpha_start).
__device__ __forceinline__ int flow_wait(unsigned *fl, unsigned *bar, int tiles_m, int ntiles, int tile, int l,
                                         int L, int j, int fin_need, int *sh)
{
    if (threadIdx.x < 64) {
        const int x = threadIdx.x;
        const int tm = tile % tiles_m;
        int dep = -1;  // the tile whose iteration j - 1 this lane waits for
        if (j > 0) {
            if (x == 0) dep = tile;
            else if (x == 1 && tm > 0) dep = tile - 1;
            else if (x == 2 && tm < tiles_m - 1 && tile + 1 < ntiles) dep = tile + 1;
            else if (x == 3 && tile >= tiles_m) dep = tile - tiles_m;
            else if (x == 4 && tile + tiles_m < ntiles) dep = tile + tiles_m;
        }
        if (dep >= 0) dep = dep * L + l;
        unsigned spins = 0;
        int go = 1;
        while (true) {
            bool ok = true, leave = false;
            if (dep >= 0) ok = __hip_atomic_load(fl + FL_DONE + dep, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= (unsigned)j;
            else if (x == 5 && fin_need > 0) ok = __hip_atomic_load(fl + FL_FIN, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= (unsigned)fin_need;
            else if (x == 6) {  // the run stopped at an earlier iteration (st - 1 < j)
                const unsigned st = __hip_atomic_load(fl + FL_STOP, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                leave = st != 0 && (int)st - 1 < j;
            } else if (x == 7) {
                leave = __hip_atomic_load(bar + BAR_FAIL, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
            } else if (x == 8) {  // injected failure (tests): at the first item of iteration j
                leave = __hip_atomic_load(bar + BAR_INJECT, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (unsigned)(j + 1);
                if (leave) __hip_atomic_store(bar + BAR_FAIL, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            if (__any(leave)) { go = 0; break; }
            if (__all(ok)) break;
            if (++spins > BAR_SPIN_LIMIT) {
                if (x == 0) __hip_atomic_store(bar + BAR_FAIL, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                go = 0;
                break;
            }
            __builtin_amdgcn_s_sleep(GQ_PERSIST_SLEEP);
        }
        // The lanes read the finalized count and the stop word in the same
        // poll, unordered: lane 6 may have read a stop word older than the
        // count lane 5 saw.  finalize(s) stores the stop word before it
        // publishes the count (release), so after an acquire load of the
        // count the stop word is current: an item past a stop never runs
        // (at lag 2 an item of iteration s + 2 would overwrite state s).
        if (x == 0 && go && fin_need > 0) {
            (void)__hip_atomic_load(fl + FL_FIN, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
            const unsigned st = __hip_atomic_load(fl + FL_STOP, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (st != 0 && (int)st - 1 < j) go = 0;
        }
        if (x == 0) *sh = go;
    }
    __syncthreads();
    return *sh;
}

// The last tile of iteration j to arrive: finalize(j) after finalize(j - 1).
__device__ void flow_finalize(const FinParams &F, unsigned *fl, unsigned *bar, unsigned long long *slot, int j,
                              double *tot, unsigned long long *sh, int *shf)
{
    if (threadIdx.x == 0) {
        unsigned spins = 0;
        int go = 1;
        while (__hip_atomic_load(fl + FL_FIN, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < (unsigned)j) {
            if (__hip_atomic_load(bar + BAR_FAIL, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0 ||
                ++spins > BAR_SPIN_LIMIT) {
                __hip_atomic_store(bar + BAR_FAIL, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                go = 0;
                break;
            }
            __builtin_amdgcn_s_sleep(GQ_PERSIST_SLEEP);
        }
        // a run stopped at an earlier iteration: Ctl keeps that iteration
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");  // (the stop word is stored before FL_FIN)
        if (go && __hip_atomic_load(fl + FL_STOP, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) go = 2;
        *shf = go;
    }
    __syncthreads();
    const int go = *shf;
    if (go == 0) return;
    if (go == 1) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");  // Ctl and the trace as the previous finalizer left them
        fin_reduce_acc(F, tot, sh, slot);
        if (threadIdx.x == 0) {
            fin_apply(F, tot);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
            if (F.ctl->stop) __hip_atomic_store(fl + FL_STOP, (unsigned)(j + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    if (threadIdx.x == 0) {
        __hip_atomic_store(fl + FL_ARR + (j % FL_SLOTS) * FL_LINE, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(fl + FL_FIN, (unsigned)(j + 1), __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// snap: Ctl as the launch found it (k_persist_snap, launched just before):
// a workgroup dispatched late must not read Ctl after a finalize changed it.
// GQ_FLOW_TL (diagnostic builds): per item (j, tile) of a launch that starts
// at iteration 1, four words at (j * items + tile) -- the claim, the end of the dependency wait,
// the end of the item, and (XCC_ID << 32 | HW_ID) -- read back with
// gqmap_debug_flow_timeline (scripts/flow_timeline.py).
#ifndef GQ_FLOW_TL
#define GQ_FLOW_TL 0
#endif
#if GQ_FLOW_TL
constexpr int FLOW_TL_WORDS = 1 << 18;
__device__ unsigned long long g_flow_tl[FLOW_TL_WORDS];
#endif
// Waves per SIMD the allocation must allow at one lane per node.  2 (<= 256
// VGPRs): the C2 fp64 kernel takes 215 and spills nothing (at 3, as k_iter
// on C2: 167 + 144 bytes of scratch), and the 512 resident slots leave a band
// of 116 tiles ~64 items in flight -- more slack for the neighbour
// dependencies; C2 fp64 142.9 -> 139.6 us/it (graph), the 480x640 ctf level
// ~278 -> ~275 (profiles/r06_flow_2waves_ab.txt, same checksums).
#ifndef GQ_FLOW_WAVES
#define GQ_FLOW_WAVES 2
#endif
#ifndef GQ_FLOW_LIT_WAVES  // the same for the literal-order instantiation (2: <= 256 VGPRs, no spills)
#define GQ_FLOW_LIT_WAVES 2
#endif
#ifndef GQ_FLOW_MIX  // node-first / edge-first alternation among co-resident workgroups
#define GQ_FLOW_MIX 1
#endif
#ifndef GQ_FLOW_LIT_MIX
#define GQ_FLOW_LIT_MIX 0
#endif
#ifndef GQ_FLOW_COH  // device-coherent state access (0: plain -- timing experiments only, not coherent)
#define GQ_FLOW_COH 1
#endif
#ifndef GQ_FLOW_PREFETCH  // claim the next item while the current one runs (measured: +18%, reservation skew)
#define GQ_FLOW_PREFETCH 0
#endif
#ifndef GQ_FLOW_PAIR  // the next claim issued together with the arrival ticket (one round trip)
#define GQ_FLOW_PAIR 0
#endif
// Each XCD queue walks its band row by row (band_row_tile) instead of down
// the tile columns: a tile's left / right neighbours are then one queue
// position away instead of a tile column (C2: 25 positions), so the items
// of iteration j + 1 rarely find a neighbour of iteration j still running
// (about 96 items are in flight per XCD against a band of 116).
#ifndef GQ_FLOW_ROWS
#define GQ_FLOW_ROWS 1
#endif
// W > 0: the waves per SIMD, overriding the defaults above (the large-frame
// instantiation, launch_flow_q)
template <typename R, typename VT, int ENG, int Q, bool LIT = false, int W = 0>
__global__ __launch_bounds__(BLOCK, W > 0 ? W : LIT ? GQ_FLOW_LIT_WAVES : Q == 1 ? GQ_FLOW_WAVES : ENG == 1 ? 2 : min_waves(ENG, Q))
void k_iter_flow(IterParams<R, VT> P, int n_iter, unsigned *fl, int ntiles, const Ctl *snap)
{
    static_assert(Q >= 1 && Q <= 4, "1..4 lanes per node");
    static_assert(!LIT || (ENG == 0 && Q == 1), "literal order: the mixture engine at one lane per node");
    unsigned *bar = P.bar;
    // a stopped run, or a failed launch earlier in the replay (whose
    // snapshot the host restores): nothing to do but take the exit ticket.
    // (Ctl's own stop word too: after a stop the snapshot is not refreshed;
    // within this launch it only turns to 1 once the run has stopped.)
    const bool run = !snap->stop && __hip_atomic_load(&P.ctl->stop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0 &&
                     __hip_atomic_load(bar + BAR_FAIL, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0;
    const int it0 = snap->it, done0 = snap->done;
    const double T0 = snap->T;
    const int b = blockIdx.x, xcd = b & 7;
    int s0 = 0;
    for (int y = 0; y < xcd; ++y) s0 += (ntiles - y + 7) >> 3;
    const int nb = (ntiles - xcd + 7) >> 3;  // this XCD's band: tiles [s0, s0 + nb)
    // items per tile and iteration: one per mixture component for the super
    // engine (its node grid is small; a tile's components run back to back
    // in the queue), one otherwise (L = 1)
    const int L = ENG == 1 ? P.L : 1, nbl = nb * L, nitems = ntiles * L;
    constexpr int INV = ENG == 2 && Q == 1 ? GQ_PHASE_MIX_CTF_Q1_INV : GQ_PHASE_MIX_OTHER_INV;
    // (the phase mix: the fast mixture engine; the literal kernel's with
    // GQ_FLOW_LIT_MIX -- its second instantiation spilled at 3 waves)
    constexpr bool MIX = GQ_FLOW_MIX && ENG == 0 && (!LIT || GQ_FLOW_LIT_MIX);
    const bool edge_first = MIX && ((((b >> 3) / P.cu_slots) & 1) != INV);
    __shared__ TileLdsQ<R, Q> lds;
    __shared__ int sh_i, sh_go, sh_last;
    __shared__ double tot[NFIX + GQMAP_LMAX];
    __shared__ unsigned long long sh_acc[4 * (NFIX + GQMAP_LMAX)];
    unsigned long long *acc = reinterpret_cast<unsigned long long *>(fl + FL_ACC);
    unsigned *q = fl + FL_Q + xcd * FL_LINE;
    unsigned nxt = 0;  // thread 0: the claim issued during the previous item
    if (run && nb > 0 && GQ_FLOW_PREFETCH && threadIdx.x == 0)
        nxt = __hip_atomic_fetch_add(q, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    bool have = false;  // GQ_FLOW_PAIR: sh_i already holds the next claim
    while (run && nb > 0) {
        if (threadIdx.x == 0 && !(GQ_FLOW_PAIR && have)) {
            if (GQ_FLOW_PREFETCH) {
                sh_i = (int)nxt;
                // the next claim goes out now; its latency hides behind this
                // item's first state loads (a claim past the last item is harmless)
                if ((int)nxt / nbl < n_iter) nxt = __hip_atomic_fetch_add(q, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            } else {
                sh_i = (int)__hip_atomic_fetch_add(q, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
        __syncthreads();
        const int i = sh_i, j = i / nbl, pos = (i % nbl) / L, l = ENG == 1 ? i % L : 0;
        if (j >= n_iter) break;
        const int tile = GQ_FLOW_ROWS ? band_row_tile(pos, s0, s0 + nb, P.tiles_m) : s0 + pos;
        const int it = it0 + j, parity = (done0 + j) & 1;
        // finalize(j - 1) changed alpha (fin_apply: it - 1 > alpha_start, L > 1)
        const bool alpha_moved = P.L > 1 && it - 1 > P.fin.alpha_start;
#if GQ_FLOW_TL
        const unsigned long long tl_claim = __builtin_amdgcn_s_memrealtime();
#endif
        if (!flow_wait(fl, bar, P.tiles_m, ntiles, tile, l, L, j, alpha_moved ? j : j - GQ_FLOW_LAG + 1, &sh_go)) break;
        if (GQ_FLOW_LAG > 2 && threadIdx.x == 0)  // (for the overshoot check at the exit)
            __hip_atomic_fetch_max(fl + FL_MAXJ, (unsigned)(j + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#if GQ_FLOW_TL
        const unsigned long long tl_go = __builtin_amdgcn_s_memrealtime();
#endif
        double T = T0;  // fin_apply's temperature decay after each earlier iteration
        if (P.fin.t_decay_every > 0)
            for (int q = it0; q < it; ++q)
                if (q % P.fin.t_decay_every == 0) T = fmax(T * P.fin.drate, P.fin.t_min);
        unsigned long long *slot = acc + (size_t)(j % FL_SLOTS) * FL_ACC_SLOT;
        const int l0 = ENG == 1 ? l : 0, l1 = ENG == 1 ? l + 1 : 1;  // (L = 1 unless super)
        if (MIX && edge_first)
            iter_tile<R, VT, ENG, Q, true, GQ_FLOW_COH, false, LIT>(P, tile, it, parity, 0, lds, l0, l1, T, false, slot);
        else
            iter_tile<R, VT, ENG, Q, false, GQ_FLOW_COH, false, LIT>(P, tile, it, parity, 0, lds, l0, l1, T, false, slot);
        // publish: every wave's stores (state, rou, the slot's sums) are done
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
#if GQ_FLOW_TL
        const size_t tli = (size_t)j * nitems + (size_t)tile * L + l;  // (iteration, tile, component)
        if (threadIdx.x == 0 && (tli + 1) * 4 <= (size_t)FLOW_TL_WORDS && snap->it == 1) {
            unsigned long long *w = g_flow_tl + tli * 4;
            w[0] = tl_claim;
            w[1] = tl_go;
            w[2] = __builtin_amdgcn_s_memrealtime();
            w[3] = ((unsigned long long)__builtin_amdgcn_s_getreg((31 << 11) | 20) << 32) |
                   (unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 4);
        }
#endif
        if (threadIdx.x == 0) {
            __hip_atomic_store(fl + FL_DONE + tile * L + l, (unsigned)(j + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const unsigned tk = __hip_atomic_fetch_add(fl + FL_ARR + (j % FL_SLOTS) * FL_LINE, 1u, __ATOMIC_RELAXED,
                                                       __HIP_MEMORY_SCOPE_AGENT);
            if (GQ_FLOW_PAIR) sh_i = (int)__hip_atomic_fetch_add(q, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            sh_last = tk == (unsigned)(nitems - 1);
        }
        have = true;
        __syncthreads();
        if (sh_last) flow_finalize(P.fin, fl, bar, slot, j, tot, sh_acc, &sh_go);
        __syncthreads();
    }
    // the last workgroup out clears the queue state for the next launch
    __syncthreads();
    if (threadIdx.x == 0)
        sh_last = __hip_atomic_fetch_add(fl + FL_EXIT, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1;
    __syncthreads();
    if (sh_last) {
        if (threadIdx.x == 0 && GQ_FLOW_LAG > 2) {
            // an item of iteration >= s + 2 ran after the stop at s: the
            // buffer of state s may be overwritten -- the host recovers
            const unsigned st = __hip_atomic_load(fl + FL_STOP, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const unsigned mj = __hip_atomic_load(fl + FL_MAXJ, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (st != 0 && mj >= st + 2) __hip_atomic_store(&P.ctl->ovr, (int)st, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        __syncthreads();
        for (int w = threadIdx.x; w < flow_words(nitems); w += blockDim.x)
            __hip_atomic_store(fl + w, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

__global__ __launch_bounds__(256) void k_finalize(FinParams F)
{
    if (F.ctl->stop) return;
    __shared__ fix128 sh[256];
    __shared__ double tot[NFIX + GQMAP_LMAX];
    fin_reduce(F, tot, sh);
    if (threadIdx.x == 0) fin_apply(F, tot);
}

// Deferred-totals RCCL sequence (launch_seq_deferred): the state buffer the
// sequence starts from and Ctl, unless the run has stopped (an earlier
// sequence's snapshot is then the one a recovery needs).
template <typename R>
__global__ __launch_bounds__(256) void k_seq_snap(const Ctl *ctl, const R *st0, const R *st1, R *snap, Ctl *snap_ctl,
                                                  int64_t n)
{
    if (ctl->stop) return;
    const R *cur = (ctl->done & 1) ? st1 : st0;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        snap[i] = cur[i];
    if (blockIdx.x == 0) {
        constexpr int W = (int)(sizeof(Ctl) / sizeof(uint32_t));
        const uint32_t *a = reinterpret_cast<const uint32_t *>(ctl);
        uint32_t *d = reinterpret_cast<uint32_t *>(snap_ctl);
        for (int w = threadIdx.x; w < W; w += blockDim.x) d[w] = a[w];
    }
}

// The end of a deferred sequence of n iterations: rows [rank][n][NP] of all
// tiles' exact totals (the all-gather of d_rows), reduced row by row in
// iteration order and applied with fin_apply -- the trace, it / done / T and
// the stop rule exactly as the whole grid's finalize.  A stop met before the
// last row means the sequence's later iterations have already run: Ctl::ovr
// = row + 1 tells the host to recover (ovr_recover).  One workgroup.
__global__ __launch_bounds__(256) void k_finalize_seq(FinParams F, const fix128 *rows, int n)
{
    Ctl *ctl = F.ctl;
    const int NP = NFIX + F.L;
    // every row's exact totals at once (n NP sums over the ranks), then the
    // rows applied in iteration order by one thread
    __shared__ double tot[GRAPH_CHUNK][NFIX + GQMAP_LMAX];
    if (ctl->stop) return;
    for (int t = threadIdx.x; t < n * NP; t += blockDim.x) {
        const int i = t / NP, q = t - i * NP;
        fix128 v = 0;
        for (int r = 0; r < F.nranks; ++r) v += rows[((int64_t)r * n + i) * NP + q];
        tot[i][q] = from_fix(v);
    }
    __syncthreads();
    if (threadIdx.x != 0) return;
    for (int i = 0; i < n; ++i) {
        fin_apply(F, tot[i]);
        if (ctl->stop) {
            if (i < n - 1) ctl->ovr = i + 1;
            return;
        }
    }
}

// Tiled mode: this tile's block partials -> its exact totals (one row of the
// gathered table; the other rows arrive from the other tiles).
__global__ __launch_bounds__(256) void k_reduce_local(const fix128 *partials, int nblocks, int NP,
                                                      fix128 *out, const Ctl *ctl)
{
    if (ctl->stop) return;
    __shared__ fix128 sh[256];
    const int tid = threadIdx.x;
    for (int q = 0; q < NP; ++q) {
        fix128 v = 0;
        for (int b = tid; b < nblocks; b += 256) {
            const uint64_t *w = reinterpret_cast<const uint64_t *>(partials);
            v += (fix128)(((unsigned __int128)w[part_word(nblocks, b, q, 1)] << 64) | w[part_word(nblocks, b, q, 0)]);
        }
        sh[tid] = v;
        __syncthreads();
        for (int st = 128; st > 0; st >>= 1) {
            if (tid < st) sh[tid] += sh[tid + st];
            __syncthreads();
        }
        if (tid == 0) out[q] = sh[0];
        __syncthreads();
    }
}

// Ghost-column exchange: the column k_iter just wrote (the ping-pong
// destination, chosen by the device-side parity) <-> a contiguous buffer of
// np x L x M values, the planes listed 4 bits each in `planes`.  Column-major
// planes make each (plane, component) column one contiguous run of M.
//
// Only what the neighbour reads travels.  A tile recomputes the edges between
// its left ghost and its first owned column -- they are the ghost's right
// edges (dir 2): u1, o1 and rou(dir 2) of the ghost, gqmap_gpu_mixture.m:31-35
// -- and its last owned column's right edges into the right ghost read that
// ghost's mu and sigma.  pn and rou(dir 1) of a ghost are never read.
constexpr uint32_t HALO_TO_LEFT = 0x3210;      // mu_u, mu_v, sigma_u, sigma_v
constexpr int HALO_TO_LEFT_N = 4;
constexpr uint32_t HALO_TO_RIGHT = 0x863210;   // + rou(dir 2, u), rou(dir 2, v) (planes 6, 8)
constexpr int HALO_TO_RIGHT_N = 6;

// One side of an exchange: column col <-> buf, planes listed 4 bits each.
template <typename R>
struct HaloSide {
    int col, np;
    uint32_t planes;
    R *buf;
};
// Pack: the tile's boundary columns of the buffer the iteration just wrote
// -> the send buffers, both sides in one launch (blockIdx.y picks the side;
// the strip ends have one).
template <typename R>
__global__ void k_halo_copy(const Ctl *ctl, R *st0, R *st1, int M, int64_t MN, int64_t MNL, int L,
                            HaloSide<R> s0, HaloSide<R> s1, int spec)
{
    if (ctl->stop) return;
    R *dst = ((spec ? ctl->done_i : ctl->done) & 1) ? st0 : st1;
    const HaloSide<R> &hs = blockIdx.y == 0 ? s0 : s1;
    const int col = hs.col, np = hs.np;
    const uint32_t planes = hs.planes;
    R *buf = hs.buf;
    const int64_t n = (int64_t)np * L * M;
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < n; t += (int64_t)gridDim.x * blockDim.x) {
        const int m = (int)(t % M);
        const int64_t ql = t / M;  // qi * L + l
        const int q = (int)((planes >> (4 * (int)(ql / L))) & 15u), l = (int)(ql % L);
        R *p = dst + (int64_t)q * MNL + (int64_t)l * MN + (int64_t)col * M + m;
        buf[t] = *p;
    }
}

// A tile's ghost-column unpack and its finalize in one launch (one
// workgroup): the received columns go into the state buffer the iteration
// just wrote (parity read before fin_apply flips it), then the exact
// reduction of all tiles' totals and the iteration's control step.
template <typename R>
__global__ __launch_bounds__(256) void k_unpack_finalize(FinParams F, R *st0, R *st1, int M, int64_t MN,
                                                         int64_t MNL, int L, HaloSide<R> s0, HaloSide<R> s1,
                                                         int nsides)
{
    Ctl *ctl = F.ctl;
    if (ctl->stop) return;
    R *dst = (ctl->done & 1) ? st0 : st1;
    for (int k = 0; k < nsides; ++k) {
        const HaloSide<R> &hs = k == 0 ? s0 : s1;
        const int64_t n = (int64_t)hs.np * L * M;
        for (int64_t t = threadIdx.x; t < n; t += 256) {
            const int m = (int)(t % M);
            const int64_t ql = t / M;
            const int q = (int)((hs.planes >> (4 * (int)(ql / L))) & 15u), l = (int)(ql % L);
            dst[(int64_t)q * MNL + (int64_t)l * MN + (int64_t)hs.col * M + m] = hs.buf[t];
        }
    }
    __shared__ fix128 sh[256];
    __shared__ double tot[NFIX + GQMAP_LMAX];
    fin_reduce(F, tot, sh);  // (its barriers order every thread's parity read before fin_apply)
    if (threadIdx.x == 0) {
        fin_apply(F, tot);
        ctl->it_i = ctl->it;  // the kernels' counters follow (a later deferred sequence starts here)
        ctl->done_i = ctl->done;
        ctl->T_i = ctl->T;
    }
}

// Deferred-totals RCCL tile (L = 1): the received ghost columns into the state
// buffer the iteration just wrote, then the iteration counters the kernels
// run by -- the same steps fin_apply takes (temperature decay after
// iteration it_i, it + 1, done + 1), without waiting for the totals: nothing
// of the next iteration depends on them but the stop rule, which the
// sequence's finalize (k_finalize_seq) judges at the end of the sequence.
template <typename R>
__global__ __launch_bounds__(256) void k_unpack_advance(Ctl *ctl, R *st0, R *st1, int M, int64_t MN, int64_t MNL,
                                                        int L, HaloSide<R> s0, HaloSide<R> s1, int nsides,
                                                        int t_decay_every, double drate, double t_min)
{
    if (ctl->stop) return;
    R *dst = (ctl->done_i & 1) ? st0 : st1;
    for (int k = 0; k < nsides; ++k) {
        const HaloSide<R> &hs = k == 0 ? s0 : s1;
        const int64_t n = (int64_t)hs.np * L * M;
        for (int64_t t = threadIdx.x; t < n; t += 256) {
            const int m = (int)(t % M);
            const int64_t ql = t / M;
            const int q = (int)((hs.planes >> (4 * (int)(ql / L))) & 15u), l = (int)(ql % L);
            dst[(int64_t)q * MNL + (int64_t)l * MN + (int64_t)hs.col * M + m] = hs.buf[t];
        }
    }
    __syncthreads();  // every thread's parity read before the advance
    if (threadIdx.x == 0) {
        const int it = ctl->it_i;
        if (t_decay_every > 0 && it % t_decay_every == 0) ctl->T_i = fmax(ctl->T_i * drate, t_min);
        ctl->it_i = it + 1;
        ctl->done_i = ctl->done_i + 1;
    }
}

template <typename R>
__global__ void k_init_state(R *st0, R *st1, int64_t MNL, uint64_t b1, uint64_t b2, uint64_t b3,
                             uint64_t b4, double minu, double maxu, double minv, double maxv,
                             double sig_init, int M, int N, int n_off, int Ng)
{
    const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (i >= MNL) return;
    // the random streams are indexed by the GLOBAL node index, so a tile draws
    // exactly the values the untiled grid has in its columns
    const int64_t MN = (int64_t)M * N;
    const int64_t l = i / MN, rem = i % MN;
    const int64_t g = rem % M + (int64_t)M * (rem / M + n_off) + (int64_t)M * Ng * l;
    // gqmap_gpu_mixture.m:19-24 (gqmap_ctf.m:14-17: sigma = rand + 3); no
    // contraction: same bits as the host formula
    const double su = sig_init < 0 ? maxu - minu : sig_init, sv = sig_init < 0 ? maxv - minv : sig_init;
    const R v[NPLANES] = {R(minu + u01(b1, g) * (maxu - minu)), R(minv + u01(b2, g) * (maxv - minv)),
                          R(u01(b3, g) + su),                   R(u01(b4, g) + sv),
                          R(0), R(0), R(0), R(0), R(0)};
#pragma unroll
    for (int q = 0; q < NPLANES; ++q) {
        st0[i + MNL * q] = v[q];
        st1[i + MNL * q] = v[q];
    }
}

__device__ __forceinline__ double wave_sum(double v)
{
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// profile_logP (gqmap_gpu_mixture.m:148-154; super :152-169): per-block partials.
template <typename R, typename VT, bool SUPER>
__global__ __launch_bounds__(256) void k_logp(IterParams<R, VT> P, const R *__restrict__ map,
                                              double *partials)
{
    const int64_t MN = (int64_t)P.M * P.N;
    const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    double v = 0;
    if (i < MN) {
        const int m = (int)(i % P.M), n = (int)(i / P.M);
        if (m >= 1 && m <= P.M - 2 && n >= 1 && n <= P.N - 2) {
            const R u = map[i], w = map[i + MN];
            if constexpr (!SUPER) {
                const R d = P.I1[m + (int64_t)P.Mo * n] - sample(P.VV, P.M2, P.Mo, P.No, m + 1, n + 1, u, w);
                v += (double)(-P.lamd * gq_sqrt_dev(P.epsn + d * d));
            } else {
                for (int q = 0; q < 16; ++q) {
                    const int ii = 4 * m + (q >> 2), jj = 4 * n + (q & 3);
                    const R d = P.I1[ii + (int64_t)P.Mo * jj] -
                                sample(P.VV, P.M2, P.Mo, P.No, ii + 1, jj + 1, u, w);
                    v += (double)(-P.lamd * gq_sqrt_dev(P.epsn + d * d));
                }
            }
            // edge_pot(cat(4,uv,uv), cat(4,circshift(uv,-1),circshift(uv,-1,2)))
            const int64_t jd = (m + 1) % P.M + (int64_t)P.M * n;
            const int64_t jr = m + (int64_t)P.M * ((n + 1) % P.N);
            for (int c = 0; c < 2; ++c) {
                const R x = map[i + MN * c];
                const R dd = x - map[jd + MN * c], dr = x - map[jr + MN * c];
                v += (double)(-P.lams * gq_sqrt_dev(P.epsn + dd * dd));
                v += (double)(-P.lams * gq_sqrt_dev(P.epsn + dr * dr));
            }
        }
    }
    __shared__ double red[4];
    v = wave_sum(v);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    if (threadIdx.x == 0) partials[blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
}

// math self-test (not part of the public ABI): fn 0 sqrt, 1 log, 2 exp
__global__ void k_selftest(int fn, const double *in, double *out, int64_t n)
{
    const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (i >= n) return;
    const double x = in[i];
    out[i] = fn == 0 ? gq_sqrt_dev(x) : fn == 1 ? gq_log(x) : fn == 2 ? gq_exp(x)
           : (double)gq_sqrt_dev((float)x);  // 3: the f32 sqrt of (float)x
}

}  // namespace gq

// ===========================================================================
// host runtime
// ===========================================================================
using namespace gq;

namespace gq {
hipError_t mixture_map_device(const double *alpha_host, const void *st, bool fp32, int64_t MNL,
                              int M, int N, int L, double *out_dev, hipStream_t s);
}

// Execution policies that never change a result (placement, caching, launch
// shape; tests/test_gpu_parity.py, test_gpu_persist.py hold them to the same
// bits): chosen automatically, overridable only through the debug entry
// gqmap_debug_policy (tests and A/B scripts; not in the public header).  The
// library reads no environment variables.  A context copies the process-wide
// setting when it is created (gqmap_ctx::pol) and reads only its copy, so a
// later gqmap_debug_policy call never changes a context already running.
namespace gq {
struct Policy {
    int nt_state = -1;     // non-temporal state stores: -1 auto (state > 32 MiB), 0 off, 1 on
    int band_rows = -1;    // row-by-row walk of each XCD's band: -1 auto (padded VV > 4 MiB), 0, 1
    int cu_group = -1;     // co-resident tile grouping: -1 from the occupancy query, 0 off, n > 0 forced
    int lpar = -1;         // super engine L > 1: -1 one block per (tile, component), 1 one block per tile
    int lpar_xcd = 1;      // a tile's component blocks on one XCD (whole-grid fused launch)
    int fused_finalize = 1;
    int persist = 1;       // persistent launch of the small ctf levels
    int persist_cap = -1;  // resident workgroups assumed by the persistent launch (-1: occupancy query)
    int graph = 1;         // replayed hipGraphs (0: direct launches)
    int flow = -1;         // dataflow launch (k_iter_flow): -1 auto (fp64 whole grids at Q = 1, 2), 0 off, 1 on
    int vv_float = 1;      // float padded-frame store when exact
    int vv_pair = 1;       // binary16 column-pair store when exact (fp64 single-scale mixture, Q = 1)
    int verbose = 0;       // recovery messages on stderr
};
Policy g_pol;
}  // namespace gq

struct gqmap_ctx {
    gqmap_options opt;
    int device = 0;
    hipStream_t stream = nullptr;
    bool fp32 = false, super_ = false;
    int Mo = 0, No = 0, M = 0, N = 0, L = 0, K = 0, K2 = 0;
    int64_t MNL = 0;
    size_t rsz = 8;
    void *d_VV = nullptr, *d_I1 = nullptr, *d_st[2] = {nullptr, nullptr}, *d_tab = nullptr;
    Ctl *d_ctl = nullptr;
    fix128 *d_partials = nullptr;  // 2 x nblocks rows (k_iter_persist alternates halves)
    unsigned *d_bar = nullptr;      // k_iter_persist barrier counters (BAR_WORDS)
    // k_iter_persist recovery: the state a launch starts from (k_persist_snap);
    // after a failed launch the context runs one launch per iteration
    void *d_snap = nullptr;
    Ctl *d_snap_ctl = nullptr;
    size_t snap_bytes = 0;
    bool persist_off = false;
    double *d_trace = nullptr;
    // pinned host mirrors: Ctl, the trace ring and the persistent failure
    // word, read back together at the end of a run chunk (one sync)
    Ctl *h_ctl = nullptr;
    double *h_ring = nullptr;
    unsigned *h_fail = nullptr;
    // Ctl::it as the host last saw it (read_ctl / upload_ctl / the end of
    // gqmap_run_aepe); every launch that may advance Ctl clears ctl_known, so
    // back-to-back runs skip the round trip that reads the starting iteration
    int ctl_it = 0;
    bool ctl_known = false;
    double *d_truth = nullptr;  // gqmap_set_truth: M x N x 2 (ctf engine)
    size_t truth_elems = 0;     // doubles d_truth was allocated for
    int tiles_m = 0, tiles_n = 0, nblocks = 0;
    bool have_images = false, have_state = false;
    bool vv32 = false;  // VV stored as float (exact: integer-valued frames)
    bool vvp = false;   // VV stored as binary16 column pairs (vvh2_t; gqmap_math.h, policy vv_pair)
    bool lit = false;   // GQMAP_ARITH_LITERAL: k_iter_lit, literal table layout
    int split = 1;      // lanes per node of the arithmetic (Q): 1, 2, 4, 8, 16, 64
    int kq = 1;         // kernel shape: split, or 0 = role split (Q = 1 arithmetic, 16 x 8 tiles)
    int lpar = 1;       // k_iter blocks per tile (components spread over blocks)
    hipGraphExec_t graph = nullptr;
    // graphs of 2^k iterations (k < SUB_GRAPHS) for the part of a run below
    // GRAPH_CHUNK: every count runs as replayed graphs (gqmap_prepare builds them)
    hipGraphExec_t sub[6] = {nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};
    bool own_stream = true;
    double tab_host[NTAB * TS];
    // column-strip tiling (gqmap_create_tile): node columns [col0, col1) of Ng
    // owned, plus one ghost column per neighbour; M x N above is the LOCAL grid
    int n_tiles = 1, tile = 0, Ng = 0, col0 = 0, col1 = 0, n_off = 0, own_lo = 0, own_hi = 0;
    // cross-tile exchange: per-tile exact totals [nranks][NFIX+L] (nranks = 0:
    // single context, k_finalize reduces its own partials), ghost-column
    // send/recv buffers (left send, right send, left recv, right recv)
    int nranks = 0;
    fix128 *d_gathered = nullptr;
    bool own_gathered = false;
    // d_halo: send left (HALO_TO_LEFT planes), send right (HALO_TO_RIGHT),
    // receive left (the left neighbour's send right), receive right
    void *d_halo[4] = {nullptr, nullptr, nullptr, nullptr};
    struct RcclComm *comm = nullptr;
    bool in_group = false;
    bool host_xfer = false;  // gqmap_tile_attach_host: the caller moves the data
    // deferred-totals RCCL step (L = 1, launch_seq_deferred): each iteration
    // of a sequence writes this tile's exact totals to row `pos` of d_rows; the
    // sequence ends with one all-gather of its rows into d_seqg
    // [nranks][n][NP] and k_finalize_seq
    fix128 *d_rows = nullptr, *d_seqg = nullptr;
    fix128 *seq_row = nullptr;  // the row of the iteration being issued
    bool spec_now = false;      // the launches being issued run by Ctl::it_i / done_i / T_i
    gq::Policy pol = gq::g_pol;  // execution policies, fixed at creation
    unsigned *d_flow = nullptr;  // k_iter_flow queue state (flow_words(tiles) words, zero between launches)
    int flow_n = 0;
};


namespace {

// Lanes per node Q (a node's quadrature split over Q lanes of one wave: more
// lanes in flight; the lane-varying table index is served from an LDS copy of
// the quadrature table).  Measured per-iteration k_iter times (scripts/
// level_sweep.py, ctf engine K=11, us for Q = 1 / 2 / 4 / 16, round 2):
// 30x40 109/81/53/34, 60x80 112/83/54/43, 120x160 113/87/67/100, 240x320
// 173/142/145/332, 480x640 302/374/423/1207; C2 (mixture K=9, 388x584)
// Q=1 173, Q=2 227 -> single-pixel engines: Q = 16 below 2^13 nodes, 4
// below 2^16, 2 below 2^17, else 1; round 3 (profiles/r03_midq_sweep.txt):
// one wave per node (Q = 64, k_iter_wn) below 2^11 nodes (30x40 26.1 -> 19.1
// us), Q = 8 (8 x 4 tiles) below 2^13 (60x80 35.0 -> 31.1 us; Q = 64 58.6).  The super engine runs its L components as separate blocks
// (choose_lpar) and counts node-components: C4 (120x160 x L=3 = 57,600)
// Q = 16 / 4 / 1 -> 616 / 509 / 613-717 us with global table reads (one block
// per tile: 680 / 829 / 1687); Q = 4 with the LDS table 376 us.
// Lanes per node from the node count.  Single-scale mixture (round 5,
// profiles/r05_strip_q_sweep.txt, RubberWhale strips 388 x 21..294): Q = 1
// from 98,304 nodes (114k: 87 vs 101 us at Q = 2), Q = 2 from 16,384 (76k:
// 80 vs 86 at Q = 1; 57k: 57 vs 69 at Q = 4; 20k: 38.7 vs 39.5), Q = 4
// below (15k: 30 vs 38).  Coarse-to-fine levels (K = 11; round 2-3 sweeps,
// profiles/r03_midq_sweep.txt): Q = 1 from 2^17, 2 from 2^16, 4 from 2^13.
int choose_split(int M, int N, int L, int forced, bool super_, bool ctf)
{
    if (forced == 1 || forced == 2 || forced == 4 || forced == 8 || forced == 16 || (forced == 64 && !super_))
        return forced;
    const int64_t nodes = (int64_t)M * N;
    if (!super_ && !ctf)
        return nodes >= 98304 ? 1 : nodes >= (1 << 14) ? 2 : nodes >= (1 << 13) ? 4 : nodes >= (1 << 11) ? 8 : 64;
    if (!super_)
        return nodes >= (1 << 17) ? 1 : nodes >= (1 << 16) ? 2 : nodes >= (1 << 13) ? 4 : nodes >= (1 << 11) ? 8 : 64;
    const int64_t nl = nodes * L;
    if (nl >= (1 << 17)) return 1;
    if (nl >= (1 << 14)) return 4;
    return 16;
}

// Components per k_iter block: the super engine's node grid is 16x smaller
// than the frame, so its L components run as separate blocks (more
// workgroups, fewer lanes per node).  Sums are exact fixed point: the split
// never changes results.  Policy lpar = 1 forces one block per tile.
int choose_lpar(const gqmap_ctx *c)
{
    if (c->pol.lpar == 1) return 1;
    return c->super_ && c->L > 1 ? c->L : 1;
}

// Bytes of ghost-column buffer k (send left, send right, receive left,
// receive right): a column of M values per (plane, component).
size_t halo_bytes(const gqmap_ctx *c, int k)
{
    const int np = (k == 0 || k == 3) ? HALO_TO_LEFT_N : HALO_TO_RIGHT_N;
    return (size_t)np * c->L * c->M * c->rsz;
}

// Column strip of tile c->tile of a Mo x No frame: the local node grid
// (owned columns + one ghost column per neighbour).  No allocation.
void strip_geometry(gqmap_ctx *c, int Mo, int No)
{
    const int M = c->super_ ? Mo / 4 : Mo, Ng = c->super_ ? No / 4 : No;
    // column strip [col0, col1) + one ghost column per neighbour
    const int col0 = (int)((int64_t)Ng * c->tile / c->n_tiles);
    const int col1 = (int)((int64_t)Ng * (c->tile + 1) / c->n_tiles);
    const int gl = c->tile > 0, gr = c->tile < c->n_tiles - 1;
    c->Mo = Mo;
    c->No = No;
    c->M = M;
    c->N = (col1 - col0) + gl + gr;
    c->Ng = Ng;
    c->col0 = col0;
    c->col1 = col1;
    c->n_off = col0 - gl;
    c->own_lo = gl;
    c->own_hi = gl + (col1 - col0);
    c->MNL = (int64_t)c->M * c->N * c->L;
}

// Lanes per node, kernel shape and the tile grid of the local node grid.
void tile_grid(gqmap_ctx *c)
{
    // from the whole grid (Ng columns), so every column-strip tile sums its
    // quadrature in the same order as the untiled solve
    c->split = c->lit ? 1
                      : choose_split(c->M, c->Ng > 0 ? c->Ng : c->N, c->super_ ? c->L : 1, c->opt.split, c->super_,
                                     c->opt.engine == GQMAP_ENGINE_CTF);
    c->kq = c->split;
    if (c->opt.split == GQMAP_SPLIT_ROLE && !c->super_) {  // role split: Q = 1 arithmetic
        c->split = 1;
        c->kq = 0;
    }
    const int tr = tile_rows(c->kq), tc = tile_cols(c->kq);
    c->tiles_m = (c->M + tr - 1) / tr;
    c->tiles_n = (c->N + tc - 1) / tc;
    c->lpar = choose_lpar(c);
    c->nblocks = c->tiles_m * c->tiles_n * c->lpar;
}

gqmap_status alloc_grid(gqmap_ctx *c)
{
    tile_grid(c);
    const size_t bytes = (size_t)c->MNL * NPLANES * c->rsz;
    for (int b = 0; b < 2; ++b) {
        if (c->d_st[b]) (void)hipFree(c->d_st[b]);
        c->d_st[b] = nullptr;
        GQ_HIP(hipMalloc(&c->d_st[b], bytes));
    }
    if (c->d_partials) (void)hipFree(c->d_partials);
    c->d_partials = nullptr;
    GQ_HIP(hipMalloc((void **)&c->d_partials, sizeof(fix128) * (size_t)2 * c->nblocks * (NFIX + c->L) + 64));
    return GQMAP_OK;
}

// A subset of the tiles for one k_iter launch (tile contexts: boundary tile
// columns / interior), see IterParams::seg_lo.
struct TileSegs {
    int lo[2], n[2];
    int part_off;
};

// The boundary tile columns of a column-strip tile (those holding its first
// and last owned node columns: their results are what the neighbours need)
// and the rest.  Together they cover every tile once; block partial rows
// [0, bnd) and [bnd, nblocks).
void tile_segments(const gqmap_ctx *c, TileSegs &bnd, TileSegs &inr)
{
    const int TN = tile_cols(c->kq);  // tile columns
    const int tm = c->tiles_m, cb0 = c->own_lo / TN, cb1 = (c->own_hi - 1) / TN;
    bnd.lo[0] = cb0 * tm; bnd.n[0] = tm;
    bnd.lo[1] = cb1 * tm; bnd.n[1] = cb1 != cb0 ? tm : 0;
    bnd.part_off = 0;
    inr.lo[0] = (cb0 + 1) * tm; inr.n[0] = std::max(0, cb1 - cb0 - 1) * tm;
    inr.lo[1] = (cb1 + 1) * tm; inr.n[1] = (c->tiles_n - cb1 - 1) * tm;
    inr.part_off = (bnd.n[0] + bnd.n[1]) * c->lpar;
    // tile columns before cb0 hold ghost columns only (one-column tiles,
    // Q = 64, of a strip with a left neighbour): never launched
}

// Workgroups of one RCCL-tile iteration (its one launch over the strip's
// tiles, strip_launch): the count the last-arrival ticket of
// tile_totals_tail waits for.
// Not c->nblocks -- a ghost-only tile column is not launched.
int iteration_blocks(const gqmap_ctx *c)
{
    TileSegs bnd, inr;
    tile_segments(c, bnd, inr);
    return (bnd.n[0] + bnd.n[1] + inr.n[0] + inr.n[1]) * c->lpar;
}



FinParams fin_params(const gqmap_ctx *c);

// Non-temporal state stores for a state buffer larger than the XCDs' L2s
// together (8 x 4 MiB): it is streamed once per iteration and would evict
// the frame's gather lines (C5 fetch 691 -> 582 MB per launch, time -0.4%);
// a C2-sized buffer (16 MB) is partly still in L2 when the next iteration
// reads it (round 3: NT stores on C2 +0.8%).  Policy nt_state = 0/1 forces.
bool state_nt(const gqmap_ctx *c)
{
    if (c->pol.nt_state >= 0) return c->pol.nt_state == 1;
    return (size_t)c->MNL * NPLANES * c->rsz > ((size_t)32 << 20);
}

// Row-by-row tile walk within each XCD's band (tile_of_block) for frames
// whose padded VV is larger than one XCD's 4 MiB L2.  Policy band_rows = 0/1 forces.
bool band_rows(const gqmap_ctx *c)
{
    if (c->pol.band_rows >= 0) return c->pol.band_rows == 1;
    const size_t vsz = c->fp32 ? sizeof(float) : c->vvp ? sizeof(vvh2_t) : c->vv32 ? sizeof(vvs_t) : sizeof(double);
    return vv_elems(c->Mo, c->No) * vsz > ((size_t)4 << 20);
}

bool fused_finalize(const gqmap_ctx *c)
{
    return c->nranks == 0 && c->pol.fused_finalize;
}

template <typename R, typename VT>
IterParams<R, VT> iter_params(const gqmap_ctx *c)
{
    IterParams<R, VT> P;
    const gqmap_options &o = c->opt;
    P.VV = (const VT *)c->d_VV;
    P.I1 = (const R *)c->d_I1;
    P.st0 = (R *)c->d_st[0];
    P.st1 = (R *)c->d_st[1];
    P.tab = (const R *)c->d_tab;
    P.ctl = c->d_ctl;
    P.partials = c->d_partials;
    P.M = c->M; P.N = c->N; P.Mo = c->Mo; P.No = c->No; P.M2 = c->Mo + 2;
    P.L = c->L; P.K2 = c->K2;
    P.tiles_m = c->tiles_m; P.tiles_n = c->tiles_n;
    P.seg_lo[0] = P.seg_lo[1] = 0;
    P.seg_n[0] = c->tiles_m * c->tiles_n;
    P.seg_n[1] = 0;
    P.part_off = 0;
    P.epsn = R(o.epsn); P.lamd = R(o.lambdad); P.lams = R(o.lambdas);
    P.minu = R(o.minu); P.maxu = R(o.maxu); P.minv = R(o.minv); P.maxv = R(o.maxv);
    P.sig_lo = R(o.sig_lo); P.sig_hi = R(o.sig_hi); P.corr = R(o.corr_tor);
    P.sig_step = R(o.sig_step);
    double xmax = 0;
    for (int k = 0; k < c->K2; ++k) xmax = std::max(xmax, std::fabs(c->tab_host[tab_at(T_XI, k)]));
    P.gh_xmax = R(xmax);
    P.truth = c->d_truth;
    P.step0 = o.step0; P.step_decay = o.step_decay;
    P.guard = o.guard_a;
    P.MNL = c->MNL;
    P.n_off = c->n_off; P.own_lo = c->own_lo; P.own_hi = c->own_hi; P.Ng = c->Ng;
    P.fused = fused_finalize(c);
    P.lpar = c->lpar;
    P.lpar_xcd = 0;
    // RCCL tiles: exact totals straight from the k_iter launches (no
    // k_reduce_local between the launches and the all-gather)
    P.tile_acc = c->comm != nullptr;
    P.ticket_total = c->comm ? iteration_blocks(c) : c->nblocks;
    P.tile_totals = c->seq_row ? c->seq_row : c->d_gathered ? c->d_gathered + (size_t)c->tile * (NFIX + c->L) : nullptr;
    P.spec = c->spec_now ? 1 : 0;
    P.fin = fin_params(c);
    P.cu_group = 1; P.cu_slots = 32;  // set per kernel by launch_iter_q
    P.band_rows = 0;
    P.bar = c->d_bar;
    return P;
}

FinParams fin_params(const gqmap_ctx *c)
{
    FinParams F;
    const gqmap_options &o = c->opt;
    F.partials = c->d_partials;
    F.nblocks = c->nblocks;
    F.L = c->L;
    F.ctl = c->d_ctl;
    F.trace = c->d_trace;
    F.aepe = c->d_truth != nullptr;
    F.count = (double)(c->M - 2) * (double)(c->Ng - 2) * c->L;  // global interior
    F.gathered = c->d_gathered;
    F.nranks = c->nranks;
    F.step0 = o.step0; F.step_decay = o.step_decay;
    F.alpha_mode = o.alpha_mode; F.alpha_start = o.alpha_start; F.alpha_lr = o.alpha_lr;
    F.t_decay_every = o.t_decay_every; F.drate = o.drate; F.t_min = o.t_min; F.tor = o.tor;
    return F;
}

// Resident workgroups per CU for a k_iter instantiation, and CUs per XCD:
// the tile grouping of k_iter (speed only, never results).
template <typename K>
int2 kernel_shape(K kern)
{
    int per_cu = 1, dev = 0, cus = 256;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, BLOCK, 0) != hipSuccess) per_cu = 1;
    if (hipGetDevice(&dev) == hipSuccess && hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        cus = 256;
    return make_int2(std::max(1, per_cu), std::max(8, cus));
}

template <typename R, typename VT, int ENG, int Q>
void launch_k_iter(gqmap_ctx *c, const TileSegs *sg)
{
    IterParams<R, VT> P = iter_params<R, VT>(c);
    int nblocks = c->nblocks;
    if (sg) {
        for (int k = 0; k < 2; ++k) {
            P.seg_lo[k] = sg->lo[k];
            P.seg_n[k] = sg->n[k];
        }
        P.part_off = sg->part_off;
        nblocks = (sg->n[0] + sg->n[1]) * c->lpar;
        if (nblocks == 0) return;
    }
    static const int2 shape = kernel_shape(k_iter<R, VT, ENG, Q>);
    if (c->pol.cu_group != 0) {
        P.cu_group = c->pol.cu_group > 0 ? c->pol.cu_group : shape.x;
        P.cu_slots = std::max(1, shape.y / 8);
    }
    if (c->lpar > 1 && P.fused && !sg && c->pol.lpar_xcd) {
        P.lpar_xcd = 1;
        nblocks = 8 * c->lpar * ((c->tiles_m * c->tiles_n + 7) / 8);
    }
    // (whole grid, one block per tile; lpar_xcd interleaves components instead)
    if (!sg && !P.lpar_xcd) P.band_rows = band_rows(c) ? 1 : 0;
    if constexpr (Q == 1 && ENG == 0 && sizeof(R) == 8 && !is_vvh2<VT>::value) {
        if (c->lit) {  // literal-order arithmetic (one instantiation per VV storage and store kind)
            static const int2 lshape = kernel_shape(k_iter_lit<VT>);
            if (P.cu_group > 1) P.cu_group = lshape.x;
            if (state_nt(c))
                k_iter_lit<VT, true><<<nblocks, BLOCK, 0, c->stream>>>(P);
            else
                k_iter_lit<VT><<<nblocks, BLOCK, 0, c->stream>>>(P);
            return;
        }
    }
    if constexpr (Q == 1 && ENG != 1) {
        if (state_nt(c)) {  // frames beyond the L2s: non-temporal state stores
            k_iter<R, VT, ENG, 1, true><<<nblocks, BLOCK, 0, c->stream>>>(P);
            return;
        }
    }
    k_iter<R, VT, ENG, Q><<<nblocks, BLOCK, 0, c->stream>>>(P);
}

// Q = 64 (one wave per node, k_iter_wn): tiles of 4 x 1 nodes
template <typename R, typename VT, int ENG>
void launch_k_iter_wn(gqmap_ctx *c, const TileSegs *sg)
{
    IterParams<R, VT> P = iter_params<R, VT>(c);
    int nblocks = c->nblocks;
    if (sg) {
        for (int k = 0; k < 2; ++k) {
            P.seg_lo[k] = sg->lo[k];
            P.seg_n[k] = sg->n[k];
        }
        P.part_off = sg->part_off;
        nblocks = sg->n[0] + sg->n[1];
        if (nblocks == 0) return;
    }
    static const int2 shape = kernel_shape(k_iter_wn<R, VT, ENG>);
    P.cu_group = 1;
    P.cu_slots = std::max(1, shape.y / 8);
    k_iter_wn<R, VT, ENG><<<nblocks, WN_THREADS, 0, c->stream>>>(P);
}

template <typename R, typename VT, int ENG>
void launch_iter_q(gqmap_ctx *c, const TileSegs *sg)
{
    if constexpr (ENG != 1) {
        if (c->kq == 64) return launch_k_iter_wn<R, VT, ENG>(c, sg);
        if (c->kq == 0) return launch_k_iter<R, VT, ENG, 0>(c, sg);
    }
    if (c->split == 16)
        launch_k_iter<R, VT, ENG, 16>(c, sg);
    else if (c->split == 8)
        launch_k_iter<R, VT, ENG, 8>(c, sg);
    else if (c->split == 4)
        launch_k_iter<R, VT, ENG, 4>(c, sg);
    else if (c->split == 2)
        launch_k_iter<R, VT, ENG, 2>(c, sg);
    else
        launch_k_iter<R, VT, ENG, 1>(c, sg);
}

template <typename R, typename VT>
void launch_iter_t(gqmap_ctx *c, const TileSegs *sg)
{
    switch (c->opt.engine) {
    case GQMAP_ENGINE_SUPER: launch_iter_q<R, VT, 1>(c, sg); break;
    case GQMAP_ENGINE_CTF: launch_iter_q<R, VT, 2>(c, sg); break;
    default: launch_iter_q<R, VT, 0>(c, sg); break;
    }
}

// sg: a subset of the tiles (default: all, one launch)
void launch_iter(gqmap_ctx *c, const TileSegs *sg = nullptr)
{
    c->ctl_known = false;
    if (c->fp32) {
        if (c->vvp) launch_k_iter<float, vvh2_t, 0, 1>(c, sg);
        else launch_iter_t<float, float>(c, sg);
    }
    else if (c->vvp) launch_k_iter<double, vvh2_t, 0, 1>(c, sg);  // (the pair store: mixture at Q = 1)
    else if (c->vv32) launch_iter_t<double, vvs_t>(c, sg);
    else launch_iter_t<double, double>(c, sg);
}


void launch_finalize(gqmap_ctx *c) { k_finalize<<<1, 256, 0, c->stream>>>(fin_params(c)); }

// ---- persistent small-grid launches (k_iter_persist) ------------------------
// Whole-grid ctf contexts with L = 1 and Q >= 8 (grids below 2^13 nodes)
// whose tiles plus the finalizer fit the device's resident workgroups
// (the context's policy persist = 0: one launch per iteration instead).
template <typename R, typename VT, int Q>
int persist_capacity(const gqmap_ctx *c)
{
    static int cap = -1;
    if (cap < 0) {
        int per_cu = 0, dev = 0, cus = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_iter_persist<R, VT, 2, Q>,
                                                         Q == 64 ? WN_THREADS : BLOCK, 0) != hipSuccess)
            per_cu = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
            cus = 0;
        // a 5-wave k_iter_wn workgroup: one per CU (the occupancy API answered
        // 2 for the 165-VGPR fp32 instantiation, but 265 workgroups on 256 CUs
        // were not co-resident: the barrier timed out); 4-wave workgroups
        // take one wave slot per SIMD each, as the API counts them
        if (Q == 64) per_cu = std::min(per_cu, 1);
        cap = std::max(0, per_cu) * std::max(0, cus);
    }
    // policy persist_cap: resident workgroups assumed (tests force the
    // per-iteration path with a capacity too small for the grid)
    return c->pol.persist_cap >= 0 ? c->pol.persist_cap : cap;
}

// The snapshot buffers of the persistent path (allocated outside a capture;
// a capture without them keeps per-iteration launches)
bool ensure_snap(gqmap_ctx *c)
{
    const size_t need = (size_t)c->MNL * NPLANES * c->rsz;
    if (c->d_snap && c->snap_bytes == need) return true;
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(c->stream, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) return false;
    if (hipStreamSynchronize(c->stream) != hipSuccess) return false;
    if (c->d_snap) (void)hipFree(c->d_snap);
    c->d_snap = nullptr;
    c->snap_bytes = 0;
    if (!c->d_snap_ctl && hipMalloc((void **)&c->d_snap_ctl, sizeof(Ctl)) != hipSuccess) return false;
    if (hipMalloc(&c->d_snap, need) != hipSuccess) {
        c->d_snap = nullptr;
        return false;
    }
    c->snap_bytes = need;
    return true;
}

template <typename R, typename VT, int Q>
bool launch_persist_q(gqmap_ctx *c, int n, bool dry)
{
    const int G = c->nblocks;
    if (G + 1 > persist_capacity<R, VT, Q>(c)) return false;
    if (!ensure_snap(c)) return false;
    if (dry) return true;
    {
        const int64_t n = (int64_t)c->MNL * NPLANES;
        const int grid = (int)std::min<int64_t>((n + 255) / 256, 512);
        k_persist_snap<R><<<grid, 256, 0, c->stream>>>(c->d_ctl, c->d_bar, (const R *)c->d_st[0],
                                                       (const R *)c->d_st[1], (R *)c->d_snap, c->d_snap_ctl, n);
    }
    IterParams<R, VT> P = iter_params<R, VT>(c);
    P.fused = 0;
    P.tile_acc = 0;
    P.fin.nblocks = 2 * G;  // partial row stride: iteration j writes rows (j & 1) * G + b
    const int threads = Q == 64 ? WN_THREADS : BLOCK;
    static const int2 shape = kernel_shape(k_iter_persist<R, VT, 2, Q>);
    P.cu_group = Q == 64 || c->pol.cu_group == 0 ? 1 : c->pol.cu_group > 0 ? c->pol.cu_group : shape.x;
    P.cu_slots = std::max(1, shape.y / 8);
    k_iter_persist<R, VT, 2, Q><<<G + 1, threads, 0, c->stream>>>(P, n);
    return true;
}

template <typename R, typename VT>
bool launch_persist_t(gqmap_ctx *c, int n, bool dry)
{
    // not Q = 4 (120x160): 57.3 vs 48.8 us/it measured (profiles/r03_persist_levels.txt;
    // GQ_PERSIST_Q4: experiment builds only)
#if GQ_PERSIST_Q4
    if (c->kq == 4) return launch_persist_q<R, VT, 4>(c, n, dry);
#endif
    switch (c->kq) {
    case 8: return launch_persist_q<R, VT, 8>(c, n, dry);
    case 16: return launch_persist_q<R, VT, 16>(c, n, dry);
    case 64: return launch_persist_q<R, VT, 64>(c, n, dry);
    default: return false;
    }
}

// n iterations as one k_iter_persist launch when the context qualifies;
// dry: only the check
bool launch_persist(gqmap_ctx *c, int n, bool dry = false)
{
    if (!c->pol.persist || c->persist_off || c->opt.engine != GQMAP_ENGINE_CTF || c->L != 1 || c->n_tiles != 1 || c->comm || c->nranks != 0 ||
        !fused_finalize(c) || n < 1)
        return false;
    if (c->fp32) return launch_persist_t<float, float>(c, n, dry);
    if (c->vv32) return launch_persist_t<double, vvs_t>(c, n, dry);
    return launch_persist_t<double, double>(c, n, dry);
}

// ---- RCCL, resolved at first use from librccl.so.1 (the copy torch has
// already loaded, when it has) so the library itself carries no link-time
// dependency on it.
struct Rccl {
    ncclResult_t (*GetUniqueId)(ncclUniqueId *) = nullptr;
    ncclResult_t (*CommInitRank)(ncclComm_t *, int, ncclUniqueId, int) = nullptr;
    ncclResult_t (*CommDestroy)(ncclComm_t) = nullptr;
    ncclResult_t (*GroupStart)() = nullptr;
    ncclResult_t (*GroupEnd)() = nullptr;
    ncclResult_t (*Send)(const void *, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*Recv)(void *, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*AllGather)(const void *, void *, size_t, ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
    const char *(*GetErrorString)(ncclResult_t) = nullptr;
    bool ok = false;
};

const Rccl *rccl()
{
    static Rccl r;
    static std::once_flag once;
    std::call_once(once, [] {
        void *h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
        if (!h) h = dlopen("librccl.so", RTLD_NOW | RTLD_GLOBAL);
        if (!h) return;
        auto sym = [&](auto &fn, const char *name) { fn = reinterpret_cast<std::decay_t<decltype(fn)>>(dlsym(h, name)); };
        sym(r.GetUniqueId, "ncclGetUniqueId");
        sym(r.CommInitRank, "ncclCommInitRank");
        sym(r.CommDestroy, "ncclCommDestroy");
        sym(r.GroupStart, "ncclGroupStart");
        sym(r.GroupEnd, "ncclGroupEnd");
        sym(r.Send, "ncclSend");
        sym(r.Recv, "ncclRecv");
        sym(r.AllGather, "ncclAllGather");
        sym(r.GetErrorString, "ncclGetErrorString");
        r.ok = r.GetUniqueId && r.CommInitRank && r.CommDestroy && r.GroupStart && r.GroupEnd && r.Send &&
               r.Recv && r.AllGather && r.GetErrorString;
    });
    return &r;
}

#define GQ_NCCL(call)                                                                       \
    do {                                                                                    \
        ncclResult_t r_ = (call);                                                           \
        if (r_ != ncclSuccess) {                                                            \
            gq::set_error("%s:%d %s failed: %s", __FILE__, __LINE__, #call,                \
                          rccl()->GetErrorString(r_));                                      \
            return GQMAP_ERR_HIP;                                                           \
        }                                                                                   \
    } while (0)

}  // namespace

struct LoopGroup;

// The communicator of an RCCL tile.  loop (tests only, never set by
// gqmap_tile_attach_rccl): the in-process loopback transport below stands in
// for the three NCCL calls of the strip iteration -- the grouped
// ncclSend/ncclRecv of exchange_rccl and the two ncclAllGather of
// launch_step_rccl / launch_seq_deferred -- so that n tile contexts, one host
// thread each, run the multi-rank iteration's own code with real neighbours
// on one GPU.
struct RcclComm {
    ncclComm_t comm = nullptr;
    int nranks = 0, rank = 0;
    LoopGroup *loop = nullptr;
};

// Loopback transport (gqmap_debug_loop_*).  Each rank's thread posts its
// buffers, records `ready` on its own stream after the work the collective
// follows, and meets the others at a host barrier; then each rank enqueues,
// on its own stream, a wait on every peer's `ready` and device copies of what
// it receives (from the peer's send buffer into its receive buffer -- what
// NCCL moves), records `done`, meets the others again and waits on the
// `done` of every peer that read its buffers before its stream goes on (the
// peer's copy must land before this rank's next pack overwrites the source:
// NCCL's send completes only when the peer has the data).  The collectives
// of all ranks are matched in issue order, as NCCL matches them; a peer whose
// posted sizes do not match, or a barrier that times out (a rank left the
// sequence), fails the call.
struct LoopGroup {
    struct P2p {
        int peer;
        const void *send;  // kind 0: send buffer to `peer`
        void *recv;        // kind 0: receive buffer from `peer`
        size_t bytes;
    };
    struct Post {
        int kind = -1;  // 0: grouped send/recv, 1: all-gather
        P2p sends[2], recvs[2];
        int ns = 0, nr = 0;
        const void *ag_send = nullptr;  // all-gather: this rank's block
        void *ag_recv = nullptr;        // rank-major [nranks][bytes]
        size_t ag_bytes = 0;
    };
    int n = 0, device = 0;
    std::mutex mu;
    std::condition_variable cv;
    int arrived = 0;
    unsigned long long gen = 0;
    bool broken = false;
    std::vector<hipEvent_t> ready, done;
    std::vector<Post> post;
    unsigned long long calls = 0;  // collectives completed (rank 0's count)
};

namespace {

// Host barrier of a loopback group; false: a rank did not arrive within the
// time limit (it left the collective sequence) or the group is broken.
bool loop_barrier(LoopGroup *g)
{
    std::unique_lock<std::mutex> lk(g->mu);
    if (g->broken) return false;
    const unsigned long long my = g->gen;
    if (++g->arrived == g->n) {
        g->arrived = 0;
        ++g->gen;
        g->cv.notify_all();
        return true;
    }
    if (!g->cv.wait_for(lk, std::chrono::seconds(120), [&] { return g->gen != my || g->broken; }) || g->broken) {
        g->broken = true;
        g->cv.notify_all();
        return false;
    }
    return true;
}

// One collective of rank r (see LoopGroup).
gqmap_status loop_collective(gqmap_ctx *c, const LoopGroup::Post &mine)
{
    LoopGroup *g = c->comm->loop;
    const int r = c->comm->rank;
    GQ_HIP(hipEventRecord(g->ready[r], c->stream));
    g->post[r] = mine;
    GQ_CHECK(loop_barrier(g), GQMAP_ERR_HIP, "loopback transport: rank %d: a peer did not reach the collective", r);
    std::vector<int> peers;  // ranks whose buffers this rank reads, or that read this rank's
    gqmap_status st = GQMAP_OK;
    for (int q = 0; q < g->n && st == GQMAP_OK; ++q)
        if (g->post[q].kind != mine.kind) {
            set_error("loopback transport: rank %d issued collective kind %d, rank %d kind %d", r, mine.kind, q,
                      g->post[q].kind);
            st = GQMAP_ERR_HIP;
        }
    if (st == GQMAP_OK && mine.kind == 0) {
        for (int i = 0; i < mine.nr && st == GQMAP_OK; ++i) {
            const LoopGroup::P2p &rv = mine.recvs[i];
            const LoopGroup::Post &pp = g->post[rv.peer];
            const LoopGroup::P2p *sd = nullptr;
            for (int j = 0; j < pp.ns; ++j)
                if (pp.sends[j].peer == r) sd = &pp.sends[j];
            if (!sd || sd->bytes != rv.bytes) {
                set_error("loopback transport: rank %d receives %zu bytes from rank %d, which sends %zu", r, rv.bytes,
                          rv.peer, sd ? sd->bytes : (size_t)0);
                st = GQMAP_ERR_HIP;
                break;
            }
            if (hipStreamWaitEvent(c->stream, g->ready[rv.peer], 0) != hipSuccess ||
                hipMemcpyAsync(rv.recv, sd->send, rv.bytes, hipMemcpyDeviceToDevice, c->stream) != hipSuccess)
                st = GQMAP_ERR_HIP;
            peers.push_back(rv.peer);
        }
        for (int i = 0; i < mine.ns; ++i) peers.push_back(mine.sends[i].peer);
    } else if (st == GQMAP_OK) {
        for (int q = 0; q < g->n && st == GQMAP_OK; ++q) {
            const LoopGroup::Post &pp = g->post[q];
            if (pp.ag_bytes != mine.ag_bytes) {
                set_error("loopback transport: all-gather of %zu bytes on rank %d, %zu on rank %d", mine.ag_bytes, r,
                          pp.ag_bytes, q);
                st = GQMAP_ERR_HIP;
                break;
            }
            char *dst = (char *)mine.ag_recv + (size_t)q * mine.ag_bytes;
            if (q == r && dst == pp.ag_send) continue;  // in place
            if ((q != r && hipStreamWaitEvent(c->stream, g->ready[q], 0) != hipSuccess) ||
                hipMemcpyAsync(dst, pp.ag_send, mine.ag_bytes, hipMemcpyDeviceToDevice, c->stream) != hipSuccess)
                st = GQMAP_ERR_HIP;
            if (q != r) peers.push_back(q);
        }
    }
    if (st == GQMAP_OK && hipEventRecord(g->done[r], c->stream) != hipSuccess) st = GQMAP_ERR_HIP;
    if (st != GQMAP_OK) {  // release the peers waiting at the second barrier
        std::lock_guard<std::mutex> lk(g->mu);
        g->broken = true;
        g->cv.notify_all();
        if (!gqmap_last_error()[0]) set_error("loopback transport: rank %d: HIP call failed", r);
        return st;
    }
    GQ_CHECK(loop_barrier(g), GQMAP_ERR_HIP, "loopback transport: rank %d: a peer failed in the collective", r);
    for (int q : peers) GQ_HIP(hipStreamWaitEvent(c->stream, g->done[q], 0));
    if (r == 0) ++g->calls;
    return GQMAP_OK;
}

// The ghost-column send/recv pairs of one iteration: grouped ncclSend /
// ncclRecv with the neighbour ranks, or the loopback transport.
gqmap_status comm_sendrecv(gqmap_ctx *c, const LoopGroup::P2p *sends, int ns, const LoopGroup::P2p *recvs, int nr,
                           size_t elem)
{
    if (c->comm->loop) {
        LoopGroup::Post p;
        p.kind = 0;
        p.ns = ns;
        p.nr = nr;
        for (int i = 0; i < ns; ++i) p.sends[i] = sends[i];
        for (int i = 0; i < nr; ++i) p.recvs[i] = recvs[i];
        return loop_collective(c, p);
    }
    const ncclDataType_t dt = elem == sizeof(float) ? ncclFloat : ncclDouble;
    const Rccl *R = rccl();
    GQ_NCCL(R->GroupStart());
    for (int i = 0; i < std::max(ns, nr); ++i) {
        if (i < ns) GQ_NCCL(R->Send(sends[i].send, sends[i].bytes / elem, dt, sends[i].peer, c->comm->comm, c->stream));
        if (i < nr) GQ_NCCL(R->Recv(recvs[i].recv, recvs[i].bytes / elem, dt, recvs[i].peer, c->comm->comm, c->stream));
    }
    GQ_NCCL(R->GroupEnd());
    return GQMAP_OK;
}

// All-gather of `bytes` per rank into the rank-major `recv` (in place when
// send is this rank's block of recv): ncclAllGather, or the loopback transport.
gqmap_status comm_allgather(gqmap_ctx *c, const void *send, void *recv, size_t bytes)
{
    if (c->comm->loop) {
        LoopGroup::Post p;
        p.kind = 1;
        p.ag_send = send;
        p.ag_recv = recv;
        p.ag_bytes = bytes;
        return loop_collective(c, p);
    }
    GQ_NCCL(rccl()->AllGather(send, recv, bytes, ncclUint8, c->comm->comm, c->stream));
    return GQMAP_OK;
}

// sides: the present ones (left and/or right), one launch
template <typename R>
void halo_copy(gqmap_ctx *c, hipStream_t s, const HaloSide<R> *sides, int nsides)
{
    if (nsides == 0) return;
    int64_t n = 0;
    for (int k = 0; k < nsides; ++k) n = std::max<int64_t>(n, (int64_t)sides[k].np * c->L * c->M);
    const int grid = (int)std::min<int64_t>((n + 255) / 256, 1024);
    k_halo_copy<R><<<dim3(grid, nsides), 256, 0, s>>>(c->d_ctl, (R *)c->d_st[0], (R *)c->d_st[1], c->M,
                                                     (int64_t)c->M * c->N, c->MNL, c->L, sides[0],
                                                     sides[nsides - 1], c->spec_now ? 1 : 0);
}

// This tile's boundary columns -> d_halo[0] (to the left neighbour, tile - 1)
// and d_halo[1] (to the right one), one launch; d_halo[2] / d_halo[3] (from
// the left / right neighbour) go into the ghost columns in
// k_unpack_finalize.
template <typename R>
void halo_pack_t(gqmap_ctx *c, hipStream_t s)
{
    HaloSide<R> sd[2];
    int n = 0;
    if (c->tile > 0) sd[n++] = HaloSide<R>{c->own_lo, HALO_TO_LEFT_N, HALO_TO_LEFT, (R *)c->d_halo[0]};
    if (c->tile < c->n_tiles - 1) sd[n++] = HaloSide<R>{c->own_hi - 1, HALO_TO_RIGHT_N, HALO_TO_RIGHT, (R *)c->d_halo[1]};
    halo_copy<R>(c, s, sd, n);
}
void halo_pack(gqmap_ctx *c, hipStream_t s)
{
    if (c->fp32) halo_pack_t<float>(c, s);
    else halo_pack_t<double>(c, s);
}

// The received ghost columns and the finalize of a tile, one launch on the
// tile's stream (k_unpack_finalize)
template <typename R>
void unpack_finalize_t(gqmap_ctx *c)
{
    HaloSide<R> sd[2];
    int n = 0;
    if (c->tile > 0) sd[n++] = HaloSide<R>{0, HALO_TO_RIGHT_N, HALO_TO_RIGHT, (R *)c->d_halo[2]};
    if (c->tile < c->n_tiles - 1) sd[n++] = HaloSide<R>{c->N - 1, HALO_TO_LEFT_N, HALO_TO_LEFT, (R *)c->d_halo[3]};
    if (n == 0) sd[0] = HaloSide<R>{0, 0, 0u, nullptr};
    k_unpack_finalize<R><<<1, 256, 0, c->stream>>>(fin_params(c), (R *)c->d_st[0], (R *)c->d_st[1], c->M,
                                                   (int64_t)c->M * c->N, c->MNL, c->L, sd[0], sd[n > 0 ? n - 1 : 0], n);
}
void unpack_finalize(gqmap_ctx *c)
{
    c->ctl_known = false;
    if (c->fp32) unpack_finalize_t<float>(c);
    else unpack_finalize_t<double>(c);
}

// The rest of a whole-grid iteration after k_iter: the finalize, unless the
// last k_iter workgroup ran it (fused).
gqmap_status launch_tail(gqmap_ctx *c)
{
    if (!fused_finalize(c)) launch_finalize(c);
    return GQMAP_OK;
}

// The strip's tiles of one RCCL iteration as one launch: every tile column
// from the one holding the first owned column (a ghost-only tile column --
// one-column tiles of a strip with a left neighbour -- is not launched; the
// workgroups iteration_blocks() counts).
TileSegs strip_launch(const gqmap_ctx *c)
{
    TileSegs bnd, inr, all{};
    tile_segments(c, bnd, inr);
    all.lo[0] = bnd.lo[0];
    all.n[0] = c->tiles_m * c->tiles_n - bnd.lo[0];
    all.part_off = 0;
    return all;
}

// The ghost-column exchange of an iteration on the context stream: pack the
// boundary columns, grouped ncclSend/ncclRecv with the neighbour ranks.
gqmap_status exchange_rccl(gqmap_ctx *c)
{
    const int r = c->comm->rank;
    const bool left = c->tile > 0, right = c->tile < c->n_tiles - 1;
    if (!left && !right) return GQMAP_OK;
    const size_t bl = (size_t)HALO_TO_LEFT_N * c->L * c->M * c->rsz, br = (size_t)HALO_TO_RIGHT_N * c->L * c->M * c->rsz;
    halo_pack(c, c->stream);
    LoopGroup::P2p sd[2], rv[2];
    int n = 0;
    if (left) {
        sd[n] = {r - 1, c->d_halo[0], nullptr, bl};
        rv[n++] = {r - 1, nullptr, c->d_halo[2], br};
    }
    if (right) {
        sd[n] = {r + 1, c->d_halo[1], nullptr, br};
        rv[n++] = {r + 1, nullptr, c->d_halo[3], bl};
    }
    return comm_sendrecv(c, sd, n, rv, n, c->rsz);
}

// One exact iteration of an RCCL tile (L > 1, whose alpha update needs every
// iteration's totals; and the re-run of a deferred sequence that overshot its
// stop): the strip's tiles, the exchange, this tile's exact totals
// all-gathered, then the received columns into the ghost columns and the
// finalize over all tiles' totals (identical on every rank) -- all on the
// context's stream (a cross-stream edge costs 5-10 us per iteration here,
// profiles/r05_strip8_timeline.txt).  e0 / e1 (optional) bracket the k_iter
// launch.
gqmap_status launch_step_rccl(gqmap_ctx *c, hipEvent_t e0 = nullptr, hipEvent_t e1 = nullptr)
{
    const int NP = NFIX + c->L, r = c->comm->rank;
    const TileSegs all = strip_launch(c);
    if (e0) GQ_HIP(hipEventRecord(e0, c->stream));
    launch_iter(c, &all);
    if (e1) GQ_HIP(hipEventRecord(e1, c->stream));
    gqmap_status st = exchange_rccl(c);
    if (st != GQMAP_OK) return st;
    // (this rank's totals row was written by the launch's last workgroup: tile_totals_tail)
    st = comm_allgather(c, c->d_gathered + (size_t)r * NP, c->d_gathered, (size_t)NP * sizeof(fix128));
    if (st != GQMAP_OK) return st;
    unpack_finalize(c);  // received ghost columns + finalize, one launch
    return GQMAP_OK;
}

// Deferred-totals RCCL step (L = 1).  Nothing of iteration j + 1 depends on
// iteration j's totals but the stop rule (alpha is constant, the step size
// and the temperature decay follow the iteration number), so the totals'
// all-gather and the finalize leave the iteration, and everything of an
// iteration runs on the context's one stream:
//   k_iter (all the strip's tiles) | pack | send/recv | unpack + advance
// with this tile's exact totals of iteration pos written to row pos of
// d_rows by the launch's last workgroup, and the kernels running by
// Ctl::it_i / done_i / T_i (k_unpack_advance takes fin_apply's steps for
// them).  No cross-stream edge: on MI355X each one cost 5-10 us per
// iteration (profiles/r05_strip8_timeline.txt: the round-4 boundary/interior
// split on two streams ran a one-rank 8-way strip at 63 us/it under the
// profiler, 20 us over the kernel; with neighbours it would have overlapped
// the boundary columns' exchange with the interior tiles, which the
// cross-queue edges cost as much as they saved).  A sequence of
// n <= GRAPH_CHUNK iterations
//   k_seq_snap (state + Ctl, unless stopped) | n iterations |
//   one all-gather of the n rows | k_finalize_seq (fin_apply per row: the
//   trace, it / done / T, the stop rule)
// is one captured graph.  If row i < n - 1 met the stop rule, iterations
// i + 1 .. n - 1 have already run: k_finalize_seq records Ctl::ovr = i + 1,
// later sequences turn into no-ops (Ctl::stop), and the host restores the
// snapshot and re-runs the i + 1 iterations with the exact per-iteration
// step (ovr_recover) -- the same state, trace and stop iteration as the
// whole grid.
// (the snapshot buffers are allocated outside any capture -- gqmap_tile_attach_rccl,
// capture_steps -- and follow the grid size; without them the exact step runs)
bool deferred(const gqmap_ctx *c)
{
    return c->comm && c->L == 1 && c->d_rows && c->d_snap && c->snap_bytes == (size_t)c->MNL * NPLANES * c->rsz;
}

// An L = 1 RCCL tile always runs deferred sequences: the snapshot follows
// the grid size (a later gqmap_set_images may change it) and is allocated
// here, outside any capture; failing that, the run fails on this rank --
// never a quiet switch to the exact step, whose collectives would not match
// the other ranks' sequences.
gqmap_status comm_snap(gqmap_ctx *c)
{
    if (!c->comm || c->L != 1) return GQMAP_OK;
    GQ_CHECK(c->d_rows && ensure_snap(c), GQMAP_ERR_HIP, "tile %d: deferred-sequence snapshot (%zu bytes) not allocated",
             c->tile, (size_t)c->MNL * NPLANES * c->rsz);
    return GQMAP_OK;
}

template <typename R>
void unpack_advance_t(gqmap_ctx *c)
{
    HaloSide<R> sd[2];
    int n = 0;
    if (c->tile > 0) sd[n++] = HaloSide<R>{0, HALO_TO_RIGHT_N, HALO_TO_RIGHT, (R *)c->d_halo[2]};
    if (c->tile < c->n_tiles - 1) sd[n++] = HaloSide<R>{c->N - 1, HALO_TO_LEFT_N, HALO_TO_LEFT, (R *)c->d_halo[3]};
    if (n == 0) sd[0] = HaloSide<R>{0, 0, 0u, nullptr};
    k_unpack_advance<R><<<1, 256, 0, c->stream>>>(c->d_ctl, (R *)c->d_st[0], (R *)c->d_st[1], c->M,
                                                  (int64_t)c->M * c->N, c->MNL, c->L, sd[0], sd[n > 0 ? n - 1 : 0], n,
                                                  c->opt.t_decay_every, c->opt.drate, c->opt.t_min);
}

// Iteration `pos` of a deferred sequence; e0 / e1 (optional) bracket its
// k_iter launch.
gqmap_status launch_step_deferred(gqmap_ctx *c, int pos, hipEvent_t e0 = nullptr, hipEvent_t e1 = nullptr)
{
    const TileSegs all = strip_launch(c);
    c->spec_now = true;
    c->seq_row = c->d_rows + (size_t)pos * (NFIX + c->L);
    if (e0) GQ_HIP(hipEventRecord(e0, c->stream));
    launch_iter(c, &all);
    if (e1) GQ_HIP(hipEventRecord(e1, c->stream));
    gqmap_status st = exchange_rccl(c);
    if (st == GQMAP_OK) {
        if (c->fp32) unpack_advance_t<float>(c);
        else unpack_advance_t<double>(c);
    }
    c->spec_now = false;
    c->seq_row = nullptr;
    return st;
}

// A deferred sequence of n (1..GRAPH_CHUNK) iterations; ev (optional): 2 n
// events, a pair around each iteration's k_iter launches.
gqmap_status launch_seq_deferred(gqmap_ctx *c, int n, hipEvent_t *ev = nullptr)
{
    const int NP = NFIX + c->L;
    {
        const int64_t nv = (int64_t)c->MNL * NPLANES;
        const int grid = (int)std::min<int64_t>((nv + 255) / 256, 512);
        if (c->fp32)
            k_seq_snap<float><<<grid, 256, 0, c->stream>>>(c->d_ctl, (const float *)c->d_st[0], (const float *)c->d_st[1],
                                                           (float *)c->d_snap, c->d_snap_ctl, nv);
        else
            k_seq_snap<double><<<grid, 256, 0, c->stream>>>(c->d_ctl, (const double *)c->d_st[0],
                                                            (const double *)c->d_st[1], (double *)c->d_snap,
                                                            c->d_snap_ctl, nv);
    }
    for (int i = 0; i < n; ++i) {
        gqmap_status st = launch_step_deferred(c, i, ev ? ev[2 * i] : nullptr, ev ? ev[2 * i + 1] : nullptr);
        if (st != GQMAP_OK) return st;
    }
    gqmap_status st = comm_allgather(c, c->d_rows, c->d_seqg, (size_t)n * NP * sizeof(fix128));
    if (st != GQMAP_OK) return st;
    k_finalize_seq<<<1, 256, 0, c->stream>>>(fin_params(c), c->d_seqg, n);
    return GQMAP_OK;
}

gqmap_status launch_step(gqmap_ctx *c);

// After a run: a deferred sequence, or a dataflow launch deeper than lag 2
// (GQ_FLOW_LAG), overshot its stop iteration (Ctl::ovr): restore the
// sequence's / launch's snapshot (state + Ctl at its start) and re-run its
// first ovr iterations with the exact per-iteration step, which stops at the
// same iteration as the whole grid.  Every rank sees the same all-gathered
// totals, so every rank recovers together (the re-run's collectives match).
gqmap_status ovr_recover(gqmap_ctx *c, const Ctl &h, bool *recovered)
{
    *recovered = false;
    if (h.ovr == 0 || !c->d_snap) return GQMAP_OK;
    c->ctl_known = false;
    Ctl snap;
    GQ_HIP(hipMemcpyAsync(&snap, c->d_snap_ctl, sizeof(Ctl), hipMemcpyDeviceToHost, c->stream));
    GQ_HIP(hipStreamSynchronize(c->stream));
    GQ_HIP(hipMemcpyAsync(c->d_st[snap.done & 1], c->d_snap, c->snap_bytes, hipMemcpyDeviceToDevice, c->stream));
    GQ_HIP(hipMemcpyAsync(c->d_ctl, c->d_snap_ctl, sizeof(Ctl), hipMemcpyDeviceToDevice, c->stream));
    if (c->d_flow) GQ_HIP(hipMemsetAsync(c->d_flow, 0, sizeof(unsigned) * c->flow_n, c->stream));
    for (int i = 0; i < h.ovr; ++i) {
        gqmap_status st = launch_step(c);
        if (st != GQMAP_OK) return st;
    }
    GQ_HIP(hipStreamSynchronize(c->stream));
    *recovered = true;
    return GQMAP_OK;
}

gqmap_status launch_step(gqmap_ctx *c)
{
    c->ctl_known = false;
    if (c->comm) return launch_step_rccl(c);
    launch_iter(c);
    return launch_tail(c);
}

bool launch_flow(gqmap_ctx *c, int n, bool dry = false);

// n iterations: one persistent launch for small ctf grids (or one dataflow
// launch, policy flow), else n steps
gqmap_status launch_steps(gqmap_ctx *c, int n)
{
    c->ctl_known = false;
    if (launch_persist(c, n) || launch_flow(c, n)) return GQMAP_OK;
    gqmap_status st = GQMAP_OK;
    if (deferred(c)) {
        for (int i = 0; i < n && st == GQMAP_OK; i += GRAPH_CHUNK) st = launch_seq_deferred(c, std::min(GRAPH_CHUNK, n - i));
        return st;
    }
    for (int i = 0; i < n && st == GQMAP_OK; ++i) st = launch_step(c);
    return st;
}

void drop_graph(gqmap_ctx *c);

// ---- dataflow launch (k_iter_flow, policy flow) ---------------------------
#ifndef GQ_FLOW_WIDE_ITEMS  // items per iteration above which the 3-wave form runs
#define GQ_FLOW_WIDE_ITEMS 4096
#endif
template <typename R, typename VT, int ENG, int Q, bool LIT, int W>
void flow_launch(gqmap_ctx *c, IterParams<R, VT> P, int n, int nitems, int ntiles)
{
    static const int2 shape = kernel_shape(k_iter_flow<R, VT, ENG, Q, LIT, W>);
    P.cu_group = 1;
    P.cu_slots = std::max(1, shape.y / 8);
    // one workgroup per resident slot (more would only queue behind them)
    const int G = std::max(8, std::min(shape.x * shape.y, nitems));
    k_iter_flow<R, VT, ENG, Q, LIT, W><<<G, BLOCK, 0, c->stream>>>(P, n, c->d_flow, ntiles, c->d_snap_ctl);
}

template <typename R, typename VT, int ENG, int Q, bool LIT = false>
bool launch_flow_q(gqmap_ctx *c, int n, bool dry)
{
    const int ntiles = c->tiles_m * c->tiles_n;
    const int nitems = ntiles * (ENG == 1 ? c->L : 1);  // items per iteration
    if (c->flow_n != flow_words(nitems)) {  // (re)allocate outside any capture
        hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
        if (hipStreamIsCapturing(c->stream, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) return false;
        if (hipStreamSynchronize(c->stream) != hipSuccess) return false;
        if (c->d_flow) (void)hipFree(c->d_flow);
        c->d_flow = nullptr;
        c->flow_n = 0;
        if (hipMalloc((void **)&c->d_flow, sizeof(unsigned) * flow_words(nitems)) != hipSuccess) {
            c->d_flow = nullptr;
            return false;
        }
        if (hipMemsetAsync(c->d_flow, 0, sizeof(unsigned) * flow_words(nitems), c->stream) != hipSuccess ||
            hipStreamSynchronize(c->stream) != hipSuccess)
            return false;
        c->flow_n = flow_words(nitems);
    }
    if (!ensure_snap(c)) return false;
    if (dry) return true;
    {
        const int64_t nv = (int64_t)c->MNL * NPLANES;
        const int grid = (int)std::min<int64_t>((nv + 255) / 256, 512);
        k_persist_snap<R><<<grid, 256, 0, c->stream>>>(c->d_ctl, c->d_bar, (const R *)c->d_st[0],
                                                       (const R *)c->d_st[1], (R *)c->d_snap, c->d_snap_ctl, nv);
    }
    IterParams<R, VT> P = iter_params<R, VT>(c);
    if constexpr (ENG == 0 && Q == 1 && !LIT) {
        // a large frame (C5: ~14k tiles) has slack enough at any occupancy and
        // wants the latency hiding of 3 waves per SIMD: 2 waves measured
        // 2551 -> 2726 us per iteration on C5
        if (nitems > GQ_FLOW_WIDE_ITEMS) {
            flow_launch<R, VT, ENG, Q, LIT, 3>(c, P, n, nitems, ntiles);
            return true;
        }
    }
    flow_launch<R, VT, ENG, Q, LIT, 0>(c, P, n, nitems, ntiles);
    return true;
}

// Instantiated for the whole-grid single-scale mixture at Q = 1 (C2, either
// precision) and the fp64 coarse-to-fine levels at Q = 1, 2, 4 (C3's 480x640,
// 240x320, 120x160; the smaller ones run k_iter_persist).
template <typename R, typename VT>
bool launch_flow_t(gqmap_ctx *c, int n, bool dry)
{
    if (c->opt.engine == GQMAP_ENGINE_SUPER) {
        // C4's node grid (120 x 160, L = 3) at Q = 4, a mixture component per
        // item: bit-exact, but 283 -> 308 us/it (the per-launch kernel's
        // 234 VGPRs become 255 with spills; profiles/r06_super_flow_ab.txt):
        // only when forced
        if constexpr (sizeof(R) == 8) return c->pol.flow > 0 && c->kq == 4 && launch_flow_q<R, VT, 1, 4>(c, n, dry);
        return false;
    }
    if (c->opt.engine != GQMAP_ENGINE_CTF) {
        if constexpr (sizeof(R) == 8 && sizeof(VT) == 4) {
            // the literal-order arithmetic on integer frames (C2's parity-carrying
            // engine), bit-exact as items.  At the per-launch kernel's 3 waves
            // per SIMD the dataflow wrapper spills (224 bytes; 251 -> 265 us/it,
            // profiles/r06_lit_flow_ab2.txt); allowed 2 waves (GQ_FLOW_LIT_WAVES:
            // 243 VGPRs, no scratch, 512 slots -- a band of 116 tiles then has
            // ~64 items in flight, more slack for the neighbour dependencies)
            // it runs 250.8 -> 224.5 us/it (profiles/r06_lit_flow_2waves_ab.txt)
            if (c->lit) return c->pol.flow != 0 && c->kq == 1 && launch_flow_q<R, VT, 0, 1, true>(c, n, dry);
        }
        return !c->lit && c->kq == 1 && launch_flow_q<R, VT, 0, 1>(c, n, dry);
    }
    if (c->lit) return false;
    if constexpr (sizeof(R) == 8) {
        switch (c->kq) {
        case 1: return launch_flow_q<R, VT, 2, 1>(c, n, dry);
        case 2: return launch_flow_q<R, VT, 2, 2>(c, n, dry);
        // Q = 4 (120x160: 300 tiles, all resident in one round -- no tail to
        // fill) measured 48.5 -> 51.5 us/it as items: only when forced
        case 4: return c->pol.flow > 0 && launch_flow_q<R, VT, 2, 4>(c, n, dry);
        default: return false;
        }
    }
    return false;
}

// n iterations as one k_iter_flow launch when the policy asks for it and the
// context qualifies (single-scale mixture at one lane per node, or an fp64
// coarse-to-fine level at 1, 2 or 4; L = 1, the whole grid, fast
// arithmetic); dry: only the check (and the buffers).
bool launch_flow(gqmap_ctx *c, int n, bool dry)
{
    // auto: fp64 only -- the fp32 mixture kernel (4 waves per SIMD, gather
    // latency-bound) measured slower as items (110.5 vs 107.9 us/it,
    // profiles/r06_flow_ab_v1.txt)
    const bool on = c->pol.flow > 0 || (c->pol.flow < 0 && !c->fp32);
    if (!on || c->persist_off || (c->L != 1 && c->opt.engine != GQMAP_ENGINE_SUPER) || c->n_tiles != 1 ||
        c->comm || c->nranks != 0 || !fused_finalize(c) || n < 1)
        return false;
    if (c->fp32)
        return c->vvp ? !c->lit && c->kq == 1 && launch_flow_q<float, vvh2_t, 0, 1>(c, n, dry)
                      : launch_flow_t<float, float>(c, n, dry);
    if (c->vvp) return !c->lit && c->kq == 1 && launch_flow_q<double, vvh2_t, 0, 1>(c, n, dry);
    if (c->vv32) return launch_flow_t<double, vvs_t>(c, n, dry);
    return launch_flow_t<double, double>(c, n, dry);
}

// A persistent launch whose grid barrier gave up (workgroups not all
// resident -- another process or stream holding CUs -- or descheduled past
// the spin limit) leaves the failure word set; every later persistent
// launch of the replay then returns at once, and the snapshot keeps the
// state and Ctl the failed launch started from.  Recovery: restore that
// snapshot (the failed launch may have half-written the other ping-pong
// buffer and advanced Ctl part-way), clear the barrier words, and from here
// on run this context with one launch per iteration (the graphs are
// re-captured without the persistent launch).  *recovered: the run must go
// on from the restored iteration.
gqmap_status persist_recover(gqmap_ctx *c, bool *recovered)
{
    *recovered = false;
    if (!c->d_snap) return GQMAP_OK;  // no persistent launch has run on this context
    c->ctl_known = false;
    unsigned f = 0;
    GQ_HIP(hipMemcpyAsync(&f, c->d_bar + BAR_FAIL, sizeof(f), hipMemcpyDeviceToHost, c->stream));
    GQ_HIP(hipStreamSynchronize(c->stream));
    if (f == 0) return GQMAP_OK;
    Ctl h;
    GQ_HIP(hipMemcpyAsync(&h, c->d_snap_ctl, sizeof(Ctl), hipMemcpyDeviceToHost, c->stream));
    GQ_HIP(hipStreamSynchronize(c->stream));
    GQ_HIP(hipMemcpyAsync(c->d_st[h.done & 1], c->d_snap, c->snap_bytes, hipMemcpyDeviceToDevice, c->stream));
    GQ_HIP(hipMemcpyAsync(c->d_ctl, c->d_snap_ctl, sizeof(Ctl), hipMemcpyDeviceToDevice, c->stream));
    GQ_HIP(hipMemsetAsync(c->d_bar, 0, sizeof(unsigned) * BAR_WORDS, c->stream));
    if (c->d_flow) GQ_HIP(hipMemsetAsync(c->d_flow, 0, sizeof(unsigned) * c->flow_n, c->stream));
    GQ_HIP(hipStreamSynchronize(c->stream));
    if (c->pol.verbose)
        fprintf(stderr, "gqmap: persistent launch failed (%d workgroups); restored iteration %d, "
                        "continuing with one launch per iteration\n", c->nblocks + 1, h.it);
    c->persist_off = true;
    drop_graph(c);
    *recovered = true;
    return GQMAP_OK;
}

gqmap_status upload_ctl(gqmap_ctx *c, int it, double T, const double *w, const double *alpha)
{
    Ctl h{};
    h.it = it;
    h.done = 0;
    h.stop = 0;
    h.T = T;
    h.it_i = it;
    h.done_i = 0;
    h.T_i = T;
    for (int l = 0; l < c->L; ++l) {
        h.w[l] = w[l];
        h.alpha[l] = alpha[l];
    }
    c->ctl_known = false;
    GQ_HIP(hipMemcpyAsync(c->d_ctl, &h, sizeof(Ctl), hipMemcpyHostToDevice, c->stream));
    // a new state: a persistent launch's failure word (and the snapshot it
    // guards) belongs to the old one (persist_recover would restore it)
    GQ_HIP(hipMemsetAsync(c->d_bar + BAR_FAIL, 0, sizeof(unsigned), c->stream));
    GQ_HIP(hipStreamSynchronize(c->stream));
    c->ctl_it = it;
    c->ctl_known = true;
    return GQMAP_OK;
}

gqmap_status read_ctl(gqmap_ctx *c, Ctl *h)
{
    GQ_HIP(hipMemcpyAsync(c->h_ctl, c->d_ctl, sizeof(Ctl), hipMemcpyDeviceToHost, c->stream));
    GQ_HIP(hipStreamSynchronize(c->stream));
    *h = *c->h_ctl;
    c->ctl_it = h->it;
    c->ctl_known = true;
    return GQMAP_OK;
}

// Queue the copy of the trace-ring slots of iterations [it_first, it_first + n)
// into the pinned mirror (one run of slots, two when it wraps).
gqmap_status queue_trace(gqmap_ctx *c, int it_first, int n)
{
    if (n <= 0) return GQMAP_OK;
    n = std::min(n, TRACE_CAP);
    const int s0 = (it_first - 1) % TRACE_CAP, n0 = std::min(n, TRACE_CAP - s0);
    GQ_HIP(hipMemcpyAsync(c->h_ring + (size_t)TRACE_W * s0, c->d_trace + (size_t)TRACE_W * s0,
                          sizeof(double) * TRACE_W * n0, hipMemcpyDeviceToHost, c->stream));
    if (n > n0)
        GQ_HIP(hipMemcpyAsync(c->h_ring, c->d_trace, sizeof(double) * TRACE_W * (n - n0), hipMemcpyDeviceToHost,
                              c->stream));
    return GQMAP_OK;
}

// Iterations [it_first, it_first + n) of the pinned ring into the caller's
// trace (Energy, ptdmu, ptdsigma) and aepe arrays.
void copy_trace(const gqmap_ctx *c, int it_first, int n, double *trace, double *aepe)
{
    for (int i = 0; i < n; ++i) {
        const int slot = (it_first + i - 1) % TRACE_CAP;
        if (trace)
            for (int q = 0; q < 3; ++q) trace[3 * i + q] = c->h_ring[TRACE_W * slot + q];
        if (aepe) aepe[i] = c->h_ring[TRACE_W * slot + 3];
    }
}

constexpr int SUB_GRAPHS = 6;  // 2^5 = 32 < GRAPH_CHUNK
static_assert((1 << SUB_GRAPHS) > GRAPH_CHUNK, "sub graphs cover a chunk's remainder");

// The graph of n iterations (captured once, replayed).
gqmap_status capture_steps(gqmap_ctx *c, int n, hipGraphExec_t *out)
{
    if (*out) return GQMAP_OK;
    (void)launch_persist(c, n, true);  // occupancy query, snapshot buffers: outside the capture
    (void)launch_flow(c, n, true);
    gqmap_status st0 = comm_snap(c);  // the deferred RCCL sequence's snapshot
    if (st0 != GQMAP_OK) return st0;
    hipGraph_t g;
    GQ_HIP(hipStreamBeginCapture(c->stream, hipStreamCaptureModeThreadLocal));
    gqmap_status st = launch_steps(c, n);
    hipError_t ec = hipStreamEndCapture(c->stream, &g);
    if (st != GQMAP_OK) {
        if (ec == hipSuccess) (void)hipGraphDestroy(g);
        return st;
    }
    GQ_HIP(ec);
    hipError_t e = hipGraphInstantiate(out, g, nullptr, nullptr, 0);
    (void)hipGraphDestroy(g);
    GQ_HIP(e);
    return GQMAP_OK;
}

gqmap_status ensure_graph(gqmap_ctx *c) { return capture_steps(c, GRAPH_CHUNK, &c->graph); }

// A loopback-transport tile (tests) runs its launches directly: its
// collectives are host barriers and cross-stream event waits between the
// ranks' threads, which a stream capture cannot hold.  The launches and
// their order are the captured graph's.
bool loop_comm(const gqmap_ctx *c) { return c->comm && c->comm->loop; }

gqmap_status ensure_sub_graph(gqmap_ctx *c, int k) { return capture_steps(c, 1 << k, &c->sub[k]); }

void drop_graph(gqmap_ctx *c)
{
    if (c->graph) (void)hipGraphExecDestroy(c->graph);
    c->graph = nullptr;
    for (hipGraphExec_t &g : c->sub) {
        if (g) (void)hipGraphExecDestroy(g);
        g = nullptr;
    }
}

template <typename R>
std::vector<R> convert(const double *p, size_t n)
{
    std::vector<R> v(n);
    for (size_t i = 0; i < n; ++i) v[i] = R(p[i]);
    return v;
}

gqmap_status upload(gqmap_ctx *c, void *dst, const double *src, size_t n)
{
    if (c->fp32) {
        std::vector<float> v = convert<float>(src, n);
        GQ_HIP(hipMemcpyAsync(dst, v.data(), n * sizeof(float), hipMemcpyHostToDevice, c->stream));
        GQ_HIP(hipStreamSynchronize(c->stream));
    } else {
        GQ_HIP(hipMemcpyAsync(dst, src, n * sizeof(double), hipMemcpyHostToDevice, c->stream));
        GQ_HIP(hipStreamSynchronize(c->stream));
    }
    return GQMAP_OK;
}

gqmap_status download(gqmap_ctx *c, double *dst, const void *src, size_t n)
{
    if (c->fp32) {
        std::vector<float> v(n);
        GQ_HIP(hipMemcpyAsync(v.data(), src, n * sizeof(float), hipMemcpyDeviceToHost, c->stream));
        GQ_HIP(hipStreamSynchronize(c->stream));
        for (size_t i = 0; i < n; ++i) dst[i] = v[i];
    } else {
        GQ_HIP(hipMemcpyAsync(dst, src, n * sizeof(double), hipMemcpyDeviceToHost, c->stream));
        GQ_HIP(hipStreamSynchronize(c->stream));
    }
    return GQMAP_OK;
}


// Shape checks and (re)allocation for a Mo x No frame pair; VV storage type
// Whether the binary16 column-pair store may serve this context (its values
// checked by the caller; prepare_images also needs one lane per node): the
// single-scale mixture engine (fp64 or fp32) on one whole grid (the ctf levels
// measured neutral with it, the literal-order engine slower:
// profiles/r06_vvpair_ctf_ab.txt, r06_vvpair_literal_ab.txt).
bool vv_pair_candidate(const gqmap_ctx *c)
{
    return c->pol.vv_pair && !c->lit && !c->super_ && c->n_tiles == 1 && c->opt.engine == GQMAP_ENGINE_MIXTURE;
}

// vv32 (float) or double.  Invalidates the state when the grid changes.
gqmap_status prepare_images(gqmap_ctx *c, int Mo, int No, bool vv32, bool vvp = false)
{
    GQ_CHECK(Mo >= 4 && No >= 4, GQMAP_ERR_INVALID_ARG, "image %dx%d too small", Mo, No);
    if (c->super_)
        GQ_CHECK(Mo % 4 == 0 && No % 4 == 0, GQMAP_ERR_INVALID_ARG,
                 "super engine needs Mo,No divisible by 4 (got %dx%d)", Mo, No);
    const int M = c->super_ ? Mo / 4 : Mo, Ng = c->super_ ? No / 4 : No;
    GQ_CHECK(M >= 3 && Ng >= 3, GQMAP_ERR_INVALID_ARG, "node grid %dx%d has no interior", M, Ng);
    GQ_CHECK(Ng >= c->n_tiles, GQMAP_ERR_INVALID_ARG, "%d node columns cannot feed %d tiles", Ng,
             c->n_tiles);
    DeviceGuard dg(c->device);
    const bool geom = Mo != c->Mo || No != c->No;
    strip_geometry(c, Mo, No);
    tile_grid(c);  // (the lanes per node of this grid; alloc_grid repeats it)
    // the column-pair store serves the one-lane-per-node kernels only (the
    // lanes per node follow the grid): else the float store, exact as well
    if (vvp && (c->kq != 1 || c->split != 1)) {
        vvp = false;
        vv32 = true;
    }
    const bool resize = geom || vv32 != c->vv32 || vvp != c->vvp || !c->d_VV;
    c->vv32 = vv32;
    c->vvp = vvp;
    if (resize) {
        drop_graph(c);
        // every buffer below may still be read by work queued on the context
        // stream (a replayed graph): drain it before freeing
        GQ_HIP(hipStreamSynchronize(c->stream));
        if (c->d_VV) (void)hipFree(c->d_VV);
        if (c->d_I1) (void)hipFree(c->d_I1);
        c->d_VV = c->d_I1 = nullptr;
        // a truth belongs to the previous grid (k_iter indexes it with M, N)
        if (c->d_truth) (void)hipFree(c->d_truth);
        c->d_truth = nullptr;
        c->truth_elems = 0;
        const size_t vsz = c->fp32 ? sizeof(float) : vvp ? sizeof(vvh2_t) : vv32 ? sizeof(vvs_t) : sizeof(double);
        // zero tail past the padded frame (gqmap_math.h vv_elems, axis_cell_abs).
        // Stream-ordered: the context stream is non-blocking, so a null-stream
        // memset would be unordered with the VV upload / convert_device that
        // follows on c->stream (round-2 fp64-VV race).
        GQ_HIP(hipMalloc(&c->d_VV, vv_elems(Mo, No) * vsz));
        GQ_HIP(hipMemsetAsync(c->d_VV, 0, vv_elems(Mo, No) * vsz, c->stream));
        GQ_HIP(hipMalloc(&c->d_I1, (size_t)Mo * No * c->rsz));
        gqmap_status s = alloc_grid(c);
        if (s != GQMAP_OK) return s;
        c->have_state = false;
        if (c->n_tiles > 1) {
            for (int k = 0; k < 4; ++k) {
                if (c->d_halo[k]) (void)hipFree(c->d_halo[k]);
                c->d_halo[k] = nullptr;
                GQ_HIP(hipMalloc(&c->d_halo[k], halo_bytes(c, k)));
            }
        }
    }
    return GQMAP_OK;
}

}  // namespace

// ---- internal API for the coarse-to-fine driver (gqmap_pyramid.hip) -------
namespace gq {

gqmap_status ctx_set_images_device(gqmap_ctx *c, const double *dI1, const double *dI2, int Mo, int No,
                                   double *d_scratch, int *d_flag)
{
    // getVV on the device into d_scratch ((Mo+2)*(No+2) doubles), then the
    // same float-exactness policy as gqmap_set_images
    DeviceGuard dg(c->device);
    GQ_HIP(pad_vv_device(dI2, Mo, No, d_scratch, c->stream));
    const size_t nvv = (size_t)(Mo + 2) * (No + 2);
    bool vv32 = c->fp32;
    if (!vv32 && c->pol.vv_float)
        GQ_HIP(f32_exact_device(d_scratch, nvv, d_flag, &vv32, c->stream));
    // (the column-pair store: host frames of the single-scale mixture engine
    // only -- on the ctf levels it measured neutral, profiles/r06_vvpair_ctf_ab.txt)
    gqmap_status s = prepare_images(c, Mo, No, vv32);
    if (s != GQMAP_OK) return s;
    GQ_HIP(convert_device(d_scratch, c->d_VV, nvv, vv32, c->stream));
    GQ_HIP(convert_device(dI1, c->d_I1, (size_t)Mo * No, c->fp32, c->stream));
    c->have_images = true;
    return GQMAP_OK;
}

gqmap_status ctx_flow_device(gqmap_ctx *c, const void **muu, const void **muv, bool *fp32)
{
    Ctl h;
    gqmap_status s = read_ctl(c, &h);
    if (s != GQMAP_OK) return s;
    const char *cur = (const char *)c->d_st[h.done & 1];
    *muu = cur;
    *muv = cur + (size_t)c->MNL * c->rsz;
    *fp32 = c->fp32;
    return GQMAP_OK;
}

void ctx_adopt_stream(gqmap_ctx *c, hipStream_t s)
{
    DeviceGuard dg(c->device);
    drop_graph(c);
    if (c->stream && c->own_stream) (void)hipStreamDestroy(c->stream);
    c->stream = s;
    c->own_stream = false;
}

}  // namespace gq

extern "C" {

int gqmap_abi_version(void) { return GQMAP_ABI_VERSION; }

// Not in include/gqmap.h (tests): the k_iter kernel shape a context runs --
// lanes per node, 0 for the role split (GQMAP_SPLIT_ROLE); -1 without a grid.
int gqmap_debug_kernel_shape(const gqmap_ctx *c)
{
    return c && c->have_images ? c->kq : -1;
}

#if GQ_TIMELINE
// debug builds only (not in include/gqmap.h): copy the k_iter timeline
int gqmap_debug_timeline(unsigned long long *out, int n)
{
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(gq::g_timeline), sizeof(unsigned long long) * 32 * (size_t)n) ==
                   hipSuccess ? 0 : -1;
}
#endif

void gqmap_options_default(gqmap_options *o, int engine)
{
    std::memset(o, 0, sizeof(*o));
    const bool sup = engine == GQMAP_ENGINE_SUPER;
    if (engine == GQMAP_ENGINE_CTF) {
        // legacy/optical_flow_ctf.m:13-17 + legacy/gqmap_ctf.m constants
        o->its = 3000; o->K = 11; o->L = 1;
        o->temperature = 0.0; o->drate = 0.5;
        o->epsn = 1e-6; o->lambdad = 1.0; o->lambdas = 5.0;
        o->minu = -1; o->maxu = 1; o->minv = -1; o->maxv = 1;
        o->engine = engine; o->precision = GQMAP_FP64;
        o->alpha_mode = GQMAP_ALPHA_SOFTMAX; o->alpha_start = 1 << 30; o->alpha_lr = 0;
        o->guard_a = 0; o->t_decay_every = 0; o->t_min = 0.0;
        o->step0 = 0.07;         /* constant step (:27) */
        o->step_decay = 1e300;   /* step0/(1+it/1e300) == step0 exactly */
        o->sig_lo = 0.01; o->sig_hi = 25.0;   /* :34-35 */
        o->corr_tor = 0.999;     /* :5 */
        o->tor = 1e-4;
        o->sig_step = 0.3;       /* sigma step x0.3 (:34-35) */
        o->sig_init = 3.0;       /* sigma = rand + 3 (:16-17) */
        return;
    }
    // driver values: optical_flow.m:16-23 / optical_flowSuper.m:19-26
    o->its = 30000;
    o->K = sup ? 11 : 9;
    o->L = 3;
    o->temperature = sup ? 0.2 : 0.0;
    o->drate = sup ? 0.75 : 0.5;
    o->epsn = 1e-6;
    o->lambdad = 1.0;
    o->lambdas = sup ? 16.0 : 5.0;
    o->minu = -1; o->maxu = 1; o->minv = -1; o->maxv = 1;
    o->engine = engine;
    o->precision = GQMAP_FP64;
    o->alpha_mode = GQMAP_ALPHA_SOFTMAX;
    o->alpha_start = 500;
    o->alpha_lr = 1e-7;
    o->guard_a = sup ? 0 : 1;
    o->t_decay_every = sup ? 500 : 0;
    o->t_min = 0.001;
    o->step0 = sup ? 0.001 : 0.1;
    o->step_decay = sup ? 4000.0 : 8000.0;
    o->sig_lo = 0.01;
    o->sig_hi = sup ? 25.0 : 23.0;
    o->corr_tor = 1 - 1e-5;
    o->tor = 1e-4;
    o->sig_step = 1.0;
    o->sig_init = -1.0;  /* sigma = rand + (max-min) (gqmap_gpu_mixture.m:21-22) */
}

gqmap_status gqmap_options_alpha_mode(gqmap_options *o, int mode)
{
    clear_error();
    GQ_CHECK(o, GQMAP_ERR_INVALID_ARG, "gqmap_options_alpha_mode: null options");
    GQ_CHECK(mode == GQMAP_ALPHA_SOFTMAX || mode == GQMAP_ALPHA_PROJSPLX, GQMAP_ERR_INVALID_ARG,
             "unknown alpha mode %d", mode);
    o->alpha_mode = mode;
    if (o->engine == GQMAP_ENGINE_CTF) return GQMAP_OK;  // L == 1: no alpha update
    const bool sup = o->engine == GQMAP_ENGINE_SUPER;
    if (mode == GQMAP_ALPHA_PROJSPLX && sup) {
        // gqmap_gpuSuper_mix_entropy.m:48 (commented): it>200, step*1E-6
        o->alpha_start = 200;
        o->alpha_lr = 1e-6;
    } else {
        // updateAlpha (:50, :83 / super :49, :82) and gqmap_gpu_mixture.m:49: it>500, 1E-7
        o->alpha_start = 500;
        o->alpha_lr = 1e-7;
    }
    return GQMAP_OK;
}

gqmap_status gqmap_create(gqmap_ctx **out, const gqmap_options *opt, int device)
{
    clear_error();
    GQ_CHECK(out && opt, GQMAP_ERR_INVALID_ARG, "gqmap_create: null argument");
    *out = nullptr;
    GQ_CHECK(opt->L >= 1 && opt->L <= GQMAP_LMAX, GQMAP_ERR_INVALID_ARG, "L=%d outside [1,%d]",
             opt->L, GQMAP_LMAX);
    GQ_CHECK(opt->K >= 2 && opt->K <= GQMAP_KMAX, GQMAP_ERR_INVALID_ARG, "K=%d outside [2,%d]",
             opt->K, GQMAP_KMAX);
    GQ_CHECK(opt->engine == GQMAP_ENGINE_MIXTURE || opt->engine == GQMAP_ENGINE_SUPER ||
                 opt->engine == GQMAP_ENGINE_CTF,
             GQMAP_ERR_INVALID_ARG, "unknown engine %d", opt->engine);
    GQ_CHECK(opt->precision != GQMAP_FP32 || opt->epsn >= 0x1p-96, GQMAP_ERR_INVALID_ARG,
             "fp32 needs epsn >= 2^-96 (its sqrt assumes normal arguments), got %g", opt->epsn);
    GQ_CHECK(opt->engine != GQMAP_ENGINE_CTF || opt->L == 1, GQMAP_ERR_INVALID_ARG,
             "the coarse-to-fine engine is single-Gaussian (L=1)");
    GQ_CHECK(opt->precision == GQMAP_FP64 || opt->precision == GQMAP_FP32, GQMAP_ERR_INVALID_ARG,
             "unknown precision %d", opt->precision);
    GQ_CHECK(opt->minu <= opt->maxu && opt->minv <= opt->maxv, GQMAP_ERR_INVALID_ARG,
             "empty flow range");
    GQ_CHECK(opt->arith == GQMAP_ARITH_FAST || opt->arith == GQMAP_ARITH_LITERAL, GQMAP_ERR_INVALID_ARG,
             "unknown arith %d", opt->arith);
    GQ_CHECK(opt->arith != GQMAP_ARITH_LITERAL ||
                 (opt->engine == GQMAP_ENGINE_MIXTURE && opt->precision == GQMAP_FP64 &&
                  (opt->split == 0 || opt->split == 1)),
             GQMAP_ERR_UNSUPPORTED, "literal-order arithmetic: fp64 mixture engine, split 0 or 1");
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
        set_error("no HIP device available");
        return GQMAP_ERR_NO_DEVICE;
    }
    GQ_CHECK(device >= 0 && device < ndev, GQMAP_ERR_INVALID_ARG, "device %d of %d", device, ndev);
    DeviceGuard dg(device);
    gqmap_ctx *c = new gqmap_ctx();
    c->opt = *opt;
    c->device = device;
    c->fp32 = opt->precision == GQMAP_FP32;
    c->super_ = opt->engine == GQMAP_ENGINE_SUPER;
    c->rsz = c->fp32 ? sizeof(float) : sizeof(double);
    c->L = opt->L;
    c->K = opt->K;
    c->K2 = opt->K * opt->K;
    c->lit = opt->arith == GQMAP_ARITH_LITERAL;
    // quadrature tables, MATLAB meshgrid order k = r + K*c (gqmap_gpu_mixture.m:8-10)
    double X[GQMAP_KMAX], W[GQMAP_KMAX];
    if (gauss_hermite(c->K, X, W) != 0) {
        delete c;
        set_error("Gauss-Hermite did not converge for K=%d", opt->K);
        return GQMAP_ERR_INVALID_ARG;
    }
    std::memset(c->tab_host, 0, sizeof(c->tab_host));
    for (int cc = 0; cc < c->K; ++cc)
        for (int r = 0; r < c->K; ++r) {
            const int k = r + c->K * cc;
            const double xi = X[cc], xj = X[r], w = W[cc] * W[r];
            if (c->lit) {  // the literal layout (gqmap_math.h TL_*)
                lit_table_point(&c->tab_host[tab_at(0, k)], xi, xj, W[cc], W[r]);
                continue;
            }
            c->tab_host[tab_at(T_XI, k)] = xi;
            c->tab_host[tab_at(T_XJ, k)] = xj;
            c->tab_host[tab_at(T_W, k)] = w;
            c->tab_host[tab_at(T_WXI, k)] = w * xi;
            c->tab_host[tab_at(T_WXJ, k)] = w * xj;
            c->tab_host[tab_at(T_WA, k)] = w * (xi * xi + xj * xj);
            c->tab_host[tab_at(T_WM, k)] = w * (xi * xi - xj * xj);
            c->tab_host[tab_at(T_WX, k)] = w * (xi * xj);
        }
    gqmap_status st = GQMAP_OK;
    auto fail = [&](gqmap_status s) { gqmap_destroy(c); return s; };
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
        set_error("hipStreamCreate failed");
        return fail(GQMAP_ERR_HIP);
    }
    if (hipMalloc(&c->d_tab, NTAB * TS * c->rsz) != hipSuccess ||
        hipMalloc((void **)&c->d_ctl, sizeof(Ctl)) != hipSuccess ||
        hipMalloc((void **)&c->d_trace, sizeof(double) * TRACE_W * TRACE_CAP) != hipSuccess ||
        hipMalloc((void **)&c->d_bar, sizeof(unsigned) * BAR_WORDS) != hipSuccess ||
        hipHostMalloc((void **)&c->h_ctl, sizeof(Ctl), hipHostMallocDefault) != hipSuccess ||
        hipHostMalloc((void **)&c->h_ring, sizeof(double) * TRACE_W * TRACE_CAP, hipHostMallocDefault) != hipSuccess ||
        hipHostMalloc((void **)&c->h_fail, sizeof(unsigned), hipHostMallocDefault) != hipSuccess) {
        set_error("device allocation failed");
        return fail(GQMAP_ERR_OUT_OF_MEMORY);
    }
    // synchronous: a pyramid level adopts another stream right after creation
    if (hipMemsetAsync(c->d_bar, 0, sizeof(unsigned) * BAR_WORDS, c->stream) != hipSuccess ||
        hipStreamSynchronize(c->stream) != hipSuccess) {
        set_error("hipMemsetAsync failed");
        return fail(GQMAP_ERR_HIP);
    }
    if ((st = upload(c, c->d_tab, c->tab_host, NTAB * TS)) != GQMAP_OK) return fail(st);
    *out = c;
    return GQMAP_OK;
}

gqmap_status gqmap_set_images(gqmap_ctx *c, const double *I1, const double *I2, int Mo, int No)
{
    clear_error();
    GQ_CHECK(c && I1 && I2, GQMAP_ERR_INVALID_ARG, "gqmap_set_images: null argument");
    std::vector<double> VV((size_t)(Mo + 2) * (No + 2));
    if (Mo >= 4 && No >= 4) build_padded(I2, Mo, No, VV.data());
    // fp64 engine: keep the padded image in float when that is exact (frames
    // from rgb2gray are integers; their cubic padding stays in [-510, 765]):
    // same values, half the gather bytes.
    bool vv32 = c->fp32;
    if (!vv32 && c->pol.vv_float) {
        vv32 = true;
        for (double v : VV)
            if ((double)(vvs_t)v != v) { vv32 = false; break; }
    }
    // binary16 column pairs (gqmap_math.h vvh2_t): the fp64 single-scale
    // mixture engine at one lane per node on one whole grid, every value exact
    bool vvp = vv32 && vv_pair_candidate(c);
    if (vvp)
        for (double v : VV)
            if ((double)(float)(_Float16)v != v) { vvp = false; break; }
    if (vvp) vv32 = false;
    gqmap_status s = prepare_images(c, Mo, No, vv32, vvp);  // (may fall back to float: c->vvp)
    if (s != GQMAP_OK) return s;
    vvp = c->vvp;
    vv32 = c->vv32;
    DeviceGuard dg(c->device);
    // every copy on the context stream, after prepare_images' zero fill
    if (vvp) {
        // element (r, c): rows r of columns c and c + 1 (the column past the
        // frame is the zero column of the buffer)
        const size_t M2 = (size_t)Mo + 2, N2 = (size_t)No + 2;
        std::vector<vvh2_t> vp(VV.size());
        for (size_t cc = 0; cc < N2; ++cc)
            for (size_t r = 0; r < M2; ++r) {
                vp[r + M2 * cc].lo = (_Float16)VV[r + M2 * cc];
                vp[r + M2 * cc].hi = cc + 1 < N2 ? (_Float16)VV[r + M2 * (cc + 1)] : (_Float16)0;
            }
        GQ_HIP(hipMemcpyAsync(c->d_VV, vp.data(), vp.size() * sizeof(vvh2_t), hipMemcpyHostToDevice, c->stream));
        GQ_HIP(hipStreamSynchronize(c->stream));
    } else if (vv32 && !c->fp32) {
        std::vector<vvs_t> vc(VV.size());
        for (size_t k = 0; k < VV.size(); ++k) vc[k] = (vvs_t)VV[k];
        GQ_HIP(hipMemcpyAsync(c->d_VV, vc.data(), vc.size() * sizeof(vvs_t), hipMemcpyHostToDevice, c->stream));
        GQ_HIP(hipStreamSynchronize(c->stream));
    } else if (vv32) {
        std::vector<float> v32(VV.begin(), VV.end());
        GQ_HIP(hipMemcpyAsync(c->d_VV, v32.data(), v32.size() * sizeof(float), hipMemcpyHostToDevice, c->stream));
        GQ_HIP(hipStreamSynchronize(c->stream));
    } else if ((s = upload(c, c->d_VV, VV.data(), VV.size())) != GQMAP_OK) {
        return s;
    }
    if ((s = upload(c, c->d_I1, I1, (size_t)Mo * No)) != GQMAP_OK) return s;
    c->have_images = true;
    return GQMAP_OK;
}

gqmap_status gqmap_init_state(gqmap_ctx *c, uint64_t seed)
{
    clear_error();
    GQ_CHECK(c, GQMAP_ERR_INVALID_ARG, "null context");
    GQ_CHECK(c->have_images, GQMAP_ERR_STATE, "gqmap_init_state before gqmap_set_images");
    DeviceGuard dg(c->device);
    const gqmap_options &o = c->opt;
    const int threads = 256;
    const int blocks = (int)((c->MNL + threads - 1) / threads);
    const uint64_t b1 = stream_base(seed, 1), b2 = stream_base(seed, 2);
    const uint64_t b3 = stream_base(seed, 3), b4 = stream_base(seed, 4);
    if (c->fp32)
        k_init_state<float><<<blocks, threads, 0, c->stream>>>(
            (float *)c->d_st[0], (float *)c->d_st[1], c->MNL, b1, b2, b3, b4, o.minu, o.maxu, o.minv, o.maxv, o.sig_init,
            c->M, c->N, c->n_off, c->Ng);
    else
        k_init_state<double><<<blocks, threads, 0, c->stream>>>(
            (double *)c->d_st[0], (double *)c->d_st[1], c->MNL, b1, b2, b3, b4, o.minu, o.maxu, o.minv, o.maxv, o.sig_init,
            c->M, c->N, c->n_off, c->Ng);
    GQ_HIP(hipGetLastError());
    double w[GQMAP_LMAX], alpha[GQMAP_LMAX], se = 0;
    gqmap_rand_uniform(seed, 0, 0, (size_t)c->L, w);  // w = rand(1,1,L)
    for (int l = 0; l < c->L; ++l) se += std::exp(w[l]);
    for (int l = 0; l < c->L; ++l) alpha[l] = std::exp(w[l]) / se;
    gqmap_status s = upload_ctl(c, 1, o.temperature, w, alpha);
    if (s != GQMAP_OK) return s;
    c->have_state = true;
    return GQMAP_OK;
}

gqmap_status gqmap_set_state(gqmap_ctx *c, const gqmap_state *st)
{
    clear_error();
    GQ_CHECK(c && st, GQMAP_ERR_INVALID_ARG, "gqmap_set_state: null argument");
    GQ_CHECK(c->have_images, GQMAP_ERR_STATE, "gqmap_set_state before gqmap_set_images");
    GQ_CHECK(st->muu && st->muv && st->sigu && st->sigv && st->pn && st->rou && st->w && st->alpha,
             GQMAP_ERR_INVALID_ARG, "gqmap_set_state: null state array");
    GQ_CHECK(st->it >= 1, GQMAP_ERR_INVALID_ARG, "state.it must be >= 1");
    DeviceGuard dg(c->device);
    // state arrays are the FULL node grid (M x Ng x L); a tile takes its
    // columns n_off .. n_off+N-1 (owned + ghosts): one run of M*N per (plane, l)
    const int64_t MNg = (int64_t)c->M * c->Ng, MNgL = MNg * c->L, MN = (int64_t)c->M * c->N;
    const double *planes[NPLANES] = {st->muu, st->muv, st->sigu, st->sigv, st->pn,
                                     st->rou, st->rou + MNgL, st->rou + 2 * MNgL,
                                     st->rou + 3 * MNgL};
    std::vector<double> loc((size_t)c->MNL);
    for (int q = 0; q < NPLANES; ++q) {
        for (int l = 0; l < c->L; ++l)
            std::memcpy(&loc[(size_t)(l * MN)], planes[q] + l * MNg + (int64_t)c->n_off * c->M,
                        sizeof(double) * (size_t)MN);
        for (int b = 0; b < 2; ++b) {
            gqmap_status s = upload(c, (char *)c->d_st[b] + (size_t)q * c->MNL * c->rsz, loc.data(),
                                    (size_t)c->MNL);
            if (s != GQMAP_OK) return s;
        }
    }
    gqmap_status s = upload_ctl(c, st->it, st->T, st->w, st->alpha);
    if (s != GQMAP_OK) return s;
    c->have_state = true;
    return GQMAP_OK;
}

gqmap_status gqmap_get_state(gqmap_ctx *c, gqmap_state *st)
{
    clear_error();
    GQ_CHECK(c && st, GQMAP_ERR_INVALID_ARG, "gqmap_get_state: null argument");
    GQ_CHECK(c->have_state, GQMAP_ERR_STATE, "no state");
    DeviceGuard dg(c->device);
    Ctl h;
    gqmap_status s = read_ctl(c, &h);
    if (s != GQMAP_OK) return s;
    const void *cur = c->d_st[h.done & 1];
    // full-grid arrays: a tile writes its owned columns only
    const int64_t MNg = (int64_t)c->M * c->Ng, MNgL = MNg * c->L, MN = (int64_t)c->M * c->N;
    double *planes[NPLANES] = {st->muu, st->muv, st->sigu, st->sigv, st->pn, st->rou,
                               st->rou ? st->rou + MNgL : nullptr,
                               st->rou ? st->rou + 2 * MNgL : nullptr,
                               st->rou ? st->rou + 3 * MNgL : nullptr};
    std::vector<double> loc((size_t)c->MNL);
    const size_t own = (size_t)c->M * (c->own_hi - c->own_lo);
    for (int q = 0; q < NPLANES; ++q) {
        if (!planes[q]) continue;
        s = download(c, loc.data(), (const char *)cur + (size_t)q * c->MNL * c->rsz, (size_t)c->MNL);
        if (s != GQMAP_OK) return s;
        for (int l = 0; l < c->L; ++l)
            std::memcpy(planes[q] + l * MNg + (int64_t)c->col0 * c->M,
                        &loc[(size_t)(l * MN + (int64_t)c->own_lo * c->M)], sizeof(double) * own);
    }
    for (int l = 0; l < c->L; ++l) {
        if (st->w) st->w[l] = h.w[l];
        if (st->alpha) st->alpha[l] = h.alpha[l];
    }
    st->it = h.it;
    st->T = h.T;
    return GQMAP_OK;
}

static gqmap_status fetch_trace(gqmap_ctx *c, int it_before, int n, double *trace, double *aepe = nullptr)
{
    if ((!trace && !aepe) || n <= 0) return GQMAP_OK;
    // only the ring slots of these n iterations: a short run copies a few
    // hundred bytes, not the ring
    gqmap_status s = queue_trace(c, it_before, n);
    if (s != GQMAP_OK) return s;
    GQ_HIP(hipStreamSynchronize(c->stream));
    copy_trace(c, it_before, n, trace, aepe);
    return GQMAP_OK;
}

gqmap_status gqmap_run(gqmap_ctx *c, int n_iter, int *n_done, double *trace)
{
    return gqmap_run_aepe(c, n_iter, n_done, trace, nullptr);
}

gqmap_status gqmap_set_truth(gqmap_ctx *c, const double *grdt, int Mg, int Ng)
{
    clear_error();
    GQ_CHECK(c, GQMAP_ERR_INVALID_ARG, "null context");
    GQ_CHECK(c->have_images, GQMAP_ERR_STATE, "gqmap_set_truth before gqmap_set_images");
    GQ_CHECK(c->opt.engine == GQMAP_ENGINE_CTF, GQMAP_ERR_UNSUPPORTED,
             "per-iteration AEPE is the ctf level engine's (legacy/gqmap_ctf.m:38)");
    GQ_CHECK(c->n_tiles == 1, GQMAP_ERR_UNSUPPORTED, "gqmap_set_truth on a column-strip tile");
    DeviceGuard dg(c->device);
    if (!grdt) {
        if (c->d_truth) {
            drop_graph(c);  // the captured launches hold the truth pointer
            GQ_HIP(hipStreamSynchronize(c->stream));
            GQ_HIP(hipFree(c->d_truth));
        }
        c->d_truth = nullptr;
        c->truth_elems = 0;
        return GQMAP_OK;
    }
    GQ_CHECK(Mg >= c->M && Ng >= c->N, GQMAP_ERR_INVALID_ARG, "truth %dx%d smaller than the grid %dx%d", Mg, Ng,
             c->M, c->N);
    // GRDT(M_,N_,:) of the array passed in: its top-left M x N block (the
    // reference passes the full-resolution trueFlow.*scale to every level)
    const size_t MN = (size_t)c->M * c->N;
    std::vector<double> blk(2 * MN);
    for (int k = 0; k < 2; ++k)
        for (int n = 0; n < c->N; ++n)
            std::memcpy(&blk[MN * k + (size_t)c->M * n], grdt + (size_t)Mg * Ng * k + (size_t)Mg * n,
                        sizeof(double) * c->M);
    if (c->truth_elems != 2 * MN) {
        // (re)allocate for this grid; the captured graph holds the old pointer
        // (a same-size update keeps pointer and graph)
        drop_graph(c);
        GQ_HIP(hipStreamSynchronize(c->stream));
        if (c->d_truth) (void)hipFree(c->d_truth);
        c->d_truth = nullptr;
        c->truth_elems = 0;
        GQ_HIP(hipMalloc((void **)&c->d_truth, sizeof(double) * 2 * MN));
        c->truth_elems = 2 * MN;
    }
    GQ_HIP(hipMemcpyAsync(c->d_truth, blk.data(), sizeof(double) * 2 * MN, hipMemcpyHostToDevice, c->stream));
    GQ_HIP(hipStreamSynchronize(c->stream));
    return GQMAP_OK;
}

gqmap_status gqmap_run_aepe(gqmap_ctx *c, int n_iter, int *n_done, double *trace, double *aepe)
{
    clear_error();
    GQ_CHECK(c, GQMAP_ERR_INVALID_ARG, "null context");
    GQ_CHECK(c->have_images && c->have_state, GQMAP_ERR_STATE, "gqmap_run before images/state");
    GQ_CHECK(c->n_tiles == 1 || c->comm, GQMAP_ERR_STATE,
             "tile %d/%d: attach RCCL (gqmap_tile_attach_rccl) or use gqmap_tile_group_run", c->tile,
             c->n_tiles);
    GQ_CHECK(n_iter >= 0, GQMAP_ERR_INVALID_ARG, "n_iter < 0");
    DeviceGuard dg(c->device);
    gqmap_status s = comm_snap(c);  // deferred RCCL sequences (outside any capture)
    if (s != GQMAP_OK) return s;
    Ctl h0;
    if (c->ctl_known) h0.it = c->ctl_it;
    else if ((s = read_ctl(c, &h0)) != GQMAP_OK) return s;
    int total = 0;
    while (total < n_iter) {
        // the device trace ring holds TRACE_CAP iterations: drain it per chunk
        const int chunk = std::min(n_iter - total, TRACE_CAP);
        int left = chunk;
        c->ctl_known = false;
        if (c->pol.graph && !loop_comm(c)) {
            // GRAPH_CHUNK-iteration graphs, then the remainder as graphs of
            // 2^k iterations (a short run replays graphs too)
            if (left >= GRAPH_CHUNK && (s = ensure_graph(c)) != GQMAP_OK) return s;
            while (left >= GRAPH_CHUNK) {
                GQ_HIP(hipGraphLaunch(c->graph, c->stream));
                left -= GRAPH_CHUNK;
            }
            // (a persistent small-level context or a deferred RCCL strip runs
            // the remainder as ONE launch / one sequence, directly: as 2^k
            // graphs it would pay a snapshot and a grid-barrier start-up, or
            // a snapshot, an all-gather and a finalize, per sub-graph)
            const bool one = left > 0 && (deferred(c) || launch_persist(c, left, true) || launch_flow(c, left, true));
            if (!one) {
                for (int k = SUB_GRAPHS - 1; k >= 0; --k)
                    if (left & (1 << k)) {
                        if ((s = ensure_sub_graph(c, k)) != GQMAP_OK) return s;
                        GQ_HIP(hipGraphLaunch(c->sub[k], c->stream));
                    }
                left = 0;
            }
        }
        if (left > 0 && (s = launch_steps(c, left)) != GQMAP_OK) return s;
        GQ_HIP(hipGetLastError());
        // one round trip: Ctl, the chunk's trace slots (as many as may have
        // run) and the persistent failure word
        const int it_first = h0.it + total;
        GQ_HIP(hipMemcpyAsync(c->h_ctl, c->d_ctl, sizeof(Ctl), hipMemcpyDeviceToHost, c->stream));
        if ((trace || aepe) && (s = queue_trace(c, it_first, chunk)) != GQMAP_OK) return s;
        if (c->d_snap)
            GQ_HIP(hipMemcpyAsync(c->h_fail, c->d_bar + BAR_FAIL, sizeof(unsigned), hipMemcpyDeviceToHost, c->stream));
        GQ_HIP(hipStreamSynchronize(c->stream));
        Ctl h = *c->h_ctl;
        bool recovered = false;
        if (c->d_snap && !c->comm && *c->h_fail != 0) {
            if ((s = persist_recover(c, &recovered)) != GQMAP_OK) return s;
            if ((s = read_ctl(c, &h)) != GQMAP_OK) return s;
        }
        if (h.ovr) {  // a deferred RCCL sequence / deep dataflow launch ran past its stop iteration
            bool again = false;
            if ((s = ovr_recover(c, h, &again)) != GQMAP_OK) return s;
            if ((s = read_ctl(c, &h)) != GQMAP_OK) return s;
            // (the finalize had already recorded the trace up to the stop; the
            // exact re-run rewrote the same slots -- read them again anyway)
            if ((trace || aepe) && (s = queue_trace(c, it_first, std::min(chunk, std::max(0, h.it - it_first)))) != GQMAP_OK)
                return s;
            GQ_HIP(hipStreamSynchronize(c->stream));
        }
        const int ran = h.it - it_first;
        copy_trace(c, it_first, std::min(ran, chunk), trace ? trace + 3 * total : nullptr, aepe ? aepe + total : nullptr);
        total += ran;
        c->ctl_it = h.it;
        c->ctl_known = true;
        if (h.stop || (ran < chunk && !recovered)) break;
    }
    if (n_done) *n_done = total;
    return GQMAP_OK;
}

gqmap_status gqmap_run_timed(gqmap_ctx *c, int n_iter, int *n_done, double *total_ms,
                             double *iter_kernel_ms)
{
    clear_error();
    GQ_CHECK(c, GQMAP_ERR_INVALID_ARG, "null context");
    GQ_CHECK(c->have_images && c->have_state, GQMAP_ERR_STATE, "gqmap_run before images/state");
    GQ_CHECK(c->n_tiles == 1 || c->comm, GQMAP_ERR_STATE,
             "tile %d/%d: attach RCCL (gqmap_tile_attach_rccl) or use gqmap_tile_group_run", c->tile,
             c->n_tiles);
    GQ_CHECK(n_iter >= 1, GQMAP_ERR_INVALID_ARG, "n_iter < 1");
    DeviceGuard dg(c->device);
    gqmap_status s = comm_snap(c);
    if (s != GQMAP_OK) return s;
    Ctl h0;
    s = read_ctl(c, &h0);
    if (s != GQMAP_OK) return s;
    std::vector<hipEvent_t> ev((size_t)2 * n_iter + 2);
    for (auto &e : ev) GQ_HIP(hipEventCreate(&e));
    GQ_HIP(hipEventRecord(ev[0], c->stream));
    int timed = n_iter;  // event pairs summed into iter_kernel_ms
    if (deferred(c)) {  // the production sequences, each iteration's k_iter launch bracketed
        for (int i = 0; i < n_iter; i += GRAPH_CHUNK)
            if ((s = launch_seq_deferred(c, std::min(GRAPH_CHUNK, n_iter - i), &ev[2 + 2 * i])) != GQMAP_OK) return s;
    } else if (launch_flow(c, n_iter, true)) {  // one pair around each chunk's dataflow launch
        timed = 0;
        for (int i = 0; i < n_iter; i += GRAPH_CHUNK, ++timed) {
            GQ_HIP(hipEventRecord(ev[2 + 2 * timed], c->stream));
            (void)launch_flow(c, std::min(GRAPH_CHUNK, n_iter - i));
            GQ_HIP(hipEventRecord(ev[3 + 2 * timed], c->stream));
        }
    } else {
        for (int i = 0; i < n_iter; ++i) {
            if (c->comm) {  // the iteration's one k_iter launch over the strip
                if ((s = launch_step_rccl(c, ev[2 + 2 * i], ev[3 + 2 * i])) != GQMAP_OK) return s;
                continue;
            }
            GQ_HIP(hipEventRecord(ev[2 + 2 * i], c->stream));
            launch_iter(c);
            GQ_HIP(hipEventRecord(ev[3 + 2 * i], c->stream));
            if ((s = launch_tail(c)) != GQMAP_OK) return s;
        }
    }
    GQ_HIP(hipEventRecord(ev[1], c->stream));
    GQ_HIP(hipEventSynchronize(ev[1]));
    GQ_HIP(hipGetLastError());
    float t = 0;
    GQ_HIP(hipEventElapsedTime(&t, ev[0], ev[1]));
    double sum = 0;
    for (int i = 0; i < timed; ++i) {
        float k = 0;
        GQ_HIP(hipEventElapsedTime(&k, ev[2 + 2 * i], ev[3 + 2 * i]));
        sum += k;
    }
    for (auto &e : ev) (void)hipEventDestroy(e);
    Ctl h;
    if ((s = read_ctl(c, &h)) != GQMAP_OK) return s;
    if (h.ovr) {
        bool again = false;
        if ((s = ovr_recover(c, h, &again)) != GQMAP_OK) return s;
        if ((s = read_ctl(c, &h)) != GQMAP_OK) return s;
    }
    if (c->d_snap && !c->comm) {  // a failed persistent / dataflow launch: restored, finished per launch
        bool rec = false;
        if ((s = persist_recover(c, &rec)) != GQMAP_OK) return s;
        if (rec) {
            if ((s = read_ctl(c, &h)) != GQMAP_OK) return s;
            for (int i = h.it - h0.it; i < n_iter && !h.stop; ++i) {
                launch_iter(c);
                if ((s = launch_tail(c)) != GQMAP_OK) return s;
                if ((s = read_ctl(c, &h)) != GQMAP_OK) return s;
            }
        }
    }
    if (n_done) *n_done = h.it - h0.it;
    if (total_ms) *total_ms = t;
    if (iter_kernel_ms) *iter_kernel_ms = sum;
    return GQMAP_OK;
}

gqmap_status gqmap_prepare(gqmap_ctx *c)
{
    clear_error();
    GQ_CHECK(c, GQMAP_ERR_INVALID_ARG, "null context");
    GQ_CHECK(c->have_images && c->have_state, GQMAP_ERR_STATE, "gqmap_prepare before images/state");
    GQ_CHECK(c->n_tiles == 1 || c->comm, GQMAP_ERR_STATE,
             "tile %d/%d: attach RCCL (gqmap_tile_attach_rccl) or use gqmap_tile_group_run", c->tile,
             c->n_tiles);
    DeviceGuard dg(c->device);
    if (loop_comm(c)) return comm_snap(c);
    gqmap_status s = ensure_graph(c);
    if (s != GQMAP_OK) return s;
    GQ_HIP(hipGraphUpload(c->graph, c->stream));
    for (int k = 0; k < SUB_GRAPHS; ++k) {
        if ((s = ensure_sub_graph(c, k)) != GQMAP_OK) return s;
        GQ_HIP(hipGraphUpload(c->sub[k], c->stream));
    }
    GQ_HIP(hipStreamSynchronize(c->stream));
    return GQMAP_OK;
}

// Not in the public header (tests, no device needed): the launch geometry of
// column-strip tile `tile` of n_tiles over a Mo x No frame -- out = {nblocks
// (the whole local tile grid), iteration_blocks (the workgroups of one RCCL
// iteration: the strip's launch), tiles_m, tiles_n, kernel shape}.
int gqmap_debug_strip_launch(const gqmap_options *opt, int Mo, int No, int n_tiles, int tile, int out[5])
{
    if (!opt || !out || n_tiles < 1 || tile < 0 || tile >= n_tiles) return GQMAP_ERR_INVALID_ARG;
    gqmap_ctx c;
    c.opt = *opt;
    c.super_ = opt->engine == GQMAP_ENGINE_SUPER;
    c.L = opt->L;
    c.n_tiles = n_tiles;
    c.tile = tile;
    strip_geometry(&c, Mo, No);
    tile_grid(&c);
    out[0] = c.nblocks;
    out[1] = iteration_blocks(&c);
    out[2] = c.tiles_m;
    out[3] = c.tiles_n;
    out[4] = c.kq;
    return GQMAP_OK;
}

// Not in the public header (tests): barrier j of the context's next
// persistent launch fails as a timed-out one does (j < 0: clears).
gqmap_status gqmap_debug_persist_fault(gqmap_ctx *c, int j)
{
    clear_error();
    GQ_CHECK(c, GQMAP_ERR_INVALID_ARG, "null context");
    DeviceGuard dg(c->device);
    const unsigned v = j < 0 ? 0u : (unsigned)(j + 1);
    GQ_HIP(hipMemcpyAsync(c->d_bar + BAR_INJECT, &v, sizeof(v), hipMemcpyHostToDevice, c->stream));
    GQ_HIP(hipStreamSynchronize(c->stream));
    return GQMAP_OK;
}

// Not in the public header (tests): 1 when the context has fallen back from
// the persistent launch to one launch per iteration.
int gqmap_debug_persist_off(const gqmap_ctx *c) { return c && c->persist_off ? 1 : 0; }

// Not in the public header (diagnostic builds with GQ_FLOW_TL): the flow
// timeline words (item (j, tile) at 4 (j * tiles + tile)); returns the
// words copied, or -1 in a build without it.
int gqmap_debug_flow_timeline(unsigned long long *out, int n)
{
#if GQ_FLOW_TL
    n = std::min(n, FLOW_TL_WORDS);
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_flow_tl), sizeof(unsigned long long) * n) != hipSuccess) return -1;
    return n;
#else
    (void)out;
    (void)n;
    return -1;
#endif
}

// Not in the public header (bench, tests): 1 when the context's runs take
// the dataflow launch (k_iter_flow) -- allocates its queue buffer if needed.
int gqmap_debug_flow(gqmap_ctx *c)
{
    if (!c || !c->have_images) return 0;
    DeviceGuard dg(c->device);
    return launch_flow(c, 1, true) ? 1 : 0;
}

// Not in the public header (tests, A/B scripts): set one execution policy of
// gq::Policy by name, process-wide; contexts created (or graphs captured)
// afterwards use it.  value -1 restores the automatic choice where there is
// one.  Returns 0, or -1 for an unknown name.
int gqmap_debug_policy(const char *name, int value)
{
    if (!name) return -1;
    struct Field { const char *n; int *p; int dflt; };
    const Field fields[] = {
        {"nt_state", &g_pol.nt_state, -1},   {"band_rows", &g_pol.band_rows, -1},
        {"cu_group", &g_pol.cu_group, -1},   {"lpar", &g_pol.lpar, -1},
        {"lpar_xcd", &g_pol.lpar_xcd, 1},    {"fused_finalize", &g_pol.fused_finalize, 1},
        {"persist", &g_pol.persist, 1},      {"persist_cap", &g_pol.persist_cap, -1},
        {"graph", &g_pol.graph, 1},          {"vv_float", &g_pol.vv_float, 1}, {"vv_pair", &g_pol.vv_pair, 1},
        {"verbose", &g_pol.verbose, 0},      {"flow", &g_pol.flow, -1},
    };
    for (const Field &f : fields)
        if (std::strcmp(f.n, name) == 0) {
            *f.p = value == -1 ? f.dflt : value;
            return 0;
        }
    return -1;
}

gqmap_status gqmap_get_info(gqmap_ctx *c, gqmap_info *info)
{
    clear_error();
    GQ_CHECK(c && info, GQMAP_ERR_INVALID_ARG, "null argument");
    DeviceGuard dg(c->device);
    std::memset(info, 0, sizeof(*info));
    info->Mo = c->Mo; info->No = c->No; info->M = c->M; info->N = c->have_images ? c->Ng : 0;
    info->L = c->L; info->K = c->K; info->device = c->device; info->split = c->split;
    info->n_tiles = c->n_tiles; info->tile = c->tile; info->col0 = c->col0; info->col1 = c->col1;
    if (c->have_state) {
        Ctl h;
        gqmap_status s = read_ctl(c, &h);
        if (s != GQMAP_OK) return s;
        info->it = h.it;
        info->stopped = h.stop;
        info->T = h.T;
    }
    return GQMAP_OK;
}

gqmap_status gqmap_get_map(gqmap_ctx *c, double *map)
{
    clear_error();
    GQ_CHECK(c && map, GQMAP_ERR_INVALID_ARG, "null argument");
    GQ_CHECK(c->have_state, GQMAP_ERR_STATE, "no state");
    DeviceGuard dg(c->device);
    Ctl h;
    gqmap_status s = read_ctl(c, &h);
    if (s != GQMAP_OK) return s;
    const void *cur = c->d_st[h.done & 1];
    const size_t MN = (size_t)c->M * c->N;
    std::vector<double> loc(2 * MN);
    if (c->L == 1) {  // map = cat(3, mu_u, mu_v)  (gqmap_gpu_mixture.m:55)
        if ((s = download(c, loc.data(), cur, MN)) != GQMAP_OK) return s;
        if ((s = download(c, loc.data() + MN, (const char *)cur + (size_t)c->MNL * c->rsz, MN)) != GQMAP_OK)
            return s;
    } else {
        double *d_out = nullptr;
        GQ_HIP(hipMalloc(&d_out, sizeof(double) * 2 * MN));
        hipError_t e = mixture_map_device(h.alpha, cur, c->fp32, c->MNL, c->M, c->N, c->L, d_out, c->stream);
        if (e == hipSuccess)
            e = hipMemcpyAsync(loc.data(), d_out, sizeof(double) * 2 * MN, hipMemcpyDeviceToHost, c->stream);
        if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
        (void)hipFree(d_out);
        GQ_HIP(e);
    }
    // full-grid M x Ng x 2 output: a tile writes its owned columns
    const size_t MNg = (size_t)c->M * c->Ng, own = (size_t)c->M * (c->own_hi - c->own_lo);
    for (int k = 0; k < 2; ++k)
        std::memcpy(map + k * MNg + (size_t)c->col0 * c->M, loc.data() + k * MN + (size_t)c->own_lo * c->M,
                    sizeof(double) * own);
    return GQMAP_OK;
}

gqmap_status gqmap_log_p(gqmap_ctx *c, const double *map, double *logp)
{
    clear_error();
    GQ_CHECK(c && map && logp, GQMAP_ERR_INVALID_ARG, "null argument");
    GQ_CHECK(c->have_images, GQMAP_ERR_STATE, "no images");
    GQ_CHECK(c->n_tiles == 1, GQMAP_ERR_UNSUPPORTED, "gqmap_log_p on a tile: evaluate on the whole grid");
    DeviceGuard dg(c->device);
    const size_t MN = (size_t)c->M * c->N;
    const int blocks = (int)((MN + 255) / 256);
    void *d_map = nullptr;
    double *d_part = nullptr;
    GQ_HIP(hipMalloc(&d_map, 2 * MN * c->rsz));
    GQ_HIP(hipMalloc(&d_part, sizeof(double) * blocks));
    gqmap_status s = upload(c, d_map, map, 2 * MN);
    if (s == GQMAP_OK) {
        if (c->fp32) {
            if (c->super_) k_logp<float, float, true><<<blocks, 256, 0, c->stream>>>(iter_params<float, float>(c), (const float *)d_map, d_part);
            else if (c->vvp) k_logp<float, vvh2_t, false><<<blocks, 256, 0, c->stream>>>(iter_params<float, vvh2_t>(c), (const float *)d_map, d_part);
            else k_logp<float, float, false><<<blocks, 256, 0, c->stream>>>(iter_params<float, float>(c), (const float *)d_map, d_part);
        } else if (c->vvp) {
            k_logp<double, vvh2_t, false><<<blocks, 256, 0, c->stream>>>(iter_params<double, vvh2_t>(c), (const double *)d_map, d_part);
        } else if (c->vv32) {
            if (c->super_) k_logp<double, vvs_t, true><<<blocks, 256, 0, c->stream>>>(iter_params<double, vvs_t>(c), (const double *)d_map, d_part);
            else k_logp<double, vvs_t, false><<<blocks, 256, 0, c->stream>>>(iter_params<double, vvs_t>(c), (const double *)d_map, d_part);
        } else {
            if (c->super_) k_logp<double, double, true><<<blocks, 256, 0, c->stream>>>(iter_params<double, double>(c), (const double *)d_map, d_part);
            else k_logp<double, double, false><<<blocks, 256, 0, c->stream>>>(iter_params<double, double>(c), (const double *)d_map, d_part);
        }
        std::vector<double> part(blocks);
        hipError_t e = hipGetLastError();
        if (e == hipSuccess)
            e = hipMemcpyAsync(part.data(), d_part, sizeof(double) * blocks, hipMemcpyDeviceToHost, c->stream);
        if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
        if (e != hipSuccess) {
            set_error("gqmap_log_p: %s", hipGetErrorString(e));
            s = GQMAP_ERR_HIP;
        }
        double v = 0;
        for (double x : part) v += x;
        *logp = v;
    }
    (void)hipFree(d_map);
    (void)hipFree(d_part);
    return s;
}

// Not in the public header: device math self-test used by tests/ (fn 0 sqrt,
// 1 log, 2 exp) to pin the device primitives against the host ones.
int gqmap_selftest_math(int fn, const double *in, double *out, int64_t n)
{
    double *d = nullptr;
    if (hipMalloc(&d, sizeof(double) * 2 * n) != hipSuccess) return GQMAP_ERR_HIP;
    hipError_t e = hipMemcpy(d, in, sizeof(double) * n, hipMemcpyHostToDevice);
    if (e == hipSuccess) {
        k_selftest<<<(int)((n + 255) / 256), 256>>>(fn, d, d + n, n);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipMemcpy(out, d + n, sizeof(double) * n, hipMemcpyDeviceToHost);
    (void)hipFree(d);
    return e == hipSuccess ? GQMAP_OK : GQMAP_ERR_HIP;
}

// Not in the public header: the padded frame VV (getVV, gqmap_gpu_mixture.m:
// 191-208) as the kernels will read it, widened to double; *stored_f32 = 1
// when it is held in float.  Tests pin that VV == getVV(I2) after
// gqmap_set_images / ctx_set_images_device (the round-2 upload race).
gqmap_status gqmap_debug_read_vv(gqmap_ctx *c, double *out, size_t n, int *stored_f32)
{
    clear_error();
    GQ_CHECK(c && out, GQMAP_ERR_INVALID_ARG, "null argument");
    GQ_CHECK(c->have_images, GQMAP_ERR_STATE, "no images");
    const size_t nvv = (size_t)(c->Mo + 2) * (c->No + 2);
    GQ_CHECK(n >= nvv, GQMAP_ERR_INVALID_ARG, "buffer holds %zu of %zu values", n, nvv);
    DeviceGuard dg(c->device);
    const bool f32 = c->fp32 || c->vv32 || c->vvp;
    if (stored_f32) *stored_f32 = f32;
    if (c->vvp) {  // the low half of each column pair
        std::vector<vvh2_t> raw(nvv);
        GQ_HIP(hipMemcpyAsync(raw.data(), c->d_VV, nvv * sizeof(vvh2_t), hipMemcpyDeviceToHost, c->stream));
        GQ_HIP(hipStreamSynchronize(c->stream));
        for (size_t k = 0; k < nvv; ++k) out[k] = (double)(float)raw[k].lo;
        return GQMAP_OK;
    }
    if (!f32) {
        GQ_HIP(hipMemcpyAsync(out, c->d_VV, nvv * sizeof(double), hipMemcpyDeviceToHost, c->stream));
        GQ_HIP(hipStreamSynchronize(c->stream));
        return GQMAP_OK;
    }
    const size_t esz = c->fp32 ? sizeof(float) : sizeof(vvs_t);
    std::vector<unsigned char> raw(nvv * esz);
    GQ_HIP(hipMemcpyAsync(raw.data(), c->d_VV, raw.size(), hipMemcpyDeviceToHost, c->stream));
    GQ_HIP(hipStreamSynchronize(c->stream));
    for (size_t k = 0; k < nvv; ++k) {
        if (c->fp32) out[k] = ((const float *)raw.data())[k];
        else out[k] = (double)((const vvs_t *)raw.data())[k];
    }
    return GQMAP_OK;
}

gqmap_status gqmap_synchronize(gqmap_ctx *c)
{
    clear_error();
    GQ_CHECK(c, GQMAP_ERR_INVALID_ARG, "null context");
    DeviceGuard dg(c->device);
    GQ_HIP(hipStreamSynchronize(c->stream));
    return GQMAP_OK;
}

gqmap_status gqmap_create_tile(gqmap_ctx **out, const gqmap_options *opt, int device, int n_tiles, int tile)
{
    clear_error();
    GQ_CHECK(n_tiles >= 1 && n_tiles <= 1024, GQMAP_ERR_INVALID_ARG, "n_tiles=%d outside [1,1024]", n_tiles);
    GQ_CHECK(tile >= 0 && tile < n_tiles, GQMAP_ERR_INVALID_ARG, "tile %d of %d", tile, n_tiles);
    gqmap_status s = gqmap_create(out, opt, device);
    if (s != GQMAP_OK) return s;
    (*out)->n_tiles = n_tiles;
    (*out)->tile = tile;
    return GQMAP_OK;
}

// A transport for a tile context: the per-tile totals table [n_tiles][NP].
static gqmap_status attach_common(gqmap_ctx *c)
{
    const size_t NP = NFIX + c->L;
    GQ_HIP(hipMalloc((void **)&c->d_gathered, sizeof(fix128) * NP * c->n_tiles));
    GQ_HIP(hipMemsetAsync(c->d_gathered, 0, sizeof(fix128) * NP * c->n_tiles, c->stream));
    GQ_HIP(hipStreamSynchronize(c->stream));
    c->own_gathered = true;
    c->nranks = c->n_tiles;
    drop_graph(c);
    return GQMAP_OK;
}

// The buffers of an RCCL tile (either communicator): the totals table, and
// for L = 1 the deferred-totals sequence's rows, gathered rows and snapshot.
// Allocated here, once, so that every rank runs the same collective
// sequence: a rank that cannot allocate them fails the attach instead of
// quietly taking the exact per-iteration step (whose collectives would not
// match its peers' sequences).
static gqmap_status attach_comm(gqmap_ctx *c)
{
    gqmap_status s = attach_common(c);
    if (s != GQMAP_OK) return s;
    if (c->L == 1) {  // deferred-totals sequences (launch_seq_deferred)
        const size_t NP = NFIX + c->L;
        GQ_HIP(hipMalloc((void **)&c->d_rows, sizeof(fix128) * NP * GRAPH_CHUNK));
        GQ_HIP(hipMalloc((void **)&c->d_seqg, sizeof(fix128) * NP * GRAPH_CHUNK * c->n_tiles));
        GQ_CHECK(ensure_snap(c), GQMAP_ERR_HIP, "tile %d: deferred-sequence snapshot (%zu bytes) not allocated",
                 c->tile, (size_t)c->MNL * NPLANES * c->rsz);
    }
    return GQMAP_OK;
}

gqmap_status gqmap_comm_unique_id(uint8_t id[128])
{
    clear_error();
    GQ_CHECK(id, GQMAP_ERR_INVALID_ARG, "null id");
    const Rccl *R = rccl();
    GQ_CHECK(R->ok, GQMAP_ERR_UNSUPPORTED, "librccl.so.1 not loadable: %s", dlerror());
    ncclUniqueId u;
    GQ_NCCL(R->GetUniqueId(&u));
    static_assert(sizeof(u) == 128, "ncclUniqueId size");
    std::memcpy(id, &u, 128);
    return GQMAP_OK;
}

gqmap_status gqmap_tile_attach_rccl(gqmap_ctx *c, const uint8_t id[128])
{
    clear_error();
    GQ_CHECK(c && id, GQMAP_ERR_INVALID_ARG, "null argument");
    GQ_CHECK(c->have_images, GQMAP_ERR_STATE, "attach after gqmap_set_images");
    GQ_CHECK(!c->comm && !c->in_group && !c->host_xfer, GQMAP_ERR_STATE, "tile already has a transport");
    const Rccl *R = rccl();
    GQ_CHECK(R->ok, GQMAP_ERR_UNSUPPORTED, "librccl.so.1 not loadable");
    DeviceGuard dg(c->device);
    ncclUniqueId u;
    std::memcpy(&u, id, 128);
    RcclComm *cm = new RcclComm();
    cm->nranks = c->n_tiles;
    cm->rank = c->tile;
    const ncclResult_t r = R->CommInitRank(&cm->comm, cm->nranks, u, cm->rank);
    if (r != ncclSuccess) {
        delete cm;
        set_error("ncclCommInitRank(%d ranks, rank %d): %s", c->n_tiles, c->tile, R->GetErrorString(r));
        return GQMAP_ERR_HIP;
    }
    c->comm = cm;
    return attach_comm(c);
}

// Not in the public header (tests): the loopback transport of n tile
// contexts in one process (LoopGroup) -- gqmap_debug_loop_create, then
// gqmap_debug_tile_attach_loop for tiles 0..n-1 (each tile then run from its
// own host thread, exactly as RCCL ranks), gqmap_debug_loop_destroy after
// every tile context is destroyed.  Returns the group or null.
void *gqmap_debug_loop_create(int n, int device)
{
    if (n < 1) return nullptr;
    DeviceGuard dg(device);
    LoopGroup *g = new LoopGroup();
    g->n = n;
    g->device = device;
    g->post.resize(n);
    g->ready.assign(n, nullptr);
    g->done.assign(n, nullptr);
    for (int i = 0; i < n; ++i)
        if (hipEventCreateWithFlags(&g->ready[i], hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&g->done[i], hipEventDisableTiming) != hipSuccess) {
            for (hipEvent_t e : g->ready) if (e) (void)hipEventDestroy(e);
            for (hipEvent_t e : g->done) if (e) (void)hipEventDestroy(e);
            delete g;
            return nullptr;
        }
    return g;
}

void gqmap_debug_loop_destroy(void *group)
{
    LoopGroup *g = (LoopGroup *)group;
    if (!g) return;
    DeviceGuard dg(g->device);
    for (hipEvent_t e : g->ready) if (e) (void)hipEventDestroy(e);
    for (hipEvent_t e : g->done) if (e) (void)hipEventDestroy(e);
    delete g;
}

// The collectives the group has completed (each counted once).
unsigned long long gqmap_debug_loop_calls(void *group) { return group ? ((LoopGroup *)group)->calls : 0; }

gqmap_status gqmap_debug_tile_attach_loop(gqmap_ctx *c, void *group)
{
    clear_error();
    LoopGroup *g = (LoopGroup *)group;
    GQ_CHECK(c && g, GQMAP_ERR_INVALID_ARG, "null argument");
    GQ_CHECK(c->have_images, GQMAP_ERR_STATE, "attach after gqmap_set_images");
    GQ_CHECK(!c->comm && !c->in_group && !c->host_xfer, GQMAP_ERR_STATE, "tile already has a transport");
    GQ_CHECK(g->n == c->n_tiles && c->device == g->device, GQMAP_ERR_INVALID_ARG,
             "loop group of %d ranks on device %d, tile %d of %d on device %d", g->n, g->device, c->tile, c->n_tiles,
             c->device);
    DeviceGuard dg(c->device);
    RcclComm *cm = new RcclComm();
    cm->nranks = c->n_tiles;
    cm->rank = c->tile;
    cm->loop = g;
    c->comm = cm;
    return attach_comm(c);
}

gqmap_status gqmap_tile_attach_host(gqmap_ctx *c)
{
    clear_error();
    GQ_CHECK(c, GQMAP_ERR_INVALID_ARG, "null context");
    GQ_CHECK(c->have_images, GQMAP_ERR_STATE, "attach after gqmap_set_images");
    GQ_CHECK(!c->comm && !c->in_group && !c->host_xfer, GQMAP_ERR_STATE, "tile already has a transport");
    DeviceGuard dg(c->device);
    gqmap_status s = attach_common(c);
    if (s != GQMAP_OK) return s;
    c->host_xfer = true;
    return GQMAP_OK;
}

gqmap_status gqmap_tile_exchange_sizes(gqmap_ctx *c, size_t sizes[6])
{
    clear_error();
    GQ_CHECK(c && sizes, GQMAP_ERR_INVALID_ARG, "null argument");
    GQ_CHECK(c->have_images, GQMAP_ERR_STATE, "sizes before gqmap_set_images");
    const size_t NPb = sizeof(fix128) * (NFIX + c->L);
    const bool left = c->tile > 0, right = c->tile < c->n_tiles - 1;
    sizes[0] = left ? halo_bytes(c, 0) : 0;
    sizes[1] = right ? halo_bytes(c, 1) : 0;
    sizes[2] = left ? halo_bytes(c, 2) : 0;
    sizes[3] = right ? halo_bytes(c, 3) : 0;
    sizes[4] = NPb;
    sizes[5] = NPb * c->n_tiles;
    return GQMAP_OK;
}

gqmap_status gqmap_tile_exchange_begin(gqmap_ctx *c, void *send_left, void *send_right, void *totals)
{
    clear_error();
    GQ_CHECK(c && totals, GQMAP_ERR_INVALID_ARG, "null argument");
    GQ_CHECK(c->host_xfer, GQMAP_ERR_STATE, "gqmap_tile_exchange_begin without gqmap_tile_attach_host");
    GQ_CHECK(c->have_state, GQMAP_ERR_STATE, "no state");
    GQ_CHECK((c->tile == 0 || send_left) && (c->tile == c->n_tiles - 1 || send_right), GQMAP_ERR_INVALID_ARG,
             "tile %d of %d: missing send buffer", c->tile, c->n_tiles);
    DeviceGuard dg(c->device);
    const int NP = NFIX + c->L;
    launch_iter(c);
    k_reduce_local<<<1, 256, 0, c->stream>>>(c->d_partials, c->nblocks, NP, c->d_gathered + (size_t)c->tile * NP,
                                             c->d_ctl);
    halo_pack(c, c->stream);
    GQ_HIP(hipGetLastError());
    if (c->tile > 0)
        GQ_HIP(hipMemcpyAsync(send_left, c->d_halo[0], halo_bytes(c, 0), hipMemcpyDeviceToHost, c->stream));
    if (c->tile < c->n_tiles - 1)
        GQ_HIP(hipMemcpyAsync(send_right, c->d_halo[1], halo_bytes(c, 1), hipMemcpyDeviceToHost, c->stream));
    GQ_HIP(hipMemcpyAsync(totals, c->d_gathered + (size_t)c->tile * NP, sizeof(fix128) * NP, hipMemcpyDeviceToHost,
                          c->stream));
    GQ_HIP(hipStreamSynchronize(c->stream));
    return GQMAP_OK;
}

gqmap_status gqmap_tile_exchange_end(gqmap_ctx *c, const void *recv_left, const void *recv_right,
                                     const void *totals_all, double *trace3)
{
    clear_error();
    GQ_CHECK(c && totals_all, GQMAP_ERR_INVALID_ARG, "null argument");
    GQ_CHECK(c->host_xfer, GQMAP_ERR_STATE, "gqmap_tile_exchange_end without gqmap_tile_attach_host");
    GQ_CHECK((c->tile == 0 || recv_left) && (c->tile == c->n_tiles - 1 || recv_right), GQMAP_ERR_INVALID_ARG,
             "tile %d of %d: missing receive buffer", c->tile, c->n_tiles);
    DeviceGuard dg(c->device);
    const int NP = NFIX + c->L;
    Ctl h0;
    gqmap_status s = read_ctl(c, &h0);
    if (s != GQMAP_OK) return s;
    if (c->tile > 0)
        GQ_HIP(hipMemcpyAsync(c->d_halo[2], recv_left, halo_bytes(c, 2), hipMemcpyHostToDevice, c->stream));
    if (c->tile < c->n_tiles - 1)
        GQ_HIP(hipMemcpyAsync(c->d_halo[3], recv_right, halo_bytes(c, 3), hipMemcpyHostToDevice, c->stream));
    GQ_HIP(hipMemcpyAsync(c->d_gathered, totals_all, sizeof(fix128) * NP * c->n_tiles, hipMemcpyHostToDevice,
                          c->stream));
    unpack_finalize(c);
    GQ_HIP(hipGetLastError());
    GQ_HIP(hipStreamSynchronize(c->stream));
    if (trace3) {
        for (int q = 0; q < 3; ++q) trace3[q] = __builtin_nan("");
        if (!h0.stop) {
            Ctl h;
            if ((s = read_ctl(c, &h)) != GQMAP_OK) return s;
            if (h.it > h0.it && (s = fetch_trace(c, h0.it, 1, trace3)) != GQMAP_OK) return s;
        }
    }
    return GQMAP_OK;
}

gqmap_status gqmap_tile_group_run(gqmap_ctx **tiles, int n, int n_iter, int *n_done, double *trace)
{
    clear_error();
    GQ_CHECK(tiles && n >= 1 && n_iter >= 0, GQMAP_ERR_INVALID_ARG, "gqmap_tile_group_run: bad arguments");
    gqmap_ctx *t0 = tiles[0];
    for (int t = 0; t < n; ++t) {
        gqmap_ctx *c = tiles[t];
        GQ_CHECK(c && c->n_tiles == n && c->tile == t, GQMAP_ERR_INVALID_ARG,
                 "tiles[%d] is not tile %d of %d", t, t, n);
        GQ_CHECK(c->device == t0->device && c->fp32 == t0->fp32 && c->L == t0->L && c->M == t0->M &&
                     c->Ng == t0->Ng,
                 GQMAP_ERR_INVALID_ARG, "tiles of one group must share device, precision and grid");
        GQ_CHECK(c->have_images && c->have_state && !c->comm && !c->host_xfer, GQMAP_ERR_STATE,
                 "tile %d: images/state missing or another transport attached", t);
    }
    DeviceGuard dg(t0->device);
    const int NP = NFIX + t0->L;
    if (!t0->in_group) {  // shared totals table owned by tile 0
        GQ_HIP(hipMalloc((void **)&t0->d_gathered, sizeof(fix128) * NP * n));
        t0->own_gathered = true;
        for (int t = 0; t < n; ++t) {
            tiles[t]->d_gathered = t0->d_gathered;
            tiles[t]->nranks = n;
            tiles[t]->in_group = true;
        }
    }
    // every launch of the group goes to tile 0's stream (restored below)
    std::vector<hipStream_t> saved(n);
    for (int t = 0; t < n; ++t) {
        saved[t] = tiles[t]->stream;
        tiles[t]->stream = t0->stream;
    }
    Ctl h0;
    gqmap_status s = read_ctl(t0, &h0);
    // The device trace is a ring of TRACE_CAP iterations: copy out what ran
    // since the last drain at every stop check (every 64 iterations) and at the end.
    int fetched = 0;
    auto drain = [&](const Ctl &h) -> gqmap_status {
        const int ran = h.it - h0.it;
        const gqmap_status r = fetch_trace(t0, h0.it + fetched, ran - fetched, trace ? trace + 3 * (size_t)fetched : nullptr);
        fetched = ran;
        return r;
    };
    for (int i = 0; i < n_iter && s == GQMAP_OK; ++i) {
        for (int t = 0; t < n; ++t) launch_iter(tiles[t]);
        for (int t = 0; t < n; ++t) {
            gqmap_ctx *c = tiles[t];
            k_reduce_local<<<1, 256, 0, c->stream>>>(c->d_partials, c->nblocks, NP, c->d_gathered + (size_t)t * NP,
                                                     c->d_ctl);
            halo_pack(c, c->stream);
        }
        for (int t = 0; t < n && s == GQMAP_OK; ++t) {
            if (t < n - 1 && hipMemcpyAsync(tiles[t + 1]->d_halo[2], tiles[t]->d_halo[1], halo_bytes(t0, 1),
                                            hipMemcpyDeviceToDevice, t0->stream) != hipSuccess)
                s = GQMAP_ERR_HIP;
            if (t > 0 && hipMemcpyAsync(tiles[t - 1]->d_halo[3], tiles[t]->d_halo[0], halo_bytes(t0, 0),
                                        hipMemcpyDeviceToDevice, t0->stream) != hipSuccess)
                s = GQMAP_ERR_HIP;
        }
        for (int t = 0; t < n; ++t) unpack_finalize(tiles[t]);
        if (hipGetLastError() != hipSuccess) s = GQMAP_ERR_HIP;
        if (i % 64 == 63 && s == GQMAP_OK) {  // stop test, bounded queue depth, trace drain
            Ctl h;
            if ((s = read_ctl(t0, &h)) == GQMAP_OK) s = drain(h);
            if (s == GQMAP_OK && h.stop) break;
        }
    }
    if (s != GQMAP_OK && !gqmap_last_error()[0]) set_error("gqmap_tile_group_run: HIP launch failed");
    Ctl h;
    if (s == GQMAP_OK) s = read_ctl(t0, &h);
    if (s == GQMAP_OK) s = drain(h);
    for (int t = 0; t < n; ++t) tiles[t]->stream = saved[t];
    if (s != GQMAP_OK) return s;
    if (n_done) *n_done = h.it - h0.it;
    return GQMAP_OK;
}

void gqmap_destroy(gqmap_ctx *c)
{
    if (!c) return;
    DeviceGuard dg(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    drop_graph(c);
    if (c->comm) {
        if (c->comm->comm) (void)rccl()->CommDestroy(c->comm->comm);
        delete c->comm;
    }
    for (void *p : {(void *)c->d_rows, (void *)c->d_seqg})
        if (p) (void)hipFree(p);
    if (c->own_gathered && c->d_gathered) (void)hipFree(c->d_gathered);
    for (void *p : c->d_halo)
        if (p) (void)hipFree(p);
    void *bufs[] = {c->d_VV, c->d_I1, c->d_st[0], c->d_st[1], c->d_tab, c->d_ctl, (void *)c->d_partials, c->d_trace,
                    c->d_truth, (void *)c->d_bar, c->d_snap, (void *)c->d_snap_ctl, (void *)c->d_flow};
    for (void *p : bufs)
        if (p) (void)hipFree(p);
    for (void *p : {(void *)c->h_ctl, (void *)c->h_ring, (void *)c->h_fail})
        if (p) (void)hipHostFree(p);
    if (c->stream && c->own_stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

}  // extern "C"
