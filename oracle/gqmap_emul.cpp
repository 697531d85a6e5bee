// gqmap_emul.cpp -- CPU model of the HIP iteration (TEST INFRASTRUCTURE).
//
// Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use
// this library.  It evaluates one QGMAP iteration exactly as libgqmap.so's
// kernels define it -- per-element arithmetic from the shared specification
// header gqmap-opticalflow_amd/csrc/gqmap_math.h, exact fixed-point sums,
// the same finalize step -- but with plain loops over the node grid instead
// of tiles, LDS halos, ping-pong buffers, XCD remapping and graphs.  Its
// output must therefore be bit-identical to the GPU's for any number of
// iterations; that checks everything the kernel does around the arithmetic.
// The arithmetic itself is checked against the literal restatement of the
// MATLAB (gqmap_oracle.c) one step at a time.
//
// It is also the CPU baseline: the same algorithm as the GPU kernel, OpenMP
// over columns.
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>
#ifdef _OPENMP
#include <omp.h>
#endif

#include "gqmap_oracle.h"

namespace gq {
using std::floor;
using std::fma;
using std::fmax;
using std::fmin;
}  // namespace gq
#define GQ_HD inline
#define GQ_SQRT(x) std::sqrt(x)
#define GQ_UNROLL2
#define GQ_PAIR_UNROLL
#define GQ_PAIR_UNROLL_K(n)
#define GQ_NODE_UNROLL
#define GQ_UNROLL_FULL
#include "../gqmap-opticalflow_amd/csrc/gqmap_math.h"

using namespace gq;

namespace {

constexpr int NFIX = 4;
constexpr int LMAX = 8;  // GQMAP_LMAX

template <typename R>
struct Work {
    const orc_params *P;
    int M, N, L, K2, Mo, No, M2;
    int64_t MN, MNL;
    std::vector<R> tab, VV, I1;
    std::vector<R> st, nst;                  // 9 planes of MNL
    std::vector<Grad<R>> node, edge;         // node [MNL], edge [MNL*4] (e = dir + 2*uv)
};

// Column-strip tile geometry (gqmap_create_tile): local column n is global
// column n + n_off of Ng; only [own_lo, own_hi) is updated.  Whole grid:
// n_off = 0, [0, N), Ng = N.
struct Geo {
    int n_off, own_lo, own_hi, Ng;
    bool upd(int m, int n, int M) const
    {
        return m >= 1 && m <= M - 2 && n >= own_lo && n < own_hi && n + n_off >= 1 && n + n_off <= Ng - 2;
    }
};
inline bool finite_d(double x) { return std::isfinite(x); }

// one term's quadrature sum split over Q lanes (k = j, j+Q, ...) + butterfly
template <typename F>
auto split_sums(int Q, F part) -> decltype(part(0, 1))
{
    if (Q == 1) return part(0, 1);
    decltype(part(0, 1)) parts[64];
    for (int j = 0; j < Q; ++j) parts[j] = part(j, Q);
    return butterfly(parts, Q);
}

// LIT: the literal-order arithmetic of gqmap_math.h (lit_*; fp64 mixture, Q = 1)
template <typename R, int ENG, bool LIT = false>
int run_t(const orc_params *P, const double *X, const double *W, const double *I1,
          const double *VV, orc_state *S, double *T_io, int it_first, int n_iter, double *trace,
          int Q, const Geo &G, int64_t *totals_out)
{
    Work<R> w;
    w.P = P;
    w.M = P->M; w.N = P->N; w.L = P->L; w.K2 = P->K * P->K;
    w.Mo = P->Mo; w.No = P->No; w.M2 = P->Mo + 2;
    w.MN = (int64_t)w.M * w.N;
    w.MNL = w.MN * w.L;
    const int M = w.M, N = w.N, L = w.L;
    const int64_t MN = w.MN, MNL = w.MNL;
    // quadrature tables exactly as gqmap_create builds them
    std::vector<double> tabd(NTAB * TAB_STRIDE, 0.0);
    for (int cc = 0; cc < P->K; ++cc)
        for (int r = 0; r < P->K; ++r) {
            const int k = r + P->K * cc;
            const double xi = X[cc], xj = X[r], ww = W[cc] * W[r];
            if (LIT) {
                lit_table_point(&tabd[tab_at(0, k)], xi, xj, W[cc], W[r]);
                continue;
            }
            tabd[tab_at(T_XI, k)] = xi;
            tabd[tab_at(T_XJ, k)] = xj;
            tabd[tab_at(T_W, k)] = ww;
            tabd[tab_at(T_WXI, k)] = ww * xi;
            tabd[tab_at(T_WXJ, k)] = ww * xj;
            tabd[tab_at(T_WA, k)] = ww * (xi * xi + xj * xj);
            tabd[tab_at(T_WM, k)] = ww * (xi * xi - xj * xj);
            tabd[tab_at(T_WX, k)] = ww * (xi * xj);
        }
    w.tab.assign(tabd.begin(), tabd.end());
    const size_t nvv = (size_t)(w.Mo + 2) * (w.No + 2), ni = (size_t)w.Mo * w.No;
    w.VV.assign(VV, VV + nvv);
    w.VV.resize(vv_elems(w.Mo, w.No), R(0));  // zero tail (axis_cell_abs)
    w.I1.assign(I1, I1 + ni);
    double *planes_in[9] = {S->muu, S->muv, S->sigu, S->sigv, S->pn, S->rou, S->rou + MNL,
                            S->rou + 2 * MNL, S->rou + 3 * MNL};
    w.st.resize((size_t)MNL * 9);
    for (int q = 0; q < 9; ++q)
        for (int64_t i = 0; i < MNL; ++i) w.st[q * MNL + i] = R(planes_in[q][i]);
    w.nst = w.st;
    w.node.assign(MNL, Grad<R>{});
    w.edge.assign(MNL * 4, Grad<R>{});

    const R eps = R(P->epsn), lamd = R(P->lambdad), lams = R(P->lambdas);
    const R minu = R(P->minu), maxu = R(P->maxu), minv = R(P->minv), maxv = R(P->maxv);
    const R sig_lo = R(P->sig_lo), sig_hi = R(P->sig_hi), corr = R(P->corr_tor);
    const R sig_step = R(P->sig_step);
    const bool guard = P->guard_a != 0;
    const R *tab = w.tab.data();
    const R *VVp = w.VV.data();
    const R *I1p = w.I1.data();
    double T = *T_io;
    int done = 0;
    for (int it = it_first; it < it_first + n_iter; ++it) {
        const R Tr = R(T);
        const R step = R(P->step0 / (1.0 + it / P->step_decay));
        const R *st = w.st.data();
        // 1. node and edge gradients (as the kernel decides which are needed)
#pragma omp parallel for schedule(dynamic, 1)
        for (int n = 0; n < N; ++n)
            for (int l = 0; l < L; ++l) {
                const R a = R(S->alpha[l]);
                for (int m = 0; m < M; ++m) {
                    const int64_t i = m + (int64_t)M * n + MN * l;
                    const bool inner = G.upd(m, n, M);
                    if (inner && LIT) {
                        if constexpr (LIT)
                            w.node[i] = lit_node_grad(tab, w.K2, VVp, w.M2, I1p, w.Mo, w.No, eps, lamd, guard, Tr, a,
                                                      st[i], st[i + MNL], st[i + 2 * MNL], st[i + 3 * MNL],
                                                      st[i + 4 * MNL], m, n + G.n_off);
                    } else if (inner) {
                        const NodeCoef<R> c = node_coef(st[i + 2 * MNL], st[i + 3 * MNL], st[i + 4 * MNL]);
                        const Sums<R> Sn = split_sums(Q, [&](int k0, int dk) {
                            return node_sums<ENG>(tab, k0, w.K2, dk, frame_view(VVp, w.M2), I1p, w.Mo, w.No, eps,
                                                  c, st[i], st[i + MNL], m, n + G.n_off);
                        });
                        w.node[i] = node_epi(Sn, c, lamd, guard, Tr, a, st[i + 2 * MNL],
                                             st[i + 3 * MNL], st[i + 4 * MNL], ENG == 2);
                    }
                    for (int e = 0; e < 4; ++e) {
                        const int dir = e & 1, uv = e >> 1;
                        const int rm = dir == 0 ? m + 1 : m, rn = dir == 1 ? n + 1 : n;
                        const bool r_inner = rm < M && rn < N && G.upd(rm, rn, M);
                        Grad<R> g{};
                        if (inner || r_inner) {
                            const int64_t r = rm + (int64_t)M * rn + MN * l;
                            const R o1 = st[i + MNL * (2 + uv)], o2 = st[r + MNL * (2 + uv)];
                            const R p = st[i + MNL * (5 + e)];
                            if constexpr (LIT) {
                                w.edge[i * 4 + e] = lit_edge_grad(tab, w.K2, eps, lams, guard, Tr, a, st[i + MNL * uv],
                                                                  st[r + MNL * uv], o1, o2, p);
                                continue;
                            }
                            const EdgeCoef<R> c = edge_coef(st[i + MNL * uv], st[r + MNL * uv], o1, o2, p);
                            // Q = 64 (one wave per node): the edges run on 16-lane groups
                            const Sums<R> Se = split_sums(edge_parts(Q), [&](int k0, int dk) {
                                return edge_sums(tab, k0, w.K2, dk, eps, c);
                            });
                            g = edge_epi(Se, c, lams, guard, Tr, a, o1, o2, p, ENG == 2);
                        }
                        w.edge[i * 4 + e] = g;
                    }
                }
            }
        // 2. gradient assembly, clamped ascent, exact sums
        fix128 fE = 0, fmu = 0, fsg = 0, fnf = 0, fda[LMAX] = {0};
#pragma omp parallel
        {
            fix128 lE = 0, lmu = 0, lsg = 0, lnf = 0, lda[LMAX] = {0};
#pragma omp for schedule(static)
            for (int n = 0; n < N; ++n)
                for (int l = 0; l < L; ++l)
                    for (int m = 1; m < M - 1; ++m) {
                        if (!G.upd(m, n, M)) continue;
                        const int64_t i = m + (int64_t)M * n + MN * l;
                        const int64_t iu = i - 1, il = i - M;  // (m-1,n), (m,n-1)
                        const Grad<R> &nd = w.node[i];
                        const Grad<R> *ed = &w.edge[i * 4];
                        R sum_mu0 = 0, sum_mu1 = 0, sum_sg0 = 0, sum_sg1 = 0, eE = 0, eda = 0;
                        for (int e = 0; e < 4; ++e) {
                            if ((e >> 1) == 0) { sum_mu0 = sum_mu0 + ed[e].du1; sum_sg0 = sum_sg0 + ed[e].do1; }
                            else               { sum_mu1 = sum_mu1 + ed[e].du1; sum_sg1 = sum_sg1 + ed[e].do1; }
                            eE = eE + ed[e].E;
                            eda = eda + ed[e].da;
                        }
                        const Grad<R> &up_u = w.edge[iu * 4 + 0], &up_v = w.edge[iu * 4 + 2];
                        const Grad<R> &lf_u = w.edge[il * 4 + 1], &lf_v = w.edge[il * 4 + 3];
                        const R gmu_u = ((nd.du1 + sum_mu0) + up_u.du2) + lf_u.du2;
                        const R gmu_v = ((nd.du2 + sum_mu1) + up_v.du2) + lf_v.du2;
                        const R gsg_u = ((nd.do1 + sum_sg0) + up_u.do2) + lf_u.do2;
                        const R gsg_v = ((nd.do2 + sum_sg1) + up_v.do2) + lf_v.do2;
                        auto cl = [](R x, R lo, R hi) { return fmin(fmax(x, lo), hi); };
                        R *ns = w.nst.data();
                        ns[i + MNL * 0] = cl(st[i] + gmu_u * step, minu, maxu);
                        ns[i + MNL * 1] = cl(st[i + MNL] + gmu_v * step, minv, maxv);
                        const R su = ENG == 2 ? (gsg_u * step) * sig_step : gsg_u * step;
                        const R sv = ENG == 2 ? (gsg_v * step) * sig_step : gsg_v * step;
                        ns[i + MNL * 2] = cl(st[i + 2 * MNL] + su, sig_lo, sig_hi);
                        ns[i + MNL * 3] = cl(st[i + 3 * MNL] + sv, sig_lo, sig_hi);
                        ns[i + MNL * 4] = cl(st[i + 4 * MNL] + nd.dp * step, -corr, corr);
                        for (int e = 0; e < 4; ++e)
                            ns[i + MNL * (5 + e)] = cl(st[i + MNL * (5 + e)] + ed[e].dp * step, -corr, corr);
                        const double cE = (double)nd.E + (double)eE, cda = (double)nd.da + (double)eda;
                        const double cmu = std::fabs((double)gmu_u), csg = std::fabs((double)gsg_u);
                        lnf += !finite_d(cE) + !finite_d(cda) + !finite_d(cmu) + !finite_d(csg);
                        lE += to_fix(cE);
                        lda[l] += to_fix(cda);
                        lmu += to_fix(cmu);
                        lsg += to_fix(csg);
                    }
#pragma omp critical
            {
                fE += lE; fmu += lmu; fsg += lsg; fnf += lnf;
                for (int l = 0; l < L; ++l) fda[l] += lda[l];
            }
        }
        std::swap(w.st, w.nst);
        // border nodes keep their values in both buffers
        w.nst = w.st;
        if (totals_out) {  // this tile's exact totals, fix128 as (lo, hi) int64 pairs
            const fix128 v[NFIX] = {fE, fmu, fsg, fnf};
            for (int q = 0; q < NFIX + L; ++q) {
                const fix128 x = q < NFIX ? v[q] : fda[q - NFIX];
                totals_out[2 * q] = (int64_t)(uint64_t)x;
                totals_out[2 * q + 1] = (int64_t)(x >> 64);
            }
        }
        // 3. finalize (k_finalize)
        double tot[NFIX + LMAX];
        tot[0] = from_fix(fE); tot[1] = from_fix(fmu); tot[2] = from_fix(fsg); tot[3] = from_fix(fnf);
        for (int l = 0; l < L; ++l) tot[NFIX + l] = from_fix(fda[l]);
        const double count = (double)(M - 2) * (double)(G.Ng - 2) * L;
        const double step_d = P->step0 / (1.0 + it / P->step_decay);
        const bool bad = tot[3] != 0.0;
        const double nan = std::nan("");
        const double energy = bad ? nan : tot[0];
        const double ptdmu = bad ? nan : tot[1] / count, ptdsig = bad ? nan : tot[2] / count;
        if (it > P->alpha_start && L != 1) {
            double dal[LMAX];
            for (int l = 0; l < L; ++l) dal[l] = bad ? nan : tot[NFIX + l];
            if (P->alpha_mode == 0) {
                double sda = 0;
                for (int l = 0; l < L; ++l) sda = sda + dal[l] * S->alpha[l];
                double se = 0, ew[LMAX];
                for (int l = 0; l < L; ++l) {
                    const double dw = S->alpha[l] * (dal[l] - sda);
                    S->w[l] = fmin(fmax(S->w[l] + dw * step_d * P->alpha_lr, -300.0), 300.0);
                    ew[l] = gq_exp(S->w[l]);
                    se = se + ew[l];
                }
                for (int l = 0; l < L; ++l) S->alpha[l] = ew[l] / se;
            } else {
                double y[LMAX], s[LMAX];
                for (int l = 0; l < L; ++l) s[l] = y[l] = S->alpha[l] + dal[l] * step_d * P->alpha_lr;
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
                for (int l = 0; l < L; ++l) S->alpha[l] = fmax(y[l] - tmax, 0.0);
            }
        }
        trace[3 * done + 0] = energy;
        trace[3 * done + 1] = ptdmu;
        trace[3 * done + 2] = ptdsig;
        if (P->t_decay_every > 0 && it % P->t_decay_every == 0) T = fmax(T * P->drate, P->t_min);
        ++done;
        if (ptdmu < P->tor) break;
    }
    for (int q = 0; q < 9; ++q)
        for (int64_t i = 0; i < MNL; ++i) planes_in[q][i] = (double)w.st[q * MNL + i];
    *T_io = T;
    return done;
}

}  // namespace

template <typename R>
static int run_eng(const orc_params *P, const double *X, const double *W, const double *I1,
                   const double *VV, orc_state *S, double *T_io, int it_first, int n_iter, double *trace,
                   int Q, const Geo &G, int64_t *tot)
{
    if (P->ctf) return run_t<R, 2>(P, X, W, I1, VV, S, T_io, it_first, n_iter, trace, Q, G, tot);
    if (P->super_) return run_t<R, 1>(P, X, W, I1, VV, S, T_io, it_first, n_iter, trace, Q, G, tot);
    return run_t<R, 0>(P, X, W, I1, VV, S, T_io, it_first, n_iter, trace, Q, G, tot);
}

/* One tile of a column-strip decomposition: P->N is the LOCAL node-column
 * count (owned + ghosts), geo = {n_off, own_lo, own_hi, Ng}; the state is the
 * local grid.  totals (2*(NFIX+L) int64) receive the last iteration's exact
 * per-tile sums; the finalize inside uses the local sums (callers combine the
 * tiles' totals themselves). */
extern "C" int emu_run_tile(const orc_params *P, const double *X, const double *W, const double *I1,
                            const double *VV, orc_state *S, double *T_io, int it_first, int n_iter,
                            double *trace, int nthreads, int fp32, int split, const int *geo,
                            int64_t *totals)
{
    if (split != 1 && split != 2 && split != 4 && split != 8 && split != 16 && split != 64) return -2;
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#endif
    const Geo G{geo[0], geo[1], geo[2], geo[3]};
    return fp32 ? run_eng<float>(P, X, W, I1, VV, S, T_io, it_first, n_iter, trace, split, G, totals)
                : run_eng<double>(P, X, W, I1, VV, S, T_io, it_first, n_iter, trace, split, G, totals);
}

extern "C" int emu_run(const orc_params *P, const double *X, const double *W, const double *I1,
                       const double *VV, orc_state *S, double *T_io, int it_first, int n_iter,
                       double *trace, int nthreads, int fp32, int split)
{
    const int Q = split;
    if (Q != 1 && Q != 2 && Q != 4 && Q != 8 && Q != 16 && Q != 64) return -2;
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#endif
    const Geo G{0, 0, P->N, P->N};
    return fp32 ? run_eng<float>(P, X, W, I1, VV, S, T_io, it_first, n_iter, trace, Q, G, nullptr)
                : run_eng<double>(P, X, W, I1, VV, S, T_io, it_first, n_iter, trace, Q, G, nullptr);
}

/* The literal-order arithmetic (gqmap_options.arith = GQMAP_ARITH_LITERAL):
 * fp64 single-scale mixture engine, one lane per node; geo as emu_run_tile
 * (NULL: the whole grid), totals may be NULL.  Returns -2 for another engine. */
extern "C" int emu_run_lit(const orc_params *P, const double *X, const double *W, const double *I1,
                           const double *VV, orc_state *S, double *T_io, int it_first, int n_iter,
                           double *trace, int nthreads, const int *geo, int64_t *totals)
{
    if (P->ctf || P->super_) return -2;
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#endif
    const Geo G = geo ? Geo{geo[0], geo[1], geo[2], geo[3]} : Geo{0, 0, P->N, P->N};
    return run_t<double, 0, true>(P, X, W, I1, VV, S, T_io, it_first, n_iter, trace, 1, G, totals);
}

extern "C" void emu_math(int fn, const double *in, double *out, int64_t n)
{
    for (int64_t i = 0; i < n; ++i)
        out[i] = fn == 0 ? std::sqrt(in[i]) : fn == 1 ? gq_log(in[i]) : fn == 2 ? gq_exp(in[i])
                                                                   : (double)std::sqrt((float)in[i]);
}

// the device's deterministic exp as a plain function (orc_set_map_exp)
extern "C" double emu_gq_exp(double x) { return gq_exp(x); }
extern "C" double emu_gq_log(double x) { return gq_log(x); }



// sample4_abs (fp64) / sample4 (fp32 relative form) at one position, for the
// cap identity test (tests/test_spec_identities.py): cap = 0 is the kernel's
// axis arithmetic (cell n at fraction 0 for X == n); cap = 1 the reference's
// interp2 cell choice (cell n-1 at fraction 1), same Keys fma chains.
template <typename R>
static R emu_sample_t(const std::vector<R> &V, int Mo, int No, double X, double Y, int cap)
{
    const int M2 = Mo + 2;
    if (!cap) {
        if (sizeof(R) == 8)
            return (R)sample4_abs<true>(V.data(), M2, Mo, No, X, Y);
        const int jj = (int)std::floor(X), ii = (int)std::floor(Y);
        return sample4<true>(V.data(), M2, Mo, No, ii, jj, (R)(X - jj), (R)(Y - ii));
    }
    auto axis = [](double P, int n, int &ix, R &fr) {
        P = std::fmin(std::fmax(P, 1.0), (double)n);
        ix = (int)P;
        if (ix > n - 1) ix = n - 1;
        fr = (R)(P - ix);
    };
    int ix, iy;
    R so, to;
    axis(X, No, ix, so);
    axis(Y, Mo, iy, to);
    return bicubic_cell4<R>(V.data(), cell_elem(iy, ix, M2), (uint32_t)M2, so, to);
}
extern "C" void emu_sample(const double *VV, int Mo, int No, const double *X, const double *Y, double *out,
                           int64_t n, int fp32, int cap)
{
    const size_t nvv = (size_t)(Mo + 2) * (No + 2);
    if (fp32) {
        std::vector<float> V(VV, VV + nvv);
        V.resize(vv_elems(Mo, No), 0.f);
        for (int64_t i = 0; i < n; ++i) out[i] = emu_sample_t<float>(V, Mo, No, X[i], Y[i], cap);
    } else {
        std::vector<double> V(VV, VV + nvv);
        V.resize(vv_elems(Mo, No), 0.0);
        for (int64_t i = 0; i < n; ++i) out[i] = emu_sample_t<double>(V, Mo, No, X[i], Y[i], cap);
    }
}
