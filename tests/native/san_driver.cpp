// san_driver.cpp -- AddressSanitizer / UndefinedBehaviorSanitizer run of the
// CPU code: the oracle (literal restatements, CPU kernel model, pyramid and
// legacy restatements) and the host side of the C ABI (gqmap_host.cpp:
// Gauss-Hermite, RNG, .flo I/O, AEPE, error strings).
// TEST INFRASTRUCTURE ("ASan/UBSan on the CPU oracle"); built by
// tests/native/Makefile, run by tests/test_sanitizers.py.  Exit 0 = clean;
// any sanitizer report aborts with a non-zero status.
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../../include/gqmap.h"
#include "../../oracle/gqmap_oracle.h"

extern "C" {
int emu_run(const orc_params *P, const double *X, const double *W, const double *I1, const double *VV,
            orc_state *S, double *T_io, int it_first, int n_iter, double *trace, int nthreads, int fp32, int split);
void emu_math(int fn, const double *in, double *out, int64_t n);
double emu_gq_exp(double x);
}

static int fails = 0;
#define CHECK(c)                                                            \
    do {                                                                    \
        if (!(c)) {                                                         \
            std::fprintf(stderr, "%s:%d check failed: %s\n", __FILE__, __LINE__, #c); \
            ++fails;                                                        \
        }                                                                   \
    } while (0)

static uint64_t rng_state = 88172645463325252ULL;
static double urand()
{
    rng_state ^= rng_state << 13; rng_state ^= rng_state >> 7; rng_state ^= rng_state << 17;
    return (double)(rng_state >> 11) * (1.0 / 9007199254740992.0);
}

struct Case {
    orc_params p{};
    std::vector<double> I1, I2, VV, st[8];
    orc_state s{};
};

static void make_case(Case &c, int engine, int Mo, int No, int L, int K)
{
    orc_params &p = c.p;
    p.Mo = Mo; p.No = No; p.L = L; p.K = K;
    p.super_ = engine == 1; p.ctf = engine == 2;
    p.M = p.super_ ? Mo / 4 : Mo; p.N = p.super_ ? No / 4 : No;
    p.guard_a = engine == 0; p.T = engine == 1 ? 0.2 : 0.05; p.drate = 0.75; p.t_min = 1e-3; p.t_decay_every = 2;
    p.epsn = 1e-6; p.lambdad = 1; p.lambdas = engine == 1 ? 16 : 5;
    p.minu = -3; p.maxu = 3; p.minv = -2; p.maxv = 2;
    p.step0 = engine == 2 ? 0.07 : 0.1; p.step_decay = engine == 2 ? 1e300 : 8000;
    p.sig_lo = 0.01; p.sig_hi = 23; p.corr_tor = 1 - 1e-5;
    p.alpha_mode = 0; p.alpha_start = 1; p.alpha_lr = 1e-4; p.tor = 1e-30; p.sig_step = engine == 2 ? 0.3 : 1;
    c.I1.resize((size_t)Mo * No); c.I2.resize((size_t)Mo * No);
    for (size_t i = 0; i < c.I1.size(); ++i) { c.I1[i] = std::floor(255 * urand()); c.I2[i] = std::floor(255 * urand()); }
    c.VV.resize((size_t)(Mo + 2) * (No + 2));
    orc_get_vv(c.I2.data(), Mo, No, c.VV.data());
    const size_t MNL = (size_t)p.M * p.N * L;
    const size_t sz[8] = {MNL, MNL, MNL, MNL, MNL, 4 * MNL, (size_t)L, (size_t)L};
    for (int k = 0; k < 8; ++k) c.st[k].assign(sz[k], 0.0);
    for (size_t i = 0; i < MNL; ++i) {
        c.st[0][i] = -3 + 6 * urand(); c.st[1][i] = -2 + 4 * urand();
        c.st[2][i] = 0.3 + 3 * urand(); c.st[3][i] = 0.3 + 3 * urand(); c.st[4][i] = 0.5 * (urand() - 0.5);
    }
    for (size_t i = 0; i < 4 * MNL; ++i) c.st[5][i] = 0.5 * (urand() - 0.5);
    double se = 0;
    for (int l = 0; l < L; ++l) { c.st[6][l] = urand(); se += std::exp(c.st[6][l]); }
    for (int l = 0; l < L; ++l) c.st[7][l] = std::exp(c.st[6][l]) / se;
    c.s.muu = c.st[0].data(); c.s.muv = c.st[1].data(); c.s.sigu = c.st[2].data(); c.s.sigv = c.st[3].data();
    c.s.pn = c.st[4].data(); c.s.rou = c.st[5].data(); c.s.w = c.st[6].data(); c.s.alpha = c.st[7].data();
}

static void engines()
{
    const int cfg[3][5] = {{0, 19, 23, 2, 7}, {1, 24, 28, 3, 5}, {2, 17, 21, 1, 7}};
    for (auto &g : cfg) {
        for (int model = 0; model < 2; ++model) {
            Case c;
            make_case(c, g[0], g[1], g[2], g[3], g[4]);
            std::vector<double> X(g[4]), W(g[4]), tr(3 * 4);
            orc_gauss_hermite(g[4], X.data(), W.data());
            double T = c.p.T;
            const int done = model == 0 ? orc_run(&c.p, c.I1.data(), c.VV.data(), &c.s, &T, 1, 4, tr.data(), 3)
                                        : emu_run(&c.p, X.data(), W.data(), c.I1.data(), c.VV.data(), &c.s, &T, 1, 4,
                                                  tr.data(), 3, 0, g[0] == 1 ? 4 : 1);
            CHECK(done == 4);
            for (double v : tr) CHECK(std::isfinite(v));
        }
    }
    Case c;
    make_case(c, 0, 13, 11, 2, 5);
    std::vector<double> node(7 * 13 * 11 * 2), edge(7 * 13 * 11 * 2 * 4);
    orc_gradients(&c.p, c.I1.data(), c.VV.data(), &c.s, 0.05, node.data(), edge.data(), 2);
    CHECK(orc_interp_cubic(c.VV.data(), 13, 11, 3.25, 4.5) == orc_interp_cubic(c.VV.data(), 13, 11, 3.25, 4.5));
}

static void plumbing()
{
    const int M = 37, N = 29;
    std::vector<double> A((size_t)M * N * 2), out;
    for (double &v : A) v = 255 * urand();
    for (double scale : {0.5, 0.25, 2.0, 4.0}) {
        const int oM = orc_resize_len(M, scale), oN = orc_resize_len(N, scale);
        CHECK(oM == (int)std::ceil(scale * M) && oN == (int)std::ceil(scale * N));
        out.assign((size_t)oM * oN * 2, 0.0);
        orc_imresize(A.data(), M, N, 2, scale, scale < 1, out.data());
    }
    std::vector<double> warp((size_t)M * N * 2), W((size_t)M * N);
    for (double &v : warp) v = 6 * (urand() - 0.5);
    orc_warp_image(A.data(), M, N, warp.data(), W.data());
    orc_fillmissing_nearest(W.data(), M, N, 1);
    orc_fillmissing_nearest(W.data(), M, N, 2);
    for (double v : W) CHECK(std::isfinite(v));

    std::vector<double> flow((size_t)M * N * 2), flo(flow.size()), stats(4);
    std::vector<unsigned char> img((size_t)M * N * 3), unk((size_t)M * N);
    for (size_t i = 0; i < flow.size(); ++i) flow[i] = i % 97 == 0 ? 2e9 : 8 * (urand() - 0.5);
    orc_flow_to_color(flow.data(), M, N, 0.0, img.data(), flo.data(), stats.data(), unk.data());
    const double e = orc_aepe(flo.data(), flow.data(), unk.data(), M, N, 1);
    CHECK(std::isfinite(e));

    const int L = 3;
    std::vector<double> mu((size_t)M * N * L), sg(mu.size()), map((size_t)M * N * 2);
    for (size_t i = 0; i < mu.size(); ++i) { mu[i] = 4 * (urand() - 0.5); sg[i] = 0.1 + urand(); }
    const double al[3] = {0.5, 0.3, 0.2};
    orc_get_map(al, mu.data(), sg.data(), mu.data(), sg.data(), M, N, L, map.data(), 2);
    orc_set_map_exp(emu_gq_exp);
    orc_get_map(al, mu.data(), sg.data(), mu.data(), sg.data(), M, N, L, map.data(), 2);
    orc_set_map_exp(nullptr);
    double y[5], x[5];
    for (double &v : y) v = urand() - 0.3;
    orc_projsplx(y, x, 5);
    double s = 0;
    for (double v : x) { CHECK(v >= 0); s += v; }
    CHECK(std::fabs(s - 1) < 1e-12);

    orc_cpu_params cp{};
    cp.its = 5; cp.K = 7; cp.var = 1; cp.gama = 1; cp.dta = 2.5; cp.step0 = 0.1; cp.step_decay = 1000;
    cp.corr_tor = 0.97; cp.tor = 1e-3; cp.min_its = 100;
    std::vector<double> X(7), Wt(7), mu2(flow.size()), sg2(flow.size()), rou((size_t)M * N * 4), tr(3 * 5);
    orc_gauss_hermite(7, X.data(), Wt.data());
    for (size_t i = 0; i < flow.size(); ++i) { flow[i] = 4 * (urand() - 0.5); mu2[i] = flow[i]; sg2[i] = 2 + urand(); }
    CHECK(orc_cpu_run(&cp, X.data(), Wt.data(), flow.data(), M, N, mu2.data(), sg2.data(), rou.data(), tr.data(), 3) == 5);

    std::vector<double> in(1000), o(1000);
    for (double &v : in) v = 1e-6 + 100 * urand();
    for (int fn = 0; fn < 4; ++fn) emu_math(fn, in.data(), o.data(), (int64_t)in.size());
}

static void host_abi()
{
    double x[16], w[16];
    CHECK(gqmap_gauss_hermite(9, x, w) == GQMAP_OK);
    CHECK(gqmap_gauss_hermite(0, x, w) != GQMAP_OK && gqmap_last_error()[0] != 0);
    std::vector<double> u(1000);
    gqmap_rand_uniform(7, 3, 12345, u.size(), u.data());
    for (double v : u) CHECK(v >= 0 && v < 1);
    const int M = 9, N = 13;
    std::vector<double> f((size_t)M * N * 2), g(f.size());
    for (double &v : f) v = (float)(10 * (urand() - 0.5));
    const char *path = "/tmp/gq_san_roundtrip.flo";
    CHECK(gqmap_write_flo(path, f.data(), M, N) == GQMAP_OK);
    int m = 0, n = 0;
    CHECK(gqmap_read_flo(path, &m, &n, nullptr) == GQMAP_OK && m == M && n == N);
    CHECK(gqmap_read_flo(path, &m, &n, g.data()) == GQMAP_OK);
    CHECK(std::memcmp(f.data(), g.data(), sizeof(double) * f.size()) == 0);
    std::remove(path);
    CHECK(gqmap_read_flo("/nonexistent/x.flo", &m, &n, nullptr) != GQMAP_OK);
    std::vector<uint8_t> unk((size_t)M * N, 0);
    double e = -1;
    CHECK(gqmap_aepe(f.data(), f.data(), unk.data(), M, N, 1, &e) == GQMAP_OK && e == 0.0);
}

int main()
{
    engines();
    plumbing();
    host_abi();
    if (fails) {
        std::fprintf(stderr, "%d checks failed\n", fails);
        return 1;
    }
    std::printf("sanitizer driver: clean\n");
    return 0;
}
