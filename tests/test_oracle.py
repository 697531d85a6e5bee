"""The C oracle (oracle/gqmap_oracle.c) against known answers and against
the independent numpy restatement's golden vectors (tests/golden)."""
import numpy as np
import pytest

from tests import _golden as G


def test_gauss_hermite_matches_numpy(oracle_lib):
    for K in (2, 3, 5, 9, 11, 16):
        x, w = oracle_lib.gauss_hermite(K)
        xr, wr = np.polynomial.hermite.hermgauss(K)
        assert np.max(np.abs(x - xr)) < 1e-13
        assert np.max(np.abs(w - wr)) < 1e-13


def test_gauss_hermite_numpy_restatement():
    from oracle import gqmap_np
    for K in (9, 11):
        x, w = gqmap_np.gauss_hermite(K)
        xr, wr = np.polynomial.hermite.hermgauss(K)
        assert np.max(np.abs(x - xr)) < 1e-13 and np.max(np.abs(w - wr)) < 1e-13


def test_getvv_and_cubic_reproduce_quadratics(oracle_lib):
    # Keys cubic convolution (a=-1/2) with 3f1-3f2+f3 padding reproduces
    # polynomials up to degree 2 exactly, boundary cells included.
    M, N = 12, 17
    m, n = np.meshgrid(np.arange(1, M + 1), np.arange(1, N + 1), indexing="ij")
    f = lambda y, x: 0.3 * x * x - 0.2 * x * y + 0.05 * y * y + 1.5 * x - 2 * y + 7
    I = np.asfortranarray(f(m, n).astype(np.float64))
    VV = oracle_lib.get_vv(I)
    rng = np.random.default_rng(0)
    for _ in range(200):
        X, Y = rng.uniform(1, N), rng.uniform(1, M)
        assert abs(oracle_lib.interp_cubic(VV, M, N, X, Y) - f(Y, X)) < 1e-9
    # integer positions return the samples exactly
    assert oracle_lib.interp_cubic(VV, M, N, 5.0, 3.0) == pytest.approx(I[2, 4], abs=1e-12)


def test_getvv_matches_numpy(oracle_lib):
    from oracle import gqmap_np
    I = np.asfortranarray(np.random.default_rng(1).random((9, 13)) * 255)
    assert np.array_equal(oracle_lib.get_vv(I), gqmap_np.get_vv(I))


@pytest.mark.parametrize("name", G.CASES)
def test_oracle_gradients_match_golden(oracle_lib, name):
    d = G.load(name)
    st = oracle_lib.State(*G.state(d).values())
    node, edge = oracle_lib.gradients(d["opts"], d["I1"], d["I2"], st, T=d["opts"]["temperature"])
    np.testing.assert_allclose(node, d["node0"], rtol=1e-11, atol=1e-9)
    np.testing.assert_allclose(edge, d["edge0"], rtol=1e-11, atol=1e-9)


@pytest.mark.parametrize("name", G.CASES)
def test_oracle_one_step_matches_golden(oracle_lib, name):
    d = G.load(name)
    st = oracle_lib.State(*G.state(d).values())
    done, trace, _ = oracle_lib.run(d["opts"], d["I1"], d["I2"], st, 1, 1)
    assert done == 1
    np.testing.assert_allclose(trace[0], d["trace"][0], rtol=1e-11)
    for k, a in zip(G.STATE_KEYS, st.arrays()):
        np.testing.assert_allclose(a, d["step1_" + k], rtol=1e-11, atol=1e-11, err_msg=k)


@pytest.mark.parametrize("name", G.CASES)
def test_oracle_iterations_match_golden(oracle_lib, name):
    # Multi-step tolerance: once pn/rou reach the +-(1-1e-5) clamp every
    # gradient carries a 1/(1-p^2) ~ 5e4 factor, so last-bit differences in
    # summation order (C loop vs numpy reductions) grow to ~1e-6 in 3-4 steps.
    d = G.load(name)
    st = oracle_lib.State(*G.state(d).values())
    its = d["trace"].shape[0]
    done, trace, T = oracle_lib.run(d["opts"], d["I1"], d["I2"], st, 1, its)
    assert done == its
    np.testing.assert_allclose(trace, d["trace"], rtol=1e-8)
    assert T == pytest.approx(float(d["T_final"]))
    for k, a in zip(G.STATE_KEYS, st.arrays()):
        np.testing.assert_allclose(a, d["final_" + k], rtol=1e-5, atol=1e-5, err_msg=k)


def test_oracle_chunked_run_equals_single_run(oracle_lib):
    d = G.load("mixture_L3_T")
    s1 = oracle_lib.State(*G.state(d).values())
    s2 = oracle_lib.State(*G.state(d).values())
    _, t1, _ = oracle_lib.run(d["opts"], d["I1"], d["I2"], s1, 1, 3)
    _, ta, T = oracle_lib.run(d["opts"], d["I1"], d["I2"], s2, 1, 1)
    _, tb, _ = oracle_lib.run(d["opts"], d["I1"], d["I2"], s2, 2, 2, T=T)
    np.testing.assert_array_equal(t1, np.vstack([ta, tb]))
    for a, b in zip(s1.arrays(), s2.arrays()):
        np.testing.assert_array_equal(a, b)


def test_projsplx_known_answers(oracle_lib):
    from oracle import gqmap_np
    assert np.allclose(oracle_lib.projsplx([0.2, 0.3, 0.5]), [0.2, 0.3, 0.5])
    assert np.allclose(oracle_lib.projsplx([1.0, 1.0, 1.0]), [1 / 3] * 3)
    assert np.allclose(oracle_lib.projsplx([2.0, 0.0, 0.0]), [1.0, 0.0, 0.0])
    rng = np.random.default_rng(3)
    for _ in range(100):
        y = rng.normal(size=rng.integers(1, 9))
        x = oracle_lib.projsplx(y)
        assert np.all(x >= 0) and abs(x.sum() - 1) < 1e-12
        np.testing.assert_array_equal(x, gqmap_np.projsplx(y))
        # idempotent on the simplex
        np.testing.assert_allclose(oracle_lib.projsplx(x), x, atol=1e-15)


def test_flow_to_color_matches_golden(oracle_lib):
    d = dict(np.load(G.GOLDEN + "/flow_to_color.npz"))
    img, flo, stats, unk = oracle_lib.flow_to_color(d["flow"])
    assert np.array_equal(img, d["img"])
    assert np.array_equal(unk, d["unknown"])
    np.testing.assert_array_equal(flo, d["flo"])
    np.testing.assert_array_equal(stats, d["stats"])


def test_colorwheel_table():
    from oracle import gqmap_np
    cw = gqmap_np.colorwheel()
    assert cw.shape == (55, 3)
    # RY ramp, the YG/GC/CB/BM/MR segment starts (legacy/computeColor.m:88-115)
    assert list(cw[0]) == [255, 0, 0] and list(cw[14]) == [255, 238, 0]
    assert list(cw[15]) == [255, 255, 0] and list(cw[21]) == [0, 255, 0]
    assert list(cw[25]) == [0, 255, 255] and list(cw[36]) == [0, 0, 255]
    assert list(cw[49]) == [255, 0, 255] and list(cw[54]) == [255, 0, 43]


def test_aepe_of_ground_truth_is_zero(oracle_lib):
    from gqmap_opticalflow_amd.flowio import load_pair
    _, _, gt = load_pair("rubberwhale")
    _, flo, _, unk = oracle_lib.flow_to_color(gt)
    assert oracle_lib.aepe(flo, flo, unk, 1) == 0.0
    assert oracle_lib.aepe(flo, flo + np.array([3.0, 4.0]), unk, 1) > 0


def test_get_map_single_component_is_mean(oracle_lib):
    rng = np.random.default_rng(5)
    mu = rng.normal(size=(6, 7, 1)); sg = rng.random((6, 7, 1)) + 0.1
    out = oracle_lib.get_map([1.0], mu, sg, -mu, sg)
    np.testing.assert_allclose(out[:, :, 0], mu[:, :, 0], atol=1e-12)
    np.testing.assert_allclose(out[:, :, 1], -mu[:, :, 0], atol=1e-12)


def test_get_map_mixture_between_modes(oracle_lib):
    # two equal-weight, heavily overlapping components: the MAP lies between the means
    mu = np.zeros((1, 1, 2)); mu[0, 0] = [0.0, 0.5]
    sg = np.ones((1, 1, 2))
    out = oracle_lib.get_map([0.5, 0.5], mu, sg, mu, sg)
    assert abs(out[0, 0, 0] - 0.25) < 1e-3


def test_map_deterministic_exp_mode(oracle_lib):
    """get_map with det_exp uses the device's gq_exp (within 1 ulp of libm):
    maxima agree to the fminbnd tolerance on well-separated mixtures, and the
    libm default is restored afterwards."""
    rng = np.random.default_rng(3)
    M, N, L = 12, 14, 2
    mu = np.asfortranarray(np.stack([rng.normal(-4, 0.3, (M, N)), rng.normal(4, 0.3, (M, N))], axis=2))
    sg = np.asfortranarray(rng.random((M, N, L)) * 0.5 + 0.2)
    a = np.array([0.7, 0.3])
    x = oracle_lib.get_map(a, mu, sg, mu, sg)
    y = oracle_lib.get_map(a, mu, sg, mu, sg, det_exp=True)
    np.testing.assert_allclose(x, y, atol=1e-4)
    np.testing.assert_array_equal(oracle_lib.get_map(a, mu, sg, mu, sg), x)


@pytest.mark.parametrize("name", ["mixture_L1", "mixture_L3_T", "super_L3"])
def test_oracle_log_p_matches_numpy_restatement(oracle_lib, name):
    # profile_logP (gqmap_gpu_mixture.m:148-154; super node_lp,
    # gqmap_gpuSuper_mix_entropy.m:152-169): the C restatement against the
    # independent array-form numpy one, on the golden frames with a MAP that
    # crosses the border clamps (displacements up to several pixels)
    from oracle import gqmap_np
    d = G.load(name)
    o = d["opts"]
    ne = gqmap_np.Engine(o, d["I1"], d["I2"])
    rng = np.random.default_rng(7)
    mp = np.asfortranarray(rng.uniform(-6, 6, size=(ne.M, ne.N, 2)))
    ref = gqmap_np.log_p(ne, mp)
    assert oracle_lib.log_p(o, d["I1"], d["I2"], mp) == pytest.approx(ref, rel=1e-12)
    # a smooth MAP (the typical case) as well
    mp2 = np.asfortranarray(np.stack(np.meshgrid(np.linspace(-1, 2, ne.N), np.linspace(0.5, -1.5, ne.M)), axis=2))
    assert oracle_lib.log_p(o, d["I1"], d["I2"], mp2) == pytest.approx(gqmap_np.log_p(ne, mp2), rel=1e-12)
