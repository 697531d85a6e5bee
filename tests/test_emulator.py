"""The CPU model of the kernel arithmetic (oracle/gqmap_emul.cpp) against the
literal restatement: one step at rounding level, exact sums independent of
thread count, deterministic math within 1 ulp of libm."""
import numpy as np
import pytest

from tests import _golden as G


def _gh(K):
    from gqmap_opticalflow_amd import gauss_hermite
    return gauss_hermite(K)


@pytest.mark.parametrize("name", G.CASES)
def test_emulator_one_step_matches_literal_restatement(oracle_lib, name):
    d = G.load(name)
    X, W = _gh(d["opts"]["K"])
    st = oracle_lib.State(*G.state(d).values())
    done, tr, _ = oracle_lib.emu_run(d["opts"], d["I1"], d["I2"], st, 1, 1, X, W)
    assert done == 1
    np.testing.assert_allclose(tr[0], d["trace"][0], rtol=1e-12)
    for k, a in zip(G.STATE_KEYS, st.arrays()):
        np.testing.assert_allclose(a, d["step1_" + k], rtol=1e-12, atol=1e-12, err_msg=k)


@pytest.mark.parametrize("name", G.CASES)
def test_emulator_fp32_one_step(oracle_lib, name):
    d = G.load(name)
    X, W = _gh(d["opts"]["K"])
    st = oracle_lib.State(*G.state(d).values())
    oracle_lib.emu_run(d["opts"], d["I1"], d["I2"], st, 1, 1, X, W, fp32=True)
    # ctf: raw (un-normalised) energies and 1/64-grid lookups -> larger fp32 step error
    atol = 3e-4 if name.startswith("ctf") else 2e-5
    for k in ("muu", "muv", "sigu", "sigv"):
        np.testing.assert_allclose(getattr(st, k), d["step1_" + k], atol=atol, err_msg=k)


def test_emulator_sums_are_order_independent(oracle_lib):
    # exact fixed-point sums: thread count (and so summation order) cannot change a bit
    d = G.load("mixture_L3_T")
    X, W = _gh(9)
    res = []
    for nt in (1, 3, 8):
        st = oracle_lib.State(*G.state(d).values())
        _, tr, _ = oracle_lib.emu_run(d["opts"], d["I1"], d["I2"], st, 1, 3, X, W, nthreads=nt)
        res.append((tr, st.arrays()))
    for tr, arrs in res[1:]:
        np.testing.assert_array_equal(tr, res[0][0])
        for a, b in zip(arrs, res[0][1]):
            np.testing.assert_array_equal(a, b)


def test_emulator_multi_step_tracks_literal_restatement(oracle_lib):
    d = G.load("mixture_L1")
    X, W = _gh(9)
    st = oracle_lib.State(*G.state(d).values())
    _, tr, _ = oracle_lib.emu_run(d["opts"], d["I1"], d["I2"], st, 1, 4, X, W)
    np.testing.assert_allclose(tr, d["trace"], rtol=1e-8)


def test_deterministic_math_within_one_ulp(oracle_lib):
    rng = np.random.default_rng(0)
    x = np.exp(rng.uniform(-12, 7, 20000))
    lg = oracle_lib.emu_math(1, x)
    assert np.max(np.abs(lg - np.log(x)) / np.spacing(np.abs(np.log(x)) + 1e-300)) <= 1.0
    y = rng.uniform(-700, 300, 20000)
    ex = oracle_lib.emu_math(2, y)
    assert np.max(np.abs(ex - np.exp(y)) / np.spacing(np.exp(y))) <= 1.0
    assert oracle_lib.emu_math(2, [-800.0])[0] == 0.0
    s = rng.uniform(1e-6, 1e4, 1000)
    np.testing.assert_array_equal(oracle_lib.emu_math(0, s), np.sqrt(s))


def test_emulator_role_split_option_is_the_q1_arithmetic(oracle_lib):
    # options["split"] = GQMAP_SPLIT_ROLE (-1) names a kernel shape with the
    # Q = 1 arithmetic: the CPU model run with it equals split 1 bit for bit
    d = G.load("mixture_L3_T")
    X, W = _gh(9)
    res = []
    for split in (1, -1):
        st = oracle_lib.State(*G.state(d).values())
        _, tr, _ = oracle_lib.emu_run(dict(d["opts"], split=split), d["I1"], d["I2"], st, 1, 3, X, W)
        res.append((tr, st.arrays()))
    np.testing.assert_array_equal(res[0][0], res[1][0])
    for a, b in zip(res[0][1], res[1][1]):
        np.testing.assert_array_equal(a, b)
