"""HIP path (libgqmap.so through the C ABI) against the oracle and the goldens.

Tolerances (fp64):
  * one iteration from identical state: 1e-10 (different summation order /
    FMA contraction in the kernel vs the literal MATLAB restatement);
  * several iterations from the golden random init: 1e-5 -- pn/rou reach
    the +-(1-1e-5) clamp where gradients carry 1/(1-p^2) ~ 5e4 (see
    tests/test_oracle.py, same tolerance between the two CPU restatements);
  * reference-style init (pn = rou = 0) at full Middlebury size: AEPE of the
    GPU flow within 1e-4 of the oracle's after 500 iterations (the north-star
    gate), state within 1e-6 after 30.
fp32 is a separate fast path; its tolerances are stated per test.
"""
import os

import numpy as np
import pytest

from tests import _golden as G

pytestmark = pytest.mark.gpu


def _engine(d, precision="fp64"):
    from gqmap_opticalflow_amd import Engine
    o = d["opts"]
    eng = Engine(o, d["I1"], d["I2"], o.get("engine", "mixture"), precision)
    return eng


def _set(eng, d, prefix="init_"):
    from gqmap_opticalflow_amd import State
    s = G.state(d, prefix)
    eng.set_state(State(**s, it=1, T=d["opts"]["temperature"]))


def _cmp_state(st, d, prefix, rtol, atol):
    for k in G.STATE_KEYS:
        np.testing.assert_allclose(getattr(st, k), d[prefix + k], rtol=rtol, atol=atol, err_msg=k)


@pytest.mark.parametrize("name", G.CASES)
def test_one_iteration_matches_golden_fp64(name):
    d = G.load(name)
    with _engine(d) as eng:
        _set(eng, d)
        done, tr = eng.run(1)
        assert done == 1
        np.testing.assert_allclose(tr[0], d["trace"][0], rtol=1e-10)
        _cmp_state(eng.get_state(), d, "step1_", 1e-10, 1e-10)


@pytest.mark.parametrize("name", G.CASES)
def test_iterations_match_golden_fp64(name):
    d = G.load(name)
    its = d["trace"].shape[0]
    with _engine(d) as eng:
        _set(eng, d)
        done, tr = eng.run(its)
        assert done == its
        np.testing.assert_allclose(tr, d["trace"], rtol=1e-8)
        st = eng.get_state()
        _cmp_state(st, d, "final_", 1e-5, 1e-5)
        assert st.it == its + 1
        assert st.T == pytest.approx(float(d["T_final"]))


@pytest.mark.parametrize("name", G.CASES)
def test_one_iteration_fp32(name):
    # fp32 fast path: one step from the golden state.  Gradients carry ~1e-6
    # relative error; the step moves mu by O(1) px, so 2e-4 absolute on mu/sigma.
    d = G.load(name)
    with _engine(d, "fp32") as eng:
        _set(eng, d)
        done, tr = eng.run(1)
        st = eng.get_state()
    np.testing.assert_allclose(tr[0], d["trace"][0], rtol=2e-4)
    for k in ("muu", "muv", "sigu", "sigv"):
        np.testing.assert_allclose(getattr(st, k), d["step1_" + k], atol=2e-3, rtol=1e-4, err_msg=k)


def test_chunked_runs_and_graph_replay_are_bit_identical():
    # 120 iterations: one run (two 50-iteration graph replays + 20 launches)
    # vs 120 single-iteration runs; device-side control must make them equal.
    d = G.load("mixture_L3_T")
    o = dict(d["opts"], its=120)
    from gqmap_opticalflow_amd import Engine, State
    s = G.state(d)
    with Engine(o, d["I1"], d["I2"]) as a, Engine(o, d["I1"], d["I2"]) as b:
        for e in (a, b):
            e.set_state(State(**{k: v.copy() for k, v in s.items()}, it=1, T=o["temperature"]))
        na, ta = a.run(120)
        tb = np.vstack([b.run(1)[1] for _ in range(120)])
        assert na == 120
        np.testing.assert_array_equal(ta, tb)
        sa, sb = a.get_state(), b.get_state()
        for k in G.STATE_KEYS:
            np.testing.assert_array_equal(getattr(sa, k), getattr(sb, k))


def test_device_init_equals_host_init():
    from gqmap_opticalflow_amd import Engine, initial_state
    d = G.load("mixture_L3_T")
    o = d["opts"]
    with Engine(o, d["I1"], d["I2"]) as eng:
        eng.init_state(seed=11)
        st = eng.get_state()
    ref = initial_state(o, d["I1"].shape[0], d["I1"].shape[1], seed=11)
    for k in G.STATE_KEYS:
        np.testing.assert_array_equal(getattr(st, k), getattr(ref, k))
    assert st.it == 1 and st.T == o["temperature"]


def test_stop_rule_ptdmu_below_tor():
    # gqmap_gpu_mixture.m:75: break once ptdmu < tor; later launches are no-ops
    from gqmap_opticalflow_amd import Engine
    d = G.load("mixture_L1")
    o = dict(d["opts"], tor=1e9)
    with Engine(o, d["I1"], d["I2"]) as eng:
        _set(eng, d)
        done, tr = eng.run(200)
        assert done == 1 and tr.shape == (1, 3)
        st1 = eng.get_state()
        assert eng.run(60)[0] == 0
        assert eng.info().stopped == 1
        st2 = eng.get_state()
        for k in G.STATE_KEYS:
            np.testing.assert_array_equal(getattr(st1, k), getattr(st2, k))


def _reference_init_case(name, M, N, r0=0, c0=0, L=1, K=9, engine="mixture", **extra):
    from gqmap_opticalflow_amd import flowio, initial_state
    from oracle import gqmap_np
    I1, I2, gt = flowio.load_pair(name)
    I1 = np.asfortranarray(I1[r0:r0 + M, c0:c0 + N]); I2 = np.asfortranarray(I2[r0:r0 + M, c0:c0 + N])
    gt = gt[r0:r0 + M, c0:c0 + N]
    _, flo, (minu, maxu, minv, maxv), unk = gqmap_np.flow_to_color(gt)
    sup = engine == "super"
    o = dict(engine=engine, K=K, L=L, temperature=0.2 if sup else 0.0, drate=0.75 if sup else 0.5,
             epsn=1e-6, lambdad=1.0, lambdas=16.0 if sup else 5.0,
             minu=minu, maxu=maxu, minv=minv, maxv=maxv, **extra)
    Mn, Nn = (M // 4, N // 4) if sup else (M, N)
    st = initial_state(o, Mn, Nn, seed=0)
    return I1, I2, flo, unk, o, st


def _oracle_state(st):
    from oracle import oracle
    return oracle.State(st.muu.copy(order="F"), st.muv.copy(order="F"), st.sigu.copy(order="F"),
                        st.sigv.copy(order="F"), st.pn.copy(order="F"), st.rou.copy(order="F"),
                        st.w.copy(), st.alpha.copy())


@pytest.mark.parametrize("engine,L,K,M,N", [("mixture", 1, 9, 96, 128), ("mixture", 3, 9, 64, 80),
                                            ("super", 3, 11, 96, 128)])
def test_reference_init_30_iterations_vs_oracle(engine, L, K, M, N):
    from gqmap_opticalflow_amd import Engine
    from oracle import oracle
    I1, I2, _, _, o, st = _reference_init_case("rubberwhale", M, N, 150, 200, L=L, K=K,
                                               engine=engine, alpha_start=10)
    ost = _oracle_state(st)
    done_o, tr_o, T_o = oracle.run(o, I1, I2, ost, 1, 30)
    with Engine(o, I1, I2, engine) as eng:
        eng.set_state(st)
        done, tr = eng.run(30)
        g = eng.get_state()
    assert done == done_o == 30
    np.testing.assert_allclose(tr, tr_o, rtol=1e-8)
    for k, a in zip(G.STATE_KEYS, ost.arrays()):
        np.testing.assert_allclose(getattr(g, k), a, rtol=1e-6, atol=1e-6, err_msg=k)


def test_full_rubberwhale_aepe_parity_500_iterations():
    """North-star gate (BASELINE config C2): RubberWhale 388x584,
    gqmap_gpu_mixture, L=1, K=9, 500 iterations, same seeded init: AEPE of
    the HIP flow within 1e-4 of the oracle's."""
    from gqmap_opticalflow_amd import Engine, aepe
    from oracle import oracle
    I1, I2, flo, unk, o, st = _reference_init_case("rubberwhale", 388, 584)
    its = 500
    ost = _oracle_state(st)
    done_o, tr_o, _ = oracle.run(o, I1, I2, ost, 1, its, nthreads=min(16, os.cpu_count() or 1))
    with Engine(o, I1, I2) as eng:
        eng.set_state(st)
        done, tr = eng.run(its)
        mp = eng.map()
    assert done == done_o
    a_gpu = aepe(flo, mp, unk)
    a_cpu = aepe(flo, np.stack([ost.muu[:, :, 0], ost.muv[:, :, 0]], axis=2), unk)
    print(f"AEPE gpu={a_gpu:.6f} cpu={a_cpu:.6f} |diff|={abs(a_gpu - a_cpu):.2e}")
    assert abs(a_gpu - a_cpu) <= 1e-4
    np.testing.assert_allclose(tr[:, 0], tr_o[:, 0], rtol=1e-6)


def test_flow_to_color_device_bit_exact():
    from gqmap_opticalflow_amd import flow_to_color
    d = dict(np.load(G.GOLDEN + "/flow_to_color.npz"))
    img, flo, stats, unk = flow_to_color(d["flow"])
    assert np.array_equal(img, d["img"])
    assert np.array_equal(unk, d["unknown"])
    np.testing.assert_array_equal(flo, d["flo"])
    np.testing.assert_array_equal(np.array(stats), d["stats"])


def test_flow_to_color_full_gt_matches_oracle():
    from gqmap_opticalflow_amd import flow_to_color, flowio
    from oracle import oracle
    for name in ("rubberwhale", "Urban3"):
        gt = flowio.load_pair(name)[2]
        a = flow_to_color(gt)
        b = oracle.flow_to_color(gt)
        assert np.array_equal(a[0], b[0]) and np.array_equal(a[3], b[3])
        np.testing.assert_array_equal(np.array(a[2]), b[2])


def test_projsplx_device_vs_oracle():
    from gqmap_opticalflow_amd import projsplx
    from oracle import oracle
    rng = np.random.default_rng(0)
    Y = np.asfortranarray(rng.normal(size=(5, 3000)))
    X = projsplx(Y)
    for c in range(0, 3000, 37):
        np.testing.assert_array_equal(X[:, c], oracle.projsplx(Y[:, c]))
    assert np.allclose(X.sum(axis=0), 1) and X.min() >= 0
    np.testing.assert_array_equal(projsplx([2.0, 0.0, 0.0]), [1.0, 0.0, 0.0])


def test_mixture_map_device_vs_oracle():
    from gqmap_opticalflow_amd import mixture_map
    from oracle import oracle
    rng = np.random.default_rng(1)
    M, N, L = 40, 50, 3
    mu = np.asfortranarray(rng.normal(size=(M, N, L)) * 2)
    sg = np.asfortranarray(rng.random((M, N, L)) * 2 + 0.05)
    mv = np.asfortranarray(rng.normal(size=(M, N, L)))
    sv = np.asfortranarray(rng.random((M, N, L)) + 0.05)
    a = np.array([0.5, 0.3, 0.2])
    g = mixture_map(a, mu, sg, mv, sv)
    c = oracle.get_map(a, mu, sg, mv, sv)
    np.testing.assert_allclose(g, c, atol=1e-9)


def test_engine_map_and_logp():
    from gqmap_opticalflow_amd import Engine
    from oracle import gqmap_np, oracle
    d = G.load("mixture_L3_T")
    with _engine(d) as eng:
        _set(eng, d)
        mp = eng.map()
        st = eng.get_state()
        lp = eng.log_p(mp)
    ref = oracle.get_map(st.alpha, st.muu, st.sigu, st.muv, st.sigv)
    np.testing.assert_allclose(mp, ref, atol=1e-9)
    # profile_logP restated in numpy (gqmap_gpu_mixture.m:148-154)
    ne = gqmap_np.Engine(d["opts"], d["I1"], d["I2"])
    M, N = mp.shape[:2]
    ns, ms = np.meshgrid(np.arange(1, N + 1), np.arange(1, M + 1))
    npot = ne.node_pot(mp[:, :, 0], mp[:, :, 1], ms, ns)
    sh = lambda X: (np.roll(X, -1, axis=0), np.roll(X, -1, axis=1))
    ep = sum(ne.edge_pot(mp, s) for s in sh(mp))
    lp_ref = npot[1:-1, 1:-1].sum() + ep[1:-1, 1:-1].sum()
    assert lp == pytest.approx(lp_ref, rel=1e-10)


def test_invalid_arguments_raise():
    from gqmap_opticalflow_amd import Engine, _lib
    d = G.load("mixture_L1")
    with pytest.raises(_lib.GqmapError):
        Engine(dict(d["opts"], L=99), d["I1"], d["I2"])
    with pytest.raises(_lib.GqmapError):  # super needs sizes divisible by 4
        Engine(d["opts"], d["I1"][:18, :27], d["I2"][:18, :27], "super")
    with Engine(d["opts"], d["I1"], d["I2"]) as eng:
        with pytest.raises(_lib.GqmapError):
            eng.run(1)  # no state yet
