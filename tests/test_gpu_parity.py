"""HIP path (libgqmap.so through the C ABI) against the oracle library.

Two references:
  * oracle/gqmap_emul.cpp, the CPU model of the kernel's arithmetic: the GPU
    must be BIT-IDENTICAL to it for any number of iterations, fp64 and fp32
    (assert_array_equal) -- this is the gate that survives the solver's
    chaotic transient (a 1e-13 perturbation of the init grows to O(1) state
    differences within ~30 iterations, see DESIGN.md "Parity");
  * the literal restatement of the MATLAB (oracle/gqmap_oracle.c, goldens
    from oracle/gqmap_np.py): one iteration within 1e-10 (fp64); several
    iterations from the golden random init within 1e-5 (pn/rou reach the
    +-(1-1e-5) clamp where gradients carry 1/(1-p^2) ~ 5e4).
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


@pytest.mark.parametrize("name", ["mixture_L3_T", "ctf_L1"])
def test_device_init_equals_host_init(name):
    from gqmap_opticalflow_amd import Engine, initial_state
    d = G.load(name)
    o = d["opts"]
    eng_name = o.get("engine", "mixture")
    with Engine(o, d["I1"], d["I2"], eng_name) as eng:
        eng.init_state(seed=11)
        st = eng.get_state()
    ref = initial_state(o, d["I1"].shape[0], d["I1"].shape[1], seed=11, engine=eng_name)
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
    if engine == "ctf":
        # pyramid levels see resampled (non-integer) frames: exercises the fp64 VV store
        I1 = np.asfortranarray(I1 * 0.7); I2 = np.asfortranarray(I2 * 0.7 + 0.1)
    o = dict(engine=engine, K=K, L=L, temperature=0.2 if sup else 0.0, drate=0.75 if sup else 0.5,
             epsn=1e-6, lambdad=1.0, lambdas=16.0 if sup else 5.0,
             minu=minu, maxu=maxu, minv=minv, maxv=maxv, **extra)
    Mn, Nn = (M // 4, N // 4) if sup else (M, N)
    st = initial_state(o, Mn, Nn, seed=0, engine=engine)
    return I1, I2, flo, unk, o, st


def _oracle_state(st):
    from oracle import oracle
    return oracle.State(st.muu.copy(order="F"), st.muv.copy(order="F"), st.sigu.copy(order="F"),
                        st.sigv.copy(order="F"), st.pn.copy(order="F"), st.rou.copy(order="F"),
                        st.w.copy(), st.alpha.copy())


def _gh(K):
    from gqmap_opticalflow_amd import gauss_hermite
    return gauss_hermite(K)


def _emulate(o, I1, I2, st, its, precision, split):
    from oracle import oracle
    ost = _oracle_state(st)
    X, W = _gh(o["K"])
    done, tr, T = oracle.emu_run(o, I1, I2, ost, st.it, its, X, W, T=st.T,
                                 nthreads=min(16, os.cpu_count() or 1), fp32=precision == "fp32",
                                 split=split)
    return done, tr, T, ost


def _assert_bit_exact(g, tr, done, e_done, e_tr, ost):
    assert done == e_done
    np.testing.assert_array_equal(tr, e_tr)
    for k, a in zip(G.STATE_KEYS, ost.arrays()):
        np.testing.assert_array_equal(getattr(g, k), a, err_msg=k)


@pytest.mark.parametrize("precision", ["fp64", "fp32"])
@pytest.mark.parametrize("name", G.CASES)
def test_bit_exact_vs_emulator_golden_init(name, precision):
    from gqmap_opticalflow_amd import State
    d = G.load(name)
    o = d["opts"]
    st = State(**G.state(d), it=1, T=o["temperature"])
    with _engine(d, precision) as eng:
        eng.set_state(State(**G.state(d), it=1, T=o["temperature"]))
        done, tr = eng.run(25)
        g = eng.get_state()
        split = eng.info().split
    e_done, e_tr, e_T, ost = _emulate(o, d["I1"], d["I2"], st, 25, precision, split)
    _assert_bit_exact(g, tr, done, e_done, e_tr, ost)
    assert g.T == e_T


@pytest.mark.parametrize("precision", ["fp64", "fp32"])
@pytest.mark.parametrize("engine,L,K,M,N,split", [("mixture", 1, 9, 96, 128, 1),
                                                  ("mixture", 1, 9, 96, 128, 4),
                                                  ("mixture", 3, 9, 70, 90, 16),
                                                  ("mixture", 3, 9, 70, 90, 1),
                                                  ("super", 3, 11, 96, 128, 16),
                                                  ("super", 3, 11, 96, 128, 4),
                                                  ("super", 1, 11, 100, 132, 1),
                                                  ("ctf", 1, 11, 96, 128, 1),
                                                  ("ctf", 1, 11, 60, 70, 4),
                                                  ("ctf", 1, 11, 30, 44, 16),
                                                  ("ctf", 1, 11, 30, 44, 64),
                                                  ("ctf", 1, 11, 60, 70, 8),
                                                  ("mixture", 3, 9, 30, 44, 64)])
def test_bit_exact_vs_emulator_reference_init(engine, L, K, M, N, split, precision):
    # reference-style init (pn = rou = 0), many tiles (halo edges across tiles),
    # ragged last tiles, alpha update from iteration 10, every lanes-per-node Q
    from gqmap_opticalflow_amd import Engine
    I1, I2, _, _, o, st = _reference_init_case("rubberwhale", M, N, 150, 200, L=L, K=K,
                                               engine=engine, alpha_start=10, t_decay_every=20,
                                               split=split)
    e_done, e_tr, e_T, ost = _emulate(o, I1, I2, st, 40, precision, split)
    with Engine(o, I1, I2, engine, precision) as eng:
        assert eng.info().split == split
        eng.set_state(st)
        done, tr = eng.run(40)
        g = eng.get_state()
    _assert_bit_exact(g, tr, done, e_done, e_tr, ost)


def test_full_rubberwhale_500_iterations_bit_exact():
    """North-star gate (BASELINE config C2): RubberWhale 388x584,
    gqmap_gpu_mixture, L=1, K=9, 500 iterations from the same seeded init.
    The GPU state is bit-identical to the CPU model's, so AEPE(GPU) ==
    AEPE(CPU) exactly (gate: <= 1e-4)."""
    from gqmap_opticalflow_amd import Engine, aepe
    I1, I2, flo, unk, o, st = _reference_init_case("rubberwhale", 388, 584)
    its = 500
    e_done, e_tr, _, ost = _emulate(o, I1, I2, st, its, "fp64", 1)
    with Engine(o, I1, I2) as eng:
        assert eng.info().split == 1
        eng.set_state(st)
        done, tr = eng.run(its)
        g = eng.get_state()
        mp = eng.map()
    _assert_bit_exact(g, tr, done, e_done, e_tr, ost)
    a_gpu = aepe(flo, mp, unk)
    a_cpu = aepe(flo, np.stack([ost.muu[:, :, 0], ost.muv[:, :, 0]], axis=2), unk)
    print(f"AEPE after {its} its: gpu={a_gpu:.9f} cpu-model={a_cpu:.9f}")
    assert a_gpu == a_cpu


class _policy:
    """Execution policies (gqmap_debug_policy) for the duration of a block."""

    def __init__(self, **kw):
        self.kw = kw

    def __enter__(self):
        from gqmap_opticalflow_amd import _lib
        for k, v in self.kw.items():
            _lib.debug_policy(k, v)

    def __exit__(self, *a):
        from gqmap_opticalflow_amd import _lib
        for k in self.kw:
            _lib.debug_policy(k, -1)


def _run_engine(o, I1, I2, engine, precision, st, its):
    from gqmap_opticalflow_amd import Engine
    with Engine(o, I1, I2, engine, precision) as eng:
        eng.set_state(st)
        done, tr = eng.run(its)
        return done, tr, eng.get_state(), eng.info()


@pytest.mark.parametrize("precision", ["fp64", "fp32"])
@pytest.mark.parametrize("engine,K,M,N,split", [("mixture", 9, 96, 128, 1),
                                                ("mixture", 9, 96, 128, 2),
                                                ("mixture", 9, 70, 90, 4),
                                                ("super", 11, 96, 128, 16),
                                                ("super", 11, 100, 132, 1),
                                                ("ctf", 11, 96, 128, 1),
                                                ("ctf", 11, 96, 128, 2),
                                                ("ctf", 11, 60, 70, 4),
                                                ("ctf", 11, 30, 44, 16),
                                                ("ctf", 11, 30, 44, 64),
                                                ("ctf", 11, 60, 70, 8),
                                                ("mixture", 9, 60, 70, 8),
                                                ("mixture", 9, 60, 70, 64)])
def test_single_gaussian_every_split_bit_exact_vs_emulator(engine, K, M, N, split, precision):
    # L = 1, constant temperature, every lanes-per-node Q (16 x 16, 16 x 8,
    # 8 x 8, 4 x 4 node tiles) against the CPU model
    I1, I2, _, _, o, st = _reference_init_case("rubberwhale", M, N, 150, 200, L=1, K=K, engine=engine,
                                               split=split, t_decay_every=0)
    e_done, e_tr, e_T, ost = _emulate(o, I1, I2, st, 40, precision, split)
    done, tr, g, info = _run_engine(o, I1, I2, engine, precision, st, 40)
    assert info.split == split
    _assert_bit_exact(g, tr, done, e_done, e_tr, ost)


def test_graph_replay_equals_per_iteration_launches():
    # full C2 frame, 120 iterations: 2 captured 50-iteration graphs + 20
    # single launches against 120 single launches (policy graph = 0)
    I1, I2, _, _, o, st = _reference_init_case("rubberwhale", 388, 584)
    a = _run_engine(o, I1, I2, "mixture", "fp64", st, 120)
    with _policy(graph=0):
        b = _run_engine(o, I1, I2, "mixture", "fp64", st, 120)
    assert a[0] == b[0] == 120
    np.testing.assert_array_equal(a[1], b[1])
    for k in G.STATE_KEYS:
        np.testing.assert_array_equal(getattr(a[2], k), getattr(b[2], k), err_msg=k)


def test_prepared_graph_and_timed_replay_are_bit_identical():
    # bench.py's two legs: gqmap_prepare + gqmap_run (the timed region) and
    # gqmap_run_timed (per-launch HIP events) from the same initial state
    from gqmap_opticalflow_amd import Engine
    I1, I2, _, _, o, st = _reference_init_case("rubberwhale", 388, 584)
    with Engine(o, I1, I2) as eng:
        eng.set_state(st)
        eng.prepare()
        done, _ = eng.run(70)
        a = eng.get_state()
        eng.set_state(st)
        done2, total_ms, kernel_ms = eng.run_timed(70)
        b = eng.get_state()
    assert done == done2 == 70
    assert 0 < kernel_ms <= total_ms
    for k in G.STATE_KEYS:
        np.testing.assert_array_equal(getattr(a, k), getattr(b, k), err_msg=k)


def test_stop_inside_a_graph_chunk():
    # the stop rule (ptdmu < tor, gqmap_gpu_mixture.m:75) firing inside a
    # replayed 50-iteration graph: the remaining launches are no-ops, the
    # state is that of the stopping iteration, later runs do nothing
    I1, I2, _, _, o, st = _reference_init_case("rubberwhale", 96, 128, 150, 200)
    _, tr, _, _ = _run_engine(o, I1, I2, "mixture", "fp64", st, 60)
    ptd = tr[:, 1]
    k = int(np.argmin(ptd[:45]))  # stop at row k (< 50: inside the first graph chunk)
    o = dict(o, tor=float(ptd[k]) * (1 + 1e-12))
    if np.any(ptd[:k] < o["tor"]):
        k = int(np.argmax(ptd < o["tor"]))
    from gqmap_opticalflow_amd import Engine
    with Engine(o, I1, I2) as eng:
        eng.set_state(st)
        done, tr2 = eng.run(60)
        g = eng.get_state()
        assert eng.info().stopped == 1
        assert eng.run(30)[0] == 0
        np.testing.assert_array_equal(eng.get_state().muu, g.muu)
    assert done == k + 1
    np.testing.assert_array_equal(tr2, tr[:k + 1])
    ref = _run_engine(o, I1, I2, "mixture", "fp64", st, k + 1)
    for key in G.STATE_KEYS:
        np.testing.assert_array_equal(getattr(g, key), getattr(ref[2], key), err_msg=key)
    assert g.it == ref[2].it == k + 2


def test_device_math_matches_host():
    from gqmap_opticalflow_amd import _lib
    from oracle import oracle
    import ctypes as C
    lib = _lib.load()
    f = lib.gqmap_selftest_math
    f.restype = C.c_int
    f.argtypes = [C.c_int, C.POINTER(C.c_double), C.POINTER(C.c_double), C.c_int64]
    rng = np.random.default_rng(0)
    inputs = {0: np.concatenate([rng.uniform(1e-6, 1e3, 200000), 1e-6 + rng.random(50000) ** 4,
                                 1 + rng.uniform(-1, 1, 50000) * (1 - 1e-5)]),
              1: np.exp(rng.uniform(-12, 7, 100000)),
              2: rng.uniform(-740, 300, 100000),
              # f32 sqrt on the arguments the fp32 engine passes (eps + d^2, 1 +- p, 1 - p^2)
              3: np.concatenate([np.float32(1e-6) + rng.uniform(0, 1e4, 200000).astype(np.float32) ** 2,
                                 rng.uniform(1e-5, 2.0, 100000).astype(np.float32),
                                 np.exp(rng.uniform(-66, 80, 100000)).astype(np.float32)]).astype(np.float64)}
    for fn, x in inputs.items():
        x = np.ascontiguousarray(x)
        out = np.zeros_like(x)
        assert f(fn, _lib.dptr(x), _lib.dptr(out), x.size) == 0
        np.testing.assert_array_equal(out, oracle.emu_math(fn, x), err_msg=f"fn {fn}")


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
    # bit-exact against the restatement evaluated with the device's exp
    # (gq_exp): same fminbnd path, same bits
    np.testing.assert_array_equal(g, oracle.get_map(a, mu, sg, mv, sv, det_exp=True))
    # against libm's exp: fminbnd is a local search, so on flat multimodal
    # mixtures a last-bit difference in exp() can send Brent's path to another
    # local optimum -- reported, not gated tightly
    c = oracle.get_map(a, mu, sg, mv, sv)
    close = np.abs(g - c) <= 1e-6
    print(f"mixture MAP agreement with the libm-exp restatement: {close.mean():.4f}")
    assert close.mean() >= 0.97
    # well-separated / unimodal case: exact agreement
    mu1 = np.asfortranarray(rng.normal(size=(M, N, 1)))
    s1 = np.asfortranarray(rng.random((M, N, 1)) + 0.1)
    np.testing.assert_allclose(mixture_map([1.0], mu1, s1, -mu1, s1), np.stack([mu1[:, :, 0], -mu1[:, :, 0]], axis=2), atol=1e-12)


def test_engine_map_and_logp():
    from gqmap_opticalflow_amd import Engine
    from oracle import gqmap_np, oracle
    d = G.load("mixture_L3_T")
    with _engine(d) as eng:
        _set(eng, d)
        mp = eng.map()
        st = eng.get_state()
        lp = eng.log_p(mp)
    np.testing.assert_array_equal(mp, oracle.get_map(st.alpha, st.muu, st.sigu, st.muv, st.sigv, det_exp=True))
    ref = oracle.get_map(st.alpha, st.muu, st.sigu, st.muv, st.sigv)
    assert (np.abs(mp - ref) <= 1e-6).mean() >= 0.97
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


@pytest.mark.parametrize("precision", ["fp64", "fp32"])
def test_super_bit_exact_on_preprocessed_frames(precision):
    # optical_flowSuper.m preprocessed=true: non-integer structure-texture frames
    # (fp64 VV store), 20 iterations, bit-exact vs the CPU model
    from gqmap_opticalflow_amd import Engine
    from tests.test_preprocessed import _case
    I1, I2, o, st = _case()
    e_done, e_tr, e_T, ost = _emulate(o, I1, I2, st, 20, precision, None)
    with Engine(o, I1, I2, "super", precision) as eng:
        eng.set_state(st)
        done, tr = eng.run(20)
        g = eng.get_state()
    _assert_bit_exact(g, tr, done, e_done, e_tr, ost)


def _placement_runs(o, I1, I2, engine, precision, st, its, split, policies):
    """The same run under each policy setting (gqmap_debug_policy): a list of
    (trace, state); each run asserts the lanes per node it was meant to use."""
    outs = []
    for pol in policies:
        with _policy(**pol):
            done, tr, g, info = _run_engine(dict(o, split=split), I1, I2, engine, precision, st, its)
        assert info.split == split and done == its
        outs.append((tr, g))
    return outs


def _same_runs(outs):
    for tr, g in outs[1:]:
        np.testing.assert_array_equal(tr, outs[0][0])
        for k in G.STATE_KEYS:
            np.testing.assert_array_equal(getattr(g, k), getattr(outs[0][1], k), err_msg=k)


@pytest.mark.parametrize("engine", ["mixture", "ctf"])
def test_nontemporal_state_stores_same_bits(engine):
    # state_nt (non-temporal state stores) is a cache policy: forced on, a
    # crop at split 1 -- the only split whose kernel has the NT variant
    # (k_iter<..,Q=1,NT=true>; the default for frames whose state exceeds
    # 32 MiB, C5 and the large ctf levels) -- gives the trace and state of
    # forced off, and both equal the CPU model
    I1, I2, _, _, o, st = _reference_init_case("rubberwhale", 128, 160, 100, 150, L=1, K=9 if engine == "mixture"
                                               else 11, engine=engine)
    outs = _placement_runs(o, I1, I2, engine, "fp64", st, 60, 1, [dict(nt_state=0), dict(nt_state=1)])
    _same_runs(outs)
    e_done, e_tr, _, ost = _emulate(o, I1, I2, st, 60, "fp64", 1)
    _assert_bit_exact(outs[1][1], outs[1][0], 60, e_done, e_tr, ost)


@pytest.mark.parametrize("precision", ["fp64", "fp32"])
@pytest.mark.parametrize("split", [1, 4])
def test_band_row_tile_order_same_bits(precision, split):
    # band_rows (each XCD walks its band of tile columns row by row,
    # gqmap_engine.hip band_row_tile) is a placement: forced on, a 100 x 150
    # frame -- at split 1 16 x 16 tiles, 7 tile rows x 10 tile columns; at
    # split 4 8 x 8 tiles, 13 x 19: the bands start and end inside a tile
    # column -- gives the trace and state of forced off
    I1, I2, _, _, o, st = _reference_init_case("rubberwhale", 100, 150, 100, 150, L=2, K=9)
    _same_runs(_placement_runs(o, I1, I2, "mixture", precision, st, 60, split,
                               [dict(band_rows=0), dict(band_rows=1)]))


def test_c5_default_policies_together_same_bits():
    # the C5 default combination -- non-temporal stores and the band-row walk
    # together, on the ctf engine (ENG = 2) and the mixture engine at split 1
    # -- against both off
    for engine, K in (("ctf", 11), ("mixture", 9)):
        I1, I2, _, _, o, st = _reference_init_case("rubberwhale", 100, 150, 100, 150, L=1, K=K, engine=engine)
        _same_runs(_placement_runs(o, I1, I2, engine, "fp64", st, 40, 1,
                                   [dict(nt_state=0, band_rows=0), dict(nt_state=1, band_rows=1)]))
