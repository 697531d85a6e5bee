"""The persistent small-grid launch (k_iter_persist): ctf contexts with L = 1
and Q >= 4 run a whole chunk of iterations in one launch, state handed
between workgroups through device-coherent stores behind a grid barrier, the
finalize step of iteration j - 1 overlapped with iteration j.

Gates: bit-identical to the CPU model (oracle/gqmap_emul.cpp) across graph
chunks (50-iteration replays + a leftover launch) with the temperature decay
on, and the stop rule (legacy/gqmap_ctf.m's `ptdmu < tor` exit, shared with
gqmap_gpu_mixture.m:75) firing at any point of a chunk: the speculative
iteration after the stopping one leaves no trace in the state, the trace or
Ctl::it / done.
"""
import numpy as np
import pytest

from tests import _golden as G
from tests.test_gpu_parity import _assert_bit_exact, _emulate, _reference_init_case, _run_engine

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("precision", ["fp64", "fp32"])
@pytest.mark.parametrize("M,N,split", [(60, 70, 4), (60, 70, 8), (30, 44, 16), (30, 44, 64)])
def test_persistent_chunks_bit_exact_vs_emulator(M, N, split, precision):
    import dataclasses
    I1, I2, _, _, o, st = _reference_init_case("rubberwhale", M, N, 150, 200, L=1, K=11, engine="ctf",
                                               split=split, t_decay_every=20)
    # a non-zero temperature, so the workgroups' own copy of the decay matters
    o = dict(o, temperature=0.3)
    st = dataclasses.replace(st, T=0.3)
    its = 130  # two replayed 50-iteration chunks + one 30-iteration launch
    e_done, e_tr, e_T, ost = _emulate(o, I1, I2, st, its, precision, split)
    done, tr, g, info = _run_engine(o, I1, I2, "ctf", precision, st, its)
    assert info.split == split
    _assert_bit_exact(g, tr, done, e_done, e_tr, ost)
    assert g.T == e_T
    assert g.it == st.it + its


@pytest.mark.parametrize("split", [8, 64])
@pytest.mark.parametrize("where", ["first", "inside", "chunk_end", "leftover"])
def test_persistent_stop_rule(split, where):
    from gqmap_opticalflow_amd import Engine
    M, N = (60, 70) if split == 8 else (30, 44)
    I1, I2, _, _, o, st = _reference_init_case("rubberwhale", M, N, 150, 200, L=1, K=11, engine="ctf",
                                               split=split)
    its = 80
    _, tr, _, _ = _run_engine(o, I1, I2, "ctf", "fp64", st, its)
    ptd = tr[:, 1]
    if where == "first":
        tor = 1e9
    else:
        k = {"inside": 17, "chunk_end": 49, "leftover": 63}[where]
        tor = float(ptd[k]) * (1 + 1e-12)
    o = dict(o, tor=tor)
    k = int(np.argmax(ptd < tor))  # first row that meets the rule
    assert ptd[k] < tor
    with Engine(o, I1, I2, "ctf", "fp64") as eng:
        eng.set_state(st)
        done, tr2 = eng.run(its)
        g = eng.get_state()
        assert eng.info().stopped == 1
        assert eng.run(30)[0] == 0
        np.testing.assert_array_equal(eng.get_state().muu, g.muu)
    assert done == k + 1
    np.testing.assert_array_equal(tr2, tr[:k + 1])
    ref = _run_engine(o, I1, I2, "ctf", "fp64", st, k + 1)
    for key in G.STATE_KEYS:
        np.testing.assert_array_equal(getattr(g, key), getattr(ref[2], key), err_msg=key)
    assert g.it == ref[2].it == st.it + k + 1


@pytest.mark.parametrize("split", [8, 64])
@pytest.mark.parametrize("barrier", [0, 7, 49])
def test_persistent_failure_recovers_bit_exact(split, barrier):
    # A persistent launch whose grid barrier gives up (workgroups not
    # co-resident, or descheduled past the spin limit) is simulated by failing
    # barrier `barrier` of the first launch (gqmap_debug_persist_fault): the
    # run restores the snapshot the failed launch started from and goes on
    # with one launch per iteration -- same trace, same state, same bits as
    # an undisturbed run, and no error.
    import ctypes as C
    import dataclasses
    from gqmap_opticalflow_amd import Engine, _lib
    # grids whose persistent launch fits the device (Q = 64: one 5-wave
    # workgroup per CU, 6 x 40 tiles + the finalizer <= 256)
    M, N = (60, 70) if split == 8 else (30, 40)
    I1, I2, _, _, o, st = _reference_init_case("rubberwhale", M, N, 150, 200, L=1, K=11, engine="ctf",
                                               split=split, t_decay_every=20)
    o = dict(o, temperature=0.3)
    st = dataclasses.replace(st, T=0.3)
    its = 130
    _, ref_tr, ref, _ = _run_engine(o, I1, I2, "ctf", "fp64", st, its)
    lib = _lib.load()
    lib.gqmap_debug_persist_fault.argtypes = [C.c_void_p, C.c_int]
    lib.gqmap_debug_persist_off.argtypes = [C.c_void_p]
    with Engine(o, I1, I2, "ctf", "fp64") as eng:
        eng.set_state(st)
        eng.prepare()  # graphs captured with the persistent launch
        assert lib.gqmap_debug_persist_off(eng.ctx) == 0
        assert lib.gqmap_debug_persist_fault(eng.ctx, barrier) == 0
        done, tr = eng.run(its)
        assert lib.gqmap_debug_persist_off(eng.ctx) == 1  # fell back
        g = eng.get_state()
        # and it keeps running correctly afterwards (per-iteration graphs)
        done2, tr2 = eng.run(20)
        g2 = eng.get_state()
    assert done == its
    np.testing.assert_array_equal(tr, ref_tr)
    for key in G.STATE_KEYS:
        np.testing.assert_array_equal(getattr(g, key), getattr(ref, key), err_msg=key)
    assert g.it == ref.it and g.T == ref.T
    _, tr3, ref2, _ = _run_engine(o, I1, I2, "ctf", "fp64", st, its + 20)
    np.testing.assert_array_equal(tr2, tr3[its:])
    for key in G.STATE_KEYS:
        np.testing.assert_array_equal(getattr(g2, key), getattr(ref2, key), err_msg=key)


def test_persistent_capacity_override_runs_per_iteration():
    # policy persist_cap: a capacity too small for the grid keeps the level on
    # one launch per iteration (the path a device without room takes) -- the
    # same bits as the persistent launch
    from tests.test_gpu_parity import _policy, _reference_init_case, _run_engine
    I1, I2, _, _, o, st = _reference_init_case("rubberwhale", 30, 40, 150, 200, L=1, K=11, engine="ctf", split=64)
    outs = []
    for cap in (-1, 1):
        with _policy(persist_cap=cap):
            _, tr, g, _ = _run_engine(o, I1, I2, "ctf", "fp64", st, 70)
        outs.append(np.concatenate([tr.ravel(), g.muu.ravel(), g.sigv.ravel(), g.rou.ravel()]))
    np.testing.assert_array_equal(outs[0], outs[1])
