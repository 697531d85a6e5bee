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
