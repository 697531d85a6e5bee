"""The literal-order arithmetic (gqmap_options.arith = "literal", gqmap_math.h
lit_*) against the literal restatement of the MATLAB (oracle/gqmap_oracle.c),
on the CPU: the CPU model run in literal mode must equal the restatement bit
for bit -- every state plane after every iteration -- when both use the same
Gauss-Hermite rule (the product's; the restatement's own GaussHermite_2.m
eig differs from it by a few ulps, tests/test_oracle.py pins both against
numpy.hermgauss) and, for T != 0, the same log (gq_log).  The GPU side of
the same claim is tests/test_gpu_literal.py.

Reference lines: gqmap_gpu_mixture.m:27-46 (iteration), :87-182 (the element
functions whose expression order the mode keeps)."""
import numpy as np
import pytest

from tests import _fullsize as F
from tests import _golden as G


def _gh(K):
    from gqmap_opticalflow_amd import gauss_hermite
    return gauss_hermite(K)


def _bit_equal(a_state, b_state):
    for k, x, y in zip(G.STATE_KEYS, a_state.arrays(), b_state.arrays()):
        np.testing.assert_array_equal(x, y, err_msg=k)


@pytest.mark.parametrize("name,drop_alpha", [("mixture_L1", False), ("mixture_L3_T", True)])
def test_literal_model_bit_exact_vs_restatement_golden(oracle_lib, name, drop_alpha):
    d = G.load(name)
    o = dict(d["opts"])
    if drop_alpha:  # the alpha update sums dalpha over pixels: exact here, sequential in MATLAB
        o.pop("alpha_start"), o.pop("alpha_lr")
    X, W = _gh(o["K"])
    a = oracle_lib.State(*G.state(d).values())
    b = oracle_lib.State(*G.state(d).values())
    na, ta, _ = oracle_lib.run(o, d["I1"], d["I2"], a, 1, 60, X=X, W=W, det_log=True)
    nb, tb, _ = oracle_lib.emu_run_lit(o, d["I1"], d["I2"], b, 1, 60, X, W)
    assert na == nb == 60
    _bit_equal(a, b)
    # the traces: correctly rounded (exact) pixel sums vs MATLAB's sequential sums
    np.testing.assert_allclose(tb, ta, rtol=1e-12)


def test_literal_model_bit_exact_c2_full_frame(oracle_lib):
    # BASELINE config C2 (RubberWhale 388x584, L=1, K=9) at the bench's 20 steps
    I1, I2, flo, unk, o, st = F.case("c2")
    X, W = _gh(9)
    a, b = F.oracle_state(st), F.oracle_state(st)
    na, ta, _ = oracle_lib.run(o, I1, I2, a, 1, 20, X=X, W=W)
    nb, tb, _ = oracle_lib.emu_run_lit(o, I1, I2, b, 1, 20, X, W)
    assert na == nb == 20
    _bit_equal(a, b)
    np.testing.assert_allclose(tb, ta, rtol=1e-12)


def test_literal_model_tiles_bit_exact(oracle_lib):
    # column strips (ghost columns from the whole-grid state each step) in
    # literal mode equal the whole grid: the arithmetic is per node
    I1, I2, flo, unk, o, st = F.case("c2")
    I1, I2 = np.asfortranarray(I1[:48, :64]), np.asfortranarray(I2[:48, :64])
    crop = lambda x: np.asfortranarray(x[:48, :64])
    ref = oracle_lib.State(crop(st.muu), crop(st.muv), crop(st.sigu), crop(st.sigv), crop(st.pn),
                           crop(st.rou), st.w, st.alpha)
    X, W = _gh(9)
    whole = ref.copy()
    oracle_lib.emu_run_lit(o, I1, I2, whole, 1, 5, X, W)
    cur = ref.copy()
    for it in range(1, 6):
        nxt = cur.copy()
        for t in range(3):
            c0, c1, n_off, lo, hi, Nl = oracle_lib.tile_geometry(64, 3, t)
            sl = slice(n_off, n_off + Nl)
            loc = oracle_lib.State(*(np.array(x[:, sl], order="F", copy=True) for x in cur.arrays()[:6]), cur.w, cur.alpha)
            oracle_lib.emu_run_lit(o, I1, I2, loc, it, 1, X, W, geo=(n_off, lo, hi, 64))
            for full, part in zip(nxt.arrays()[:6], loc.arrays()[:6]):
                full[:, c0:c1] = part[:, lo:hi]
        cur = nxt
    _bit_equal(whole, cur)


def test_literal_differs_from_fast_spec(oracle_lib):
    # the two specifications are different arithmetic (a rounding or two per
    # gradient): same to 1e-12 after one step, not bit-identical
    d = G.load("mixture_L1")
    X, W = _gh(9)
    a = oracle_lib.State(*G.state(d).values())
    b = oracle_lib.State(*G.state(d).values())
    oracle_lib.emu_run(d["opts"], d["I1"], d["I2"], a, 1, 1, X, W, split=1)
    oracle_lib.emu_run_lit(d["opts"], d["I1"], d["I2"], b, 1, 1, X, W)
    np.testing.assert_allclose(a.muu, b.muu, rtol=1e-12, atol=1e-12)
    assert any(np.any(x != y) for x, y in zip(a.arrays(), b.arrays()))


def test_literal_mode_rejects_other_engines(oracle_lib):
    d = G.load("super_L3")
    X, W = _gh(11)
    st = oracle_lib.State(*G.state(d).values())
    with pytest.raises(RuntimeError):
        oracle_lib.emu_run_lit(d["opts"], d["I1"], d["I2"], st, 1, 1, X, W)
