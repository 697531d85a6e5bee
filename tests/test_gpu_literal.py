"""The literal-order engine (options arith="literal", k_iter_lit) on the GPU
against the literal restatement of the MATLAB (oracle/gqmap_oracle.c) on
BASELINE config C2 (RubberWhale 388x584, gqmap_gpu_mixture, L=1, K=9):
bit-identical state after 20 and after 500 iterations, so the flow, its
AEPE against the .flo ground truth and its uint8 colour coding are identical
too (aepe_delta_literal = 0).  Both sides use the product's Gauss-Hermite
rule (tests/test_literal.py: the CPU model of this mode equals the
restatement bit for bit; the restatement's own eig-based rule differs by a
few ulps).  Tolerance on the trace (Energy, ptdmu, ptdsigma): 1e-12
relative -- the device sums pixels exactly (correctly rounded), MATLAB
sequentially; the state does not depend on either.

Reference: gqmap_gpu_mixture.m:27-46 (the iteration), :87-182 (the element
functions), :63-64 (AEPE)."""
import numpy as np
import pytest

from tests import _fullsize as F
from tests import _golden as G

pytestmark = pytest.mark.gpu


def _gpu_lit(o, I1, I2, st, its, **kw):
    from gqmap_opticalflow_amd import Engine
    with Engine(dict(o, arith="literal"), I1, I2, **kw) as eng:
        assert eng.info().split == 1
        eng.set_state(st)
        done, tr = eng.run(its)
        return done, tr, eng.get_state(), eng.map()


def _oracle(o, I1, I2, st, its):
    from gqmap_opticalflow_amd import gauss_hermite
    from oracle import oracle
    X, W = gauss_hermite(o["K"])
    ost = F.oracle_state(st)
    done, tr, _ = oracle.run(o, I1, I2, ost, 1, its, nthreads=16, X=X, W=W)
    return done, tr, ost


def _same(g, ost):
    for k in G.STATE_KEYS:
        np.testing.assert_array_equal(getattr(g, k), getattr(ost, k), err_msg=k)


@pytest.mark.parametrize("its", [20, 500])
def test_c2_literal_engine_bit_exact_vs_restatement(its):
    from gqmap_opticalflow_amd import aepe, flow_to_color
    from oracle import oracle
    I1, I2, flo, unk, o, st = F.case("c2")
    done, tr, g, mp = _gpu_lit(o, I1, I2, st, its)
    odone, otr, ost = _oracle(o, I1, I2, st, its)
    assert done == odone == its
    _same(g, ost)
    np.testing.assert_allclose(tr, otr, rtol=1e-12)
    omap = np.stack([ost.muu[:, :, 0], ost.muv[:, :, 0]], axis=2)
    np.testing.assert_array_equal(mp, omap)
    assert aepe(flo, mp, unk) == aepe(flo, omap, unk)
    np.testing.assert_array_equal(flow_to_color(mp)[0], oracle.flow_to_color(omap)[0])


@pytest.mark.parametrize("cfg,init", [("c2", "tight"), ("c2_dimetrodon", "ref"), ("c2_hydrangea", "tight")])
def test_literal_engine_other_pairs_and_states_bit_exact(cfg, init):
    # the same bar on the other 584x388 pairs and from a converging state
    # (mu near the ground truth: most samples interior), 20 iterations
    I1, I2, flo, unk, o, st = F.case(cfg, init)
    done, tr, g, mp = _gpu_lit(o, I1, I2, st, 20)
    odone, otr, ost = _oracle(o, I1, I2, st, 20)
    assert done == odone == 20
    _same(g, ost)
    np.testing.assert_allclose(tr, otr, rtol=1e-12)


def test_literal_engine_tiles_bit_exact_vs_whole_grid():
    # the in-process strip transport (ghost columns, exact totals) in literal mode
    from gqmap_opticalflow_amd import Engine, tile_group_run
    I1, I2, flo, unk, o, st = F.case("c2")
    I1, I2 = np.asfortranarray(I1[:96, :160]), np.asfortranarray(I2[:96, :160])
    ol = dict(o, arith="literal")
    with Engine(ol, I1, I2) as e:
        e.init_state(5)
        init = e.get_state()
        done, tr = e.run(30)
        ref = e.get_state()
    tiles = [Engine(ol, I1, I2, n_tiles=3, tile=t) for t in range(3)]
    try:
        for t in tiles:
            t.set_state(init)
        tdone, ttr = tile_group_run(tiles, 30)
        assert tdone == done == 30
        np.testing.assert_array_equal(ttr, tr)
        for t in tiles:
            s = t.get_state()
            for k in G.STATE_KEYS[:6]:
                np.testing.assert_array_equal(getattr(s, k)[:, t.col0:t.col1], getattr(ref, k)[:, t.col0:t.col1],
                                              err_msg=k)
    finally:
        for t in tiles:
            t.close()


def test_literal_engine_rejects_what_it_does_not_cover():
    from gqmap_opticalflow_amd import Engine
    from gqmap_opticalflow_amd._lib import GqmapError
    I1, I2, flo, unk, o, st = F.case("c2")
    I1, I2 = np.asfortranarray(I1[:64, :64]), np.asfortranarray(I2[:64, :64])
    for kw, extra in (({"precision": "fp32"}, {}), ({}, {"split": 4})):
        with pytest.raises(GqmapError):
            Engine(dict(o, arith="literal", **extra), I1, I2, **kw)
