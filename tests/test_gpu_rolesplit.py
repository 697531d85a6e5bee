"""The role-split kernel shape (gqmap_options.split = GQMAP_SPLIT_ROLE): Q = 1
arithmetic on 16 x 8 node tiles whose node phase (waves 0-1) and edge phase
(waves 2-3) run side by side, the node gradients handed over in LDS
(DESIGN.md §4).  Same arithmetic as the Q = 1 kernel, so it must be
bit-identical to the CPU model at split 1 and to the whole-grid Q = 1 engine,
tiled or not."""
import ctypes as C

import numpy as np
import pytest

from tests import _golden as G
from tests.test_gpu_parity import _assert_bit_exact, _emulate, _reference_init_case
from tests.test_gpu_tiles import _assemble, _problem

pytestmark = pytest.mark.gpu

ROLE = -1  # GQMAP_SPLIT_ROLE (gqmap_opticalflow_amd._lib.SPLIT_ROLE)


def _shape(eng):
    f = eng.lib.gqmap_debug_kernel_shape
    f.restype = C.c_int
    f.argtypes = [C.c_void_p]
    return f(eng.ctx)


@pytest.mark.parametrize("precision", ["fp64", "fp32"])
@pytest.mark.parametrize("engine,L,K,M,N", [("mixture", 1, 9, 96, 128), ("mixture", 3, 9, 70, 90),
                                            ("ctf", 1, 11, 96, 128), ("ctf", 1, 11, 60, 70)])
def test_role_split_bit_exact_vs_emulator(engine, L, K, M, N, precision):
    from gqmap_opticalflow_amd import Engine
    I1, I2, _, _, o, st = _reference_init_case("rubberwhale", M, N, 150, 200, L=L, K=K, engine=engine,
                                               alpha_start=10, t_decay_every=20, split=ROLE)
    e_done, e_tr, e_T, ost = _emulate(o, I1, I2, st, 40, precision, 1)
    with Engine(o, I1, I2, engine, precision) as eng:
        assert eng.info().split == 1  # the arithmetic's lanes per node
        assert _shape(eng) == 0       # the role-split kernel
        eng.set_state(st)
        done, tr = eng.run(40)
        g = eng.get_state()
    _assert_bit_exact(g, tr, done, e_done, e_tr, ost)


def test_role_split_equals_q1_kernel_on_a_full_level():
    # 240 x 320 ctf level from Grove3 (the C3 level the shape is meant for):
    # 60 iterations (a replayed graph + leftover), role split vs the Q = 1 kernel
    from bench import gt_options
    from gqmap_opticalflow_amd import Engine, ctf_options, imresize
    I1, I2, _, _, og = gt_options("Grove3", 1, 11)
    a, b = (np.asfortranarray(imresize(x, 0.5)) for x in (I1, I2))
    res = []
    for split in (1, ROLE):
        o = ctf_options(its=500, minu=og["minu"], maxu=og["maxu"], minv=og["minv"], maxv=og["maxv"], split=split)
        with Engine(o, a, b, "ctf", "fp64") as e:
            assert _shape(e) == (0 if split == ROLE else 1)
            e.init_state(0)
            done, tr = e.run(60)
            res.append((done, tr, e.get_state()))
    assert res[0][0] == res[1][0] == 60
    np.testing.assert_array_equal(res[0][1], res[1][1])
    for k in G.STATE_KEYS:
        np.testing.assert_array_equal(getattr(res[0][2], k), getattr(res[1][2], k), err_msg=k)


def test_role_split_tiles_bit_exact_vs_whole_grid():
    from gqmap_opticalflow_amd import Engine, tile_group_run
    I1, I2, o = _problem("mixture", 1, 96, 128)
    its = 40
    with Engine(dict(o, split=1), I1, I2) as e:
        e.init_state(3)
        _, tr = e.run(its)
        ref = e.get_state()
    tiles = [Engine(dict(o, split=ROLE), I1, I2, n_tiles=3, tile=t) for t in range(3)]
    try:
        for t in tiles:
            assert _shape(t) == 0
            t.init_state(3)
        done, ttr = tile_group_run(tiles, its)
        assert done == its
        np.testing.assert_array_equal(ttr, tr)
        got = _assemble(tiles, lambda t: t.get_state())
        for k in G.STATE_KEYS:
            np.testing.assert_array_equal(getattr(got, k), getattr(ref, k), err_msg=k)
    finally:
        for t in tiles:
            t.close()
