"""The staged-tap window of the single-pixel engines (gqmap_engine.hip:
each tile copies the padded-frame rectangle its samples can reach into LDS
and reads every tap there).  The rectangle is the union over the tile's
nodes of gqmap_math.h tap_rect; the CPU model of the kernel counts every tap
a node's samples read outside that node's own rectangle -- it must be none,
on every engine and precision, from the reference init (samples far apart,
clamped at the border) and on pyramid-level frames (the ctf lookup's capped
last cell)."""
import dataclasses

import numpy as np
import pytest


@pytest.mark.parametrize("precision", ["fp64", "fp32"])
@pytest.mark.parametrize("engine,M,N,split,K,its", [("ctf", 60, 70, 8, 11, 60), ("ctf", 30, 44, 16, 11, 40),
                                                     ("ctf", 48, 64, 1, 11, 20), ("mixture", 64, 80, 1, 9, 30),
                                                     ("mixture", 40, 50, 4, 9, 20)])
def test_every_tap_inside_its_window(engine, M, N, split, K, its, precision):
    from gqmap_opticalflow_amd import gauss_hermite
    from oracle import oracle
    from tests.test_gpu_parity import _reference_init_case
    I1, I2, _, _, o, st = _reference_init_case("rubberwhale", M, N, 150, 200, L=1, K=K, engine=engine, split=split,
                                               t_decay_every=20)
    o = dict(o, temperature=0.3)
    st = dataclasses.replace(st, T=0.3)
    ost = oracle.State(*(np.array(getattr(st, k), order="F", copy=True)
                         for k in ("muu", "muv", "sigu", "sigv", "pn", "rou", "w", "alpha")))
    X, W = gauss_hermite(K)
    oracle.emu_window_check(True)
    try:
        oracle.emu_run(o, I1, I2, ost, st.it, its, X, W, T=st.T, nthreads=4, fp32=precision == "fp32", split=split)
    finally:
        bad = oracle.emu_window_check(False)
    assert bad == 0


def test_window_check_detects_a_tap_outside():
    # the check itself: with every rectangle one column short it must count
    # taps outside
    from gqmap_opticalflow_amd import gauss_hermite
    from oracle import oracle
    from tests.test_gpu_parity import _reference_init_case
    I1, I2, _, _, o, st = _reference_init_case("rubberwhale", 40, 50, 150, 200, L=1, K=9)
    ost = oracle.State(*(np.array(getattr(st, k), order="F", copy=True)
                         for k in ("muu", "muv", "sigu", "sigv", "pn", "rou", "w", "alpha")))
    X, W = gauss_hermite(9)
    oracle.emu_window_check(2)
    try:
        oracle.emu_run(o, I1, I2, ost, st.it, 2, X, W, T=st.T, nthreads=4)
    finally:
        bad = oracle.emu_window_check(False)
    assert bad > 0
