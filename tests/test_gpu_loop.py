"""The multi-rank RCCL strip iteration's own code, with real neighbours, on
one GPU (gqmap_gpu_mixture.m:29-46 sharded as column strips).

Every RCCL test elsewhere uses a one-rank communicator, where
exchange_rccl returns before any send/recv and the all-gathers move only
the rank's own row.  Here n tile contexts are attached to the loopback
transport (tests/_loop.py: only the three NCCL calls -- grouped
ncclSend/ncclRecv and the two ncclAllGather -- become device copies between
the ranks' buffers, matched in issue order behind host barriers) and each is
driven from its own host thread through the public calls, as bench.py's
tiled_solve drives an RCCL rank.  So these run with neighbours:
launch_seq_deferred / launch_step_deferred, strip_launch for tile > 0,
k_unpack_advance with real ghost sides, k_finalize_seq over every rank's
rows, deferred_recover across ranks, and the exact step launch_step_rccl
with k_unpack_finalize.  Launches run directly (a loopback collective
cannot be held in a stream capture); their sequence is the captured
graph's.  The bar: bit-identical to the whole-grid solve."""
import numpy as np
import pytest

from tests import _golden as G
from tests._loop import LoopGroup, ranks
from tests.test_gpu_tiles import _problem, _whole

pytestmark = pytest.mark.gpu


def _strips(o, I1, I2, n, engine="mixture", precision="fp64"):
    from gqmap_opticalflow_amd import Engine
    grp = LoopGroup(n)
    tiles = [Engine(o, I1, I2, engine, precision, n_tiles=n, tile=t) for t in range(n)]
    for t in tiles:
        grp.attach(t)
    return grp, tiles


def _close(grp, tiles):
    for t in tiles:
        t.close()
    grp.destroy()


def _check_strips(states, tiles, ref, keys=G.STATE_KEYS[:6]):
    for t, s in zip(tiles, states):
        for k in keys:
            np.testing.assert_array_equal(getattr(s, k)[:, t.col0:t.col1], getattr(ref, k)[:, t.col0:t.col1],
                                          err_msg=f"tile {t.tile} {k}")
        np.testing.assert_array_equal(s.alpha, ref.alpha, err_msg=f"tile {t.tile} alpha")
        np.testing.assert_array_equal(s.w, ref.w, err_msg=f"tile {t.tile} w")
        assert s.it == ref.it and s.T == ref.T


@pytest.mark.parametrize("n_tiles", [2, 4, 8])
def test_loop_c2_strips_bench_sequence_bit_exact(n_tiles):
    """The headline pair (RubberWhale 388x584, L = 1, K = 9) as n_tiles
    strips at the per-strip lanes per node (strip_split), each rank making
    bench.py tiled_solve's calls: warm-up run, prepare, clock-settle chunks
    from a fresh init, the timed run (one 50-iteration deferred sequence + an
    11-iteration one), then the instrumented replay (run_timed).  Both end
    bit-identical to the whole grid at the same Q: state, trace, map."""
    from gqmap_opticalflow_amd import Engine, flow_to_color, flowio, strip_split
    I1, I2, gt = flowio.load_pair("rubberwhale")
    _, _, (minu, maxu, minv, maxv), _ = flow_to_color(gt)
    q = strip_split(*I1.shape, n_tiles)
    o = dict(K=9, L=1, temperature=0.0, drate=0.5, epsn=1e-6, lambdad=1.0, lambdas=5.0,
             minu=minu, maxu=maxu, minv=minv, maxv=maxv, split=q)
    its = 61
    init, ref, tr = _whole(I1, I2, o, "mixture", "fp64", its, seed=0)
    with Engine(o, I1, I2) as e:
        e.init_state(0)
        e.run(its)
        ref_map = e.map()
    grp, tiles = _strips(o, I1, I2, n_tiles)
    try:
        assert all(t.info().split == q for t in tiles)

        def rank(t):
            t.init_state(seed=1)
            t.run(5)
            t.prepare()
            for _ in range(2):
                t.init_state(seed=0)
                t.run(20)
            t.init_state(seed=0)
            done, ttr = t.run(its)
            st, mp = t.get_state(), t.map()
            t.init_state(seed=0)
            done2, _, kernel_ms = t.run_timed(its)
            return done, ttr, st, mp, done2, t.get_state(), kernel_ms

        res = ranks(rank, tiles)
        assert grp.calls() > 0
        for t, (done, ttr, st, mp, done2, st2, kms) in zip(tiles, res):
            assert done == its and done2 == its and kms > 0
            np.testing.assert_array_equal(ttr, tr, err_msg=f"tile {t.tile} trace")
            np.testing.assert_array_equal(mp[:, t.col0:t.col1], ref_map[:, t.col0:t.col1])
        _check_strips([r[2] for r in res], tiles, ref)
        _check_strips([r[5] for r in res], tiles, ref)
    finally:
        _close(grp, tiles)


@pytest.mark.parametrize("n_tiles,precision", [(3, "fp64"), (5, "fp32")])
def test_loop_deferred_sequences_with_decay(n_tiles, precision):
    """L = 1 strips with the temperature decay on: replayed sequences +
    leftover sequences, a run_timed in between, then more -- the kernels'
    own counters (Ctl::it_i / done_i / T_i advanced by k_unpack_advance) and
    the finalize's stay the whole grid's."""
    I1, I2, o = _problem("mixture", 1)
    o = dict(o, temperature=0.3, t_decay_every=7)
    init, ref, tr = _whole(I1, I2, o, "mixture", precision, 133, seed=1)
    grp, tiles = _strips(o, I1, I2, n_tiles, precision=precision)
    try:
        def rank(t):
            t.set_state(init.copy())
            d1, t1 = t.run(61)
            d2, _, _ = t.run_timed(11)
            d3, t3 = t.run(61)
            return (d1, d2, d3), t1, t3, t.get_state()

        res = ranks(rank, tiles)
        for t, (d, t1, t3, _) in zip(tiles, res):
            assert d == (61, 11, 61)
            np.testing.assert_array_equal(t1, tr[:61], err_msg=f"tile {t.tile}")
            np.testing.assert_array_equal(t3, tr[72:133], err_msg=f"tile {t.tile}")
        _check_strips([r[3] for r in res], tiles, ref)
    finally:
        _close(grp, tiles)


def _stop_case(k, its=70):
    I1, I2, o = _problem("mixture", 1)
    init, _, tr = _whole(I1, I2, o, "mixture", "fp64", its, seed=1)
    ptd = tr[:, 1]
    tor = 1e9 if k == 0 else float(ptd[k]) * (1 + 1e-12)
    k = int(np.argmax(ptd < tor))
    o = dict(o, tor=tor)
    _, ref, tr_ref = _whole(I1, I2, o, "mixture", "fp64", its, seed=1)
    return I1, I2, o, init, ref, tr_ref, k


@pytest.mark.parametrize("k", [0, 23, 49, 57])
def test_loop_deferred_stop_recovered_across_ranks(k):
    """The stop rule met at sequence row k (the first row, inside the first
    sequence, its last row, inside the leftover sequence) on 4 ranks: every
    rank's k_finalize_seq sees the same all-gathered rows, records the same
    overshoot, and deferred_recover restores the snapshot and re-runs the
    exact step on every rank together -- state, trace and stop iteration are
    the whole grid's; a later run does nothing."""
    I1, I2, o, init, ref, tr_ref, k = _stop_case(k)
    grp, tiles = _strips(o, I1, I2, 4)
    try:
        def rank(t):
            t.set_state(init.copy())
            done, tr = t.run(70)
            stopped = t.info().stopped
            return done, tr, stopped, t.get_state(), t.run(20)[0]

        res = ranks(rank, tiles)
        for t, (done, tr, stopped, _, again) in zip(tiles, res):
            assert done == k + 1 and stopped == 1 and again == 0, (t.tile, done, k)
            np.testing.assert_array_equal(tr, tr_ref, err_msg=f"tile {t.tile}")
        _check_strips([r[3] for r in res], tiles, ref)
    finally:
        _close(grp, tiles)


@pytest.mark.parametrize("k", [5, 30])
def test_loop_deferred_stop_in_run_timed(k):
    I1, I2, o, init, ref, _, k = _stop_case(k, 60)
    grp, tiles = _strips(o, I1, I2, 3)
    try:
        def rank(t):
            t.set_state(init.copy())
            done, _, _ = t.run_timed(60)
            return done, t.info().stopped, t.get_state()

        res = ranks(rank, tiles)
        for t, (done, stopped, _) in zip(tiles, res):
            assert done == k + 1 and stopped == 1
        _check_strips([r[2] for r in res], tiles, ref)
    finally:
        _close(grp, tiles)


@pytest.mark.parametrize("engine,L,precision,n_tiles", [("mixture", 3, "fp64", 3), ("mixture", 2, "fp32", 4),
                                                        ("super", 3, "fp64", 2)])
def test_loop_exact_step_mixture_components(engine, L, precision, n_tiles):
    """L > 1: every iteration is the exact step (launch_step_rccl: the strip's
    k_iter, the ghost send/recv, the all-gather of the tiles' exact totals,
    k_unpack_finalize) -- with the alpha update from iteration 10 and the
    temperature decay every 15: bit-identical to the whole grid."""
    M, N = (96, 128) if engine == "mixture" else (96, 160)
    I1, I2, o = _problem(engine, L, M, N)
    its = 120
    init, ref, tr = _whole(I1, I2, o, engine, precision, its, seed=3)
    grp, tiles = _strips(o, I1, I2, n_tiles, engine, precision)
    try:
        def rank(t):
            t.set_state(init.copy())
            d1, t1 = t.run(70)
            d2, t2 = t.run(its - 70)
            return d1 + d2, np.concatenate([t1, t2]), t.get_state()

        res = ranks(rank, tiles)
        for t, (done, ttr, _) in zip(tiles, res):
            assert done == its
            np.testing.assert_array_equal(ttr, tr, err_msg=f"tile {t.tile}")
        _check_strips([r[2] for r in res], tiles, ref)
    finally:
        _close(grp, tiles)


def test_loop_literal_arith_strips():
    """arith = literal (the MATLAB-expression-order engine) as 3 strips over
    the deferred sequences: the whole grid's bits."""
    I1, I2, o = _problem("mixture", 1)
    o = dict(o, arith="literal", split=1)
    init, ref, tr = _whole(I1, I2, o, "mixture", "fp64", 55, seed=2)
    grp, tiles = _strips(o, I1, I2, 3)
    try:
        def rank(t):
            t.set_state(init.copy())
            done, ttr = t.run(55)
            return done, ttr, t.get_state()

        res = ranks(rank, tiles)
        for t, (done, ttr, _) in zip(tiles, res):
            assert done == 55
            np.testing.assert_array_equal(ttr, tr)
        _check_strips([r[2] for r in res], tiles, ref)
    finally:
        _close(grp, tiles)

