"""Column-strip tiles on the device (gqmap_create_tile): the in-process
transport (gqmap_tile_group_run, several tiles on one GPU exchanging ghost
columns and exact totals) and a one-rank RCCL communicator must reproduce
the whole-grid engine BIT FOR BIT."""
import numpy as np
import pytest

from tests import _golden as G

pytestmark = pytest.mark.gpu


def _problem(engine="mixture", L=1, M=96, N=128):
    from gqmap_opticalflow_amd import flow_to_color, flowio
    name = "Urban3" if engine == "super" else "rubberwhale"
    I1, I2, gt = flowio.load_pair(name)
    I1, I2, gt = (np.asfortranarray(a[100:100 + M, 120:120 + N]) for a in (I1, I2, gt))
    _, _, (minu, maxu, minv, maxv), _ = flow_to_color(gt)
    sup = engine == "super"
    o = dict(K=11 if sup else 9, L=L, temperature=0.2 if sup else 0.05, drate=0.75, epsn=1e-6, lambdad=1.0,
             lambdas=16.0 if sup else 5.0, minu=minu, maxu=maxu, minv=minv, maxv=maxv, alpha_start=10,
             t_decay_every=15)
    return I1, I2, o


def _whole(I1, I2, o, engine, precision, its, seed):
    from gqmap_opticalflow_amd import Engine
    with Engine(o, I1, I2, engine, precision) as e:
        e.init_state(seed)
        init = e.get_state()
        done, tr = e.run(its)
        return init, e.get_state(), tr


def _assemble(tiles, getter):
    out = None
    for t in tiles:
        s = getter(t)
        if out is None:
            out = s
        else:
            for k in G.STATE_KEYS[:6]:
                getattr(out, k)[:, t.col0:t.col1] = getattr(s, k)[:, t.col0:t.col1]
    return out


@pytest.mark.parametrize("engine,L,precision,n_tiles", [("mixture", 1, "fp64", 2), ("mixture", 1, "fp64", 5),
                                                        ("mixture", 3, "fp32", 3), ("super", 3, "fp64", 4),
                                                        ("super", 2, "fp32", 2)])
def test_tile_group_bit_exact_vs_whole_grid(engine, L, precision, n_tiles):
    from gqmap_opticalflow_amd import Engine, tile_group_run
    M, N = (96, 128) if engine == "mixture" else (96, 160)
    I1, I2, o = _problem(engine, L, M, N)
    its = 40
    init, ref, tr = _whole(I1, I2, o, engine, precision, its, seed=3)
    tiles = [Engine(o, I1, I2, engine, precision, n_tiles=n_tiles, tile=t) for t in range(n_tiles)]
    try:
        for t in tiles:
            t.init_state(3)  # global RNG indexing: each tile draws its columns of the whole grid
        got0 = _assemble(tiles, lambda t: t.get_state())
        for k in G.STATE_KEYS[:6]:
            np.testing.assert_array_equal(getattr(got0, k), getattr(init, k), err_msg="init " + k)
        done, ttr = tile_group_run(tiles, its)
        assert done == its
        np.testing.assert_array_equal(ttr, tr)
        got = _assemble(tiles, lambda t: t.get_state())
        for k in G.STATE_KEYS:
            np.testing.assert_array_equal(getattr(got, k), getattr(ref, k), err_msg=k)
        mp = np.zeros((tiles[0].M, tiles[0].N, 2), order="F")
        for t in tiles:
            m = t.map()
            mp[:, t.col0:t.col1] = m[:, t.col0:t.col1]
        with Engine(o, I1, I2, engine, precision) as e:
            e.set_state(ref)
            np.testing.assert_array_equal(mp, e.map())
    finally:
        for t in tiles:
            t.close()


def test_tile_set_state_from_full_grid():
    from gqmap_opticalflow_amd import Engine, tile_group_run
    I1, I2, o = _problem()
    init, ref, tr = _whole(I1, I2, o, "mixture", "fp64", 25, seed=5)
    tiles = [Engine(o, I1, I2, n_tiles=3, tile=t) for t in range(3)]
    for t in tiles:
        t.set_state(init.copy())
    tile_group_run(tiles, 25)
    got = _assemble(tiles, lambda t: t.get_state())
    for k in G.STATE_KEYS:
        np.testing.assert_array_equal(getattr(got, k), getattr(ref, k), err_msg=k)
    with pytest.raises(Exception, match="attach RCCL"):
        tiles[0].run(1)
    for t in tiles:
        t.close()


def test_single_rank_rccl_tile_matches_whole_grid():
    # exercises the RCCL transport (communicator, in-place all-gather of the
    # exact totals, graph capture of the collective) on one GPU
    from gqmap_opticalflow_amd import Engine, comm_unique_id
    I1, I2, o = _problem("mixture", 3)
    init, ref, tr = _whole(I1, I2, o, "mixture", "fp64", 120, seed=1)
    e = Engine(o, I1, I2, n_tiles=1, tile=0)
    try:
        e.attach_rccl(comm_unique_id())
        e.set_state(init.copy())
        done, t2 = e.run(120)  # two 50-iteration graph replays + 20 launches
        np.testing.assert_array_equal(t2, tr)
        got = e.get_state()
        for k in G.STATE_KEYS:
            np.testing.assert_array_equal(getattr(got, k), getattr(ref, k), err_msg=k)
    finally:
        e.close()


def test_c5_frame_eight_tiles_bit_exact_vs_whole_grid():
    """BASELINE C5's unit of work: one Middlebury pair upsampled 4x
    (RubberWhale, 1552x2336, imresize of the uint8 RGB frames as
    optical_flow_temp.m:7-8 does) split into 8 column-strip tiles -- the
    driver's 8-GPU layout -- on one GPU through the in-process transport:
    bit-identical to the whole-grid solve after 20 iterations."""
    from gqmap_opticalflow_amd import Engine, flow_to_color, flowio, tile_group_run
    I1, I2, gt = flowio.load_pair_scaled("rubberwhale", 4.0)
    assert I1.shape == (1552, 2336)
    _, _, (minu, maxu, minv, maxv), _ = flow_to_color(gt)
    o = dict(K=9, L=1, temperature=0.0, drate=0.5, epsn=1e-6, lambdad=1.0, lambdas=5.0,
             minu=minu, maxu=maxu, minv=minv, maxv=maxv)
    its, n = 20, 8
    init, ref, tr = _whole(I1, I2, o, "mixture", "fp64", its, seed=0)
    tiles = [Engine(o, I1, I2, n_tiles=n, tile=t) for t in range(n)]
    try:
        for t in tiles:
            t.init_state(0)
        done, ttr = tile_group_run(tiles, its)
        assert done == its
        np.testing.assert_array_equal(ttr, tr)
        for t in tiles:
            s = t.get_state()
            for k in G.STATE_KEYS[:6]:
                np.testing.assert_array_equal(getattr(s, k)[:, t.col0:t.col1], getattr(ref, k)[:, t.col0:t.col1],
                                              err_msg=f"tile {t.tile} {k}")
    finally:
        for t in tiles:
            t.close()


def test_tile_group_long_run_trace_drained():
    """gqmap_tile_group_run copies the device trace ring out every 64
    iterations: a run longer than the ring (8192) returns every row."""
    from gqmap_opticalflow_amd import Engine, tile_group_run
    I1, I2, o = _problem("mixture", 1, 24, 40)
    its = 8192 + 150
    with Engine(dict(o, tor=0.0), I1, I2) as e:
        e.init_state(2)
        init = e.get_state()
        done, tr = e.run(its)
    assert done == its
    tiles = [Engine(dict(o, tor=0.0), I1, I2, n_tiles=2, tile=t) for t in range(2)]
    try:
        for t in tiles:
            t.set_state(init.copy())
        done, ttr = tile_group_run(tiles, its)
        assert done == its and ttr.shape == (its, 3)
        np.testing.assert_array_equal(ttr, tr)
    finally:
        for t in tiles:
            t.close()


def test_host_staged_tiles_three_processes_bit_exact(tmp_path):
    """Three processes share cuda:0, each holding one column-strip tile of
    libgqmap (L=3 mixture, alpha update and temperature decay inside the
    run).  Boundary columns (4 planes leftwards, 6 rightwards) and exact
    totals travel through torch.distributed gloo between
    gqmap_tile_exchange_begin and _end -- the library's own pack / unpack and
    cross-process finalize, as a multi-node MPI caller would drive them.
    Bit-identical to the whole-grid solve."""
    import os
    import socket
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    I1, I2, o = _problem("mixture", 3, 96, 128)
    its, world = 30, 3
    init, ref, tr = _whole(I1, I2, o, "mixture", "fp64", its, seed=3)
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    env = dict(os.environ, PYTHONPATH=root + os.pathsep + os.environ.get("PYTHONPATH", ""))
    procs = [subprocess.Popen([sys.executable, "-m", "tests._tile_host_worker", str(r), str(world), str(port),
                               str(its), str(tmp_path / f"r{r}.npz")], cwd=root, env=env)
             for r in range(world)]
    try:
        for p in procs:
            assert p.wait(timeout=200) == 0
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    cols = []
    for r in range(world):
        d = np.load(tmp_path / f"r{r}.npz")
        c0, c1 = int(d["col0"]), int(d["col1"])
        cols.append((c0, c1))
        np.testing.assert_array_equal(d["trace"], tr, err_msg=f"rank {r} trace")
        for k in ("muu", "muv", "sigu", "sigv", "pn", "rou"):
            np.testing.assert_array_equal(d[k], getattr(ref, k)[:, c0:c1], err_msg=f"rank {r} {k}")
        np.testing.assert_array_equal(d["alpha"], ref.alpha)
    assert cols[0][0] == 0 and cols[-1][1] == ref.muu.shape[1]


@pytest.mark.parametrize("n_tiles", [2, 4, 8])
def test_c2_pair_strips_at_per_strip_split_bit_exact(n_tiles):
    """The strong-scaling layout of the headline pair (bench.py strong_scaling):
    the full RubberWhale frame (388x584) as n_tiles column strips whose lanes
    per node come from ONE strip (strip_split: Q = 1 for 2 strips, 2 for 4 and 8),
    on one GPU through the in-process transport -- bit-identical to the
    whole-grid solve run at the same Q."""
    from gqmap_opticalflow_amd import Engine, flow_to_color, flowio, strip_split, tile_group_run
    I1, I2, gt = flowio.load_pair("rubberwhale")
    _, _, (minu, maxu, minv, maxv), _ = flow_to_color(gt)
    q = strip_split(*I1.shape, n_tiles)
    assert q == {2: 1, 4: 2, 8: 2}[n_tiles]
    o = dict(K=9, L=1, temperature=0.0, drate=0.5, epsn=1e-6, lambdad=1.0, lambdas=5.0,
             minu=minu, maxu=maxu, minv=minv, maxv=maxv, split=q)
    its = 30
    init, ref, tr = _whole(I1, I2, o, "mixture", "fp64", its, seed=0)
    tiles = [Engine(o, I1, I2, n_tiles=n_tiles, tile=t) for t in range(n_tiles)]
    try:
        assert all(t.info().split == q for t in tiles)
        for t in tiles:
            t.init_state(0)
        done, ttr = tile_group_run(tiles, its)
        assert done == its
        np.testing.assert_array_equal(ttr, tr)
        for t in tiles:
            s = t.get_state()
            for k in G.STATE_KEYS[:6]:
                np.testing.assert_array_equal(getattr(s, k)[:, t.col0:t.col1], getattr(ref, k)[:, t.col0:t.col1],
                                              err_msg=f"tile {t.tile} {k}")
    finally:
        for t in tiles:
            t.close()


def test_single_rank_rccl_deferred_step_l1():
    """L = 1 RCCL tiles run deferred-totals sequences (launch_seq_deferred:
    per iteration only the k_iter launches, the exchange and the unpack; the
    totals of a whole sequence all-gathered once and finalized row by row at
    its end): bit-identical to the whole grid over replayed graphs + leftover
    sequences with the temperature decay on, and a run_timed (the same
    sequences, instrumented) in between keeps the counters."""
    from gqmap_opticalflow_amd import Engine, comm_unique_id
    I1, I2, o = _problem("mixture", 1)
    o = dict(o, temperature=0.3, t_decay_every=7)
    init, ref, tr = _whole(I1, I2, o, "mixture", "fp64", 133, seed=1)
    e = Engine(o, I1, I2, n_tiles=1, tile=0)
    try:
        e.attach_rccl(comm_unique_id())
        e.set_state(init.copy())
        done, t1 = e.run(61)   # one graph + 11 launches
        done2, _, _ = e.run_timed(11)
        done3, t3 = e.run(61)
        assert (done, done2, done3) == (61, 11, 61)
        np.testing.assert_array_equal(t1, tr[:61])
        np.testing.assert_array_equal(t3, tr[72:133])
        got = e.get_state()
        for k in G.STATE_KEYS:
            np.testing.assert_array_equal(getattr(got, k), getattr(ref, k), err_msg=k)
        assert got.T == ref.T and got.it == ref.it
    finally:
        e.close()


@pytest.mark.parametrize("k", [0, 23, 49, 57])
def test_single_rank_rccl_deferred_stop(k):
    # the stop rule met at row k (inside a graph chunk, at its last iteration,
    # in the leftover sequence): the sequence's iterations after it are undone
    # (snapshot + exact re-run, deferred_recover); the state and trace are the
    # whole grid's after k + 1 iterations
    from gqmap_opticalflow_amd import Engine, comm_unique_id
    I1, I2, o = _problem("mixture", 1)
    init, _, tr = _whole(I1, I2, o, "mixture", "fp64", 70, seed=1)
    ptd = tr[:, 1]
    tor = 1e9 if k == 0 else float(ptd[k]) * (1 + 1e-12)
    k = int(np.argmax(ptd < tor))
    o = dict(o, tor=tor)
    _, ref, tr_ref = _whole(I1, I2, o, "mixture", "fp64", 70, seed=1)
    e = Engine(o, I1, I2, n_tiles=1, tile=0)
    try:
        e.attach_rccl(comm_unique_id())
        e.set_state(init.copy())
        done, t2 = e.run(70)
        assert done == k + 1 and e.info().stopped == 1
        np.testing.assert_array_equal(t2, tr_ref)
        got = e.get_state()
        for key in G.STATE_KEYS:
            np.testing.assert_array_equal(getattr(got, key), getattr(ref, key), err_msg=key)
        assert e.run(20)[0] == 0
    finally:
        e.close()


@pytest.mark.parametrize("k", [5, 30])
def test_single_rank_rccl_deferred_stop_in_run_timed(k):
    # the instrumented replay runs the same deferred sequences: a stop inside
    # one is recovered the same way
    from gqmap_opticalflow_amd import Engine, comm_unique_id
    I1, I2, o = _problem("mixture", 1)
    init, _, tr = _whole(I1, I2, o, "mixture", "fp64", 60, seed=1)
    tor = float(tr[k, 1]) * (1 + 1e-12)
    k = int(np.argmax(tr[:, 1] < tor))
    o = dict(o, tor=tor)
    _, ref, _ = _whole(I1, I2, o, "mixture", "fp64", 60, seed=1)
    e = Engine(o, I1, I2, n_tiles=1, tile=0)
    try:
        e.attach_rccl(comm_unique_id())
        e.set_state(init.copy())
        done, _, _ = e.run_timed(60)
        assert done == k + 1 and e.info().stopped == 1
        got = e.get_state()
        for key in G.STATE_KEYS:
            np.testing.assert_array_equal(getattr(got, key), getattr(ref, key), err_msg=key)
    finally:
        e.close()
