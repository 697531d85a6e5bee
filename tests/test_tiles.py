"""Column-strip tiling (multi-GPU decomposition) on the CPU
model of the kernel: tiles with ghost columns, exchanged every iteration, and
per-tile exact totals summed across tiles must reproduce the whole-grid
solve BIT FOR BIT.  The protocol is the one the RCCL transport
(gqmap_tile_attach_rccl) and the in-process transport (gqmap_tile_group_run)
run on the device; here it runs in one process and over torch.distributed
gloo with two ranks."""
import os

import numpy as np
import pytest

from tests import _golden as G


def _case(L=1, engine="mixture", M=30, N=41):
    from gqmap_opticalflow_amd import flowio
    from oracle import gqmap_np
    I1, I2, gt = flowio.load_pair("rubberwhale")
    sup = engine == "super"
    Mo, No = (4 * M, 4 * N) if sup else (M, N)
    I1, I2, gt = (np.asfortranarray(a[100:100 + Mo, 150:150 + No]) for a in (I1, I2, gt))
    _, _, (minu, maxu, minv, maxv), _ = gqmap_np.flow_to_color(gt)
    o = dict(engine=engine, K=7, L=L, temperature=0.1, drate=0.5, epsn=1e-6, lambdad=1.0,
             lambdas=16.0 if sup else 5.0, minu=minu, maxu=maxu, minv=minv, maxv=maxv, tor=-1.0,
             alpha_start=1 << 30, t_decay_every=3)
    rng = np.random.default_rng(7)
    du, dv = maxu - minu, maxv - minv
    f = lambda a: np.asfortranarray(a)
    st = dict(muu=f(minu + rng.random((M, N, L)) * du), muv=f(minv + rng.random((M, N, L)) * dv),
              sigu=f(rng.random((M, N, L)) + 1), sigv=f(rng.random((M, N, L)) + 1),
              pn=f(0.4 * (2 * rng.random((M, N, L)) - 1)), rou=f(0.4 * (2 * rng.random((M, N, L, 2, 2)) - 1)),
              w=np.zeros(L), alpha=np.full(L, 1.0 / L))
    return I1, I2, o, st


def _gh(K):
    from oracle import oracle
    return oracle.gauss_hermite(K)


def _local(st, n_off, Nl):
    from oracle import oracle
    return oracle.State(*(np.array(st[k][:, n_off:n_off + Nl], order="F", copy=True) if k not in ("w", "alpha")
                          else np.array(st[k], copy=True) for k in G.STATE_KEYS))


def _whole(I1, I2, o, st, its):
    from oracle import oracle
    X, W = _gh(o["K"])
    s = oracle.State(*(np.array(st[k], order="F", copy=True) for k in G.STATE_KEYS))
    done, tr, T = oracle.emu_run(o, I1, I2, s, 1, its, X, W, split=1)
    return s, tr


def _tiled_one_process(I1, I2, o, st, its, n_tiles):
    from oracle import oracle
    X, W = _gh(o["K"])
    M, N, L = st["muu"].shape
    glob = {k: np.array(v, order="F", copy=True) for k, v in st.items()}
    T = o["temperature"]
    trace = []
    for it in range(1, its + 1):
        tot = [0] * (4 + L)
        new = {k: v.copy(order="F") for k, v in glob.items()}
        for t in range(n_tiles):
            col0, col1, n_off, lo, hi, Nl = oracle.tile_geometry(N, n_tiles, t)
            s = _local(glob, n_off, Nl)
            _, _, T_next, totals = oracle.emu_run_tile(o, I1, I2, s, it, 1, X, W, (n_off, lo, hi, N), T=T)
            tot = [a + b for a, b in zip(tot, totals)]
            for k, a in zip(G.STATE_KEYS[:6], s.arrays()[:6]):
                new[k][:, col0:col1] = a[:, lo:hi]
        T = T_next
        glob = new
        cnt = (M - 2) * (N - 2) * L
        trace.append((oracle.from_fix(tot[0]), oracle.from_fix(tot[1]) / cnt, oracle.from_fix(tot[2]) / cnt))
    return glob, np.array(trace)


@pytest.mark.parametrize("n_tiles", [2, 3, 5])
@pytest.mark.parametrize("L,engine", [(1, "mixture"), (3, "mixture"), (2, "super")])
def test_tiles_reproduce_whole_grid_bit_exact(oracle_lib, n_tiles, L, engine):
    I1, I2, o, st = _case(L, engine, *((8, 11) if engine == "super" else (30, 41)))
    its = 5
    ref, tr = _whole(I1, I2, o, st, its)
    glob, ttr = _tiled_one_process(I1, I2, o, st, its, n_tiles)
    for k, a in zip(G.STATE_KEYS[:6], ref.arrays()[:6]):
        np.testing.assert_array_equal(glob[k], a, err_msg=k)
    np.testing.assert_array_equal(ttr, tr)


def test_tile_geometry_matches_library_rule():
    from oracle import oracle
    for Ng, n in ((584, 8), (97, 3), (10, 10), (146, 4)):
        cols = []
        for t in range(n):
            col0, col1, n_off, lo, hi, Nl = oracle.tile_geometry(Ng, n, t)
            assert col1 > col0 and n_off + lo == col0 and n_off + hi == col1 and Nl == hi + (t < n - 1)
            cols.append((col0, col1))
        assert cols[0][0] == 0 and cols[-1][1] == Ng
        assert all(a[1] == b[0] for a, b in zip(cols, cols[1:]))


def _gloo_worker(rank, world, port, its, result_q):
    import torch.distributed as dist
    from oracle import oracle
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        I1, I2, o, st = _case(3, "mixture")
        X, W = _gh(o["K"])
        M, N, L = st["muu"].shape
        col0, col1, n_off, lo, hi, Nl = oracle.tile_geometry(N, world, rank)
        s = _local(st, n_off, Nl)
        T = o["temperature"]
        trace = []
        import torch
        for it in range(1, its + 1):
            _, _, T, totals = oracle.emu_run_tile(o, I1, I2, s, it, 1, X, W, (n_off, lo, hi, N), T=T)
            # ghost columns <- the neighbours' boundary columns: only what the
            # library ships (gqmap_engine.hip HALO_TO_LEFT / HALO_TO_RIGHT):
            # mu, sigma leftwards; mu, sigma and rou of the right edges
            # (dir 2, u and v) rightwards.  pn / rou(dir 1) of a ghost stay stale.
            muu, muv, sigu, sigv, _, rou = s.arrays()[:6]
            views = lambda c, right: ([muu[:, c], muv[:, c], sigu[:, c], sigv[:, c]] +
                                      ([rou[:, c, :, 1, 0], rou[:, c, :, 1, 1]] if right else []))
            pack = lambda c, right: torch.from_numpy(np.concatenate([v.ravel(order="F") for v in views(c, right)]))
            def unpack(c, right, buf):
                off = 0
                for v in views(c, right):
                    n = v.size
                    v[...] = buf[off:off + n].numpy().reshape(v.shape, order="F")
                    off += n
            reqs, bufs = [], {}
            if rank > 0:
                bufs["l"] = torch.empty_like(pack(0, True))
                reqs += [dist.isend(pack(lo, False), rank - 1), dist.irecv(bufs["l"], rank - 1)]
            if rank < world - 1:
                bufs["r"] = torch.empty_like(pack(Nl - 1, False))
                reqs += [dist.isend(pack(hi - 1, True), rank + 1), dist.irecv(bufs["r"], rank + 1)]
            for r in reqs:
                r.wait()
            if "l" in bufs:
                unpack(0, True, bufs["l"])
            if "r" in bufs:
                unpack(Nl - 1, False, bufs["r"])
            # per-tile exact totals -> every rank sums all of them
            allt = [None] * world
            dist.all_gather_object(allt, totals)
            tot = [sum(x) for x in zip(*allt)]
            cnt = (M - 2) * (N - 2) * L
            trace.append((oracle.from_fix(tot[0]), oracle.from_fix(tot[1]) / cnt))
        # bench.py's strong-scaling check: the strips gathered to rank 0
        import bench
        owned = [a[:, lo:hi] for a in s.arrays()[:6]]
        gathered = bench.gather_strips(dist, world, owned, col0, col1)
        if rank == 0:
            result_q.put((gathered, trace))
        else:
            assert gathered is None
    finally:
        dist.destroy_process_group()


def test_tiles_over_gloo_two_ranks(oracle_lib):
    import socket

    import torch.multiprocessing as mp
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    its = 4
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_gloo_worker, args=(r, 2, port, its, q)) for r in range(2)]
    for p in procs:
        p.start()
    gathered, trace = q.get(timeout=300)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    I1, I2, o, st = _case(3, "mixture")
    ref, tr = _whole(I1, I2, o, st, its)
    import bench
    rec = bench.strip_parity(gathered, ref.arrays()[:6], np.array(trace), tr[:, :2], its, len(tr))
    assert rec["bit_exact"], rec
    assert rec["columns_not_covered_once"] == 0 and rec["trace_bit_exact"]
    # the check itself catches a differing strip, a missing column and a different stop
    bad = [(c0, c1, [a.copy() for a in ow]) for c0, c1, ow in gathered]
    bad[1][2][0][3, 0, 0] += 1e-15
    assert bench.strip_parity(bad, ref.arrays()[:6])["mismatch"]["muu"] == 1
    assert not bench.strip_parity(gathered[:1], ref.arrays()[:6])["bit_exact"]
    assert not bench.strip_parity(gathered, ref.arrays()[:6], strip_done=its - 1, whole_done=its)["bit_exact"]


def test_strip_split_mirrors_library_thresholds():
    # engine.strip_split restates gqmap_engine.hip choose_split on one strip's
    # node count; oracle.split_for restates it for a whole grid
    from gqmap_opticalflow_amd import strip_split
    from oracle import oracle
    for M in (30, 60, 120, 240, 388, 480):
        for N in (40, 80, 160, 320, 584, 640):
            assert strip_split(M, N, 1) == oracle.split_for(M, N), (M, N)
    # the headline pair's strips (round 5 mixture thresholds): 2-way Q=1, 4- and 8-way Q=2, 16-way Q=4
    assert [strip_split(388, 584, n) for n in (1, 2, 4, 8, 16)] == [1, 1, 2, 2, 4]
    assert strip_split(30, 40, 2) == 64
    # the coarse-to-fine levels keep their own thresholds
    assert oracle.split_for(240, 320, ctf=True) == 2 and oracle.split_for(240, 320) == 2
    assert oracle.split_for(120, 160, ctf=True) == 4 and oracle.split_for(120, 160) == 2
    assert oracle.split_for(388, 300, ctf=True) == 2 and oracle.split_for(388, 300) == 1


@pytest.mark.parametrize("engine", ["mixture", "super"])
def test_rccl_iteration_ticket_counts_launched_blocks(engine):
    # The last-arrival ticket of an RCCL tile iteration (tile_totals_tail)
    # must count the workgroups the boundary + interior launches actually run.
    # One-column tiles (Q = 64) never launch the ghost-only tile column 0 of
    # a strip with a left neighbour: the ticket must be nblocks - tiles_m there
    # (round-3 advisor finding: it was nblocks, so the totals row was never
    # written).  Host-only geometry (gqmap_debug_strip_launch), no device.
    import ctypes as C
    from gqmap_opticalflow_amd import _lib
    from gqmap_opticalflow_amd.engine import make_options
    lib = _lib.load()
    f = lib.gqmap_debug_strip_launch
    f.restype = C.c_int
    f.argtypes = [C.POINTER(_lib.GqmapOptions), C.c_int, C.c_int, C.c_int, C.c_int, C.POINTER(C.c_int)]
    tile_cols = {64: 1, 16: 4, 8: 4, 4: 8, 2: 8, 1: 16, 0: 8}
    sup = engine == "super"
    cases = ([(120, 160, 2, 0), (120, 160, 3, 0), (480, 640, 4, 0), (120, 160, 2, 16)] if sup else
             [(30, 40, 2, 0), (30, 40, 3, 64), (60, 80, 4, 0), (60, 80, 2, 64), (388, 584, 8, 4),
              (388, 584, 2, 0), (240, 320, 4, 8), (120, 160, 5, 16), (388, 584, 3, -1)])
    hit_wn = False
    for Mo, No, n, split in cases:
        o = make_options(dict(K=11 if sup else 9, L=3 if sup else 1, split=split, minu=-1, maxu=1, minv=-1, maxv=1),
                         engine)
        for t in range(n):
            out = (C.c_int * 5)()
            assert f(C.byref(o), Mo, No, n, t, out) == 0
            nblocks, it_blocks, tm, tn, kq = list(out)
            lpar = o.L if sup else 1
            own_lo = int(t > 0)
            # launched: every tile column from the one holding the first owned
            # node column to the last tile column (a right ghost-only column
            # runs, computing nothing)
            assert it_blocks == (tn - own_lo // tile_cols[kq]) * tm * lpar, (Mo, No, n, t, split, list(out))
            assert nblocks == tn * tm * lpar
            if kq == 64 and t > 0:
                hit_wn = True
                assert it_blocks == nblocks - tm
    assert sup or hit_wn
