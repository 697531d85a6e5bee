"""The dataflow launch of the single-scale engine (policy flow, k_iter_flow):
resident workgroups claim (iteration, tile) items from per-XCD queues and
start a tile's next iteration as soon as it and its four neighbours have
finished the previous one (gqmap_gpu_mixture.m:29-46 is a Jacobi update), a
chunk of up to 50 iterations per launch.  An execution form only: the
arithmetic is k_iter's iter_tile, so the trace and state must be the
per-launch path's bit for bit -- over graph chunks and leftovers, with the
stop rule firing anywhere in a chunk, and after a failed launch (restored
from its snapshot, finished with one launch per iteration)."""
import numpy as np
import pytest

from tests import _golden as G
from tests.test_gpu_parity import _policy

pytestmark = pytest.mark.gpu


def _c2(its_tor=None):
    from gqmap_opticalflow_amd import flow_to_color, flowio
    I1, I2, gt = flowio.load_pair("rubberwhale")
    _, _, (minu, maxu, minv, maxv), _ = flow_to_color(gt)
    o = dict(K=9, L=1, temperature=0.0, drate=0.5, epsn=1e-6, lambdad=1.0, lambdas=5.0,
             minu=minu, maxu=maxu, minv=minv, maxv=maxv)
    return I1, I2, o


def _run(o, I1, I2, its, flow, precision="fp64", seed=0, timed=False, fault=None):
    from gqmap_opticalflow_amd import Engine
    with _policy(flow=1 if flow else 0):
        e = Engine(o, I1, I2, "mixture", precision)
    try:
        e.init_state(seed)
        if fault is not None:
            _inject(e, fault)
        if timed:
            done, _, kms = e.run_timed(its)
            tr = None
        else:
            done, tr = e.run(its)
        return done, tr, e.get_state()
    finally:
        e.close()


def _inject(e, j):
    import ctypes as C
    from gqmap_opticalflow_amd import _lib
    f = _lib.load().gqmap_debug_persist_fault
    f.restype = C.c_int
    f.argtypes = [C.c_void_p, C.c_int]
    assert f(e.ctx, j) == 0


def _same(a, b):
    for k in G.STATE_KEYS:
        np.testing.assert_array_equal(getattr(a, k), getattr(b, k), err_msg=k)
    assert a.it == b.it and a.T == b.T


@pytest.mark.parametrize("precision", ["fp64", "fp32"])
def test_flow_c2_bit_exact_vs_per_launch(precision):
    """The full C2 frame, 133 iterations (two 50-iteration graph chunks, a
    leftover of 33 as one launch): trace and state equal the per-launch
    path's, and run_timed through the dataflow launches ends in the same
    state."""
    I1, I2, o = _c2()
    d0, t0, s0 = _run(o, I1, I2, 133, False, precision)
    d1, t1, s1 = _run(o, I1, I2, 133, True, precision)
    assert d0 == d1 == 133
    np.testing.assert_array_equal(t1, t0)
    _same(s1, s0)
    d2, _, s2 = _run(o, I1, I2, 133, True, precision, timed=True)
    assert d2 == 133
    _same(s2, s0)


def test_flow_temperature_decay_bit_exact():
    """T != 0 with a decay every 7 iterations: each workgroup replays the
    decay up to its item's iteration as fin_apply applies it."""
    I1, I2, o = _c2()
    o = dict(o, temperature=0.3, t_decay_every=7)
    d0, t0, s0 = _run(o, I1, I2, 61, False)
    d1, t1, s1 = _run(o, I1, I2, 61, True)
    np.testing.assert_array_equal(t1, t0)
    _same(s1, s0)


@pytest.mark.parametrize("k", [0, 1, 23, 48, 49, 57])
def test_flow_stop_rule_anywhere_in_a_chunk(k):
    """The stop rule met at iteration k (launch-local row k of a 50-iteration
    chunk, or of the leftover launch): items of iteration k + 1 may already
    have run (they wrote the buffer of state k - 1), later ones see the stop
    word and leave; state, trace and stop iteration are the per-launch
    path's."""
    I1, I2, o = _c2()
    _, tr, _ = _run(o, I1, I2, 70, False)
    tor = 1e9 if k == 0 else float(tr[k, 1]) * (1 + 1e-12)
    k = int(np.argmax(tr[:, 1] < tor))
    o = dict(o, tor=tor)
    d0, t0, s0 = _run(o, I1, I2, 70, False)
    d1, t1, s1 = _run(o, I1, I2, 70, True)
    assert d0 == d1 == k + 1
    np.testing.assert_array_equal(t1, t0)
    _same(s1, s0)


@pytest.mark.parametrize("j", [0, 7, 49])
def test_flow_failed_launch_recovers_bit_exact(j):
    """A dataflow launch that gives up (the failure word raised at the first
    item of iteration j, as a spin timeout raises it) leaves the state the
    chunk started from to the host, which restores it and finishes with one
    launch per iteration: the per-launch path's bits."""
    I1, I2, o = _c2()
    d0, t0, s0 = _run(o, I1, I2, 80, False)
    d1, t1, s1 = _run(o, I1, I2, 80, True, fault=j)
    assert d1 == 80
    np.testing.assert_array_equal(t1, t0)
    _same(s1, s0)


@pytest.mark.parametrize("scale,q", [(1.0, 1), (0.5, 2), (0.25, 4)])
def test_flow_ctf_levels_bit_exact(scale, q):
    """The coarse-to-fine levels the dataflow launch takes (fp64, L = 1):
    Grove3 at full resolution (Q = 1), 240 x 320 (Q = 2) and 120 x 160
    (Q = 4, its table staged in LDS per item), with the truth set (the
    AEPE trace of gqmap_ctf.m:38): trace, AEPE and state equal the
    per-launch path's over 61 iterations."""
    from gqmap_opticalflow_amd import Engine, ctf_options, flow_to_color, flowio, imresize
    I1, I2, gt = flowio.load_pair("Grove3")
    _, flo, (minu, maxu, minv, maxv), _ = flow_to_color(gt)
    if scale != 1.0:
        I1, I2 = imresize(I1, scale), imresize(I2, scale)
    o = ctf_options(its=61, minu=minu * scale, maxu=maxu * scale, minv=minv * scale, maxv=maxv * scale)
    out = []
    for flow in (0, 1):
        with _policy(flow=flow):
            e = Engine(o, I1, I2, "ctf")
        try:
            assert e.info().split == q
            e.set_truth(np.asfortranarray(flo * scale))
            e.init_state(3)
            done, tr, ae = e.run_aepe(61)
            out.append((done, tr, ae, e.get_state()))
        finally:
            e.close()
    (d0, t0, a0, s0), (d1, t1, a1, s1) = out
    assert d0 == d1 == 61
    np.testing.assert_array_equal(t1, t0)
    np.testing.assert_array_equal(a1, a0)
    _same(s1, s0)


def test_flow_c3_pyramid_same_flow():
    """BASELINE C3 (Grove3, 5 levels) with every qualifying level on the
    dataflow launch: the final flow and every level's intermediates equal
    the per-launch pyramid's."""
    from gqmap_opticalflow_amd import C3_SCALES, Pyramid, ctf_options, flow_to_color, flowio
    I1, I2, gt = flowio.load_pair("Grove3")
    _, _, (minu, maxu, minv, maxv), _ = flow_to_color(gt)
    opts = ctf_options(its=40, minu=minu, maxu=maxu, minv=minv, maxv=maxv)
    res = []
    for flow in (0, 1):
        with _policy(flow=flow):
            p = Pyramid(opts, C3_SCALES)
            p.set_images(I1, I2)
        try:
            f, its, _ = p.run(seed=5)
            res.append((f, its, [p.level(l) for l in range(len(C3_SCALES))]))
        finally:
            p.close()
    (f0, i0, l0), (f1, i1, l1) = res
    assert i0 == i1
    np.testing.assert_array_equal(f1, f0)
    for a, b in zip(l0, l1):
        for k in ("I1w", "I2", "flow", "warp"):
            np.testing.assert_array_equal(b[k], a[k], err_msg=k)


def test_flow_literal_order_forced_bit_exact():
    """The literal-order engine (arith = literal) on the dataflow launch when
    forced (policy flow = 1; its default stays per launch): the per-launch
    literal engine's bits over a graph chunk and a leftover."""
    I1, I2, o = _c2()
    o = dict(o, arith="literal", split=1)
    d0, t0, s0 = _run(o, I1, I2, 61, False)
    d1, t1, s1 = _run(o, I1, I2, 61, True)
    assert d0 == d1 == 61
    np.testing.assert_array_equal(t1, t0)
    _same(s1, s0)


@pytest.mark.parametrize("alpha_start,its", [(500, 61), (10, 61)])
def test_flow_super_mixture_components_bit_exact(alpha_start, its):
    """BASELINE C4 (Urban3, super engine, L = 3, K = 11, Q = 4): each mixture
    component of a tile is its own item.  Past alpha_start the alpha update
    of finalize(j - 1) feeds iteration j, so items then wait for it (lag 1
    instead of 2); with the temperature decay every 15 iterations.  The
    per-launch path's trace, alpha and state bit for bit."""
    from gqmap_opticalflow_amd import Engine, flow_to_color, flowio
    I1, I2, gt = flowio.load_pair("Urban3")
    _, _, (minu, maxu, minv, maxv), _ = flow_to_color(gt)
    o = dict(K=11, L=3, temperature=0.2, drate=0.75, epsn=1e-6, lambdad=1.0, lambdas=16.0,
             minu=minu, maxu=maxu, minv=minv, maxv=maxv, alpha_start=alpha_start, t_decay_every=15)
    out = []
    for flow in (0, 1):
        with _policy(flow=flow):
            e = Engine(o, I1, I2, "super")
        try:
            assert e.info().split == 4 and e.dataflow() == bool(flow)
            e.init_state(4)
            done, tr = e.run(its)
            out.append((done, tr, e.get_state()))
        finally:
            e.close()
    (d0, t0, s0), (d1, t1, s1) = out
    assert d0 == d1 == its
    np.testing.assert_array_equal(t1, t0)
    _same(s1, s0)


def test_flow_wide_frame_bit_exact():
    """A frame beyond GQ_FLOW_WIDE_ITEMS items per iteration (RubberWhale
    upsampled 3x, 1164 x 1752: 8030 tiles) takes the 3-wave instantiation of
    the dataflow launch (C5's frames): per-launch trace and state bit for bit
    over a graph chunk and a leftover."""
    from gqmap_opticalflow_amd import flow_to_color, flowio
    I1, I2, gt = flowio.load_pair_scaled("rubberwhale", 3.0)
    _, _, (minu, maxu, minv, maxv), _ = flow_to_color(gt)
    o = dict(K=9, L=1, temperature=0.0, drate=0.5, epsn=1e-6, lambdad=1.0, lambdas=5.0,
             minu=minu, maxu=maxu, minv=minv, maxv=maxv)
    d0, t0, s0 = _run(o, I1, I2, 61, False)
    d1, t1, s1 = _run(o, I1, I2, 61, True)
    assert d0 == d1 == 61
    np.testing.assert_array_equal(t1, t0)
    _same(s1, s0)
