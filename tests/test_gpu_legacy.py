"""legacy/gqmap_cpu.m on the device (gqmap_cpu_run) against the C
restatement: plain fp64 in the same operation order, so bit-identical."""
import os

import numpy as np
import pytest

from tests import _golden as G

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("dta", [np.inf, 2.5])
def test_legacy_device_bit_exact_vs_oracle(dta):
    from gqmap_opticalflow_amd import gauss_hermite, gqmap_cpu
    from oracle import oracle
    d = dict(np.load(os.path.join(G.GOLDEN, "legacy_cpu.npz"), allow_pickle=False))
    o = dict(its=30, K=9, var=1.0, gama=1.0, dta=dta)
    X, W = gauss_hermite(9)
    ref = oracle.cpu_run(o, d["flow"], d["sigma0"], X, W)
    got = gqmap_cpu(o, d["flow"], sigma0=d["sigma0"], return_trace=True)
    for a, b, k in zip(got, ref, ("mu", "sigma", "rou", "trace")):
        np.testing.assert_array_equal(a, b, err_msg=k)


def test_legacy_c1_dimetrodon_50_iterations():
    """BASELINE config C1: Dimetrodon 388x584 GT flow (unknowns zeroed), 50
    iterations, K=9, sigma0 = U + 2 from the library RNG (seed 0)."""
    from gqmap_opticalflow_amd import flow_to_color, flowio, gauss_hermite, gqmap_cpu, rand_uniform
    from oracle import oracle
    gt = flowio.load_pair("Dimetrodon")[2]
    _, flo, _, unk = flow_to_color(gt)
    M, N, _ = flo.shape
    sg0 = np.asfortranarray(rand_uniform(0, 3, 2 * M * N).reshape((M, N, 2), order="F") + 2)
    o = dict(its=50, K=9)
    mu, sg, rou, tr = gqmap_cpu(o, flo, seed=0, return_trace=True)
    X, W = gauss_hermite(9)
    r = oracle.cpu_run(o, flo, sg0, X, W)
    np.testing.assert_array_equal(mu, r[0])
    np.testing.assert_array_equal(sg, r[1])
    np.testing.assert_array_equal(rou, r[2])
    np.testing.assert_array_equal(tr, r[3])
    e = np.sqrt(((mu - flo) ** 2).sum(axis=2))[~unk].mean()
    print(f"C1: {tr.shape[0]} its, mean |mu - flow| {e:.4f}, last max|dmu| {tr[-1, 0]:.3e}")


@pytest.mark.parametrize("shape", [(37, 41), (5, 7), (61, 3)])
def test_legacy_ragged_sizes_bit_exact(shape):
    """2*M*N not a multiple of 64 (the last workgroup of k_legacy_update has
    idle threads that still take part in the block maximum): bit-exact vs the
    C restatement, traces (the running maxima) included."""
    from gqmap_opticalflow_amd import gauss_hermite, gqmap_cpu, legacy
    from oracle import oracle
    M, N = shape
    assert (2 * M * N) % 64 != 0
    rng = np.random.default_rng(7)
    flow = np.asfortranarray(rng.normal(0, 3, (M, N, 2)))
    sg0 = np.asfortranarray(rng.uniform(0, 1, (M, N, 2)) + 2)
    o = dict(its=120, K=9, var=1.0, gama=1.0, dta=np.inf, min_its=100, tor=1e-3)
    X, W = gauss_hermite(9)
    ref = oracle.cpu_run(o, flow, sg0, X, W)
    got = gqmap_cpu(o, flow, sigma0=sg0, return_trace=True)
    for a, b, k in zip(got, ref, ("mu", "sigma", "rou", "trace")):
        np.testing.assert_array_equal(a, b, err_msg=k)
    legacy.release()
    with pytest.raises(ValueError):
        gqmap_cpu(o, flow, sigma0=sg0[:, :, 0])


def test_legacy_device_arrays_same_bits_as_host_arrays():
    """gqmap_cpu_run_device (flow resident in HBM, outputs left there) gives
    the host-array call's results bit for bit, with a given sigma0 and with the
    library RNG, and stops at the same iteration (the stop rule, :70)."""
    import torch
    from gqmap_opticalflow_amd import gqmap_cpu, gqmap_cpu_device
    rng = np.random.default_rng(11)
    M, N = 45, 52
    flow = np.asfortranarray(rng.normal(0, 2, (M, N, 2)))
    sg0 = np.asfortranarray(rng.uniform(0, 1, (M, N, 2)) + 2)
    dev = torch.device("cuda", 0)
    flow_d = torch.from_numpy(flow).to(dev)
    sg0_d = torch.from_numpy(sg0).to(dev)
    assert flow_d.stride() == (1, M, M * N)
    for kw_h, kw_d, its in (({"sigma0": sg0}, {"sigma0": sg0_d}, 40), ({"seed": 3}, {"seed": 3}, 150)):
        o = dict(its=its, K=9, min_its=100, tor=1e-1)
        h = gqmap_cpu(o, flow, return_trace=True, **kw_h)
        d = gqmap_cpu_device(o, flow_d, return_trace=True, **kw_d)
        for a, b, k in zip(h, d, ("mu", "sigma", "rou", "trace")):
            np.testing.assert_array_equal(a, b.cpu().numpy(), err_msg=k)
    # the input flow is left as it was
    np.testing.assert_array_equal(flow_d.cpu().numpy(), flow)


def test_legacy_device_arrays_rejects_host_and_row_major():
    import torch
    from gqmap_opticalflow_amd import gqmap_cpu_device, legacy
    from gqmap_opticalflow_amd._lib import load
    import ctypes as C
    flow = np.zeros((8, 9, 2), order="F")
    with pytest.raises(ValueError):  # row-major device tensor
        gqmap_cpu_device({}, torch.zeros((8, 9, 2), dtype=torch.float64, device="cuda"))
    with pytest.raises(TypeError):
        gqmap_cpu_device({}, torch.from_numpy(flow))  # host tensor
    # the C-ABI itself refuses host pointers
    o = legacy.cpu_options({"its": 2})
    out = [np.zeros((8, 9, 2), order="F"), np.zeros((8, 9, 2), order="F"), np.zeros((8, 9, 2, 2), order="F")]
    rc = load().gqmap_cpu_run_device(C.byref(o), flow.ctypes.data, 8, 9, None, C.c_uint64(0),
                                     *[a.ctypes.data for a in out], None, None, 0)
    assert rc != 0
    # ... and outputs that overlap an input or each other (partial overlaps
    # included), with every array on the device
    n = 8 * 9 * 2
    buf = torch.zeros(6 * n, dtype=torch.float64, device="cuda")
    base = buf.data_ptr()
    f_, mu_, sg_, rou_ = base, base + 8 * n, base + 16 * n, base + 24 * n
    ok = load().gqmap_cpu_run_device(C.byref(o), f_, 8, 9, None, C.c_uint64(0), mu_, sg_, rou_, None, None, 0)
    assert ok == 0, load().gqmap_last_error()
    for args in ((f_, f_ + 8 * 8, sg_, rou_), (f_, mu_, mu_ + 8 * n - 8, rou_), (f_, mu_, sg_, sg_ + 8)):
        rc = load().gqmap_cpu_run_device(C.byref(o), args[0], 8, 9, None, C.c_uint64(0), *args[1:], None, None, 0)
        assert rc != 0 and b"overlap" in load().gqmap_last_error()


@pytest.mark.parametrize("name", ["Hydrangea", "rubberwhale"])
def test_legacy_other_pairs_device_arrays_bit_exact(name):
    """C1's 50 iterations on the other 584x388 GT flows, through the
    device-array entry point, against the C restatement."""
    import torch
    from gqmap_opticalflow_amd import flow_to_color, flowio, gauss_hermite, gqmap_cpu_device, rand_uniform
    from oracle import oracle
    gt = flowio.load_pair(name)[2]
    _, flo, _, unk = flow_to_color(gt)
    M, N, _ = flo.shape
    sg0 = np.asfortranarray(rand_uniform(0, 3, 2 * M * N).reshape((M, N, 2), order="F") + 2)
    o = dict(its=50, K=9)
    mu, sg, rou, tr = gqmap_cpu_device(o, torch.from_numpy(np.asfortranarray(flo)).to("cuda:0"), seed=0,
                                       return_trace=True)
    X, W = gauss_hermite(9)
    r = oracle.cpu_run(o, flo, sg0, X, W, nthreads=min(16, os.cpu_count() or 1))
    for a, b, k in zip((mu, sg, rou, tr), r, ("mu", "sigma", "rou", "trace")):
        np.testing.assert_array_equal(a.cpu().numpy(), b, err_msg=k)
