"""Coarse-to-fine path on the device (gqmap_imresize / gqmap_warp_image /
gqmap_pyramid through the C ABI) against the oracle's restatement.

The plumbing kernels are plain fp64 with contraction off in the oracle's
operation order, and each level runs the CTF engine, which is bit-identical
to the CPU model of the kernel (oracle/gqmap_emul.cpp): so every level's
warped frame, flow and warp must be BIT-IDENTICAL to the oracle pipeline fed
the same seeded per-level initial states."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _rand(shape, seed=0):
    return np.asfortranarray(np.random.default_rng(seed).random(shape) * 255)


@pytest.mark.parametrize("scale", [1 / 16, 1 / 8, 0.25, 0.5, 1.0, 2.0])
@pytest.mark.parametrize("shape", [(480, 640), (37, 29), (30, 40, 2)])
def test_imresize_device_bit_exact(scale, shape):
    from gqmap_opticalflow_amd import imresize
    from oracle import oracle
    A = _rand(shape, 1)
    np.testing.assert_array_equal(imresize(A, scale), oracle.imresize(A, scale))


@pytest.mark.parametrize("fill", [False, True])
def test_warp_image_device_bit_exact(fill):
    from gqmap_opticalflow_amd import warp_image
    from oracle import oracle
    rng = np.random.default_rng(3)
    V = _rand((120, 160), 4)
    warp = np.asfortranarray(rng.normal(scale=4.0, size=(120, 160, 2)))
    warp[:6, :, 1] = -9.0
    a = warp_image(V, warp, fill)
    b = oracle.warp_image(V, warp, fill)
    np.testing.assert_array_equal(a, b)  # NaN positions included
    assert np.isnan(a).any() != fill


def _pipeline_pair(name, crop=None):
    from gqmap_opticalflow_amd import flow_to_color, flowio
    I1, I2, gt = flowio.load_pair(name)
    if crop:
        r0, c0, M, N = crop
        I1, I2, gt = (np.asfortranarray(a[r0:r0 + M, c0:c0 + N]) for a in (I1, I2, gt))
    _, flo, (minu, maxu, minv, maxv), unk = flow_to_color(gt)
    return I1, I2, flo, unk, dict(minu=minu, maxu=maxu, minv=minv, maxv=maxv)


def _oracle_pipeline(opts, I1, I2, scales, seed, precision):
    from gqmap_opticalflow_amd import gauss_hermite, initial_state
    from oracle import oracle

    def init_fn(l, lo, M, N):  # host replica of gqmap_init_state(seed + level)
        st = initial_state(lo, M, N, seed=seed + l, engine="ctf")
        return oracle.State(st.muu, st.muv, st.sigu, st.sigv, st.pn, st.rou, st.w, st.alpha)

    X, W = gauss_hermite(opts["K"])
    return oracle.ctf_pipeline(opts, I1, I2, scales, init_fn, solver="emu", X=X, W=W,
                               nthreads=min(16, os.cpu_count() or 1), fp32=precision == "fp32")


def _check_levels(p, levels, warp, flow):
    for l, lv in enumerate(levels):
        g = p.level(l)
        for k in ("I2", "I1w", "flow", "warp"):
            np.testing.assert_array_equal(g[k], lv[k], err_msg=f"level {l} {k}")
    np.testing.assert_array_equal(flow, warp)


@pytest.mark.parametrize("precision", ["fp64", "fp32"])
def test_pyramid_bit_exact_vs_oracle_pipeline(precision):
    from gqmap_opticalflow_amd import Pyramid, ctf_options
    I1, I2, _, _, rng = _pipeline_pair("Grove3", (150, 200, 64, 96))
    scales = (0.25, 0.5, 1.0)
    opts = ctf_options(its=30, **rng)
    warp, levels = _oracle_pipeline(opts, I1, I2, scales, 7, precision)
    with Pyramid(opts, scales, precision) as p:
        p.set_images(I1, I2)
        flow, its, ms = p.run(seed=7)
        assert its == [lv["its"] for lv in levels]
        _check_levels(p, levels, warp, flow)
        # a second run from the same seed repeats bit for bit
        flow2, _, _ = p.run(seed=7)
        np.testing.assert_array_equal(flow2, flow)


def test_pyramid_grove3_five_levels_bit_exact():
    """BASELINE config C3 geometry: Grove3 480x640, 5 levels 30x40 .. 480x640
    (few iterations per level to keep the CPU model short)."""
    from gqmap_opticalflow_amd import C3_SCALES, Pyramid, aepe, ctf_options
    I1, I2, flo, unk, rng = _pipeline_pair("Grove3")
    opts = ctf_options(its=12, **rng)
    warp, levels = _oracle_pipeline(opts, I1, I2, C3_SCALES, 0, "fp64")
    with Pyramid(opts, C3_SCALES) as p:
        p.set_images(I1, I2)
        flow, its, ms = p.run(seed=0)
        assert [p.level(l)["I1w"].shape for l in range(5)] == [(30, 40), (60, 80), (120, 160),
                                                               (240, 320), (480, 640)]
        _check_levels(p, levels, warp, flow)
    print(f"C3 geometry, 12 its/level: AEPE {aepe(flo, flow, unk):.4f}, {ms:.1f} ms")


def test_gqmap_ctf_single_level_and_driver():
    from gqmap_opticalflow_amd import gqmap_ctf, optical_flow_ctf
    I1, I2, flo, unk, rng = _pipeline_pair("Grove3", (100, 100, 64, 96))
    mu, sigma, rou, AEPE, Energy = gqmap_ctf(dict(K=11, its=40, epsn=1e-6, lambdas=5, lambdad=1),
                                             I1, I2, flo)
    assert mu.shape == (64, 96, 2) and rou.shape == (64, 96, 2, 2)
    assert np.isfinite(AEPE).all() and (Energy != 0).all()
    # the last AEPE is gqmap_ctf.m:38 on the returned mean
    d = flo[1:-1, 1:-1] - mu[1:-1, 1:-1]
    assert AEPE[-1] == pytest.approx(np.mean(np.mean(np.sqrt(np.sum(d ** 2, axis=2)), axis=0)), rel=1e-12)
    flow, a, its, ms = optical_flow_ctf(I1, I2, flo, dict(its=20), scales=(0.25, 0.5, 1.0))
    assert flow.shape == (64, 96, 2) and np.isfinite(a) and len(its) == 3


def test_pyramid_rejects_inconsistent_geometry():
    from gqmap_opticalflow_amd import C3_SCALES, Pyramid, ctf_options
    from gqmap_opticalflow_amd._lib import GqmapError
    I1 = _rand((388, 584), 1)  # 388/16 -> 25, but 2*ceil(388/32) = 26: imresize(warp,2) mismatch
    with Pyramid(ctf_options(its=5, minu=-1, maxu=1, minv=-1, maxv=1), C3_SCALES) as p:
        with pytest.raises(GqmapError, match="twice the previous"):
            p.set_images(I1, I1)
    with pytest.raises(GqmapError, match="scale 1"):
        Pyramid(ctf_options(minu=-1, maxu=1, minv=-1, maxv=1), (0.25, 0.5))


def test_ctf_aepe_every_iteration_matches_host():
    """gqmap_ctf.m:38 records AEPE every iteration: the device reduction
    (exact fixed-point sum inside the iteration kernel) equals the host mean
    of means on the state after each iteration; a GRDT larger than the level
    contributes its top-left block, as the reference indexes it."""
    from gqmap_opticalflow_amd import Engine
    I1, I2, flo, unk, rng = _pipeline_pair("Grove3", (100, 100, 64, 96))
    big = np.asfortranarray(np.pad(flo, ((0, 7), (0, 5), (0, 0)), constant_values=3.0) * 0.5)
    o = dict(K=11, its=30, epsn=1e-6, lambdas=5, lambdad=1, minu=-2, maxu=2, minv=-2, maxv=2)
    with Engine(o, I1, I2, "ctf") as a, Engine(o, I1, I2, "ctf") as b:
        a.init_state(4)
        b.init_state(4)
        a.set_truth(big)
        done, tr, ae = a.run_aepe(12)
        assert done == 12
        g = big[:64, :96]
        for k in range(12):
            _, trb = b.run(1)
            np.testing.assert_array_equal(trb[0], tr[k])  # the truth does not perturb the solve
            st = b.get_state()
            d = g[1:-1, 1:-1] - np.stack([st.muu[1:-1, 1:-1, 0], st.muv[1:-1, 1:-1, 0]], axis=2)
            ref = np.mean(np.mean(np.sqrt(np.sum(d ** 2, axis=2)), axis=0))
            assert ae[k] == pytest.approx(ref, rel=1e-12, abs=0)
        a.set_truth(None)
        _, _, ae2 = a.run_aepe(2)
        assert np.isnan(ae2).all()


def test_pyramid_level_aepe_traces():
    """optical_flow_ctf.m:33: each level's gqmap_ctf gets trueFlow.*scale;
    its per-iteration AEPE (gqmap_ctf.m:38) is kept per level."""
    from gqmap_opticalflow_amd import Pyramid, ctf_options
    I1, I2, flo, unk, rng = _pipeline_pair("Grove3", (100, 100, 64, 96))
    scales = (0.25, 0.5, 1.0)
    with Pyramid(ctf_options(its=15, **rng), scales) as p:
        p.set_images(I1, I2)
        p.set_truth(flo)
        flow, its, ms = p.run(seed=2)
        for l, s in enumerate(scales):
            e, a = p.trace(l)
            assert len(a) == its[l] and np.isfinite(a).all() and (e != 0).all()
            lev = p.level(l)
            m, n = lev["flow"].shape[:2]
            d = (flo[:m, :n] * s)[1:-1, 1:-1] - lev["flow"][1:-1, 1:-1]
            assert a[-1] == pytest.approx(np.mean(np.mean(np.sqrt(np.sum(d ** 2, axis=2)), axis=0)), rel=1e-12)
        p.set_truth(None)
        p.run(seed=2)
        assert np.isnan(p.trace(0)[1]).all()
