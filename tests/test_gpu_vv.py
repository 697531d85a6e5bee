"""The padded frame VV the kernels read equals getVV(I2)
(gqmap_gpu_mixture.m:12, 191-208) right after the images are set.

Round 2's driver run failed one fp64 test because prepare_images zeroed VV
with a null-stream memset that was unordered with the VV upload on the
context's non-blocking stream.  These tests read VV back through the debug
export gqmap_debug_read_vv and compare it with the oracle's getVV: they pin
the invariant (every copy stream-ordered), they do not try to provoke a race.
Also: the ctf truth buffer follows a frame-size change.
"""
import ctypes as C

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _lib():
    from gqmap_opticalflow_amd import _lib
    lib = _lib.load()
    for name, args in (("gqmap_debug_read_vv", [C.c_void_p, C.POINTER(C.c_double), C.c_size_t, C.POINTER(C.c_int)]),
                       ("gqmap_ctf_debug_read_vv", [C.c_void_p, C.c_int, C.POINTER(C.c_double), C.c_size_t,
                                                    C.POINTER(C.c_int)])):
        f = getattr(lib, name)
        f.restype, f.argtypes = C.c_int, args
    return lib


def _read_vv(ctx, Mo, No):
    from gqmap_opticalflow_amd import _lib as L
    out = np.zeros((Mo + 2) * (No + 2))
    f32 = C.c_int(-1)
    L.check(_lib().gqmap_debug_read_vv(ctx, L.dptr(out), out.size, C.byref(f32)), "gqmap_debug_read_vv")
    return out.reshape((Mo + 2, No + 2), order="F"), f32.value


def _frames(M, N, integer, seed=0):
    rng = np.random.default_rng(seed)
    I1 = rng.integers(0, 256, (M, N)).astype(np.float64)
    I2 = rng.integers(0, 256, (M, N)).astype(np.float64)
    if not integer:  # the ctf test frames / resampled pyramid levels
        I1, I2 = I1 * 0.7, I2 * 0.7 + 0.1
    return np.asfortranarray(I1), np.asfortranarray(I2)


def _opts(engine):
    return dict(K=11 if engine != "mixture" else 9, L=1, minu=-2.0, maxu=2.0, minv=-1.0, maxv=1.5,
                temperature=0.0, epsn=1e-6, lambdad=1.0, lambdas=5.0, drate=0.5)


@pytest.mark.parametrize("engine,precision,integer", [("mixture", "fp64", True), ("mixture", "fp64", False),
                                                      ("ctf", "fp64", False), ("ctf", "fp64", True),
                                                      ("mixture", "fp32", False)])
def test_vv_equals_getvv_after_set_images(engine, precision, integer):
    from gqmap_opticalflow_amd import Engine, _lib as L
    from oracle import oracle
    sizes = [(30, 44), (60, 70), (96, 128), (30, 44)]  # fresh context, then resizes on the same one
    I1, I2 = _frames(*sizes[0], integer)
    with Engine(_opts(engine), I1, I2, engine, precision) as eng:
        for k, (M, N) in enumerate(sizes):
            I1, I2 = _frames(M, N, integer, seed=k)
            L.check(eng.lib.gqmap_set_images(eng.ctx, L.dptr(I1), L.dptr(I2), M, N), "gqmap_set_images")
            vv, f32 = _read_vv(eng.ctx, M, N)
            ref = oracle.get_vv(I2)
            if precision == "fp32":
                assert f32 == 1
                np.testing.assert_array_equal(vv, ref.astype(np.float32).astype(np.float64))
            else:
                assert f32 == (1 if integer else 0)  # float store only when exact
                np.testing.assert_array_equal(vv, ref)


def test_pyramid_level_vv_equals_getvv_of_level_frame():
    # device getVV (k_pad_*) + f32-exactness check + convert_device, per level
    from gqmap_opticalflow_amd import Pyramid, ctf_options, flowio
    from oracle import oracle
    I1, I2, _ = flowio.load_pair("Grove3")
    I1, I2 = np.asfortranarray(I1[:120, :160]), np.asfortranarray(I2[:120, :160])
    o = ctf_options(its=2, minu=-3.0, maxu=3.0, minv=-2.0, maxv=2.0)
    lib = _lib()
    from gqmap_opticalflow_amd import _lib as L
    with Pyramid(o, (1 / 4, 1 / 2, 1.0)) as p:
        p.set_images(I1, I2)
        for rep in range(2):
            p.run(seed=rep)
            for lv in range(3):
                d = p.level(lv)
                M, N = d["I2"].shape
                out = np.zeros((M + 2) * (N + 2))
                f32 = C.c_int(-1)
                L.check(lib.gqmap_ctf_debug_read_vv(p.ptr, lv, L.dptr(out), out.size, C.byref(f32)), "read_vv")
                ref = oracle.get_vv(d["I2"])
                np.testing.assert_array_equal(out.reshape((M + 2, N + 2), order="F"), ref, err_msg=f"level {lv}")


def test_truth_follows_frame_resize():
    # set_truth, set_images with a larger frame, set_truth,
    # run_aepe -- the truth buffer must be reallocated for the new grid and
    # the AEPE computed against the new truth
    from gqmap_opticalflow_amd import Engine, _lib as L
    o = _opts("ctf")
    I1, I2 = _frames(30, 44, False)
    rng = np.random.default_rng(3)
    with Engine(o, I1, I2, "ctf") as eng:
        eng.init_state(0)
        eng.set_truth(np.asfortranarray(rng.normal(size=(30, 44, 2))))
        assert np.isfinite(eng.run_aepe(3)[2]).all()
        I1b, I2b = _frames(60, 70, False, seed=5)
        L.check(eng.lib.gqmap_set_images(eng.ctx, L.dptr(I1b), L.dptr(I2b), 60, 70), "gqmap_set_images")
        eng.M, eng.N = 60, 70
        eng.init_state(1)
        # the resize dropped the old truth: no AEPE until a new one is set
        assert np.isnan(eng.run_aepe(2)[2]).all()
        eng.init_state(1)
        gt = np.asfortranarray(rng.normal(size=(60, 70, 2)))
        eng.set_truth(gt)
        done, tr, ae = eng.run_aepe(3)
        st = eng.get_state()
    # a fresh context on the same frames and truth gives the same trace
    with Engine(o, I1b, I2b, "ctf") as ref:
        ref.init_state(1)
        ref.set_truth(gt)
        rdone, rtr, rae = ref.run_aepe(3)
        rst = ref.get_state()
    assert done == rdone == 3
    np.testing.assert_array_equal(ae, rae)
    np.testing.assert_array_equal(tr, rtr)
    np.testing.assert_array_equal(st.muu, rst.muu)
    # and it is the mean end-point error of the updated mean against gt
    M_, N_ = slice(1, 59), slice(1, 69)
    e = np.sqrt((gt[M_, N_, 0] - st.muu[M_, N_, 0]) ** 2 + (gt[M_, N_, 1] - st.muv[M_, N_, 0]) ** 2)
    assert ae[-1] == pytest.approx(e.mean(), rel=1e-12)
