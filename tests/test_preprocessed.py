"""The structure-texture input path (optical_flowSuper.m:7-14, preprocessed=true):
the reference's preprocessed RubberWhale frames (fixture copied by
scripts/make_preprocessed_fixture.py; their generator is not in the reference,
so the frames themselves are the pin).  Non-integer frames take the fp64 VV
store of the kernels."""
import numpy as np


def _case(M=96, N=128, r0=120, c0=200):
    from gqmap_opticalflow_amd import initial_state, load_preprocessed
    from oracle import gqmap_np
    I1, I2, gt = load_preprocessed("RubberWhale")
    I1 = np.asfortranarray(I1[r0:r0 + M, c0:c0 + N]); I2 = np.asfortranarray(I2[r0:r0 + M, c0:c0 + N])
    _, flo, (minu, maxu, minv, maxv), unk = gqmap_np.flow_to_color(gt[r0:r0 + M, c0:c0 + N])
    o = dict(engine="super", K=11, L=3, temperature=0.2, drate=0.75, epsn=1e-6, lambdad=1.0, lambdas=16.0,
             minu=minu, maxu=maxu, minv=minv, maxv=maxv)
    st = initial_state(o, M // 4, N // 4, seed=0, engine="super")
    return I1, I2, o, st


def test_preprocessed_frames_load():
    from gqmap_opticalflow_amd import load_preprocessed
    I1, I2, gt = load_preprocessed("RubberWhale")
    assert I1.shape == I2.shape == (388, 584) and gt.shape == (388, 584, 2)
    assert I1.dtype == np.float64 and I1.flags.f_contiguous
    assert np.mean(I1 != np.round(I1)) > 0.99  # structure-texture output: not integer-valued
    assert 0.0 <= I1.min() and I1.max() < 256.0


def test_super_one_step_on_preprocessed_frames(oracle_lib):
    # CPU model of the kernel vs the literal restatement, one step, rounding level
    from gqmap_opticalflow_amd import gauss_hermite
    I1, I2, o, st = _case()
    X, W = gauss_hermite(11)

    def ost():
        return oracle_lib.State(st.muu.copy(order="F"), st.muv.copy(order="F"), st.sigu.copy(order="F"),
                                st.sigv.copy(order="F"), st.pn.copy(order="F"), st.rou.copy(order="F"),
                                st.w.copy(), st.alpha.copy())
    lit, emu = ost(), ost()
    oracle_lib.run(o, I1, I2, lit, 1, 1, nthreads=4)
    oracle_lib.emu_run(o, I1, I2, emu, 1, 1, X, W, T=st.T, nthreads=4)
    for k, a, b in zip(("muu", "muv", "sigu", "sigv", "pn", "rou"), emu.arrays(), lit.arrays()):
        np.testing.assert_allclose(a, b, rtol=1e-11, atol=1e-11, err_msg=k)
