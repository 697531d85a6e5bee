"""The MATLAB MEX gateways (mex/gqmap_gpu_mixture_mex.cpp, built plain and
with -DGQMAP_SUPER, and mex/gqmap_ctf_mex.cpp), compiled against the MEX API
shim (tests/native/mexshim, MATLAB being absent) and driven through their
mexFunction: their outputs equal the Python mirror of the same call bit for
bit (same C ABI underneath), their shapes are the reference's
(gqmap_gpu_mixture.m:183-188, legacy/gqmap_ctf.m:1)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _crop(name, r0, c0, M, N):
    from gqmap_opticalflow_amd import flow_to_color, flowio
    I1, I2, gt = flowio.load_pair(name)
    I1, I2, gt = (np.asfortranarray(a[r0:r0 + M, c0:c0 + N]) for a in (I1, I2, gt))
    _, flo, (minu, maxu, minv, maxv), unk = flow_to_color(gt)
    return I1, I2, flo, unk, dict(minu=minu, maxu=maxu, minv=minv, maxv=maxv)


@pytest.mark.parametrize("engine", ["mixture", "super"])
def test_mixture_and_super_gateways_equal_python_mirror(engine):
    from gqmap_opticalflow_amd import gqmap_gpu_mixture, gqmap_gpuSuper_mix_entropy
    from tests._mexshim import Gateway
    sup = engine == "super"
    I1, I2, flo, unk, rng = _crop("Urban3" if sup else "rubberwhale", 100, 120, 64, 96)
    opts = dict(its=4, K=11 if sup else 9, L=3, temperature=0.2 if sup else 0.0, drate=0.75, epsn=1e-6,
                lambdad=1.0, lambdas=16.0 if sup else 5.0, **rng)
    gw = Gateway(engine)
    mu, sigma, alpha, AEPE, Energy, logP = gw(6, dict(opts, trueFlow=flo, unknownIdx=unk, seed=5), I1, I2)
    f = gqmap_gpuSuper_mix_entropy if sup else gqmap_gpu_mixture
    r = f(dict(opts, trueFlow=flo, unknownIdx=unk), I1, I2, seed=5)
    M, N = (16, 24) if sup else (64, 96)
    assert mu.shape == (M, N, 3, 2) and sigma.shape == (M, N, 3, 2) and alpha.shape == (1, 1, 3)
    assert AEPE.shape == (4, 1) and Energy.shape == (4, 1) and logP.shape == (4, 1)
    np.testing.assert_array_equal(mu, r[0])
    np.testing.assert_array_equal(sigma, r[1])
    np.testing.assert_array_equal(alpha, r[2])
    np.testing.assert_array_equal(Energy[:, 0], r[4])
    # evaluation block at it == 1 only (gqmap_gpu_mixture.m:52): AEPE, logP there, NaN elsewhere
    assert np.isnan(AEPE[1:, 0]).all() and np.isnan(logP[1:, 0]).all()
    assert AEPE[0, 0] == pytest.approx(r[3][0], rel=1e-12)
    assert logP[0, 0] == pytest.approx(r[5][0], rel=1e-12)
    assert gw.log().count("\n") == 4  # one console line per iteration (:71)


def test_ctf_gateway_equals_python_mirror():
    from gqmap_opticalflow_amd import gqmap_ctf
    from tests._mexshim import Gateway
    I1, I2, flo, unk, _ = _crop("Grove3", 100, 100, 48, 64)
    big = np.asfortranarray(np.pad(flo, ((0, 9), (0, 3), (0, 0)), constant_values=1.5))
    opts = dict(its=25, K=11, epsn=1e-6, lambdas=5.0, lambdad=1.0)
    gw = Gateway("ctf")
    mu, sigma, rou, AEPE, Energy = gw(5, dict(opts, seed=3), I1, I2, big)
    r = gqmap_ctf(opts, I1, I2, big, seed=3)
    assert mu.shape == (48, 64, 2) and rou.shape == (48, 64, 2, 2) and AEPE.shape == (25, 1)
    for a, b in zip((mu, sigma, rou, AEPE[:, 0], Energy[:, 0]), r):
        np.testing.assert_array_equal(a, b)
    assert np.isfinite(AEPE).all()
    assert gw.log().count("best at#") == 25


def test_gateway_argument_errors():
    from tests._mexshim import Gateway
    gw = Gateway("ctf")
    with pytest.raises(RuntimeError, match="usage"):
        gw(5, dict(its=2), np.zeros((4, 4)), np.zeros((4, 4)))
    with pytest.raises(RuntimeError, match="options.K missing"):
        gw(5, dict(its=2, epsn=1e-6, lambdas=5, lambdad=1), np.zeros((8, 8)), np.zeros((8, 8)),
           np.zeros((8, 8, 2)))
    with pytest.raises(RuntimeError, match="usage"):
        Gateway("mixture")(6, dict(its=2), np.zeros((8, 8)))
