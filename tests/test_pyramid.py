"""Coarse-to-fine plumbing (legacy/optical_flow_ctf.m:21-35) on the CPU: the C
restatement (oracle/gqmap_pyramid_oracle.c) against the independent numpy
restatement (oracle/gqmap_np.py) and the committed pipeline golden.

MATLAB's imresize / interp2 / fillmissing are not vendored in the reference
and no output of them is available, so these functions are "parity
unpinned" against MATLAB itself; the two restatements pin each other."""
import ast
import os

import numpy as np
import pytest

from tests import _golden as G


def _rand(shape, seed=0):
    return np.asfortranarray(np.random.default_rng(seed).random(shape) * 255)


@pytest.mark.parametrize("scale", [1 / 16, 1 / 8, 0.25, 0.5, 0.3, 1.0, 2.0, 1.7])
@pytest.mark.parametrize("shape", [(48, 64), (37, 29), (30, 40, 2)])
def test_imresize_c_vs_numpy(oracle_lib, scale, shape):
    from oracle import gqmap_np
    A = _rand(shape, 1)
    a = oracle_lib.imresize(A, scale)
    b = gqmap_np.imresize(A, scale)
    assert a.shape == b.shape == (int(np.ceil(shape[0] * scale)), int(np.ceil(shape[1] * scale))) + shape[2:]
    np.testing.assert_allclose(a, b, rtol=1e-12, atol=1e-10)


@pytest.mark.parametrize("in_len,out_len,scale", [(480, 30, 1 / 16), (30, 60, 2.0), (64, 64, 1.0),
                                                  (97, 49, 0.5), (10, 17, 1.7)])
def test_resize_contributions_c_vs_numpy(oracle_lib, in_len, out_len, scale):
    from oracle import gqmap_np
    w, i = oracle_lib.resize_contrib(in_len, out_len, scale)
    wn, jn = gqmap_np.imresize_contrib(in_len, out_len, scale)
    assert w.shape == wn.shape
    np.testing.assert_array_equal(i, jn)
    np.testing.assert_allclose(w, wn, rtol=1e-13, atol=1e-15)
    np.testing.assert_allclose(w.sum(axis=1), 1.0, rtol=1e-13)
    assert i.min() >= 0 and i.max() < in_len


def test_imresize_known_answers(oracle_lib):
    A = _rand((40, 56), 2)
    # scale 1: all-zero tap columns are removed -> an exact copy
    np.testing.assert_array_equal(oracle_lib.imresize(A, 1.0), A)
    # constants survive any scale (normalised weights, mirrored edges)
    C = np.full((40, 30), 7.25, order="F")
    for s in (1 / 16, 0.5, 2.0):
        np.testing.assert_allclose(oracle_lib.imresize(C, s), 7.25, rtol=0, atol=1e-12)
    # x2 of a linear ramp is exact away from the mirrored border
    r = np.asfortranarray(np.tile(np.arange(1.0, 41.0)[:, None], (1, 8)))
    up = oracle_lib.imresize(r, 2.0)
    u = (np.arange(1, 81) / 2 + 0.25)[:, None]
    np.testing.assert_allclose(up[4:-4], np.broadcast_to(u, up.shape)[4:-4], atol=1e-12)


def test_warp_and_fill_c_vs_numpy(oracle_lib):
    from oracle import gqmap_np
    rng = np.random.default_rng(3)
    V = _rand((33, 45), 4)
    warp = np.asfortranarray(rng.normal(scale=3.0, size=(33, 45, 2)))
    warp[:4, :, 1] = -6.0  # rows whose samples fall below the image -> NaN
    a = oracle_lib.warp_image(V, warp, fill=False)
    b = gqmap_np.warp_image(V, warp, fill=False)
    np.testing.assert_array_equal(np.isnan(a), np.isnan(b))
    assert np.isnan(a).any()
    ok = ~np.isnan(a)
    np.testing.assert_allclose(a[ok], b[ok], rtol=1e-12, atol=1e-10)
    fa = oracle_lib.warp_image(V, warp, fill=True)
    fb = gqmap_np.warp_image(V, warp, fill=True)
    assert not np.isnan(fa).any()
    np.testing.assert_allclose(fa, fb, rtol=1e-12, atol=1e-10)


def test_warp_identity_and_integer_shift(oracle_lib):
    V = _rand((20, 25), 5)
    z = np.zeros((20, 25, 2), order="F")
    np.testing.assert_array_equal(oracle_lib.warp_image(V, z, fill=False), V)
    w = np.zeros((20, 25, 2), order="F")
    w[:, :, 0] = 2.0  # sample from x - 2: columns shift right by 2, first two missing
    out = oracle_lib.warp_image(V, w, fill=False)
    assert np.isnan(out[:, :2]).all()
    np.testing.assert_array_equal(out[:, 2:], V[:, :-2])
    filled = oracle_lib.warp_image(V, w, fill=True)
    np.testing.assert_array_equal(filled[:, 0], V[:, 0])  # nearest along dim 2
    np.testing.assert_array_equal(filled[:, 1], V[:, 0])


def test_fillmissing_nearest_rules(oracle_lib):
    from oracle import gqmap_np
    nan = np.nan
    A = np.asfortranarray(np.array([[nan, 1.0, nan], [2.0, nan, nan], [nan, nan, nan],
                                    [4.0, 3.0, nan], [nan, nan, nan]]))
    a = oracle_lib.fillmissing_nearest(A.copy(order="F"), 1)
    # col 0: row 2 is a tie between rows 1 and 3 -> the later sample (4)
    np.testing.assert_array_equal(a[:, 0], [2, 2, 4, 4, 4])
    np.testing.assert_array_equal(a[:, 1], [1, 1, 3, 3, 3])
    assert np.isnan(a[:, 2]).all()  # all-missing line stays missing
    np.testing.assert_array_equal(gqmap_np.fillmissing_nearest(A, 1), a)
    b = oracle_lib.fillmissing_nearest(a, 2)
    np.testing.assert_array_equal(b[:, 2], b[:, 1])


def _pipe_golden():
    d = dict(np.load(os.path.join(G.GOLDEN, "ctf_pipeline.npz"), allow_pickle=False))
    d["opts"] = ast.literal_eval(str(d["opts"]))
    return d


def _golden_init(d):
    from oracle import oracle

    def init_fn(l, lo, M, N):
        return oracle.State(*(np.array(d[f"L{l}_init_{k}"], order="F", copy=True) for k in G.STATE_KEYS))
    return init_fn


@pytest.mark.parametrize("solver", ["literal", "emu"])
def test_ctf_pipeline_matches_golden(oracle_lib, solver):
    d = _pipe_golden()
    from gqmap_opticalflow_amd import gauss_hermite
    X, W = gauss_hermite(d["opts"]["K"])
    warp, levels = oracle_lib.ctf_pipeline(d["opts"], d["img1"], d["img2"], tuple(d["scales"]),
                                           _golden_init(d), solver=solver, X=X, W=W)
    for l, lv in enumerate(levels):
        np.testing.assert_allclose(lv["I2"], d[f"L{l}_I2"], rtol=1e-12, atol=1e-10)
        np.testing.assert_allclose(lv["I1w"], d[f"L{l}_I1w"], rtol=1e-9, atol=1e-8)
        np.testing.assert_allclose(lv["flow"], d[f"L{l}_flow"], rtol=1e-7, atol=1e-7)
    np.testing.assert_allclose(warp, d["warp"], rtol=1e-7, atol=1e-7)
