"""The C-ABI library (libgqmap.so) loads, exports every entry point that
include/gqmap.h declares, and its host-only helpers behave; no device
compute here."""
import ctypes as C
import os
import re

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "gqmap.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(gqmap_[a-z_0-9]+)\s*\(", src)))


def test_header_declares_expected_entry_points():
    from gqmap_opticalflow_amd import _lib
    assert set(declared_functions()) == set(_lib.EXPORTS)


def test_library_exports_every_declared_symbol():
    from gqmap_opticalflow_amd import _lib
    lib = _lib.load()
    for name in declared_functions():
        assert hasattr(lib, name), name
    assert lib.gqmap_abi_version() == 2


def test_header_constants_mirrored():
    # enum values and #defines of include/gqmap.h that the Python mirror restates
    from gqmap_opticalflow_amd import _lib
    src = open(HEADER).read()
    consts = {k: int(v) for k, v in re.findall(r"\b(GQMAP_[A-Z0-9_]+)\s*=\s*(-?\d+)", src)}
    consts.update({k: int(v) for k, v in re.findall(r"#define\s+(GQMAP_[A-Z0-9_]+)\s+\(?(-?\d+)\)?", src)})
    assert consts["GQMAP_ENGINE_CTF"] == _lib.ENGINE_CTF and consts["GQMAP_FP32"] == _lib.FP32
    assert consts["GQMAP_ALPHA_PROJSPLX"] == _lib.ALPHA_PROJSPLX
    assert consts["GQMAP_SPLIT_ROLE"] == _lib.SPLIT_ROLE


def test_library_is_built_for_gfx950():
    from gqmap_opticalflow_amd import _lib
    blob = open(_lib.LIB_PATH, "rb").read()
    assert b"gfx950" in blob


def test_host_gauss_hermite_matches_numpy():
    from gqmap_opticalflow_amd import gauss_hermite
    for K in (2, 5, 9, 11, 16):
        x, w = gauss_hermite(K)
        xr, wr = np.polynomial.hermite.hermgauss(K)
        assert np.max(np.abs(x - xr)) < 1e-13 and np.max(np.abs(w - wr)) < 1e-13


def test_rng_is_deterministic_and_uniform():
    from gqmap_opticalflow_amd import rand_uniform
    a = rand_uniform(7, 1, 100000)
    assert np.array_equal(a, rand_uniform(7, 1, 100000))
    assert np.array_equal(a[500:600], rand_uniform(7, 1, 100, first=500))
    assert not np.array_equal(a[:100], rand_uniform(7, 2, 100))
    assert not np.array_equal(a[:100], rand_uniform(8, 1, 100))
    assert 0 <= a.min() and a.max() < 1 and abs(a.mean() - 0.5) < 0.01


def test_initial_state_formulas():
    from gqmap_opticalflow_amd import initial_state
    o = dict(L=3, minu=-2.0, maxu=3.0, minv=-1.0, maxv=0.5, temperature=0.2)
    st = initial_state(o, 5, 6, seed=3)
    assert st.muu.shape == (5, 6, 3) and st.rou.shape == (5, 6, 3, 2, 2)
    assert st.muu.min() >= -2 and st.muu.max() <= 3
    assert st.sigu.min() >= 5 and st.sigu.max() <= 6        # U + (maxu-minu)
    assert st.sigv.min() >= 1.5 and st.sigv.max() <= 2.5
    assert np.all(st.pn == 0) and np.all(st.rou == 0)
    assert abs(st.alpha.sum() - 1) < 1e-15 and st.T == 0.2


def test_create_fails_loudly_without_device():
    from gqmap_opticalflow_amd import _lib
    lib = _lib.load()
    if lib.gqmap_device_count() > 0:
        pytest.skip("a HIP device is present")
    o = _lib.GqmapOptions()
    lib.gqmap_options_default(C.byref(o), 0)
    ctx = C.c_void_p()
    assert lib.gqmap_create(C.byref(ctx), C.byref(o), 0) == 4  # GQMAP_ERR_NO_DEVICE
    assert b"no HIP device" in lib.gqmap_last_error()
    with pytest.raises(_lib.GqmapError):
        from gqmap_opticalflow_amd import projsplx
        projsplx([0.1, 0.2])


def test_options_defaults_mirror_reference():
    from gqmap_opticalflow_amd.engine import make_options
    o = make_options({}, "mixture")
    assert (o.K, o.lambdas, o.step0, o.step_decay, o.sig_hi, o.guard_a, o.t_decay_every) == \
        (9, 5.0, 0.1, 8000.0, 23.0, 1, 0)
    s = make_options({}, "super")
    assert (s.K, s.lambdas, s.step0, s.step_decay, s.sig_hi, s.guard_a, s.t_decay_every) == \
        (11, 16.0, 0.001, 4000.0, 25.0, 0, 500)
    assert o.corr_tor == 1 - 1e-5 and o.tor == 1e-4 and o.alpha_start == 500 and o.alpha_lr == 1e-7


def test_mex_gateways_build_and_reject_bad_calls_without_a_device():
    """The MEX gateways compile against the MEX API shim and check their
    argument lists before touching the device (gqmap:usage)."""
    import pytest
    from tests._mexshim import Gateway, build
    try:
        build()
    except Exception as e:  # no libgqmap.so in this environment
        pytest.skip(f"MEX shim build: {e}")
    for name in ("mixture", "super", "ctf"):
        with pytest.raises(RuntimeError, match="usage"):
            Gateway(name)(1, dict(its=1))


def test_context_calls_reject_a_null_context_before_touching_a_device():
    from gqmap_opticalflow_amd import _lib
    lib = _lib.load()
    for call in (lambda: lib.gqmap_prepare(None), lambda: lib.gqmap_synchronize(None)):
        assert call() == 1  # GQMAP_ERR_INVALID_ARG
        assert b"null" in lib.gqmap_last_error()
