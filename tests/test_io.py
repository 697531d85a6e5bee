"""Host I/O of the drivers: .flo read/write, rgb2gray, Middlebury fixtures."""
import os
import numpy as np
import pytest

from gqmap_opticalflow_amd import flowio


def test_flo_roundtrip(tmp_path):
    rng = np.random.default_rng(0)
    f = rng.normal(size=(7, 11, 2)).astype(np.float32).astype(np.float64)
    p = str(tmp_path / "x.flo")
    flowio.write_flow_file(f, p)
    g = flowio.read_flow_file(p)
    assert g.shape == (7, 11, 2) and np.array_equal(f, g)
    with open(p, "rb") as fh:
        assert fh.read(4) == b"PIEH"


def test_flo_errors(tmp_path):
    with pytest.raises(ValueError):
        flowio.read_flow_file(str(tmp_path / "x.png"))
    with pytest.raises(ValueError):
        flowio.write_flow_file(np.zeros((2, 2, 3)), str(tmp_path / "y.flo"))


@pytest.mark.parametrize("name,shape", [("rubberwhale", (388, 584)), ("Dimetrodon", (388, 584)),
                                        ("Grove3", (480, 640)), ("Urban3", (480, 640))])
def test_middlebury_fixtures(name, shape):
    I1, I2, gt = flowio.load_pair(name)
    assert I1.shape == shape and I2.shape == shape and gt.shape == shape + (2,)
    assert I1.min() >= 0 and I1.max() <= 255 and np.all(I1 == np.round(I1))


def test_rgb2gray_matlab_coefficients():
    rgb = np.array([[[255, 0, 0], [0, 255, 0], [0, 0, 255], [255, 255, 255], [10, 20, 30]]],
                   dtype=np.uint8)
    g = flowio.rgb2gray(rgb)
    assert g.dtype == np.uint8
    assert list(g[0]) == [76, 150, 29, 255, 18]


def test_library_flo_io_and_aepe(tmp_path, oracle_lib):
    # the C-ABI host helpers (gqmap_read_flo / gqmap_write_flo / gqmap_aepe)
    # against the Python readFlowFile / writeFlowFile and the oracle's AEPE
    import ctypes as C

    from gqmap_opticalflow_amd import _lib, flowio
    lib = _lib.load()
    path = os.path.join(flowio.DATA_DIR, "rubberwhale", "flow10.flo").encode()
    M, N = C.c_int(0), C.c_int(0)
    _lib.check(lib.gqmap_read_flo(path, C.byref(M), C.byref(N), None))
    flow = np.zeros((M.value, N.value, 2), order="F")
    _lib.check(lib.gqmap_read_flo(path, C.byref(M), C.byref(N), _lib.dptr(flow)))
    ref = flowio.read_flow_file(path.decode())
    np.testing.assert_array_equal(flow, ref)
    out = str(tmp_path / "x.flo").encode()
    _lib.check(lib.gqmap_write_flo(out, _lib.dptr(flow), M.value, N.value))
    np.testing.assert_array_equal(flowio.read_flow_file(out.decode()), ref)
    assert lib.gqmap_read_flo(b"nope.png", C.byref(M), C.byref(N), None) != 0
    # AEPE with unknowns, crop 1 and 4
    from oracle import gqmap_np
    _, flo, _, unk = gqmap_np.flow_to_color(ref)
    flo = np.asfortranarray(flo)
    rng = np.random.default_rng(0)
    est = np.asfortranarray(flo + rng.normal(scale=0.3, size=flo.shape))
    u8 = np.asfortranarray(unk.astype(np.uint8))
    for crop in (1, 4):
        v = C.c_double(0)
        _lib.check(lib.gqmap_aepe(_lib.dptr(flo), _lib.dptr(est), _lib.u8ptr(u8), M.value, N.value, crop,
                                  C.byref(v)))
        assert v.value == oracle_lib.aepe(flo, est, unk, crop)
