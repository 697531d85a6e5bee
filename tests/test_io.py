"""Host I/O of the drivers: .flo read/write, rgb2gray, Middlebury fixtures."""
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
