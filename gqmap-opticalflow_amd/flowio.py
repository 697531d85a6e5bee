"""Host I/O of the reference drivers: .flo files, frames, greyscale conversion.

readFlowFile.m:33-84 / legacy/writeFlowFile.m:33-76 (Middlebury .flo),
optical_flow.m:8-11 (imread -> rgb2gray -> double).
"""
from __future__ import annotations

import os

import numpy as np

TAG_FLOAT = 202021.25
TAG_STRING = b"PIEH"

DATA_DIR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                        "data", "middlebury")


def read_flow_file(filename: str) -> np.ndarray:
    """readFlowFile.m: H x W x 2 float64 (u, v)."""
    if not filename:
        raise ValueError("readFlowFile: empty filename")
    ext = os.path.splitext(filename)[1]
    if ext == "":
        raise ValueError(f"readFlowFile: extension required in filename {filename}")
    if ext != ".flo":
        raise ValueError(f"readFlowFile: filename {filename} should have extension '.flo'")
    with open(filename, "rb") as f:
        tag = np.frombuffer(f.read(4), dtype="<f4")[0]
        width = int(np.frombuffer(f.read(4), dtype="<i4")[0])
        height = int(np.frombuffer(f.read(4), dtype="<i4")[0])
        if tag != np.float32(TAG_FLOAT):
            raise ValueError(f"readFlowFile({filename}): wrong tag (possibly due to big-endian machine?)")
        if width < 1 or width > 99999:
            raise ValueError(f"readFlowFile({filename}): illegal width {width}")
        if height < 1 or height > 99999:
            raise ValueError(f"readFlowFile({filename}): illegal height {height}")
        tmp = np.frombuffer(f.read(), dtype="<f4")
    if tmp.size != width * height * 2:
        raise ValueError(f"readFlowFile({filename}): truncated data")
    # tmp reshaped [width*2, height]' -> rows are image rows, bands interleaved
    tmp = tmp.reshape(height, width * 2).astype(np.float64)
    return np.asfortranarray(np.stack([tmp[:, 0::2], tmp[:, 1::2]], axis=2))


def write_flow_file(img: np.ndarray, filename: str) -> None:
    """legacy/writeFlowFile.m: tag 'PIEH', int32 W, int32 H, interleaved float32."""
    if not filename:
        raise ValueError("writeFlowFile: empty filename")
    ext = os.path.splitext(filename)[1]
    if ext != ".flo":
        raise ValueError(f"writeFlowFile: filename {filename} should have extension '.flo'")
    img = np.asarray(img)
    if img.ndim != 3 or img.shape[2] != 2:
        raise ValueError("writeFlowFile: image must have two bands")
    height, width, _ = img.shape
    tmp = np.empty((height, width * 2), dtype="<f4")
    tmp[:, 0::2] = img[:, :, 0]
    tmp[:, 1::2] = img[:, :, 1]
    with open(filename, "wb") as f:
        f.write(TAG_STRING)
        f.write(np.array([width, height], dtype="<i4").tobytes())
        f.write(tmp.tobytes())


# MATLAB rgb2gray coefficients (luma of the NTSC YIQ transform as MATLAB stores them)
RGB2GRAY = (0.298936021293775, 0.587043074451121, 0.114020904255103)


def rgb2gray(rgb: np.ndarray) -> np.ndarray:
    """MATLAB rgb2gray for uint8 input: weighted sum in double, rounded
    half away from zero and saturated to uint8."""
    rgb = np.asarray(rgb)
    if rgb.ndim == 2:
        return rgb
    x = rgb[:, :, 0].astype(np.float64) * RGB2GRAY[0] + rgb[:, :, 1].astype(np.float64) * RGB2GRAY[1] \
        + rgb[:, :, 2].astype(np.float64) * RGB2GRAY[2]
    if rgb.dtype == np.uint8:
        return np.clip(np.floor(x + 0.5), 0, 255).astype(np.uint8)
    return x


def imread(path: str) -> np.ndarray:
    from PIL import Image  # PIL ships in this image; only used for PNG decode
    with Image.open(path) as im:
        return np.array(im.convert("RGB") if im.mode not in ("L", "RGB") else im)


def imwrite(img: np.ndarray, path: str) -> None:
    from PIL import Image
    Image.fromarray(np.ascontiguousarray(img)).save(path)


def middlebury_names():
    return sorted(d for d in os.listdir(DATA_DIR)
                  if d != "preprocessed" and os.path.isdir(os.path.join(DATA_DIR, d)))


def load_pair(name: str, root: str = DATA_DIR):
    """optical_flow.m:8-13 at scale 1: greyscale double frames + GT flow."""
    d = os.path.join(root, name)
    I1 = rgb2gray(imread(os.path.join(d, "frame10.png"))).astype(np.float64)
    I2 = rgb2gray(imread(os.path.join(d, "frame11.png"))).astype(np.float64)
    gt = read_flow_file(os.path.join(d, "flow10.flo"))
    return np.asfortranarray(I1), np.asfortranarray(I2), gt


def load_preprocessed(name: str, root: str = DATA_DIR):
    """optical_flowSuper.m:7-14 with preprocessed=true: the structure-texture
    frames the reference loads from middlebury/preprocessed/<name>.mat
    (img1, img2; fp64, not integer-valued), plus the GT flow of the pair.
    Stored here as .npz (scripts/make_preprocessed_fixture.py)."""
    path = os.path.join(root, "preprocessed", name + ".npz")
    if not os.path.exists(path):
        raise FileNotFoundError(f"no preprocessed frames for {name!r} ({path})")
    with np.load(path) as d:
        I1, I2 = d["img1"], d["img2"]
    pair = name if os.path.isdir(os.path.join(root, name)) else name.lower()
    gt = read_flow_file(os.path.join(root, pair, "flow10.flo"))
    return np.asfortranarray(I1, dtype=np.float64), np.asfortranarray(I2, dtype=np.float64), gt
