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


# The eight ground-truth pairs of legacy/optical_flow_temp.m:3 (BASELINE config C5)
C5_PAIRS = ("Urban3", "Grove3", "Urban2", "Venus", "Dimetrodon", "rubberwhale", "Grove2", "Hydrangea")


def to_uint8(a: np.ndarray) -> np.ndarray:
    """MATLAB's double -> uint8 conversion (what imresize returns for uint8
    input): round half away from zero, saturate to [0, 255]."""
    return np.clip(np.sign(a) * np.floor(np.abs(a) + 0.5), 0, 255).astype(np.uint8)


def load_pair_scaled(name: str, scale: float, device: int = 0, root: str = DATA_DIR):
    """optical_flow_temp.m:7-8 / optical_flowSuper.m:8-11 at any scale:
    img = imresize(imread(frame), scale) on the uint8 RGB frame (bicubic,
    resampled on the device, rounded back to uint8), then double(rgb2gray(img)).
    The GT flow is resized to the frame (nearest, each pixel repeated) and
    multiplied by the scale -- the reference keeps its GT at scale 1, so this
    part is this build's choice for an upsampled benchmark (unknown entries
    stay > 1e9).  Returns I1, I2 (double) and the GT flow."""
    from .ops import imresize
    d = os.path.join(root, name)
    frames = []
    for f in ("frame10.png", "frame11.png"):
        rgb = imread(os.path.join(d, f))
        if scale != 1:
            rgb = to_uint8(imresize(rgb.astype(np.float64), scale, device=device))
        frames.append(np.asfortranarray(rgb2gray(rgb).astype(np.float64)))
    gt = read_flow_file(os.path.join(d, "flow10.flo"))
    if scale != 1:
        r = int(round(scale))
        if r != scale or r < 1:
            raise ValueError("GT resizing supports integer upscaling only")
        gt = np.asfortranarray(np.repeat(np.repeat(gt, r, axis=0), r, axis=1) * float(scale))
        gt = gt[:frames[0].shape[0], :frames[0].shape[1]]
    return frames[0], frames[1], gt
