"""Standalone device ops of libgqmap.so beside the iteration.

flow_to_color   flowToColor_mex (legacy/flowToColor.m:37-87 + legacy/computeColor.m:33-115)
mixture_map     get_map_mex     (legacy/findMixMax.m:39-70 semantics, fminbnd TolX 1e-4)
projsplx        projsplx.m:15-30, batched over columns (projsplx.m:34-67)
gauss_hermite   GaussHermite_2.m (host)
imresize        imresize(A, scale) bicubic + antialias (legacy/optical_flow_ctf.m:26-29)
warp_image      interp2 linear + fillmissing nearest (legacy/optical_flow_ctf.m:30-32)
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib
from ._lib import check, dptr, f64, u8ptr


def flow_to_color(flow, max_flow: float = 0.0, device: int = 0):
    """[img, flo, minu, maxu, minv, maxv, idxUnknown] = flowToColor(flow)
    returned as (img uint8 MxNx3, flo MxNx2, (minu,maxu,minv,maxv), unknown MxN bool)."""
    flow = f64(flow)
    if flow.ndim != 3 or flow.shape[2] != 2:
        raise ValueError("flowToColor: image must have two bands")
    M, N, _ = flow.shape
    img = np.zeros((M, N, 3), dtype=np.uint8, order="F")
    flo = np.zeros((M, N, 2), order="F")
    stats = np.zeros(4)
    unk = np.zeros((M, N), dtype=np.uint8, order="F")
    check(_lib.load().gqmap_flow_to_color(dptr(flow), M, N, float(max_flow), u8ptr(img), dptr(flo),
                                          dptr(stats), u8ptr(unk), device), "gqmap_flow_to_color")
    return img, flo, tuple(float(x) for x in stats), unk.astype(bool)


def mixture_map(alpha, muu, sigu, muv, sigv, device: int = 0) -> np.ndarray:
    muu, sigu, muv, sigv = map(f64, (muu, sigu, muv, sigv))
    if muu.ndim == 2:
        muu, sigu, muv, sigv = (a[:, :, None] for a in (muu, sigu, muv, sigv))
        muu, sigu, muv, sigv = map(f64, (muu, sigu, muv, sigv))
    alpha = f64(np.ravel(alpha))
    M, N, L = muu.shape
    out = np.zeros((M, N, 2), order="F")
    check(_lib.load().gqmap_mixture_map(dptr(alpha), dptr(muu), dptr(sigu), dptr(muv), dptr(sigv),
                                        M, N, L, dptr(out), device), "gqmap_mixture_map")
    return out


def projsplx(Y, device: int = 0) -> np.ndarray:
    """Project y (vector) or every column of Y onto the probability simplex."""
    Y = np.asarray(Y, dtype=np.float64)
    vec = Y.ndim == 1
    Yc = f64(Y.reshape(-1, 1) if vec else Y)
    n, ncols = Yc.shape
    X = np.zeros((n, ncols), order="F")
    check(_lib.load().gqmap_projsplx(dptr(Yc), dptr(X), n, ncols, device), "gqmap_projsplx")
    return X.ravel() if vec else X


def gauss_hermite(K: int):
    x, w = np.zeros(K), np.zeros(K)
    check(_lib.load().gqmap_gauss_hermite(K, dptr(x), dptr(w)), "gqmap_gauss_hermite")
    return x, w


def resize_len(n: int, scale: float) -> int:
    """imresize output length ceil(scale * n)."""
    return int(_lib.load().gqmap_resize_len(int(n), float(scale)))


def imresize(A, scale: float, antialias: bool = True, device: int = 0) -> np.ndarray:
    """imresize(A, scale) with MATLAB's defaults ('bicubic', Antialiasing on
    when shrinking) for an M x N (x C) double array, resampled on the device."""
    A = f64(A)
    M, N = A.shape[:2]
    Cn = 1 if A.ndim == 2 else int(np.prod(A.shape[2:]))
    oM, oN = resize_len(M, scale), resize_len(N, scale)
    out = np.zeros((oM, oN) + A.shape[2:], order="F")
    check(_lib.load().gqmap_imresize(dptr(A), M, N, Cn, float(scale), int(antialias), dptr(out),
                                     device), "gqmap_imresize")
    return out


def warp_image(V, warp, fill: bool = True, device: int = 0) -> np.ndarray:
    """interp2(V, x - warp(:,:,1), y - warp(:,:,2)) (linear, NaN outside),
    then fillmissing(.,'nearest',1) and (.,'nearest',2) when fill."""
    V, warp = f64(V), f64(warp)
    M, N = V.shape
    if warp.shape != (M, N, 2):
        raise ValueError(f"warp must be {M}x{N}x2, got {warp.shape}")
    out = np.zeros((M, N), order="F")
    check(_lib.load().gqmap_warp_image(dptr(V), M, N, dptr(warp), int(fill), dptr(out), device),
          "gqmap_warp_image")
    return out
