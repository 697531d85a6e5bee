"""Coarse-to-fine optical flow: host mirror of legacy/optical_flow_ctf.m and
legacy/gqmap_ctf.m over libgqmap.so.

gqmap_ctf            one pyramid level, [mu,sigma,rou,AEPE,Energy] = gqmap_ctf(options,I1,I2,GRDT)
                     (legacy/gqmap_ctf.m:1) on the level engine (GQMAP_ENGINE_CTF)
Pyramid              gqmap_pyramid: the whole driver loop optical_flow_ctf.m:21-35
                     (imresize, prolong, warp, fillmissing, level solves) resident on the device
optical_flow_ctf     optical_flow_ctf.m:4-35 for one frame pair
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib
from ._lib import check, dptr, f64
from .engine import Engine, aepe, make_options
from .ops import flow_to_color

# optical_flow_ctf.m:21 uses four levels (1/8..1); BASELINE config C3 adds a
# fifth (1/16, 30x40 for a 480x640 pair).
REFERENCE_SCALES = (1 / 8, 1 / 4, 1 / 2, 1.0)
C3_SCALES = (1 / 16, 1 / 8, 1 / 4, 1 / 2, 1.0)


def ctf_options(options: dict | None = None, **kw) -> dict:
    """optical_flow_ctf.m:13-17 defaults (K=11, its=3000, epsn=0.001^2,
    lambdas=5, lambdad=1) overridden by `options` / keywords."""
    o = dict(K=11, its=3000, L=1, epsn=0.001 ** 2, lambdas=5.0, lambdad=1.0, temperature=0.0)
    o.update(options or {})
    o.update(kw)
    return o


def gqmap_ctf(options: dict, I1, I2, GRDT, *, seed: int = 0, precision: str = "fp64",
              device: int = 0):
    """[mu, sigma, rou, AEPE, Energy] = gqmap_ctf(options, I1, I2, GRDT).

    minu..maxv come from GRDT (gqmap_ctf.m:4).  AEPE(it) is the reference's
    per-iteration mean(mean(sqrt((GRDT(M_,N_,1)-muu(M_,N_)).^2 + ...)))
    (gqmap_ctf.m:38), reduced exactly on the device inside the iteration
    kernel (GRDT may be larger than I1: its top-left block is used, as the
    reference indexes it).  Iterations after a stop keep the reference's
    initial value 17 (AEPE = ones(its,1)*17, :13); Energy after a stop is 0."""
    GRDT = f64(GRDT)
    o = dict(options)
    o.update(minu=float(GRDT[:, :, 0].min()), maxu=float(GRDT[:, :, 0].max()),
             minv=float(GRDT[:, :, 1].min()), maxv=float(GRDT[:, :, 1].max()))
    its = int(o["its"])
    AEPE = np.full(its, 17.0)
    Energy = np.zeros(its)
    with Engine(o, I1, I2, "ctf", precision, device) as eng:
        eng.init_state(seed)
        eng.set_truth(GRDT)
        done, tr, ae = eng.run_aepe(its)
        Energy[:done] = tr[:, 0]
        AEPE[:done] = ae
        st = eng.get_state()
    mu = np.stack([st.muu[:, :, 0], st.muv[:, :, 0]], axis=2)
    sigma = np.stack([st.sigu[:, :, 0], st.sigv[:, :, 0]], axis=2)
    rou = st.rou[:, :, 0]
    return mu, sigma, rou, AEPE, Energy


class Pyramid:
    """gqmap_pyramid: every level of optical_flow_ctf.m:21-35 on the device."""

    def __init__(self, options: dict, scales=C3_SCALES, precision: str = "fp64", device: int = 0):
        self.lib = _lib.load()
        self.scales = np.ascontiguousarray(scales, dtype=np.float64)
        self.opts = make_options(options, "ctf", precision)
        self.ptr = C.c_void_p()
        check(self.lib.gqmap_ctf_create(C.byref(self.ptr), C.byref(self.opts), dptr(self.scales),
                                        len(self.scales), device), "gqmap_ctf_create")
        self.M = self.N = 0

    def set_images(self, img1, img2) -> None:
        img1, img2 = f64(img1), f64(img2)
        if img1.shape != img2.shape or img1.ndim != 2:
            raise ValueError("img1 and img2 must be equal-size 2-D images")
        self.M, self.N = img1.shape
        check(self.lib.gqmap_ctf_set_images(self.ptr, dptr(img1), dptr(img2), self.M, self.N),
              "gqmap_ctf_set_images")

    def set_truth(self, true_flow) -> None:
        """Full-resolution trueFlow (M x N x 2, as flowToColor returns it):
        each level then records gqmap_ctf's per-iteration AEPE against
        trueFlow.*scale (optical_flow_ctf.m:33).  None clears it."""
        if true_flow is None:
            check(self.lib.gqmap_ctf_set_truth(self.ptr, None, 0, 0), "gqmap_ctf_set_truth")
            return
        t = f64(true_flow)
        check(self.lib.gqmap_ctf_set_truth(self.ptr, dptr(t), t.shape[0], t.shape[1]), "gqmap_ctf_set_truth")

    def trace(self, l: int):
        """Level l of the last run: (Energy, AEPE) per iteration (gqmap_ctf's outputs)."""
        n = C.c_int(0)
        check(self.lib.gqmap_ctf_get_trace(self.ptr, l, C.byref(n), None, None), "gqmap_ctf_get_trace")
        e, a = np.zeros(max(n.value, 1)), np.zeros(max(n.value, 1))
        check(self.lib.gqmap_ctf_get_trace(self.ptr, l, None, dptr(e), dptr(a)), "gqmap_ctf_get_trace")
        return e[:n.value], a[:n.value]

    def run(self, seed: int = 0):
        """Returns (flow M x N x 2, iterations per level, wall ms)."""
        flow = np.zeros((self.M, self.N, 2), order="F")
        its = (C.c_int * len(self.scales))()
        ms = C.c_double(0)
        check(self.lib.gqmap_ctf_run(self.ptr, C.c_uint64(seed), dptr(flow), its, C.byref(ms)),
              "gqmap_ctf_run")
        return flow, list(its), ms.value

    def level(self, l: int) -> dict:
        """Level l after a run: I1w, I2 (Ml x Nl), flow and warp (Ml x Nl x 2)."""
        Ml, Nl = C.c_int(0), C.c_int(0)
        check(self.lib.gqmap_ctf_get_level(self.ptr, l, C.byref(Ml), C.byref(Nl), None, None, None,
                                           None), "gqmap_ctf_get_level")
        m, n = Ml.value, Nl.value
        out = dict(I1w=np.zeros((m, n), order="F"), I2=np.zeros((m, n), order="F"),
                   flow=np.zeros((m, n, 2), order="F"), warp=np.zeros((m, n, 2), order="F"))
        check(self.lib.gqmap_ctf_get_level(self.ptr, l, None, None, dptr(out["I1w"]), dptr(out["I2"]),
                                           dptr(out["flow"]), dptr(out["warp"])), "gqmap_ctf_get_level")
        return out

    def close(self) -> None:
        if self.ptr:
            self.lib.gqmap_ctf_destroy(self.ptr)
            self.ptr = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()


def optical_flow_ctf(img1, img2, true_flow, options: dict | None = None, scales=C3_SCALES, *,
                     seed: int = 0, precision: str = "fp64", device: int = 0):
    """optical_flow_ctf.m:4-35 for one pair: GT range from flowToColor of the
    ground truth (:10-11), the device pyramid, AEPE of the final warp against
    the GT (unknowns zeroed, 1-px border dropped).  Returns
    (flow, aepe, iterations per level, wall ms)."""
    _, flo, (minu, maxu, minv, maxv), unk = flow_to_color(true_flow, device=device)
    o = ctf_options(options, minu=minu, maxu=maxu, minv=minv, maxv=maxv)
    with Pyramid(o, scales, precision, device) as p:
        p.set_images(img1, img2)
        flow, its, ms = p.run(seed)
    return flow, aepe(flo, flow, unk), its, ms
