"""Full-frame cases shared by the CPU (emulator vs literal restatement) and
GPU (HIP vs both) parity tests: BASELINE configs C2 (RubberWhale 388x584,
mixture L=1 K=9), C3's finest level (Grove3 480x640, ctf K=11) and C4
(Urban3 480x640, super L=3 K=11), each from two initial states:

  * "ref":   the reference init (gqmap_gpu_mixture.m:18-24; sigma = U +
             (max-min), pn = rou = 0) -- most quadrature samples are clamped
             at the border and most super blocks cross it;
  * "tight": mu near the ground truth, sigma in [0.2, 1.7], pn / rou in
             [-0.4, 0.4] -- the state of a converging run, where the
             single-scale clamp-free quadrature (gqmap_math.h node_unclamped)
             and the super 7x7 shared tap window (super_block_sum, safe
             branch) carry most of the work.

path_coverage() measures, in numpy, how often those two fast paths apply,
so a test can assert that it exercised them.
"""
from __future__ import annotations

import numpy as np

CONFIGS = {
    "c2": dict(name="rubberwhale", engine="mixture", L=1, K=9),
    "c3": dict(name="Grove3", engine="ctf", L=1, K=11),
    "c4": dict(name="Urban3", engine="super", L=3, K=11),
    # the other 584x388 pairs of the multi-GPU frame-parallel runs (bench.PAIRS)
    "c2_dimetrodon": dict(name="Dimetrodon", engine="mixture", L=1, K=9),
    "c2_hydrangea": dict(name="Hydrangea", engine="mixture", L=1, K=9),
}


def case(cfg: str, init: str = "ref", seed: int = 0, **extra):
    """-> I1, I2, GT flow, unknown mask, options dict, engine State."""
    from gqmap_opticalflow_amd import State, flowio, initial_state
    from gqmap_opticalflow_amd.ops import flow_to_color
    c = CONFIGS[cfg]
    engine = c["engine"]
    I1, I2, gt = flowio.load_pair(c["name"])
    if engine == "ctf":
        # the finest pyramid level sees a warped, non-integer I1 (fp64 I1 plane)
        I1 = np.asfortranarray(I1 * 0.7 + 0.1)
    _, flo, (minu, maxu, minv, maxv), unk = _color(gt)
    sup = engine == "super"
    o = dict(engine=engine, K=c["K"], L=c["L"], temperature=0.2 if sup else 0.0,
             drate=0.75 if sup else 0.5, epsn=1e-6, lambdad=1.0, lambdas=16.0 if sup else 5.0,
             minu=minu, maxu=maxu, minv=minv, maxv=maxv)
    o.update(extra)
    Mo, No = I1.shape
    M, N = (Mo // 4, No // 4) if sup else (Mo, No)
    st = initial_state(o, M, N, seed=seed, engine=engine)
    if init == "tight":
        rng = np.random.default_rng(seed + 100)
        L = c["L"]
        f = 4 if sup else 1
        gu = flo[f // 2::f, f // 2::f, 0][:M, :N]
        gv = flo[f // 2::f, f // 2::f, 1][:M, :N]
        sh = (M, N, L)
        st = State(
            muu=np.asfortranarray(np.clip(gu[:, :, None] + rng.normal(0, 0.5, sh), minu, maxu)),
            muv=np.asfortranarray(np.clip(gv[:, :, None] + rng.normal(0, 0.5, sh), minv, maxv)),
            sigu=np.asfortranarray(0.2 + 1.5 * rng.random(sh)),
            sigv=np.asfortranarray(0.2 + 1.5 * rng.random(sh)),
            pn=np.asfortranarray(0.8 * (rng.random(sh) - 0.5)),
            rou=np.asfortranarray(0.8 * (rng.random(sh + (2, 2)) - 0.5)),
            w=st.w, alpha=st.alpha, it=st.it, T=st.T)
    return I1, I2, flo, unk, o, st


def _color(gt):
    from oracle import gqmap_np
    return gqmap_np.flow_to_color(gt)


def oracle_state(st):
    from oracle import oracle
    return oracle.State(*(np.array(getattr(st, k), order="F", copy=True) for k in
                          ("muu", "muv", "sigu", "sigv", "pn", "rou", "w", "alpha")))


def _coefs(st, K):
    x, _ = np.polynomial.hermite.hermgauss(K)
    XI, XJ = np.meshgrid(x, x)  # XI(r,c) = x_c, XJ(r,c) = x_r (gqmap_gpu_mixture.m:8-9)
    p = st.pn
    sp, sm = np.sqrt(1 + p), np.sqrt(1 - p)
    s, t = (sp + sm) / 2, (sp - sm) / 2
    r2 = np.sqrt(2.0)
    return (x, XI.ravel(order="F"), XJ.ravel(order="F"), r2 * st.sigu * s, r2 * st.sigu * t,
            r2 * st.sigv * t, r2 * st.sigv * s)


def path_coverage(cfg: str, st, Mo: int, No: int, K: int) -> float:
    """Fraction of the work on the fast path: single-scale engines, nodes
    whose every sample is provably unclamped (node_unclamped); super, (node,
    component, quadrature point) triples whose 4x4 block lies inside the
    image (super_block_sum's shared-window branch)."""
    x, XI, XJ, ax, bx, ay, by = _coefs(st, K)
    M, N, L = st.muu.shape
    m = np.arange(M)[:, None, None]
    n = np.arange(N)[None, :, None]
    if CONFIGS[cfg]["engine"] != "super":
        xmax = np.abs(x).max()
        rx = (np.abs(ax) + np.abs(bx)) * xmax + 1e-6
        ry = (np.abs(ay) + np.abs(by)) * xmax + 1e-6
        u1, u2 = st.muu, st.muv
        ok = (u1 - rx >= -n) & (u1 + rx < No - 1 - n) & (u2 - ry >= -m) & (u2 + ry < Mo - 1 - m)
        return float(ok.mean())
    x1 = ax[..., None] * XI + bx[..., None] * XJ + st.muu[..., None]
    x2 = ay[..., None] * XI + by[..., None] * XJ + st.muv[..., None]
    j0, i0 = 4 * n[..., None], 4 * m[..., None]
    safe = (j0 + 1 + x1 >= 1) & (j0 + 4 + x1 <= No - 1) & (i0 + 1 + x2 >= 1) & (i0 + 4 + x2 <= Mo - 1)
    return float(safe.mean())
