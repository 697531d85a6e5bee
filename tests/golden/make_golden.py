"""Generate the golden vectors under tests/golden/ from the numpy fp64
restatement (oracle/gqmap_np.py) of the reference MATLAB.

The reference itself (MATLAB + Windows MEX) cannot run anywhere in this
pipeline, so these goldens pin the C oracle and the HIP kernels to an
independent restatement of the same MATLAB lines -- see DESIGN.md "Parity".

    python tests/golden/make_golden.py

Inputs are crops of the Middlebury RubberWhale pair (data/middlebury) with an
explicit seeded initial state stored in each .npz.
"""
from __future__ import annotations

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle import gqmap_np  # noqa: E402
from gqmap_opticalflow_amd.flowio import load_pair  # noqa: E402


def crop_pair(r0, c0, M, N, name="rubberwhale"):
    I1, I2, gt = load_pair(name)
    return (np.asfortranarray(I1[r0:r0 + M, c0:c0 + N]), np.asfortranarray(I2[r0:r0 + M, c0:c0 + N]),
            np.asfortranarray(gt[r0:r0 + M, c0:c0 + N]))


def random_state(rng, M, N, L, opts, corr=0.6):
    du, dv = opts["maxu"] - opts["minu"], opts["maxv"] - opts["minv"]
    w = rng.random(L)
    return dict(
        muu=np.asfortranarray(opts["minu"] + rng.random((M, N, L)) * du),
        muv=np.asfortranarray(opts["minv"] + rng.random((M, N, L)) * dv),
        sigu=np.asfortranarray(rng.random((M, N, L)) + du),
        sigv=np.asfortranarray(rng.random((M, N, L)) + dv),
        pn=np.asfortranarray(corr * (2 * rng.random((M, N, L)) - 1)),
        rou=np.asfortranarray(corr * (2 * rng.random((M, N, L, 2, 2)) - 1)),
        w=w, alpha=np.exp(w) / np.exp(w).sum())


CASES = {
    # single-scale mixture engine (gqmap_gpu_mixture.m), K=9 as optical_flow.m:16
    "mixture_L1": dict(engine="mixture", crop=(120, 200, 20, 28), K=9, L=1, temperature=0.0,
                       lambdas=5.0, lambdad=1.0, its=4, seed=1),
    "mixture_L3_T": dict(engine="mixture", crop=(60, 300, 18, 22), K=9, L=3, temperature=0.3,
                         lambdas=5.0, lambdad=1.0, its=3, seed=2, alpha_start=1, alpha_lr=1e-3),
    "mixture_L3_proj": dict(engine="mixture", crop=(200, 100, 16, 20), K=7, L=3, temperature=0.1,
                            lambdas=5.0, lambdad=1.0, its=3, seed=3, alpha_start=1, alpha_lr=1e-4,
                            alpha_mode=1),
    # 4x4 super-pixel engine (gqmap_gpuSuper_mix_entropy.m), drivers use K=11
    "super_L3": dict(engine="super", crop=(100, 240, 32, 40), K=11, L=3, temperature=0.2,
                     drate=0.75, lambdas=16.0, lambdad=1.0, its=3, seed=4, alpha_start=1,
                     alpha_lr=1e-4, t_decay_every=2),
    # coarse-to-fine level solver (legacy/gqmap_ctf.m), K=11 as optical_flow_ctf.m:13
    "ctf_L1": dict(engine="ctf", crop=(200, 300, 22, 30), K=11, L=1, temperature=0.0,
                   lambdas=5.0, lambdad=1.0, its=3, seed=5, pair="Grove3"),
}


def make_case(name, c):
    r0, c0, M, N = c["crop"]
    I1, I2, gt = crop_pair(r0, c0, M, N, c.get("pair", "rubberwhale"))
    # minu..maxv come from flowToColor of the GT (unknown pixels zeroed), optical_flow.m:12-13
    _, _, (minu, maxu, minv, maxv), _ = gqmap_np.flow_to_color(gt)
    opts = dict(engine=c["engine"], K=c["K"], L=c["L"], temperature=c["temperature"],
                drate=c.get("drate", 0.5), epsn=1e-6, lambdad=c["lambdad"], lambdas=c["lambdas"],
                minu=float(minu) - 0.5, maxu=float(maxu) + 0.5,
                minv=float(minv) - 0.5, maxv=float(maxv) + 0.5)
    for k in ("alpha_start", "alpha_lr", "alpha_mode", "t_decay_every"):
        if k in c:
            opts[k] = c[k]
    eng = gqmap_np.Engine(opts, I1, I2)
    rng = np.random.default_rng(c["seed"])
    st = random_state(rng, eng.M, eng.N, c["L"], opts)
    init = {k: v.copy() for k, v in st.items()}
    T = opts["temperature"]
    node0, edge0 = eng.gradients(st, T)
    trace = []
    step1 = None
    for it in range(1, c["its"] + 1):
        e, pm, ps, T = eng.iterate(st, it, T)
        trace.append((e, pm, ps))
        if it == 1:
            step1 = {k: v.copy() for k, v in st.items()}
    out = dict(I1=I1, I2=I2, trace=np.array(trace), T_final=T,
               node0=np.stack(node0, axis=-1), edge0=np.stack(edge0, axis=-1))
    for k, v in init.items():
        out["init_" + k] = v
    for k, v in st.items():
        out["final_" + k] = v
    for k, v in step1.items():
        out["step1_" + k] = v
    np.savez_compressed(os.path.join(HERE, f"{name}.npz"), opts=np.array(repr(opts)), **out)
    print(name, eng.M, eng.N, "trace", np.array(trace)[-1])


def make_color():
    _, _, gt = load_pair("rubberwhale")
    flow = np.asfortranarray(gt[150:214, 250:330])
    flow[3, 5, :] = 1e10  # one unknown pixel
    img, flo, stats, unk = gqmap_np.flow_to_color(flow)
    np.savez_compressed(os.path.join(HERE, "flow_to_color.npz"), flow=flow, img=img, flo=flo,
                        stats=np.array(stats), unknown=unk)
    print("flow_to_color", img.shape, stats)


# coarse-to-fine driver (legacy/optical_flow_ctf.m:21-35) on a Grove3 crop:
# 3 levels 16x24 -> 32x48 -> 64x96, a few iterations per level, explicit
# per-level initial states (sigma = U + 3, gqmap_ctf.m:16-17)
CTF_PIPE = dict(crop=(150, 200, 64, 96), scales=(0.25, 0.5, 1.0), its=4, K=11, seed=50)


def ctf_level_state(seed, l, M, N, lo):
    rng = np.random.default_rng(seed + l)
    du, dv = lo["maxu"] - lo["minu"], lo["maxv"] - lo["minv"]
    f = lambda a: np.asfortranarray(a.reshape(M, N, 1))
    return dict(muu=f(lo["minu"] + rng.random(M * N) * du), muv=f(lo["minv"] + rng.random(M * N) * dv),
                sigu=f(rng.random(M * N) + 3), sigv=f(rng.random(M * N) + 3),
                pn=np.zeros((M, N, 1), order="F"), rou=np.zeros((M, N, 1, 2, 2), order="F"),
                w=np.zeros(1), alpha=np.ones(1))


def make_ctf_pipeline():
    c = CTF_PIPE
    r0, c0, M, N = c["crop"]
    img1, img2, gt = crop_pair(r0, c0, M, N, "Grove3")
    _, _, (minu, maxu, minv, maxv), _ = gqmap_np.flow_to_color(gt)
    opts = dict(engine="ctf", K=c["K"], L=1, its=c["its"], epsn=1e-6, lambdas=5.0, lambdad=1.0,
                temperature=0.0, minu=float(minu), maxu=float(maxu), minv=float(minv), maxv=float(maxv))
    inits = {}

    def init_fn(l, lo, Ml, Nl):
        st = ctf_level_state(c["seed"], l, Ml, Nl, lo)
        inits[l] = {k: v.copy() for k, v in st.items()}
        return st

    warp, levels = gqmap_np.ctf_pipeline(opts, img1, img2, c["scales"], init_fn)
    out = dict(img1=img1, img2=img2, scales=np.array(c["scales"]), warp=warp)
    for l, lv in enumerate(levels):
        for k, v in lv.items():
            out[f"L{l}_{k}"] = v
        for k, v in inits[l].items():
            out[f"L{l}_init_{k}"] = v
    np.savez_compressed(os.path.join(HERE, "ctf_pipeline.npz"), opts=np.array(repr(opts)), **out)
    print("ctf_pipeline", [lv["I1w"].shape for lv in levels], float(np.abs(warp).max()))


# legacy flow-denoising engine (legacy/gqmap_cpu.m): Dimetrodon GT crop with
# unknowns zeroed, sigma0 = U + 2 (seeded), var = gama = 1, dta = inf and 2.5
def make_legacy():
    from gqmap_opticalflow_amd.flowio import load_pair as lp
    _, _, gt = lp("Dimetrodon")
    flow = np.asfortranarray(gt[150:190, 200:252])
    flow[np.abs(flow) > 1e9] = 0
    rng = np.random.default_rng(60)
    sigma0 = np.asfortranarray(rng.random(flow.shape) + 2)
    X, W = gqmap_np.gauss_hermite(9)
    out = dict(flow=flow, sigma0=sigma0, X=X, W=W)
    for tag, dta in (("inf", np.inf), ("trunc", 2.5)):
        opts = dict(its=12, K=9, var=1.0, gama=1.0, dta=dta)
        mu, sg, rou, tr = gqmap_np.cpu_engine(opts, flow, sigma0, X, W)
        out.update({f"{tag}_mu": mu, f"{tag}_sigma": sg, f"{tag}_rou": rou, f"{tag}_trace": tr})
    np.savez_compressed(os.path.join(HERE, "legacy_cpu.npz"), **out)
    print("legacy_cpu", flow.shape, out["inf_trace"][-1], out["trunc_trace"][-1])


if __name__ == "__main__":
    for n, c in CASES.items():
        make_case(n, c)
    make_color()
    make_ctf_pipeline()
    make_legacy()
