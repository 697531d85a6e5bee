"""Legacy flow-denoising engine: host mirror of legacy/gqmap_cpu.m over
libgqmap.so (gqmap_cpu_run, the K-point node rule and K x K edge rules on the
device)."""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib
from ._lib import check, dptr, f64

CPU_KNOBS = ("its", "K", "var", "gama", "dta", "step0", "step_decay", "corr_tor", "tor", "min_its")


def cpu_options(options: dict | None = None) -> _lib.GqmapCpuOptions:
    o = _lib.GqmapCpuOptions()
    _lib.load().gqmap_cpu_options_default(C.byref(o))
    for k, v in (options or {}).items():
        if k in CPU_KNOBS:
            setattr(o, k, type(getattr(o, k))(v))
    return o


def gqmap_cpu(options: dict, flow, *, sigma0=None, seed: int = 0, device: int = 0, return_trace: bool = False):
    """[mu, sigma, rou] = gqmap_cpu(options, flow).  sigma0: the initial sigma
    (the reference draws rand(M,N,2)+2; default: the library RNG from seed)."""
    flow = f64(flow)
    if flow.ndim != 3 or flow.shape[2] != 2:
        raise ValueError("flow must be M x N x 2")
    M, N, _ = flow.shape
    o = cpu_options(options)
    mu = np.zeros((M, N, 2), order="F")
    sigma = np.zeros((M, N, 2), order="F")
    rou = np.zeros((M, N, 2, 2), order="F")
    trace = np.zeros((max(o.its, 1), 3))
    done = C.c_int(0)
    sg = None if sigma0 is None else f64(sigma0)
    if sg is not None and sg.shape != (M, N, 2):
        raise ValueError(f"sigma0 must be {M} x {N} x 2 like flow, got {sg.shape}")
    check(_lib.load().gqmap_cpu_run(C.byref(o), dptr(flow), M, N, dptr(sg) if sg is not None else None,
                                    C.c_uint64(seed), dptr(mu), dptr(sigma), dptr(rou), dptr(trace),
                                    C.byref(done), device), "gqmap_cpu_run")
    if return_trace:
        return mu, sigma, rou, trace[:done.value]
    return mu, sigma, rou


def release() -> None:
    """Free the calling thread's device arenas of gqmap_cpu (gqmap_cpu_release)."""
    check(_lib.load().gqmap_cpu_release(), "gqmap_cpu_release")
