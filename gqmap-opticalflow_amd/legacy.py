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


def _fortran_dev(shape, device):
    """An uninitialised float64 device tensor laid out column-major (MATLAB
    order: first index fastest), as the C-ABI expects."""
    import torch
    strides, st = [], 1
    for n in shape:
        strides.append(st)
        st *= n
    return torch.empty_strided(tuple(shape), tuple(strides), dtype=torch.float64, device=device)


def _check_dev(name, t, shape):
    import torch
    if not (isinstance(t, torch.Tensor) and t.is_cuda and t.dtype == torch.float64):
        raise TypeError(f"{name} must be a float64 device tensor")
    if tuple(t.shape) != tuple(shape):
        raise ValueError(f"{name} must be {' x '.join(map(str, shape))}, got {tuple(t.shape)}")
    want, st = [], 1
    for n in shape:
        want.append(st)
        st *= n
    if tuple(t.stride()) != tuple(want):
        raise ValueError(f"{name} must be column-major (strides {tuple(want)}), got {tuple(t.stride())}")


def gqmap_cpu_device(options: dict, flow, *, sigma0=None, seed: int = 0, return_trace: bool = False):
    """gqmap_cpu on device arrays (gqmap_cpu_run_device): flow an M x N x 2
    float64 tensor on a HIP device, column-major (strides (1, M, M*N):
    `torch.from_numpy(np.asfortranarray(flow)).cuda()`); sigma0 likewise or
    None.  Returns mu, sigma (M x N x 2) and rou (M x N x 2 x 2) as device
    tensors in the same layout (and the its_done x 3 trace) -- no host copies,
    the same bits as gqmap_cpu."""
    M, N = int(flow.shape[0]), int(flow.shape[1])
    _check_dev("flow", flow, (M, N, 2))
    if sigma0 is not None:
        _check_dev("sigma0", sigma0, (M, N, 2))
        if sigma0.device != flow.device:
            raise ValueError(f"sigma0 is on {sigma0.device}, flow on {flow.device}: one device")
    o = cpu_options(options)
    dev = flow.device
    mu, sigma, rou = _fortran_dev((M, N, 2), dev), _fortran_dev((M, N, 2), dev), _fortran_dev((M, N, 2, 2), dev)
    import torch
    trace = torch.empty((max(o.its, 1), 3), dtype=torch.float64, device=dev)
    # the library runs on its own HIP runtime's queue: torch work that
    # produced flow / sigma0 must have finished (the call itself returns
    # synchronised)
    torch.cuda.synchronize(dev)
    done = C.c_int(0)
    check(_lib.load().gqmap_cpu_run_device(C.byref(o), flow.data_ptr(), M, N,
                                           sigma0.data_ptr() if sigma0 is not None else None, C.c_uint64(seed),
                                           mu.data_ptr(), sigma.data_ptr(), rou.data_ptr(), trace.data_ptr(),
                                           C.byref(done), dev.index if dev.index is not None else 0),
          "gqmap_cpu_run_device")
    if return_trace:
        return mu, sigma, rou, trace[:done.value]
    return mu, sigma, rou


def release() -> None:
    """Free the calling thread's device arenas of gqmap_cpu (gqmap_cpu_release)."""
    check(_lib.load().gqmap_cpu_release(), "gqmap_cpu_release")
