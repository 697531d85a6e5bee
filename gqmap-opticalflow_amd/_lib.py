"""ctypes binding of libgqmap.so (include/gqmap.h).

The shared library is the product: HIP kernels for gfx950 plus the host
runtime.  This module never falls back to anything else -- if the library is
missing or no GPU is present the calls raise.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("GQMAP_LIB", os.path.join(PKG_DIR, "libgqmap.so"))

GQMAP_OK = 0
ENGINE_MIXTURE, ENGINE_SUPER, ENGINE_CTF = 0, 1, 2
FP64, FP32 = 0, 1
ALPHA_SOFTMAX, ALPHA_PROJSPLX = 0, 1
ARITH_FAST, ARITH_LITERAL = 0, 1  # gqmap_options.arith (ABI 2)
ABI_VERSION = 2
SPLIT_ROLE = -1  # GQMAP_SPLIT_ROLE: options["split"] for the role-split kernel shape (Q = 1 arithmetic)
LMAX, KMAX = 8, 16

# Every entry point declared in include/gqmap.h (checked by tests/test_abi.py).
EXPORTS = (
    "gqmap_options_default", "gqmap_options_alpha_mode", "gqmap_create", "gqmap_set_images", "gqmap_init_state",
    "gqmap_set_state", "gqmap_get_state", "gqmap_run", "gqmap_run_aepe", "gqmap_set_truth", "gqmap_run_timed", "gqmap_prepare", "gqmap_get_info",
    "gqmap_get_map", "gqmap_log_p", "gqmap_synchronize", "gqmap_destroy", "gqmap_projsplx",
    "gqmap_mixture_map", "gqmap_flow_to_color", "gqmap_gauss_hermite", "gqmap_rand_uniform",
    "gqmap_last_error", "gqmap_abi_version", "gqmap_device_count", "gqmap_imresize",
    "gqmap_warp_image", "gqmap_ctf_create", "gqmap_ctf_set_images", "gqmap_ctf_run",
    "gqmap_ctf_get_level", "gqmap_ctf_set_truth", "gqmap_ctf_get_trace", "gqmap_ctf_destroy", "gqmap_resize_len", "gqmap_create_tile",
    "gqmap_comm_unique_id", "gqmap_tile_attach_rccl", "gqmap_tile_group_run", "gqmap_tile_attach_host",
    "gqmap_tile_exchange_sizes", "gqmap_tile_exchange_begin", "gqmap_tile_exchange_end",
    "gqmap_cpu_options_default", "gqmap_cpu_run", "gqmap_cpu_run_device", "gqmap_cpu_release", "gqmap_read_flo", "gqmap_write_flo", "gqmap_aepe",
)
CTF_MAX_LEVELS = 8


class GqmapOptions(C.Structure):
    _fields_ = [
        ("its", C.c_int), ("K", C.c_int), ("L", C.c_int),
        ("temperature", C.c_double), ("drate", C.c_double), ("epsn", C.c_double),
        ("lambdad", C.c_double), ("lambdas", C.c_double),
        ("minu", C.c_double), ("maxu", C.c_double), ("minv", C.c_double), ("maxv", C.c_double),
        ("engine", C.c_int), ("precision", C.c_int), ("alpha_mode", C.c_int),
        ("alpha_start", C.c_int), ("alpha_lr", C.c_double),
        ("guard_a", C.c_int), ("t_decay_every", C.c_int), ("t_min", C.c_double),
        ("step0", C.c_double), ("step_decay", C.c_double),
        ("sig_lo", C.c_double), ("sig_hi", C.c_double), ("corr_tor", C.c_double),
        ("tor", C.c_double), ("split", C.c_int), ("sig_step", C.c_double), ("sig_init", C.c_double),
        ("arith", C.c_int),
    ]


_D = C.POINTER(C.c_double)


class GqmapCpuOptions(C.Structure):
    _fields_ = [("its", C.c_int), ("K", C.c_int), ("var", C.c_double), ("gama", C.c_double),
                ("dta", C.c_double), ("step0", C.c_double), ("step_decay", C.c_double),
                ("corr_tor", C.c_double), ("tor", C.c_double), ("min_its", C.c_int)]


class GqmapState(C.Structure):
    _fields_ = [("muu", _D), ("muv", _D), ("sigu", _D), ("sigv", _D), ("pn", _D),
                ("rou", _D), ("w", _D), ("alpha", _D), ("it", C.c_int), ("T", C.c_double)]


class GqmapInfo(C.Structure):
    _fields_ = [("Mo", C.c_int), ("No", C.c_int), ("M", C.c_int), ("N", C.c_int),
                ("L", C.c_int), ("K", C.c_int), ("it", C.c_int), ("stopped", C.c_int),
                ("T", C.c_double), ("device", C.c_int), ("split", C.c_int),
                ("n_tiles", C.c_int), ("tile", C.c_int), ("col0", C.c_int), ("col1", C.c_int)]


class GqmapError(RuntimeError):
    pass


_lib = None


def load():
    """Load libgqmap.so (raises if it was not built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise GqmapError(f"{LIB_PATH} not built: run `make -C {PKG_DIR}` "
                         "(or __graft_entry__.build())")
    lib = C.CDLL(LIB_PATH)
    lib.gqmap_abi_version.restype = C.c_int
    if lib.gqmap_abi_version() != ABI_VERSION:
        raise GqmapError(f"{LIB_PATH}: ABI {lib.gqmap_abi_version()}, this binding is ABI {ABI_VERSION} "
                         "(rebuild the library)")
    P = C.POINTER
    u8 = P(C.c_uint8)
    vp = C.c_void_p
    sig = {
        "gqmap_options_default": (None, [P(GqmapOptions), C.c_int]),
        "gqmap_options_alpha_mode": (C.c_int, [P(GqmapOptions), C.c_int]),
        "gqmap_create": (C.c_int, [P(vp), P(GqmapOptions), C.c_int]),
        "gqmap_set_images": (C.c_int, [vp, _D, _D, C.c_int, C.c_int]),
        "gqmap_init_state": (C.c_int, [vp, C.c_uint64]),
        "gqmap_set_state": (C.c_int, [vp, P(GqmapState)]),
        "gqmap_get_state": (C.c_int, [vp, P(GqmapState)]),
        "gqmap_run": (C.c_int, [vp, C.c_int, P(C.c_int), _D]),
        "gqmap_run_aepe": (C.c_int, [vp, C.c_int, P(C.c_int), _D, _D]),
        "gqmap_set_truth": (C.c_int, [vp, _D, C.c_int, C.c_int]),
        "gqmap_run_timed": (C.c_int, [vp, C.c_int, P(C.c_int), _D, _D]),
        "gqmap_prepare": (C.c_int, [vp]),
        "gqmap_get_info": (C.c_int, [vp, P(GqmapInfo)]),
        "gqmap_get_map": (C.c_int, [vp, _D]),
        "gqmap_log_p": (C.c_int, [vp, _D, _D]),
        "gqmap_synchronize": (C.c_int, [vp]),
        "gqmap_destroy": (None, [vp]),
        "gqmap_projsplx": (C.c_int, [_D, _D, C.c_int, C.c_int, C.c_int]),
        "gqmap_mixture_map": (C.c_int, [_D, _D, _D, _D, _D, C.c_int, C.c_int, C.c_int, _D, C.c_int]),
        "gqmap_flow_to_color": (C.c_int, [_D, C.c_int, C.c_int, C.c_double, u8, _D, _D, u8, C.c_int]),
        "gqmap_gauss_hermite": (C.c_int, [C.c_int, _D, _D]),
        "gqmap_rand_uniform": (None, [C.c_uint64, C.c_uint32, C.c_uint64, C.c_size_t, _D]),
        "gqmap_last_error": (C.c_char_p, []),
        "gqmap_abi_version": (C.c_int, []),
        "gqmap_device_count": (C.c_int, []),
        "gqmap_imresize": (C.c_int, [_D, C.c_int, C.c_int, C.c_int, C.c_double, C.c_int, _D, C.c_int]),
        "gqmap_warp_image": (C.c_int, [_D, C.c_int, C.c_int, _D, C.c_int, _D, C.c_int]),
        "gqmap_ctf_create": (C.c_int, [P(vp), P(GqmapOptions), _D, C.c_int, C.c_int]),
        "gqmap_ctf_set_images": (C.c_int, [vp, _D, _D, C.c_int, C.c_int]),
        "gqmap_ctf_run": (C.c_int, [vp, C.c_uint64, _D, P(C.c_int), _D]),
        "gqmap_ctf_get_level": (C.c_int, [vp, C.c_int, P(C.c_int), P(C.c_int), _D, _D, _D, _D]),
        "gqmap_ctf_set_truth": (C.c_int, [vp, _D, C.c_int, C.c_int]),
        "gqmap_ctf_get_trace": (C.c_int, [vp, C.c_int, P(C.c_int), _D, _D]),
        "gqmap_ctf_destroy": (None, [vp]),
        "gqmap_resize_len": (C.c_int, [C.c_int, C.c_double]),
        "gqmap_create_tile": (C.c_int, [P(vp), P(GqmapOptions), C.c_int, C.c_int, C.c_int]),
        "gqmap_comm_unique_id": (C.c_int, [u8]),
        "gqmap_tile_attach_rccl": (C.c_int, [vp, u8]),
        "gqmap_tile_group_run": (C.c_int, [P(vp), C.c_int, C.c_int, P(C.c_int), _D]),
        "gqmap_tile_attach_host": (C.c_int, [vp]),
        "gqmap_tile_exchange_sizes": (C.c_int, [vp, P(C.c_size_t)]),
        "gqmap_tile_exchange_begin": (C.c_int, [vp, vp, vp, vp]),
        "gqmap_tile_exchange_end": (C.c_int, [vp, vp, vp, vp, _D]),
        "gqmap_cpu_options_default": (None, [P(GqmapCpuOptions)]),
        "gqmap_cpu_release": (C.c_int, []),
        "gqmap_read_flo": (C.c_int, [C.c_char_p, P(C.c_int), P(C.c_int), _D]),
        "gqmap_write_flo": (C.c_int, [C.c_char_p, _D, C.c_int, C.c_int]),
        "gqmap_aepe": (C.c_int, [_D, _D, u8, C.c_int, C.c_int, C.c_int, _D]),
        "gqmap_cpu_run": (C.c_int, [P(GqmapCpuOptions), _D, C.c_int, C.c_int, _D, C.c_uint64, _D, _D, _D, _D,
                                    P(C.c_int), C.c_int]),
        "gqmap_cpu_run_device": (C.c_int, [P(GqmapCpuOptions), vp, C.c_int, C.c_int, vp, C.c_uint64, vp, vp, vp,
                                           vp, P(C.c_int), C.c_int]),
    }
    for name, (res, args) in sig.items():
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args
    _lib = lib
    return lib


def debug_policy(name: str, value: int) -> None:
    """Set one execution policy of the library (gqmap_debug_policy, not in the
    public header): placement / caching / launch-shape choices that never
    change a result -- nt_state, band_rows, cu_group, lpar, lpar_xcd,
    fused_finalize, persist, persist_cap, graph, vv_float, vv_pair, flow,
    verbose.  value -1
    restores the automatic choice.  Contexts created afterwards use it."""
    f = load().gqmap_debug_policy
    f.restype = C.c_int
    f.argtypes = [C.c_char_p, C.c_int]
    if f(name.encode(), int(value)) != 0:
        raise GqmapError(f"unknown policy {name!r}")


def check(status: int, what: str = "gqmap") -> None:
    if status != GQMAP_OK:
        msg = load().gqmap_last_error().decode(errors="replace")
        raise GqmapError(f"{what}: status {status}: {msg}")


def dptr(a: np.ndarray):
    return a.ctypes.data_as(_D)


def u8ptr(a: np.ndarray):
    return a.ctypes.data_as(C.POINTER(C.c_uint8))


def f64(a) -> np.ndarray:
    """Column-major contiguous float64 view/copy (MATLAB layout)."""
    return np.require(np.asarray(a, dtype=np.float64), requirements=["F_CONTIGUOUS", "ALIGNED"])
