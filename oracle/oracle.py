"""ctypes front-end for the oracle library (oracle/gqmap_oracle.c literal
restatement + oracle/gqmap_emul.cpp CPU model of the kernel arithmetic).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py -- never by the product package.  The oracle is
a literal fp64 restatement of gqmap_gpu_mixture.m / gqmap_gpuSuper_mix_entropy.m
(see gqmap_oracle.h for the parity status).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None


class OrcParams(C.Structure):
    _fields_ = [
        ("M", C.c_int), ("N", C.c_int), ("Mo", C.c_int), ("No", C.c_int),
        ("L", C.c_int), ("K", C.c_int), ("super_", C.c_int), ("guard_a", C.c_int),
        ("T", C.c_double), ("drate", C.c_double), ("t_min", C.c_double),
        ("t_decay_every", C.c_int),
        ("epsn", C.c_double), ("lambdad", C.c_double), ("lambdas", C.c_double),
        ("minu", C.c_double), ("maxu", C.c_double), ("minv", C.c_double), ("maxv", C.c_double),
        ("step0", C.c_double), ("step_decay", C.c_double),
        ("sig_lo", C.c_double), ("sig_hi", C.c_double), ("corr_tor", C.c_double),
        ("alpha_mode", C.c_int), ("alpha_start", C.c_int), ("alpha_lr", C.c_double),
        ("tor", C.c_double), ("ctf", C.c_int), ("sig_step", C.c_double),
        ("gh_x", C.POINTER(C.c_double)), ("gh_w", C.POINTER(C.c_double)),
    ]


class OrcState(C.Structure):
    _fields_ = [(n, C.POINTER(C.c_double)) for n in
                ("muu", "muv", "sigu", "sigv", "pn", "rou", "w", "alpha")]


def build() -> str:
    path = os.path.join(_HERE, "liboracle.so")
    srcs = [os.path.join(_HERE, f) for f in ("gqmap_oracle.c", "gqmap_oracle.h", "gqmap_emul.cpp",
                                             "gqmap_pyramid_oracle.c", "gqmap_legacy_oracle.c", "Makefile")]
    srcs.append(os.path.join(os.path.dirname(_HERE), "gqmap-opticalflow_amd", "csrc", "gqmap_math.h"))
    if not os.path.exists(path) or os.path.getmtime(path) < max(os.path.getmtime(f) for f in srcs):
        subprocess.check_call(["make", "-s", "-C", _HERE])
    return path


def lib():
    global _LIB
    if _LIB is None:
        _LIB = C.CDLL(build())
        d = C.POINTER(C.c_double)
        _LIB.orc_run.restype = C.c_int
        _LIB.orc_run.argtypes = [C.POINTER(OrcParams), d, d, C.POINTER(OrcState), d,
                                 C.c_int, C.c_int, d, C.c_int]
        _LIB.orc_interp_cubic.restype = C.c_double
        _LIB.orc_interp_cubic.argtypes = [d, C.c_int, C.c_int, C.c_double, C.c_double]
        _LIB.orc_aepe.restype = C.c_double
    return _LIB


def _p(a):
    return a.ctypes.data_as(C.POINTER(C.c_double))


def _f64(a):
    return np.require(a, dtype=np.float64, requirements=["F_CONTIGUOUS", "ALIGNED", "WRITEABLE"])


def gauss_hermite(K: int):
    x = np.zeros(K); w = np.zeros(K)
    lib().orc_gauss_hermite(C.c_int(K), _p(x), _p(w))
    return x, w


def get_vv(I2: np.ndarray) -> np.ndarray:
    I2 = _f64(I2)
    M, N = I2.shape
    VV = np.zeros((M + 2, N + 2), order="F")
    lib().orc_get_vv(_p(I2), C.c_int(M), C.c_int(N), _p(VV))
    return VV


def interp_cubic(VV: np.ndarray, M: int, N: int, Xq: float, Yq: float) -> float:
    VV = _f64(VV)
    return lib().orc_interp_cubic(_p(VV), M, N, float(Xq), float(Yq))


def make_params(opts: dict, Mo: int, No: int) -> OrcParams:
    """opts uses the reference option names plus the engine knobs of
    gqmap_opticalflow_amd.options (engine, step0, ...)."""
    eng = opts.get("engine", "mixture")
    sup = eng == "super"
    if eng == "ctf":
        # legacy/gqmap_ctf.m constants (see gqmap_options_default)
        opts = dict(dict(step0=0.07, step_decay=1e300, sig_hi=25.0, corr_tor=0.999, guard_a=0,
                         alpha_start=1 << 30, t_decay_every=0, t_min=0.0, temperature=0.0, L=1,
                         sig_step=0.3), **opts)
    p = OrcParams()
    p.Mo, p.No = Mo, No
    p.M, p.N = (Mo // 4, No // 4) if sup else (Mo, No)
    p.L, p.K = int(opts["L"]), int(opts["K"])
    p.super_ = int(sup)
    p.guard_a = int(opts.get("guard_a", not sup))
    p.T = float(opts.get("temperature", 0.0))
    p.drate = float(opts.get("drate", 0.5))
    p.t_min = float(opts.get("t_min", 0.001))
    p.t_decay_every = int(opts.get("t_decay_every", 500 if sup else 0))
    p.epsn, p.lambdad, p.lambdas = float(opts["epsn"]), float(opts["lambdad"]), float(opts["lambdas"])
    p.minu, p.maxu = float(opts["minu"]), float(opts["maxu"])
    p.minv, p.maxv = float(opts["minv"]), float(opts["maxv"])
    p.step0 = float(opts.get("step0", 0.001 if sup else 0.1))
    p.step_decay = float(opts.get("step_decay", 4000.0 if sup else 8000.0))
    p.sig_lo = float(opts.get("sig_lo", 0.01))
    p.sig_hi = float(opts.get("sig_hi", 25.0 if sup else 23.0))
    p.corr_tor = float(opts.get("corr_tor", 1 - 1e-5))
    p.alpha_mode = int(opts.get("alpha_mode", 0))
    # reference constants of the alpha update: projsplx on the super engine
    # it>200, 1E-6 (gqmap_gpuSuper_mix_entropy.m:48), otherwise it>500, 1E-7
    proj_sup = sup and p.alpha_mode == 1
    p.alpha_start = int(opts.get("alpha_start", 200 if proj_sup else 500))
    p.alpha_lr = float(opts.get("alpha_lr", 1e-6 if proj_sup else 1e-7))
    p.tor = float(opts.get("tor", 1e-4))
    p.ctf = int(eng == "ctf")
    p.sig_step = float(opts.get("sig_step", 1.0))
    return p


class State:
    """Host copy of the engine state in MATLAB layout."""

    def __init__(self, muu, muv, sigu, sigv, pn, rou, w, alpha):
        self.muu, self.muv, self.sigu, self.sigv, self.pn = map(_f64, (muu, muv, sigu, sigv, pn))
        self.rou = _f64(rou)
        self.w, self.alpha = _f64(np.ravel(w)), _f64(np.ravel(alpha))

    def copy(self):
        return State(*(np.array(a, order="F", copy=True) for a in self.arrays()))

    def arrays(self):
        return (self.muu, self.muv, self.sigu, self.sigv, self.pn, self.rou, self.w, self.alpha)

    def cstruct(self) -> OrcState:
        s = OrcState()
        for name, a in zip(("muu", "muv", "sigu", "sigv", "pn", "rou", "w", "alpha"), self.arrays()):
            setattr(s, name, _p(a))
        return s


def run(opts: dict, I1: np.ndarray, I2: np.ndarray, state: State, it_first: int, n_iter: int,
        T: float | None = None, nthreads: int = 0, X=None, W=None, det_log: bool = False):
    """Run n_iter iterations in place on `state`.  Returns (done, trace[done,3], T).
    X, W: a Gauss-Hermite rule to use instead of the restated GaussHermite_2.m
    (orc_gauss_hermite) -- e.g. the product's, to compare the iteration
    arithmetic bit for bit with the literal-order engine.  det_log: the
    entropy terms use the device's deterministic log (gqmap_math.h gq_log)
    instead of libm's (T != 0 runs compared bit for bit)."""
    I1 = _f64(I1)
    Mo, No = I1.shape
    p = make_params(opts, Mo, No)
    if X is not None:
        X, W = _f64(np.asarray(X, dtype=np.float64)), _f64(np.asarray(W, dtype=np.float64))
        p.gh_x, p.gh_w = _p(X), _p(W)
    VV = get_vv(I2)
    Tbox = (C.c_double * 1)(p.T if T is None else T)
    trace = np.zeros((max(n_iter, 1), 3))
    cs = state.cstruct()
    L_ = lib()
    L_.orc_set_ent_log.argtypes = [C.c_void_p]
    if det_log:
        L_.orc_set_ent_log(C.cast(L_.emu_gq_log, C.c_void_p))
    try:
        done = L_.orc_run(C.byref(p), _p(I1), _p(VV), C.byref(cs), Tbox, it_first, n_iter,
                          _p(trace), nthreads)
    finally:
        L_.orc_set_ent_log(None)
    return done, trace[:done].copy(), Tbox[0]


def gradients(opts: dict, I1, I2, state: State, T: float | None = None, nthreads: int = 0):
    I1 = _f64(I1)
    Mo, No = I1.shape
    p = make_params(opts, Mo, No)
    VV = get_vv(I2)
    MNL = p.M * p.N * p.L
    node = np.zeros(7 * MNL); edge = np.zeros(7 * MNL * 4)
    lib().orc_gradients(C.byref(p), _p(I1), _p(VV), C.byref(state.cstruct()),
                        C.c_double(p.T if T is None else T), _p(node), _p(edge), nthreads)
    return (node.reshape((p.M, p.N, p.L, 7), order="F"),
            edge.reshape((p.M, p.N, p.L, 2, 2, 7), order="F"))


def log_p(opts: dict, I1, I2, mp) -> float:
    """profile_logP (gqmap_gpu_mixture.m:148-154; super node_lp,
    gqmap_gpuSuper_mix_entropy.m:152-169) of the M x N x 2 MAP flow mp."""
    I1 = _f64(I1)
    Mo, No = I1.shape
    p = make_params(opts, Mo, No)
    VV = get_vv(I2)
    mp = _f64(mp)
    if mp.shape != (p.M, p.N, 2):
        raise ValueError(f"map shape {mp.shape} != node grid {(p.M, p.N, 2)}")
    f = lib().orc_log_p
    f.restype = C.c_double
    f.argtypes = [C.POINTER(OrcParams), C.POINTER(C.c_double), C.POINTER(C.c_double), C.POINTER(C.c_double)]
    return f(C.byref(p), _p(I1), _p(VV), _p(mp))


def projsplx(y) -> np.ndarray:
    y = _f64(np.asarray(y, dtype=np.float64).ravel())
    x = np.zeros_like(y)
    lib().orc_projsplx(_p(y), _p(x), C.c_int(y.size))
    return x


def flow_to_color(flow: np.ndarray, max_flow: float = 0.0):
    flow = _f64(flow)
    M, N, _ = flow.shape
    img = np.zeros((M, N, 3), dtype=np.uint8, order="F")
    flo = np.zeros((M, N, 2), order="F")
    stats = np.zeros(4)
    unk = np.zeros((M, N), dtype=np.uint8, order="F")
    u8 = C.POINTER(C.c_ubyte)
    lib().orc_flow_to_color(_p(flow), C.c_int(M), C.c_int(N), C.c_double(max_flow),
                            img.ctypes.data_as(u8), _p(flo), _p(stats), unk.ctypes.data_as(u8))
    return img, flo, stats, unk.astype(bool)


def aepe(tflow, flow, unknown, r0: int = 1) -> float:
    tflow, flow = _f64(tflow), _f64(flow)
    unk = np.require(unknown, dtype=np.uint8, requirements=["F_CONTIGUOUS"])
    M, N = unk.shape
    f = lib().orc_aepe
    f.argtypes = [C.POINTER(C.c_double), C.POINTER(C.c_double), C.POINTER(C.c_ubyte),
                  C.c_int, C.c_int, C.c_int]
    return f(_p(tflow), _p(flow), unk.ctypes.data_as(C.POINTER(C.c_ubyte)), M, N, r0)


def get_map(alpha, muu, sigu, muv, sigv, nthreads: int = 0, det_exp: bool = False) -> np.ndarray:
    """findMixMax.m:39-70 with MATLAB fminbnd.  det_exp: the mixture density
    uses the device's deterministic exp (gqmap_math.h gq_exp) instead of
    libm's, so the result is comparable bit for bit with k_mixture_map."""
    muu, sigu, muv, sigv = map(_f64, (muu, sigu, muv, sigv))
    alpha = _f64(np.ravel(alpha))
    M, N, L = muu.shape
    out = np.zeros((M, N, 2), order="F")
    L_ = lib()
    L_.orc_set_map_exp.argtypes = [C.c_void_p]
    if det_exp:
        L_.orc_set_map_exp(C.cast(L_.emu_gq_exp, C.c_void_p))
    try:
        L_.orc_get_map(_p(alpha), _p(muu), _p(sigu), _p(muv), _p(sigv), M, N, L, _p(out), nthreads)
    finally:
        L_.orc_set_map_exp(None)
    return out


def split_for(M: int, N: int, super_: bool = False, L: int = 1, ctf: bool = False) -> int:
    """The library's default lanes-per-node policy (gqmap_engine.hip choose_split:
    single-scale mixture and coarse-to-fine levels have their own thresholds;
    the super engine runs its L components as separate blocks: nodes x L)."""
    nodes = M * N
    if not super_ and not ctf:
        return (1 if nodes >= 98304 else 2 if nodes >= (1 << 14) else 4 if nodes >= (1 << 13)
                else 8 if nodes >= (1 << 11) else 64)
    if not super_:
        return (1 if nodes >= (1 << 17) else 2 if nodes >= (1 << 16) else 4 if nodes >= (1 << 13)
                else 8 if nodes >= (1 << 11) else 64)
    nodes *= L
    return 1 if nodes >= (1 << 17) else 4 if nodes >= (1 << 14) else 16


def emu_run(opts: dict, I1, I2, state: State, it_first: int, n_iter: int, X, W,
            T: float | None = None, nthreads: int = 0, fp32: bool = False, split: int | None = None):
    """CPU model of the HIP kernel (oracle/gqmap_emul.cpp): bit-identical to
    libgqmap.so for the same quadrature nodes X, W (pass the product's
    gauss_hermite(K)).  Returns (done, trace[done,3], T)."""
    I1 = _f64(I1)
    Mo, No = I1.shape
    p = make_params(opts, Mo, No)
    VV = get_vv(I2)
    X, W = _f64(np.asarray(X, dtype=np.float64)), _f64(np.asarray(W, dtype=np.float64))
    Tbox = (C.c_double * 1)(p.T if T is None else T)
    trace = np.zeros((max(n_iter, 1), 3))
    cs = state.cstruct()
    f = lib().emu_run
    f.restype = C.c_int
    Q = int(opts.get("split", 0))
    Q = 1 if Q == -1 else Q  # GQMAP_SPLIT_ROLE: a kernel shape with the Q = 1 arithmetic
    Q = Q or (split_for(p.M, p.N, bool(p.super_), int(p.L), opts.get("engine") == "ctf")
              if split is None else split)
    done = f(C.byref(p), _p(X), _p(W), _p(I1), _p(VV), C.byref(cs), Tbox, it_first, n_iter,
             _p(trace), nthreads, int(fp32), Q)
    if done < 0:
        raise RuntimeError("emu_run failed")
    return done, trace[:done].copy(), Tbox[0]


def emu_run_lit(opts: dict, I1, I2, state: State, it_first: int, n_iter: int, X, W,
                T: float | None = None, nthreads: int = 0, geo=None):
    """CPU model of the literal-order engine (gqmap_options.arith = literal;
    gqmap_math.h lit_*): fp64 mixture, Q = 1.  geo as emu_run_tile (None: the
    whole grid).  Returns (done, trace[done,3], T)."""
    I1 = _f64(I1)
    Mo, No = I1.shape
    p = make_params(opts, Mo, No)
    if geo is not None:
        p.N = state.muu.shape[1]
    VV = get_vv(I2)
    X, W = _f64(np.asarray(X, dtype=np.float64)), _f64(np.asarray(W, dtype=np.float64))
    Tbox = (C.c_double * 1)(p.T if T is None else T)
    trace = np.zeros((max(n_iter, 1), 3))
    g = (C.c_int * 4)(*[int(v) for v in geo]) if geo is not None else None
    f = lib().emu_run_lit
    f.restype = C.c_int
    cs = state.cstruct()
    done = f(C.byref(p), _p(X), _p(W), _p(I1), _p(VV), C.byref(cs), Tbox, it_first, n_iter, _p(trace),
             nthreads, g, None)
    if done < 0:
        raise RuntimeError("emu_run_lit: literal mode is the fp64 single-scale mixture engine")
    return done, trace[:done].copy(), Tbox[0]


def emu_math(fn: int, x) -> np.ndarray:
    """Host evaluation of the shared deterministic math (0 sqrt, 1 log, 2 exp)."""
    x = _f64(np.asarray(x, dtype=np.float64).ravel())
    out = np.zeros_like(x)
    f = lib().emu_math
    f.restype = None
    f.argtypes = [C.c_int, C.POINTER(C.c_double), C.POINTER(C.c_double), C.c_int64]
    f(fn, _p(x), _p(out), x.size)
    return out


def emu_sample(VV, Mo: int, No: int, X, Y, fp32: bool = False, cap: bool = False) -> np.ndarray:
    """4 x interp2-cubic of the padded frame VV at absolute 1-based positions
    (X column, Y row) through the kernel's axis arithmetic (gqmap_math.h
    sample4_abs / sample4), or with cap=True the reference's interp2 cell
    choice at the last column / row (cell n-1 at fraction 1)."""
    VV = _f64(VV)
    X = _f64(np.asarray(X, dtype=np.float64).ravel())
    Y = _f64(np.asarray(Y, dtype=np.float64).ravel())
    out = np.zeros_like(X)
    f = lib().emu_sample
    f.restype = None
    f.argtypes = [C.POINTER(C.c_double), C.c_int, C.c_int, C.POINTER(C.c_double), C.POINTER(C.c_double),
                  C.POINTER(C.c_double), C.c_int64, C.c_int, C.c_int]
    f(_p(VV), Mo, No, _p(X), _p(Y), _p(out), X.size, int(fp32), int(cap))
    return out


# ---- coarse-to-fine plumbing (gqmap_pyramid_oracle.c) -----------------------
def resize_len(n: int, scale: float) -> int:
    f = lib().orc_resize_len
    f.restype = C.c_int
    f.argtypes = [C.c_int, C.c_double]
    return f(int(n), float(scale))


def imresize(A, scale: float, antialias: bool = True) -> np.ndarray:
    """imresize(A, scale) restated (bicubic, antialias when shrinking)."""
    A = _f64(np.asarray(A, dtype=np.float64))
    M, N = A.shape[:2]
    Cn = 1 if A.ndim == 2 else int(np.prod(A.shape[2:]))
    out = np.zeros((resize_len(M, scale), resize_len(N, scale)) + A.shape[2:], order="F")
    f = lib().orc_imresize
    f.argtypes = [C.POINTER(C.c_double), C.c_int, C.c_int, C.c_int, C.c_double, C.c_int,
                  C.POINTER(C.c_double)]
    f(_p(A), M, N, Cn, float(scale), int(antialias), _p(out))
    return out


def resize_contrib(in_len: int, out_len: int, scale: float, antialias: bool = True):
    P = lib().orc_resize_taps
    P.restype = C.c_int
    P.argtypes = [C.c_double, C.c_int]
    p = P(float(scale), int(antialias))
    w = np.zeros(out_len * p)
    idx = np.zeros(out_len * p, dtype=np.int32)
    f = lib().orc_resize_contrib
    f.restype = C.c_int
    f.argtypes = [C.c_int, C.c_int, C.c_double, C.c_int, C.POINTER(C.c_double), C.POINTER(C.c_int)]
    k = f(in_len, out_len, float(scale), int(antialias), _p(w), idx.ctypes.data_as(C.POINTER(C.c_int)))
    return w[:out_len * k].reshape(out_len, k), idx[:out_len * k].reshape(out_len, k)


def warp_image(V, warp, fill: bool = True) -> np.ndarray:
    """interp2 linear warp (+ fillmissing nearest dim 1 then 2)."""
    V, warp = _f64(V), _f64(warp)
    M, N = V.shape
    out = np.zeros((M, N), order="F")
    f = lib().orc_warp_image
    f.argtypes = [C.POINTER(C.c_double), C.c_int, C.c_int, C.POINTER(C.c_double), C.POINTER(C.c_double)]
    f(_p(V), M, N, _p(warp), _p(out))
    if fill:
        fillmissing_nearest(out, 1)
        fillmissing_nearest(out, 2)
    return out


def fillmissing_nearest(A: np.ndarray, dim: int) -> np.ndarray:
    """In place on a Fortran-ordered float64 array (returned for chaining)."""
    assert A.flags.f_contiguous and A.dtype == np.float64
    M, N = A.shape
    f = lib().orc_fillmissing_nearest
    f.argtypes = [C.POINTER(C.c_double), C.c_int, C.c_int, C.c_int]
    f(_p(A), M, N, int(dim))
    return A


def ctf_pipeline(opts: dict, img1, img2, scales, init_fn, *, solver: str = "emu", X=None, W=None,
                 nthreads: int = 0, fp32: bool = False):
    """legacy/optical_flow_ctf.m:21-35 with the restated plumbing.

    opts: level options (engine "ctf", its per level) with the FULL-RES GT
    range minu..maxv; level s uses it times s (gqmap_ctf.m:4 on trueFlow.*scale).
    init_fn(level, level_opts, M, N) -> State for the level (the caller's
    seeded initialisation).  solver "emu" (CPU model of the kernel, needs
    X, W) or "literal" (gqmap_oracle.c).  Returns (final warp, per-level dicts)."""
    img1, img2 = _f64(img1), _f64(img2)
    M, N = img1.shape
    s0 = scales[0]
    warp = np.zeros((resize_len(M, s0 / 2), resize_len(N, s0 / 2), 2), order="F")
    levels = []
    for l, s in enumerate(scales):
        I1 = imresize(img1, s)
        I2 = imresize(img2, s)
        warp = _f64(imresize(warp, 2.0) * 2)
        I1w = warp_image(I1, warp)
        lo = dict(opts, engine="ctf", minu=opts["minu"] * s, maxu=opts["maxu"] * s,
                  minv=opts["minv"] * s, maxv=opts["maxv"] * s)
        Ml, Nl = I1.shape
        st = init_fn(l, lo, Ml, Nl)
        its = int(lo["its"])
        if solver == "emu":
            done, tr, _ = emu_run(lo, I1w, I2, st, 1, its, X, W, nthreads=nthreads, fp32=fp32)
        else:
            done, tr, _ = run(lo, I1w, I2, st, 1, its, nthreads=nthreads)
        flow = np.stack([st.muu[:, :, 0], st.muv[:, :, 0]], axis=2)
        warp = _f64(warp + flow)
        levels.append(dict(I1w=I1w, I2=I2, flow=flow, warp=warp.copy(), its=done, trace=tr))
    return warp, levels


def tile_geometry(Ng: int, n_tiles: int, tile: int):
    """Column strip of tile `tile` (gqmap_create_tile): (col0, col1, n_off,
    own_lo, own_hi, N_local)."""
    col0, col1 = Ng * tile // n_tiles, Ng * (tile + 1) // n_tiles
    gl, gr = int(tile > 0), int(tile < n_tiles - 1)
    return col0, col1, col0 - gl, gl, gl + (col1 - col0), (col1 - col0) + gl + gr


def emu_run_tile(opts: dict, I1, I2, state: State, it_first: int, n_iter: int, X, W, geo, *,
                 T: float | None = None, nthreads: int = 0, fp32: bool = False, split: int = 1):
    """CPU model of one tile (local grid state incl. ghost columns, geo =
    (n_off, own_lo, own_hi, Ng)).  Returns (done, trace, T, totals) where
    totals are the last iteration's exact per-tile sums as Python ints
    (value * 2^64): Energy, sum|dmu|, sum|dsigma|, #nonfinite, dalpha[L]."""
    I1 = _f64(I1)
    Mo, No = I1.shape
    p = make_params(opts, Mo, No)
    p.N = state.muu.shape[1]  # local node columns
    VV = get_vv(I2)
    X, W = _f64(np.asarray(X, dtype=np.float64)), _f64(np.asarray(W, dtype=np.float64))
    Tbox = (C.c_double * 1)(p.T if T is None else T)
    trace = np.zeros((max(n_iter, 1), 3))
    g = (C.c_int * 4)(*[int(v) for v in geo])
    tot = np.zeros(2 * (4 + p.L), dtype=np.int64)
    f = lib().emu_run_tile
    f.restype = C.c_int
    cs = state.cstruct()
    done = f(C.byref(p), _p(X), _p(W), _p(I1), _p(VV), C.byref(cs), Tbox, it_first, n_iter, _p(trace),
             nthreads, int(fp32), int(split), g, tot.ctypes.data_as(C.POINTER(C.c_int64)))
    if done < 0:
        raise RuntimeError("emu_run_tile failed")
    totals = [(int(tot[2 * q]) & ((1 << 64) - 1)) + (int(tot[2 * q + 1]) << 64) for q in range(4 + p.L)]
    return done, trace[:done].copy(), Tbox[0], totals


def from_fix(v: int) -> float:
    """gqmap_math.h from_fix: (double)hi + (double)lo * 2^-64 of a value * 2^64."""
    hi, lo = v >> 64, v & ((1 << 64) - 1)
    return float(hi) + float(lo) * 5.42101086242752217004e-20


# ---- legacy flow-denoising engine (gqmap_legacy_oracle.c) ---------------------
class OrcCpuParams(C.Structure):
    _fields_ = [("its", C.c_int), ("K", C.c_int), ("var", C.c_double), ("gama", C.c_double),
                ("dta", C.c_double), ("step0", C.c_double), ("step_decay", C.c_double),
                ("corr_tor", C.c_double), ("tor", C.c_double), ("min_its", C.c_int)]


def cpu_params(opts: dict) -> OrcCpuParams:
    p = OrcCpuParams()
    p.its, p.K = int(opts["its"]), int(opts["K"])
    p.var, p.gama = float(opts.get("var", 1.0)), float(opts.get("gama", 1.0))
    p.dta = float(opts.get("dta", float("inf")))
    p.step0, p.step_decay = float(opts.get("step0", 0.1)), float(opts.get("step_decay", 1000.0))
    p.corr_tor, p.tor = float(opts.get("corr_tor", 0.97)), float(opts.get("tor", 1e-3))
    p.min_its = int(opts.get("min_its", 100))
    return p


def cpu_run(opts: dict, flow, sigma0, X, W, nthreads: int = 1):
    """legacy/gqmap_cpu.m from mu = flow, sigma = sigma0, rou = 0.
    Returns (mu, sigma, rou, trace[its_done, 3])."""
    flow = _f64(flow)
    M, N, _ = flow.shape
    mu = np.array(flow, order="F", copy=True)
    sigma = np.array(sigma0, dtype=np.float64, order="F", copy=True)
    rou = np.zeros((M, N, 2, 2), order="F")
    p = cpu_params(opts)
    trace = np.zeros((max(p.its, 1), 3))
    X, W = _f64(np.asarray(X, dtype=np.float64)), _f64(np.asarray(W, dtype=np.float64))
    f = lib().orc_cpu_run
    f.restype = C.c_int
    done = f(C.byref(p), _p(X), _p(W), _p(flow), M, N, _p(mu), _p(sigma), _p(rou), _p(trace), int(nthreads))
    return mu, sigma, rou, trace[:done].copy()
