"""Python mirror of the reference engines' call signature, over the C ABI.

    mu, sigma, alpha, AEPE, Energy, logP = gqmap_gpu_mixture(options, I1, I2)
        -- gqmap_gpu_mixture.m:1 (optical_flow.m:27)
    mu, sigma, alpha, AEPE, Energy, logP = gqmap_gpuSuper_mix_entropy(options, I1, I2)
        -- gqmap_gpuSuper_mix_entropy.m:1 (optical_flowSuper.m:34)

`options` is a dict with the MATLAB field names (trueFlow, unknownIdx, its,
K, L, temperature, drate, epsn, lambdad, lambdas, minu, maxu, minv, maxv,
dir).  The solver loop runs on the GPU (libgqmap.so); the host keeps what the
reference keeps on the host: the evaluation block every 300 iterations
(gqmap_gpu_mixture.m:52-68: MAP, flowToColor, PNG, AEPE, logP) and the
per-iteration console line.
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass

import numpy as np

from . import _lib
from ._lib import check, dptr, f64
from .ops import flow_to_color

ENGINES = {"mixture": _lib.ENGINE_MIXTURE, "super": _lib.ENGINE_SUPER, "ctf": _lib.ENGINE_CTF}
PRECISIONS = {"fp64": _lib.FP64, "fp32": _lib.FP32}
KNOBS = ("alpha_mode", "alpha_start", "alpha_lr", "guard_a", "t_decay_every", "t_min", "step0",
         "step_decay", "sig_lo", "sig_hi", "corr_tor", "tor", "split", "sig_step", "sig_init", "arith")
ARITH = {"fast": _lib.ARITH_FAST, "literal": _lib.ARITH_LITERAL}


def make_options(options: dict, engine: str = "mixture", precision: str = "fp64") -> _lib.GqmapOptions:
    lib = _lib.load()
    o = _lib.GqmapOptions()
    lib.gqmap_options_default(C.byref(o), ENGINES[engine])
    for k in ("its", "K", "L"):
        if k in options:
            setattr(o, k, int(options[k]))
    for k in ("temperature", "drate", "epsn", "lambdad", "lambdas", "minu", "maxu", "minv", "maxv"):
        if k in options:
            setattr(o, k, float(options[k]))
    o.engine = ENGINES[engine]
    if "alpha_mode" in options:  # the mode's reference alpha_start / alpha_lr, unless given below
        check(lib.gqmap_options_alpha_mode(C.byref(o), int(options["alpha_mode"])), "alpha_mode")
    for k in KNOBS:
        if k in options:
            cur = getattr(o, k)
            v = options[k]
            if k == "arith" and isinstance(v, str):
                v = ARITH[v]
            setattr(o, k, type(cur)(v))
    o.engine = ENGINES[engine]
    o.precision = PRECISIONS[precision]
    return o


@dataclass
class State:
    """Engine state in MATLAB layout (M x N x L, rou M x N x L x 2 x 2)."""
    muu: np.ndarray
    muv: np.ndarray
    sigu: np.ndarray
    sigv: np.ndarray
    pn: np.ndarray
    rou: np.ndarray
    w: np.ndarray
    alpha: np.ndarray
    it: int = 1
    T: float = 0.0

    def cstruct(self) -> _lib.GqmapState:
        s = _lib.GqmapState()
        for k in ("muu", "muv", "sigu", "sigv", "pn", "rou", "w", "alpha"):
            setattr(s, k, dptr(getattr(self, k)))
        s.it, s.T = int(self.it), float(self.T)
        return s

    @staticmethod
    def empty(M: int, N: int, L: int) -> "State":
        z = lambda *sh: np.zeros(sh, order="F")
        return State(z(M, N, L), z(M, N, L), z(M, N, L), z(M, N, L), z(M, N, L),
                     z(M, N, L, 2, 2), np.zeros(L), np.zeros(L))

    def copy(self) -> "State":
        return State(*(np.array(getattr(self, k), order="F", copy=True) for k in
                       ("muu", "muv", "sigu", "sigv", "pn", "rou", "w", "alpha")), self.it, self.T)


def rand_uniform(seed: int, stream: int, n: int, first: int = 0) -> np.ndarray:
    """The library's counter-based U(0,1) stream (host evaluation)."""
    out = np.empty(n)
    _lib.load().gqmap_rand_uniform(C.c_uint64(seed), C.c_uint32(stream), C.c_uint64(first),
                                   C.c_size_t(n), dptr(out))
    return out


def initial_state(options: dict, M: int, N: int, seed: int = 0, T: float | None = None,
                  engine: str = "mixture") -> State:
    """Host copy of gqmap_init_state: gqmap_gpu_mixture.m:18-24 with the
    library RNG (what the device generates for the same seed)."""
    L = int(options["L"])
    MNL = M * N * L
    sh = lambda a: a.reshape((M, N, L), order="F")
    w = rand_uniform(seed, 0, L)
    du, dv = options["maxu"] - options["minu"], options["maxv"] - options["minv"]
    # sigma offset: (max-min) for the mixture engines, 3 for ctf (gqmap_ctf.m:16-17)
    sig_init = float(options.get("sig_init", 3.0 if engine == "ctf" else -1.0))
    su, sv = (du, dv) if sig_init < 0 else (sig_init, sig_init)
    st = State(
        muu=sh(options["minu"] + rand_uniform(seed, 1, MNL) * du),
        muv=sh(options["minv"] + rand_uniform(seed, 2, MNL) * dv),
        sigu=sh(rand_uniform(seed, 3, MNL) + su),
        sigv=sh(rand_uniform(seed, 4, MNL) + sv),
        pn=np.zeros((M, N, L), order="F"), rou=np.zeros((M, N, L, 2, 2), order="F"),
        w=w, alpha=np.exp(w) / np.exp(w).sum(), it=1,
        T=float(options.get("temperature", 0.0) if T is None else T))
    return st


class Engine:
    """One device context (gqmap_ctx) holding images and state on the GPU."""

    def __init__(self, options: dict, I1, I2, engine: str = "mixture", precision: str = "fp64",
                 device: int = 0, n_tiles: int = 1, tile: int = 0):
        self.lib = _lib.load()
        self.engine, self.precision = engine, precision
        self.opts = make_options(options, engine, precision)
        self.ctx = C.c_void_p()
        if n_tiles == 1:
            check(self.lib.gqmap_create(C.byref(self.ctx), C.byref(self.opts), device), "gqmap_create")
        else:
            check(self.lib.gqmap_create_tile(C.byref(self.ctx), C.byref(self.opts), device, n_tiles, tile),
                  "gqmap_create_tile")
        I1, I2 = f64(I1), f64(I2)
        if I1.shape != I2.shape or I1.ndim != 2:
            raise ValueError("I1 and I2 must be equal-size 2-D images")
        self.Mo, self.No = I1.shape
        check(self.lib.gqmap_set_images(self.ctx, dptr(I1), dptr(I2), self.Mo, self.No),
              "gqmap_set_images")
        info = self.info()
        self.M, self.N, self.L = info.M, info.N, info.L  # full node grid (a tile owns col0:col1)
        self.n_tiles, self.tile, self.col0, self.col1 = info.n_tiles, info.tile, info.col0, info.col1

    # -- multi-GPU tiles ---------------------------------------------------
    def attach_rccl(self, unique_id: bytes) -> None:
        """Join the RCCL communicator of all tiles (rank == tile); collective."""
        buf = (C.c_uint8 * 128).from_buffer_copy(bytes(unique_id))
        check(self.lib.gqmap_tile_attach_rccl(self.ctx, buf), "gqmap_tile_attach_rccl")

    def attach_host(self) -> None:
        """Host-staged transport (gqmap_tile_attach_host): the caller moves
        the boundary columns and totals between exchange_begin / _end."""
        check(self.lib.gqmap_tile_attach_host(self.ctx), "gqmap_tile_attach_host")
        sz = (C.c_size_t * 6)()
        check(self.lib.gqmap_tile_exchange_sizes(self.ctx, sz), "gqmap_tile_exchange_sizes")
        # send_left, send_right, recv_left, recv_right, totals, totals_all (bytes)
        self.xfer_sizes = tuple(int(v) for v in sz)

    def exchange_begin(self):
        """One iteration up to the exchange: (send_left, send_right, totals)
        as uint8 arrays (send_* empty at the strip ends)."""
        sl, sr, _, _, tot, _ = self.xfer_sizes
        bufs = [np.zeros(n, np.uint8) for n in (sl, sr, tot)]
        ptrs = [b.ctypes.data_as(C.c_void_p) if b.size else None for b in bufs]
        check(self.lib.gqmap_tile_exchange_begin(self.ctx, *ptrs), "gqmap_tile_exchange_begin")
        return tuple(bufs)

    def exchange_end(self, recv_left, recv_right, totals_all) -> np.ndarray:
        """Finish the iteration with the neighbours' columns (recv_left from
        tile-1's send_right, recv_right from tile+1's send_left) and every
        tile's totals in tile order.  Returns Energy, ptdmu, ptdsigma."""
        tr = np.zeros(3)
        bufs = [np.ascontiguousarray(b, np.uint8) if b is not None else None
                for b in (recv_left, recv_right, totals_all)]
        for b, n, what in zip(bufs, self.xfer_sizes[2:4] + self.xfer_sizes[5:], ("recv_left", "recv_right", "totals_all")):
            if n and (b is None or b.size != n):
                raise ValueError(f"{what} must hold {n} bytes")
        ptrs = [b.ctypes.data_as(C.c_void_p) if b is not None and b.size else None for b in bufs]
        check(self.lib.gqmap_tile_exchange_end(self.ctx, *ptrs, dptr(tr)), "gqmap_tile_exchange_end")
        return tr

    # -- state -----------------------------------------------------------
    def init_state(self, seed: int = 0) -> None:
        check(self.lib.gqmap_init_state(self.ctx, C.c_uint64(seed)), "gqmap_init_state")

    def set_state(self, st: State) -> None:
        for k in ("muu", "muv", "sigu", "sigv", "pn", "rou", "w", "alpha"):
            setattr(st, k, f64(getattr(st, k)))
        exp = (self.M, self.N, self.L)
        if st.muu.shape != exp or st.rou.shape != exp + (2, 2):
            raise ValueError(f"state shape {st.muu.shape} != node grid {exp}")
        cs = st.cstruct()
        check(self.lib.gqmap_set_state(self.ctx, C.byref(cs)), "gqmap_set_state")

    def get_state(self) -> State:
        st = State.empty(self.M, self.N, self.L)
        cs = st.cstruct()
        check(self.lib.gqmap_get_state(self.ctx, C.byref(cs)), "gqmap_get_state")
        st.it, st.T = cs.it, cs.T
        return st

    # -- iterations ------------------------------------------------------
    def run(self, n_iter: int):
        """Run up to n_iter iterations; returns (n_done, trace[n_done, 3])."""
        trace = np.zeros((max(n_iter, 1), 3))
        done = C.c_int(0)
        check(self.lib.gqmap_run(self.ctx, int(n_iter), C.byref(done), dptr(trace)), "gqmap_run")
        return done.value, trace[:done.value]

    def set_truth(self, grdt) -> None:
        """Ground truth of the ctf level engine (gqmap_set_truth): GRDT of
        gqmap_ctf(options,I1,I2,GRDT), Mg x Ng x 2 with Mg >= M, Ng >= N (its
        top-left M x N block is used, as gqmap_ctf.m:38 does); None clears."""
        if grdt is None:
            check(self.lib.gqmap_set_truth(self.ctx, None, 0, 0), "gqmap_set_truth")
            return
        g = f64(grdt)
        if g.ndim != 3 or g.shape[2] != 2:
            raise ValueError("truth must be Mg x Ng x 2")
        check(self.lib.gqmap_set_truth(self.ctx, dptr(g), g.shape[0], g.shape[1]), "gqmap_set_truth")

    def run_aepe(self, n_iter: int):
        """run() plus the per-iteration AEPE of gqmap_ctf.m:38 (NaN without a
        truth): (n_done, trace[n_done, 3], aepe[n_done])."""
        trace = np.zeros((max(n_iter, 1), 3))
        ae = np.zeros(max(n_iter, 1))
        done = C.c_int(0)
        check(self.lib.gqmap_run_aepe(self.ctx, int(n_iter), C.byref(done), dptr(trace), dptr(ae)),
              "gqmap_run_aepe")
        return done.value, trace[:done.value], ae[:done.value]

    def run_timed(self, n_iter: int):
        done, tot, ker = C.c_int(0), C.c_double(0), C.c_double(0)
        check(self.lib.gqmap_run_timed(self.ctx, int(n_iter), C.byref(done), C.byref(tot),
                                       C.byref(ker)), "gqmap_run_timed")
        return done.value, tot.value, ker.value

    def prepare(self) -> None:
        """Build and upload the replayed iteration graph now (gqmap_prepare)."""
        check(self.lib.gqmap_prepare(self.ctx), "gqmap_prepare")

    def dataflow(self) -> bool:
        """Whether runs take the dataflow launch (k_iter_flow, one launch per
        50-iteration chunk) rather than one k_iter launch per iteration
        (gqmap_debug_flow; the library's flow policy)."""
        f = self.lib.gqmap_debug_flow
        f.restype = C.c_int
        f.argtypes = [C.c_void_p]
        return bool(f(self.ctx))

    def synchronize(self) -> None:
        check(self.lib.gqmap_synchronize(self.ctx), "gqmap_synchronize")

    def info(self) -> _lib.GqmapInfo:
        inf = _lib.GqmapInfo()
        check(self.lib.gqmap_get_info(self.ctx, C.byref(inf)), "gqmap_get_info")
        return inf

    def map(self) -> np.ndarray:
        out = np.zeros((self.M, self.N, 2), order="F")
        check(self.lib.gqmap_get_map(self.ctx, dptr(out)), "gqmap_get_map")
        return out

    def log_p(self, map_: np.ndarray) -> float:
        v = C.c_double(0)
        check(self.lib.gqmap_log_p(self.ctx, dptr(f64(map_)), C.byref(v)), "gqmap_log_p")
        return v.value

    def close(self) -> None:
        if self.ctx:
            self.lib.gqmap_destroy(self.ctx)
            self.ctx = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()


def strip_split(M: int, N: int, n_tiles: int) -> int:
    """Lanes per node Q for a single-scale mixture grid M x N cut into n_tiles
    column strips, chosen from ONE strip's node count with the library's own
    thresholds (gqmap_engine.hip choose_split, mixture: Q = 1 from 98,304
    nodes, 2 from 2^14, 4 from 2^13, 8 from 2^11, else 64 -- one wave per
    node).  The library picks Q from the whole grid so a tiled solve sums in
    the untiled order; pass this as options["split"] to every tile AND to the
    whole-grid reference to keep both bit-identical while each rank's strip
    still fills the GPU (strong scaling).  tests/test_tiles.py pins these
    thresholds against the library's."""
    nodes = M * -(-N // max(1, n_tiles))
    return (1 if nodes >= 98304 else 2 if nodes >= 1 << 14 else 4 if nodes >= 1 << 13
            else 8 if nodes >= 1 << 11 else 64)


def comm_unique_id() -> bytes:
    """An RCCL unique id for Engine.attach_rccl (draw on one rank, broadcast)."""
    buf = (C.c_uint8 * 128)()
    check(_lib.load().gqmap_comm_unique_id(buf), "gqmap_comm_unique_id")
    return bytes(buf)


def tile_group_run(tiles, n_iter: int):
    """Run the tiles of one grid (same device, tile order) n_iter iterations in
    lockstep with in-process halo exchange.  Returns (n_done, trace)."""
    lib = _lib.load()
    arr = (C.c_void_p * len(tiles))(*[t.ctx.value for t in tiles])
    trace = np.zeros((max(n_iter, 1), 3))
    done = C.c_int(0)
    check(lib.gqmap_tile_group_run(arr, len(tiles), int(n_iter), C.byref(done), dptr(trace)),
          "gqmap_tile_group_run")
    return done.value, trace[:done.value]


def aepe(tflow: np.ndarray, flow: np.ndarray, unknown: np.ndarray, crop: int = 1) -> float:
    """gqmap_gpu_mixture.m:63-64: flow(unidx)=0; mean over the interior of
    the end-point error (super engine: crop=4, gqmap_gpuSuper_mix_entropy.m:63)."""
    f = np.array(flow, dtype=np.float64)
    f[np.asarray(unknown, dtype=bool)] = 0
    M, N = f.shape[:2]
    sl = (slice(crop, M - crop), slice(crop, N - crop))
    d = tflow[sl] - f[sl]
    return float(np.mean(np.mean(np.sqrt(np.sum(d ** 2, axis=2)), axis=0)))


def _solve(engine: str, options: dict, I1, I2, *, seed: int = 0, precision: str = "fp64",
           device: int = 0, state: State | None = None, verbose: bool = False,
           eval_every: int = 300):
    its = int(options["its"])
    L = int(options["L"])
    sup = engine == "super"
    tflow = options.get("trueFlow")
    unk = options.get("unknownIdx")
    odir = options.get("dir")
    AEPE = np.full(its, np.nan)
    logP = np.full(its, np.nan)
    Energy = np.zeros(its)
    best = np.inf
    mark = None
    with Engine(options, I1, I2, engine, precision, device) as eng:
        if state is None:
            eng.init_state(seed)
        else:
            eng.set_state(state)
        it = 1
        while it <= its:
            # run up to the next evaluation point (it == 1 or it % eval_every == 0)
            nxt = 1 if it == 1 else min(its, (it // eval_every + 1) * eval_every)
            n = nxt - it + 1
            done, tr = eng.run(n)
            Energy[it - 1: it - 1 + done] = tr[:, 0]
            last = it + done - 1
            if done == n and (last == 1 or last % eval_every == 0):
                mp = eng.map()
                flow = np.repeat(np.repeat(mp, 4, axis=0), 4, axis=1) if sup else mp
                crop = 4 if sup else 1
                img = flow_to_color(flow[4:-4, 4:-4] if sup else flow, device=device)[0]
                if odir:
                    from .flowio import imwrite
                    os.makedirs(odir, exist_ok=True)
                    imwrite(img, os.path.join(odir, f"{last}.png"))
                if tflow is not None:
                    a = aepe(tflow, flow, unk, crop)
                    AEPE[last - 1] = a
                    best = min(best, a)
                logP[last - 1] = eng.log_p(mp)
                mark = last
            if verbose:
                for k in range(done):
                    print(f"[{it + k:3d}], Δ(mu) = {tr[k, 1]:e}, Δ(sigma) = {tr[k, 2]:e}, "
                          f"Energy = {tr[k, 0]:e}, AEPE={best:e},logP={logP[mark - 1] if mark else np.nan:e}")
            it += done
            if done < n:  # ptdmu < tor
                break
        st = eng.get_state()
    mu = np.stack([st.muu, st.muv], axis=3)
    sigma = np.stack([st.sigu, st.sigv], axis=3)
    alpha = st.alpha.reshape(1, 1, L)
    return mu, sigma, alpha, AEPE, Energy, logP


def gqmap_gpu_mixture(options: dict, I1, I2, **kw):
    """[mu, sigma, alpha, AEPE, Energy, logP] = gqmap_gpu_mixture(options, I1, I2)."""
    return _solve("mixture", options, I1, I2, **kw)


def gqmap_gpuSuper_mix_entropy(options: dict, I1, I2, **kw):
    """[mu, sigma, alpha, AEPE, Energy, logP] = gqmap_gpuSuper_mix_entropy(options, I1, I2)."""
    return _solve("super", options, I1, I2, **kw)
