"""Independent numpy fp64 restatement of the QGMAP iteration.

TEST INFRASTRUCTURE ONLY (golden-vector generator and cross-check of the C
oracle).  Written in the reference's own array style -- repmat/cat/circshift
become np.broadcast/np.stack/np.roll -- rather than per-element loops, so it
shares no code path with oracle/gqmap_oracle.c.

Restates:
  GaussHermite_2.m:21-32                 gauss_hermite (numpy.linalg.eigh)
  gqmap_gpu_mixture.m:191-208            get_vv
  gqmap_gpu_mixture.m:156-182            node_pot / edge_pot (vectorised)
  gqmap_gpu_mixture.m:87-146             node/edge spectral gradients
  gqmap_gpuSuper_mix_entropy.m:87-122    super node gradient
  gqmap_gpu_mixture.m:26-86              one iteration (+ updateAlpha)
  gqmap_gpuSuper_mix_entropy.m:72        temperature decay
"""
from __future__ import annotations

import numpy as np

SQRT2 = np.sqrt(2.0)


def gauss_hermite(K: int):
    i = np.arange(1, K)
    a = np.sqrt(i / 2.0)
    CM = np.diag(a, 1) + np.diag(a, -1)
    lam, V = np.linalg.eigh(CM)
    ind = np.argsort(lam)
    x = lam[ind]
    V = V[:, ind].T
    w = np.sqrt(np.pi) * V[:, 0] ** 2
    return x, w


def quad_tables(K: int):
    X, W = gauss_hermite(K)
    XI, XJ = np.meshgrid(X, X)          # XI(r,c)=X(c), XJ(r,c)=X(r)
    WI, WJ = np.meshgrid(W, W)
    # MATLAB linear order: column-major over (r,c)
    f = lambda A: A.ravel(order="F")
    return dict(XI=f(XI), XJ=f(XJ), WIWJ=f(WI * WJ), XIXJ=f(XI * XJ),
                XI2aXJ2=f(XI ** 2 + XJ ** 2), XI2mXJ2=f(XI ** 2 - XJ ** 2))


def get_vv(V: np.ndarray) -> np.ndarray:
    M, N = V.shape
    VV = np.zeros((M + 2, N + 2))
    VV[1:-1, 1:-1] = V
    VV[0, :] = (3.0 * VV[1, :] - 3.0 * VV[2, :]) + VV[3, :]
    VV[-1, :] = (3.0 * VV[-2, :] - 3.0 * VV[-3, :]) + VV[-4, :]
    VV[:, 0] = (3.0 * VV[:, 1] - 3.0 * VV[:, 2]) + VV[:, 3]
    VV[:, -1] = (3.0 * VV[:, -2] - 3.0 * VV[:, -3]) + VV[:, -4]
    return VV


def _keys(t):
    return (((2.0 - t) * t - 1.0) * t, (3.0 * t - 5.0) * t * t + 2.0,
            ((4.0 - 3.0 * t) * t + 1.0) * t, (t - 1.0) * t * t)


def interp_cubic(VV, M, N, Xq, Yq):
    """Vectorised node_pot interpolation; Xq/Yq 1-based (any shape)."""
    Xq = np.minimum(np.maximum(Xq, 1.0), N)
    Yq = np.minimum(np.maximum(Yq, 1.0), M)
    ix = np.where(Xq <= 1.0, 1, np.where(Xq <= N - 1, np.floor(Xq), N - 1)).astype(np.int64)
    iy = np.where(Yq <= 1.0, 1, np.where(Yq <= M - 1, np.floor(Yq), M - 1)).astype(np.int64)
    so, to = Xq - ix, Yq - iy
    ws, wt = _keys(so), _keys(to)
    Vq = np.zeros(np.broadcast(Xq, Yq).shape)
    for c in range(4):
        for r in range(4):
            Vq = Vq + VV[iy - 1 + r, ix - 1 + c] * ws[c] * wt[r]
    return Vq / 4


def matlab_round(v):
    """MATLAB round: half away from zero (exact: v - trunc(v) is exact)."""
    r = np.trunc(v)
    return r + np.where(np.abs(v - r) >= 0.5, np.sign(v), 0.0)


class Engine:
    def __init__(self, opts: dict, I1: np.ndarray, I2: np.ndarray):
        self.ctf = opts.get("engine", "mixture") == "ctf"
        if self.ctf:  # legacy/gqmap_ctf.m constants
            opts = dict(dict(step0=0.07, step_decay=1e300, sig_hi=25.0, corr_tor=0.999,
                             guard_a=0, alpha_start=1 << 30, t_decay_every=0, t_min=0.0, temperature=0.0,
                             sig_step=0.3), **opts)
        self.o = opts
        self.sup = opts.get("engine", "mixture") == "super"
        self.I1 = np.asarray(I1, dtype=np.float64)
        self.Mo, self.No = self.I1.shape
        self.M, self.N = (self.Mo // 4, self.No // 4) if self.sup else (self.Mo, self.No)
        self.VV = get_vv(np.asarray(I2, dtype=np.float64))
        self.q = quad_tables(int(opts["K"]))
        self.guard = bool(opts.get("guard_a", not self.sup))
        self.step0 = float(opts.get("step0", 0.001 if self.sup else 0.1))
        self.step_decay = float(opts.get("step_decay", 4000.0 if self.sup else 8000.0))
        self.sig_hi = float(opts.get("sig_hi", 25.0 if self.sup else 23.0))
        self.sig_lo = float(opts.get("sig_lo", 0.01))
        self.corr = float(opts.get("corr_tor", 1 - 1e-5))
        # projsplx on the super engine: it>200, 1E-6 (gqmap_gpuSuper_mix_entropy.m:48)
        proj_sup = self.sup and int(opts.get("alpha_mode", 0)) == 1
        self.alpha_start = int(opts.get("alpha_start", 200 if proj_sup else 500))
        self.alpha_lr = float(opts.get("alpha_lr", 1e-6 if proj_sup else 1e-7))
        self.t_every = int(opts.get("t_decay_every", 500 if self.sup else 0))
        self.t_min = float(opts.get("t_min", 0.001))

    # --- potentials -------------------------------------------------
    def node_pot(self, x1, x2, ms, ns):
        o = self.o
        if self.ctf:
            # gqmap_ctf.m:96 lookup into I2_cont = interp2(I2,6,'cubic'), returned
            # WITHOUT -lambda (the ctf gradients apply -lambda at the end)
            MM, NN = 64 * (self.Mo - 1) + 1, 64 * (self.No - 1) + 1
            r = np.clip(matlab_round((ms + x2 - 1) * 64 + 1), 1, MM)
            c = np.clip(matlab_round((ns + x1 - 1) * 64 + 1), 1, NN)
            Vq = interp_cubic(self.VV, self.Mo, self.No, (c - 1) / 64 + 1, (r - 1) / 64 + 1)
            return np.sqrt(o["epsn"] + (self.I1[ms - 1, ns - 1] - Vq) ** 2)
        if not self.sup:
            Vq = interp_cubic(self.VV, self.Mo, self.No, ns + x1, ms + x2)
            I = self.I1[ms - 1, ns - 1]
            return -o["lambdad"] * np.sqrt(o["epsn"] + (I - Vq) ** 2)
        tot = np.zeros(np.broadcast(x1, ms).shape)
        for di in range(4):
            for dj in range(4):
                i = 4 * ms - 3 + di
                j = 4 * ns - 3 + dj
                Vq = interp_cubic(self.VV, self.Mo, self.No, j + x1, i + x2)
                tot = tot + (-o["lambdad"] * np.sqrt(o["epsn"] + (self.I1[i - 1, j - 1] - Vq) ** 2))
        return tot

    def edge_pot(self, x1, x2):
        if self.ctf:
            return np.sqrt(self.o["epsn"] + (x1 - x2) ** 2)
        return -self.o["lambdas"] * np.sqrt(self.o["epsn"] + (x1 - x2) ** 2)

    def _ctf_epi(self, acc, pr, lam, o1, o2):
        # legacy/gqmap_ctf.m:104-109 and :144-149
        return (np.zeros_like(o1), -lam * acc["du1"] * (SQRT2 / (o1 * pr)) / np.pi,
                -lam * acc["du2"] * (SQRT2 / (o2 * pr)) / np.pi, -lam * acc["do1"] / np.pi / o1,
                -lam * acc["do2"] / np.pi / o2, -lam * acc["dp"] / np.pi / pr, -lam * acc["Ei"])

    def _spectral(self, pot_fn, a, u1, u2, o1, o2, p):
        q = self.q
        s = (np.sqrt(1 + p) + np.sqrt(1 - p)) / 2
        t = (np.sqrt(1 + p) - np.sqrt(1 - p)) / 2
        pr = 1 - p ** 2
        sqrtpr = np.sqrt(pr)
        acc = {k: np.zeros_like(u1) for k in ("dp", "du1", "du2", "do1", "do2", "Ei")}
        live = (a != 0) if self.guard else np.ones_like(u1, dtype=bool)
        for k in range(q["XI"].size):
            zi = s * q["XI"][k] + t * q["XJ"][k]
            zj = t * q["XI"][k] + s * q["XJ"][k]
            x1 = SQRT2 * o1 * zi + u1
            x2 = SQRT2 * o2 * zj + u2
            fval = q["WIWJ"][k] * pot_fn(x1, x2)
            fl = np.where(live, fval, 0.0)
            acc["dp"] += fl * (p - p * q["XI2aXJ2"][k] + 2 * q["XIXJ"][k])
            acc["du1"] += fl * (zi - p * zj)
            acc["du2"] += fl * (zj - p * zi)
            acc["do1"] += fl * (q["XI2aXJ2"][k] - 1 + q["XI2mXJ2"][k] / sqrtpr)
            acc["do2"] += fl * (q["XI2aXJ2"][k] - 1 - q["XI2mXJ2"][k] / sqrtpr)
            acc["Ei"] += fval
        return acc, pr, sqrtpr

    def node_grad(self, T, a, u1, u2, o1, o2, p, ms, ns):
        const1 = 1 + np.log(2 * np.pi)
        acc, pr, sqrtpr = self._spectral(lambda x1, x2: self.node_pot(x1, x2, ms, ns),
                                         a, u1, u2, o1, o2, p)
        if self.ctf:
            return self._ctf_epi(acc, pr, self.o["lambdad"], o1, o2)
        du1 = a * acc["du1"] * (SQRT2 / (o1 * pr)) / np.pi
        du2 = a * acc["du2"] * (SQRT2 / (o2 * pr)) / np.pi
        da = acc["Ei"] / np.pi - 3 * T * (const1 + np.log(sqrtpr * o1 * o2))
        do1 = a * (acc["do1"] / np.pi - 3 * T) / o1
        do2 = a * (acc["do2"] / np.pi - 3 * T) / o2
        dp = a * (acc["dp"] / np.pi + 3 * T * p) / pr
        return da, du1, du2, do1, do2, dp, a * da

    def edge_grad(self, T, a, u1, u2, o1, o2, p):
        const1 = 1 + np.log(2 * np.pi)
        acc, pr, sqrtpr = self._spectral(self.edge_pot, a, u1, u2, o1, o2, p)
        if self.ctf:
            return self._ctf_epi(acc, pr, self.o["lambdas"], o1, o2)
        du1 = a * acc["du1"] * (SQRT2 / (o1 * pr)) / np.pi
        du2 = a * acc["du2"] * (SQRT2 / (o2 * pr)) / np.pi
        da = acc["Ei"] / np.pi + T * (const1 + np.log(sqrtpr * o1 * o2))
        do1 = a * (acc["do1"] / np.pi + T) / o1
        do2 = a * (acc["do2"] / np.pi + T) / o2
        dp = a * (acc["dp"] / np.pi - T * p) / pr
        return da, du1, du2, do1, do2, dp, a * da

    # --- one iteration (gqmap_gpu_mixture.m:27-75) --------------------
    def gradients(self, st: dict, T: float):
        M, N, L = self.M, self.N, st["muu"].shape[2]
        ns, ms = np.meshgrid(np.arange(1, N + 1), np.arange(1, M + 1))
        ms3 = np.repeat(ms[:, :, None], L, axis=2)
        ns3 = np.repeat(ns[:, :, None], L, axis=2)
        A = np.broadcast_to(st["alpha"].reshape(1, 1, L), (M, N, L))
        node = self.node_grad(T, A, st["muu"], st["muv"], st["sigu"], st["sigv"], st["pn"], ms3, ns3)
        sh = lambda X: (np.roll(X, -1, axis=0), np.roll(X, -1, axis=1))
        cat45 = lambda Xu, Xv: np.stack([np.stack(Xu, axis=3), np.stack(Xv, axis=3)], axis=4)
        U1 = cat45((st["muu"], st["muu"]), (st["muv"], st["muv"]))
        U2 = cat45(sh(st["muu"]), sh(st["muv"]))
        O1 = cat45((st["sigu"], st["sigu"]), (st["sigv"], st["sigv"]))
        O2 = cat45(sh(st["sigu"]), sh(st["sigv"]))
        A5 = np.broadcast_to(st["alpha"].reshape(1, 1, L, 1, 1), U1.shape)
        edge = self.edge_grad(T, A5, U1, U2, O1, O2, st["rou"])
        return node, edge

    def iterate(self, st: dict, it: int, T: float):
        """Apply iteration `it` in place.  Returns (Energy, ptdmu, ptdsigma, T_next)."""
        o = self.o
        M, N, L = self.M, self.N, st["muu"].shape[2]
        step = self.step0 / (1 + it / self.step_decay)
        (dan, dmuu, dmuv, dsigu, dsigv, dpn, nE), (dae, dmu1, dmu2, dsg1, dsg2, drou, eE) = \
            self.gradients(st, T)
        I, J = slice(1, M - 1), slice(1, N - 1)
        dalpha = dan[I, J, :].sum(axis=(0, 1)) + dae[I, J, :, :, :].sum(axis=(0, 1, 3, 4))
        dmuu = dmuu + dmu1[:, :, :, :, 0].sum(axis=3) + np.roll(dmu2[:, :, :, 0, 0], 1, axis=0) \
            + np.roll(dmu2[:, :, :, 1, 0], 1, axis=1)
        dmuv = dmuv + dmu1[:, :, :, :, 1].sum(axis=3) + np.roll(dmu2[:, :, :, 0, 1], 1, axis=0) \
            + np.roll(dmu2[:, :, :, 1, 1], 1, axis=1)
        dsigu = dsigu + dsg1[:, :, :, :, 0].sum(axis=3) + np.roll(dsg2[:, :, :, 0, 0], 1, axis=0) \
            + np.roll(dsg2[:, :, :, 1, 0], 1, axis=1)
        dsigv = dsigv + dsg1[:, :, :, :, 1].sum(axis=3) + np.roll(dsg2[:, :, :, 0, 1], 1, axis=0) \
            + np.roll(dsg2[:, :, :, 1, 1], 1, axis=1)
        cl = lambda x, lo, hi: np.minimum(np.maximum(x, lo), hi)
        st["muu"][I, J] = cl(st["muu"][I, J] + dmuu[I, J] * step, o["minu"], o["maxu"])
        st["muv"][I, J] = cl(st["muv"][I, J] + dmuv[I, J] * step, o["minv"], o["maxv"])
        if self.ctf:  # gqmap_ctf.m:34-35: dsigmau*step*0.3
            f = float(o.get("sig_step", 0.3))
            st["sigu"][I, J] = cl(st["sigu"][I, J] + dsigu[I, J] * step * f, self.sig_lo, self.sig_hi)
            st["sigv"][I, J] = cl(st["sigv"][I, J] + dsigv[I, J] * step * f, self.sig_lo, self.sig_hi)
        else:
            st["sigu"][I, J] = cl(st["sigu"][I, J] + dsigu[I, J] * step, self.sig_lo, self.sig_hi)
            st["sigv"][I, J] = cl(st["sigv"][I, J] + dsigv[I, J] * step, self.sig_lo, self.sig_hi)
        st["rou"][I, J] = cl(st["rou"][I, J] + drou[I, J] * step, -self.corr, self.corr)
        st["pn"][I, J] = cl(st["pn"][I, J] + dpn[I, J] * step, -self.corr, self.corr)
        energy = nE[I, J].sum() + eE[I, J].sum()
        if it > self.alpha_start and L != 1:
            if int(o.get("alpha_mode", 0)) == 0:
                a = st["alpha"]
                dw = a * (dalpha - np.sum(dalpha * a))
                st["w"][:] = cl(st["w"] + dw * step * self.alpha_lr, -300, 300)
                e = np.exp(st["w"])
                st["alpha"][:] = e / e.sum()
            else:
                st["alpha"][:] = projsplx(st["alpha"] + dalpha * step * self.alpha_lr)
        ptdmu = np.abs(dmuu[I, J]).mean()
        ptdsig = np.abs(dsigu[I, J]).mean()
        if self.t_every > 0 and it % self.t_every == 0:
            T = max(T * float(o.get("drate", 0.5)), self.t_min)
        return energy, ptdmu, ptdsig, T


def log_p(eng: Engine, mp) -> float:
    """profile_logP (gqmap_gpu_mixture.m:148-154; super: node_lp,
    gqmap_gpuSuper_mix_entropy.m:152-169) in array form: np(M_,N_) + the
    circshift edge potentials, numpy sums."""
    M, N = mp.shape[:2]
    ns, ms = np.meshgrid(np.arange(1, N + 1), np.arange(1, M + 1))
    npot = eng.node_pot(mp[:, :, 0], mp[:, :, 1], ms, ns)
    ep = sum(eng.edge_pot(mp, s) for s in (np.roll(mp, -1, axis=0), np.roll(mp, -1, axis=1)))
    return float(npot[1:-1, 1:-1].sum() + ep[1:-1, 1:-1].sum())


def projsplx(y):
    y = np.asarray(y, dtype=np.float64).ravel()
    m = y.size
    s = np.sort(y)[::-1]
    tmpsum = 0.0
    bget = False
    tmax = 0.0
    for ii in range(m - 1):
        tmpsum = tmpsum + s[ii]
        tmax = (tmpsum - 1) / (ii + 1)
        if tmax >= s[ii + 1]:
            bget = True
            break
    if not bget:
        tmax = (tmpsum + s[m - 1] - 1) / m
    return np.maximum(y - tmax, 0)


# --- flowToColor / computeColor (legacy/flowToColor.m, legacy/computeColor.m) ---
def colorwheel():
    RY, YG, GC, CB, BM, MR = 15, 6, 4, 11, 13, 6
    cw = np.zeros((RY + YG + GC + CB + BM + MR, 3))
    col = 0
    cw[0:RY, 0] = 255
    cw[0:RY, 1] = np.floor(255 * np.arange(RY) / RY)
    col += RY
    cw[col:col + YG, 0] = 255 - np.floor(255 * np.arange(YG) / YG)
    cw[col:col + YG, 1] = 255
    col += YG
    cw[col:col + GC, 1] = 255
    cw[col:col + GC, 2] = np.floor(255 * np.arange(GC) / GC)
    col += GC
    cw[col:col + CB, 1] = 255 - np.floor(255 * np.arange(CB) / CB)
    cw[col:col + CB, 2] = 255
    col += CB
    cw[col:col + BM, 2] = 255
    cw[col:col + BM, 0] = np.floor(255 * np.arange(BM) / BM)
    col += BM
    cw[col:col + MR, 2] = 255 - np.floor(255 * np.arange(MR) / MR)
    cw[col:col + MR, 0] = 255
    return cw


def flow_to_color(flow, max_flow=0.0):
    u = np.array(flow[:, :, 0], dtype=np.float64)
    v = np.array(flow[:, :, 1], dtype=np.float64)
    unk = (np.abs(u) > 1e9) | (np.abs(v) > 1e9)
    u[unk] = 0
    v[unk] = 0
    flo = np.stack([u, v], axis=2)
    maxu = max(-999.0, np.nanmax(u)); minu = min(999.0, np.nanmin(u))
    maxv = max(-999.0, np.nanmax(v)); minv = min(999.0, np.nanmin(v))
    rad = np.sqrt(u ** 2 + v ** 2)
    maxrad = max(-1.0, np.nanmax(rad))
    if max_flow > 0:
        maxrad = max_flow
    eps = np.finfo(np.float64).eps
    u = u / (maxrad + eps)
    v = v / (maxrad + eps)
    nan = np.isnan(u) | np.isnan(v)
    u[nan] = 0
    v[nan] = 0
    cw = colorwheel()
    ncols = cw.shape[0]
    rad = np.sqrt(u ** 2 + v ** 2)
    a = np.arctan2(-v, -u) / np.pi
    fk = (a + 1) / 2 * (ncols - 1) + 1
    k0 = np.floor(fk).astype(np.int64)
    k1 = k0 + 1
    k1[k1 == ncols + 1] = 1
    f = fk - k0
    img = np.zeros(u.shape + (3,), dtype=np.uint8)
    for i in range(3):
        col0 = cw[k0 - 1, i] / 255
        col1 = cw[k1 - 1, i] / 255
        col = (1 - f) * col0 + f * col1
        idx = rad <= 1
        col[idx] = 1 - rad[idx] * (1 - col[idx])
        col[~idx] = col[~idx] * 0.75
        img[:, :, i] = np.clip(np.floor(255 * col * (1 - nan)), 0, 255).astype(np.uint8)
    img[unk] = 0
    return img, flo, (minu, maxu, minv, maxv), unk


# ---- coarse-to-fine plumbing (legacy/optical_flow_ctf.m:21-35), vectorised ----
# Independent of oracle/gqmap_pyramid_oracle.c: MATLAB-style whole-array
# expressions (numpy sums and powers), bilinear sampling by
# scipy.ndimage.map_coordinates.  Agreement with the C restatement is to
# rounding (~1e-13), not bitwise.
def _cubic_np(x):
    ax = np.abs(x)
    ax2, ax3 = ax ** 2, ax ** 3
    return ((1.5 * ax3 - 2.5 * ax2 + 1) * (ax <= 1)
            + (-0.5 * ax3 + 2.5 * ax2 - 4 * ax + 2) * ((1 < ax) & (ax <= 2)))


def imresize_contrib(in_len, out_len, scale, antialias=True):
    """imresize.m contributions(): (weights [out,P], 0-based indices [out,P])."""
    if scale < 1 and antialias:
        h = lambda x: scale * _cubic_np(scale * x)
        width = 4.0 / scale
    else:
        h, width = _cubic_np, 4.0
    x = np.arange(1, out_len + 1, dtype=np.float64)[:, None]
    u = x / scale + 0.5 * (1 - 1 / scale)
    left = np.floor(u - width / 2)
    P = int(np.ceil(width)) + 2
    ind = left + np.arange(P)[None, :]
    w = h(u - ind)
    w = w / w.sum(axis=1, keepdims=True)
    aux = np.concatenate([np.arange(1, in_len + 1), np.arange(in_len, 0, -1)])
    ind = aux[np.mod(ind - 1, aux.size).astype(np.int64)]
    keep = np.any(w != 0, axis=0)
    return w[:, keep], ind[:, keep] - 1


def imresize(A, scale, antialias=True):
    A = np.asarray(A, dtype=np.float64)
    M, N = A.shape[:2]
    oM, oN = int(np.ceil(scale * M)), int(np.ceil(scale * N))
    wm, im = imresize_contrib(M, oM, scale, antialias)
    wn, jn = imresize_contrib(N, oN, scale, antialias)
    B = np.einsum("ik,ik...->i...", wm, A[im])                 # dim 1
    B = np.einsum("jk,ijk...->ij...", wn, B[:, jn])            # dim 2
    return np.asfortranarray(B)


def warp_image(V, warp, fill=True):
    from scipy.ndimage import map_coordinates
    V = np.asarray(V, dtype=np.float64)
    M, N = V.shape
    xs, ys = np.meshgrid(np.arange(1, N + 1), np.arange(1, M + 1))
    xq, yq = xs - warp[:, :, 0], ys - warp[:, :, 1]
    out = map_coordinates(V, [yq - 1, xq - 1], order=1, mode="constant", cval=np.nan)
    out[~((xq >= 1) & (xq <= N) & (yq >= 1) & (yq <= M))] = np.nan
    out = np.asfortranarray(out)
    if fill:
        out = fillmissing_nearest(fillmissing_nearest(out, 1), 2)
    return out


def fillmissing_nearest(A, dim):
    A = np.array(A, dtype=np.float64, order="F")
    B = A if dim == 1 else A.T
    for c in range(B.shape[1]):
        col = B[:, c]
        ok = np.flatnonzero(~np.isnan(col))
        bad = np.flatnonzero(np.isnan(col))
        if ok.size == 0 or bad.size == 0:
            continue
        pos = np.searchsorted(ok, bad)               # next valid at ok[pos]
        nxt = ok[np.minimum(pos, ok.size - 1)]
        prv = ok[np.maximum(pos - 1, 0)]
        use_prev = (pos == ok.size) | ((pos > 0) & (bad - prv < nxt - bad))
        col[bad] = np.where(use_prev, col[prv], col[nxt])
    return np.asfortranarray(A)


def ctf_pipeline(opts, img1, img2, scales, init_fn):
    """optical_flow_ctf.m:21-35 with this module's Engine("ctf") as the level solver."""
    M, N = img1.shape
    s0 = scales[0]
    warp = np.zeros((int(np.ceil(M * s0 / 2)), int(np.ceil(N * s0 / 2)), 2))
    levels = []
    for l, s in enumerate(scales):
        I1, I2 = imresize(img1, s), imresize(img2, s)
        warp = imresize(warp, 2.0) * 2
        I1w = warp_image(I1, warp)
        lo = dict(opts, engine="ctf", minu=opts["minu"] * s, maxu=opts["maxu"] * s,
                  minv=opts["minv"] * s, maxv=opts["maxv"] * s)
        st = init_fn(l, lo, *I1.shape)
        eng = Engine(lo, I1w, I2)
        T = 0.0
        for it in range(1, int(lo["its"]) + 1):
            e, ptdmu, _ = eng.iterate(st, it, T)[:3]
            if ptdmu < lo.get("tor", 1e-4):
                break
        flow = np.stack([st["muu"][:, :, 0], st["muv"][:, :, 0]], axis=2)
        warp = warp + flow
        levels.append(dict(I1w=I1w, I2=I2, flow=flow, warp=warp.copy()))
    return warp, levels


# ---- legacy flow-denoising engine (legacy/gqmap_cpu.m), vectorised ----------
def cpu_engine(opts, flow, sigma0, X, W):
    """[mu, sigma, rou] = gqmap_cpu(options, flow) with sigma = sigma0 (the
    reference draws rand(M,N,2)+2), numpy whole-array form.  Returns
    (mu, sigma, rou, trace)."""
    its, var, gama = int(opts["its"]), float(opts.get("var", 1.0)), float(opts.get("gama", 1.0))
    dta = float(opts.get("dta", np.inf))
    X, W = np.asarray(X, dtype=np.float64), np.asarray(W, dtype=np.float64)
    XI, XJ = np.meshgrid(X, X)
    WI, WJ = np.meshgrid(W, W)
    WIWJ = WI * WJ
    flow = np.asarray(flow, dtype=np.float64)
    M, N, _ = flow.shape
    mu, sigma = flow.copy(), np.array(sigma0, dtype=np.float64)
    rou = np.zeros((M, N, 2, 2))
    dnode = np.zeros((M, N, 2, 2))
    dedge = np.zeros((M, N, 2, 5, 2))
    S = (slice(0, M - 1), slice(0, N - 1))
    trace = []
    it = 1
    while True:
        for l in range(2):
            x = SQRT2 * sigma[S + (l,)][..., None] * X + mu[S + (l,)][..., None]
            dval = W * (flow[S + (l,)][..., None] - x) / var
            dnode[S + (0, l)] = dval.sum(-1) / np.sqrt(np.pi)
            dnode[S + (1, l)] = (dval * X).sum(-1) * np.sqrt(2 / np.pi)
        for j in range(2):
            S2 = (slice(1, M), slice(0, N - 1)) if j == 0 else (slice(0, M - 1), slice(1, N))
            for l in range(2):
                e = lambda a: a[..., None, None]
                p = rou[S + (j, l)]
                o1, o2 = e(sigma[S + (l,)]), e(sigma[S2 + (l,)])
                u1, u2 = e(mu[S + (l,)]), e(mu[S2 + (l,)])
                q, r = np.sqrt(1 + p), np.sqrt(1 - p)
                s, t = e((q + r) / 2), e((q - r) / 2)
                ds, dt = e((1 / q - 1 / r) / 4), e((1 / q + 1 / r) / 4)
                ZI, ZJ = s * XI + t * XJ, t * XI + s * XJ
                x1, x2 = SQRT2 * o1 * ZI + u1, SQRT2 * o2 * ZJ + u2
                diff = x2 - x1
                diff = np.where(np.abs(diff) > dta, 0.0, diff)
                df1 = WIWJ * diff / gama
                df2 = -df1
                ss = lambda A: A.sum(axis=-2).sum(axis=-1)   # sum(sum(A))
                dedge[S + (j, 0, l)] = 1 / np.pi * ss(df1)
                dedge[S + (j, 1, l)] = 1 / np.pi * ss(df2)
                dedge[S + (j, 2, l)] = 1 / np.pi * SQRT2 * ss(df1 * ZI)
                dedge[S + (j, 3, l)] = 1 / np.pi * SQRT2 * ss(df2 * ZJ)
                dedge[S + (j, 4, l)] = 1 / np.pi * SQRT2 * ss(o1 * df1 * (ds * XI + dt * XJ)
                                                               + o2 * df2 * (dt * XI + ds * XJ))
        z1 = np.zeros((1, N, 2))
        z2 = np.zeros((M, 1, 2))
        dmu = dnode[:, :, 0, :] + dedge[:, :, :, 0, :].sum(axis=2) + (
            np.concatenate([dedge[1:, :, 0, 1, :], z1], 0) + np.concatenate([dedge[:, 1:, 1, 1, :], z2], 1))
        dsg = dnode[:, :, 1, :] + dedge[:, :, :, 2, :].sum(axis=2) + (
            np.concatenate([dedge[1:, :, 0, 3, :], z1], 0) + np.concatenate([dedge[:, 1:, 1, 3, :], z2], 1))
        drou = dedge[:, :, :, 4, :]
        step = float(opts.get("step0", 0.1)) / (1 + it / float(opts.get("step_decay", 1000.0)))
        mu = mu + dmu * step
        sigma = np.abs(sigma + dsg * step)
        c = float(opts.get("corr_tor", 0.97))
        rou = np.maximum(np.minimum(rou + drou * step, c), -c)
        mx = np.abs(dmu).max()
        trace.append((mx, np.abs(dsg).max(), np.abs(drou).max()))
        it += 1
        if it > its or (it > int(opts.get("min_its", 100)) and mx < float(opts.get("tor", 1e-3))):
            break
    return mu, sigma, rou, np.array(trace)
