"""Headline benchmark (BASELINE.json): Gpixel-iterations/s + AEPE vs the .flo
ground truth on the Middlebury 584x388 pair, 1/2/4/8 GPUs.

Default workload (BASELINE config C2): RubberWhale 388x584, gqmap_gpu_mixture
(single-scale mixture QGMAP), L=1, K=9, 500 iterations, lambda_s=5,
lambda_d=1, eps=1e-6, T=0 (optical_flow.m:16-23 with L=1).  One "step" is one
iteration of the hot path over the whole frame (gqmap_gpu_mixture.m:27-75);
frames and state are resident in HBM before the timed region.

    python bench.py [--steps 500] [--warmup 20] [--precision fp64|fp32]
    python -m torch.distributed.run --nproc-per-node N bench.py --gpus N

Multi-GPU (default) is frame-parallel (weak scaling): every rank solves its
own 584x388 pair on its own GPU, no data-path collective; `value` is the
pixels of all ranks x steps / the slowest rank's time.  The same line carries
`strong_scaling`: the RubberWhale pair itself split into one column strip per
rank (RCCL ghost-column + exact-totals exchange every iteration, lanes per
node chosen from one strip: gqmap_opticalflow_amd.strip_split), timed the
same way -- the north star's "584x388 pair at 1, 2, 4 and 8 MI355X".

The other BASELINE configs are selectable (same JSON line, their workload
named in `config`):
    --config c3   Grove3 480x640, 5-level coarse-to-fine pyramid (gqmap_ctf
                  levels + device imresize/warp/fillmissing), steps = its/level
    --config c4   Urban3 480x640, gqmap_gpuSuper_mix_entropy L=3 K=11, 1000 its
    --config c5   the eight GT pairs of legacy/optical_flow_temp.m:3 upsampled
                  4x (33.1 Mpx in all), each pair split into column-strip
                  tiles over the ranks with RCCL ghost-column exchange, pairs
                  in turn (strong scaling)
    --config c2 --tiled   the RubberWhale pair itself split over the ranks
                  (strong scaling of the headline pair)
    --config c1   Dimetrodon 388x584 legacy/gqmap_cpu.m flow denoising, 50 its
                  (gqmap_cpu_run_device on the flow resident in HBM; the
                  host-array call's PCIe-inclusive rate as `host_arrays`)
Before the timed steps (after --warmup W steps and the graph capture) the
hot path runs untimed until the GPU clocks settle (settle_clocks; reported as
`clock_settle`, with the same steps timed once cold as `cold_start_value`;
--no-settle skips it): a 20-step window started cold measures the clock ramp
(profiles/r04_clock_ramp.txt).
Rank 0 prints one JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "Gpixel-iters/s + AEPE vs .flo GT, Middlebury 584x388, 1/2/4/8 GPU"
PEAK_TFLOPS = {"fp64": 78.6, "fp32": 157.3}   # MI355X vector (non-MFMA) peaks, MI355X_MICROARCH.md
PEAK_HBM_GBPS = 8000.0
PAIRS = ("rubberwhale", "Dimetrodon", "Hydrangea")      # the 584x388 Middlebury pairs
PAIRS_480 = ("Grove3", "Urban3", "Urban2", "Grove2")     # the 640x480 pairs
# the eight GT pairs of legacy/optical_flow_temp.m:3 (config C5), as flowio.C5_PAIRS
C5_PAIRS = ("Urban3", "Grove3", "Urban2", "Venus", "Dimetrodon", "rubberwhale", "Grove2", "Hydrangea")
DEFAULT_STEPS = {"c1": 50, "c2": 500, "c3": 500, "c4": 1000, "c5": 100}


def algorithmic_flops_per_node(engine: str, L: int, K: int) -> float:
    # node qp ~128 flop (super: 16 x 92 + 36 = 1524), edge qp ~41, 4 edges
    if engine == "super":
        return L * K * K * (1524 + 4 * 41)
    return 292 * L * K * K


def algorithmic_bytes_per_node(engine: str, L: int, S: int) -> float:
    # state (9 values per component) read + write, plus I1 and I2 once per pixel
    if engine == "super":
        return 18 * L * S + 16 * 2 * S
    return (18 * L + 2) * S


def gt_options(name: str, L: int, K: int, **kw):
    from gqmap_opticalflow_amd import flow_to_color, flowio
    I1, I2, gt = flowio.load_pair(name)
    _, flo, (minu, maxu, minv, maxv), unk = flow_to_color(gt)
    opts = dict(trueFlow=flo, unknownIdx=unk, its=500, K=K, L=L, temperature=0.0, drate=0.5,
                epsn=0.001 ** 2, lambdas=5.0, lambdad=1.0, minu=minu, maxu=maxu, minv=minv, maxv=maxv)
    opts.update(kw)
    return I1, I2, flo, unk, opts


def setup_problem(name: str, L: int, K: int):
    return gt_options(name, L, K)


def host_cpus():
    """What the CPU baseline runs on: nproc, the threads this process may use
    (affinity, capped by OMP_NUM_THREADS -- the GPU box grants each GPU a
    share of its cores and sets OMP_NUM_THREADS to it), physical cores."""
    nproc = os.cpu_count() or 1
    try:
        avail = len(os.sched_getaffinity(0))
    except AttributeError:
        avail = nproc
    omp = os.environ.get("OMP_NUM_THREADS")
    threads = min(avail, int(omp)) if omp and omp.isdigit() and int(omp) > 0 else avail
    quota = None  # CPUs' worth of time the cgroup grants (cpu.max quota / period)
    for path in ("/sys/fs/cgroup/cpu.max", "/sys/fs/cgroup/cpu/cpu.cfs_quota_us"):
        try:
            parts = open(path).read().split()
            if path.endswith("cpu.max") and parts and parts[0] != "max":
                quota = int(parts[0]) / int(parts[1])
            elif path.endswith("quota_us") and int(parts[0]) > 0:
                quota = int(parts[0]) / int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
        except (OSError, ValueError, IndexError, ZeroDivisionError):
            continue
        if quota:
            break
    phys = set()
    try:
        pid = cid = None
        for line in open("/proc/cpuinfo"):
            if line.startswith("physical id"):
                pid = line.split(":")[1].strip()
            elif line.startswith("core id"):
                cid = line.split(":")[1].strip()
            elif not line.strip():
                if cid is not None:
                    phys.add((pid, cid))
                pid = cid = None
    except OSError:
        pass
    return {"nproc": nproc, "affinity": avail, "threads": threads, "physical_cores": len(phys) or None,
            "cpu_quota": quota}


def _timed_leg(run_n, budget_s):
    """Time run_n(n) on a bounded sample: one untimed warm-up iteration (the
    first call pays OpenMP start-up and first-touch page faults: 2.7 s once
    on the GPU box), one probe iteration that sizes n to about budget_s
    seconds, then n timed iterations.  Returns (iterations, seconds)."""
    run_n(1)
    t0 = time.perf_counter()
    run_n(1)
    t1 = time.perf_counter() - t0
    n = max(1, min(200, int(budget_s / max(t1, 1e-3))))
    t0 = time.perf_counter()
    done = run_n(n)
    return done, time.perf_counter() - t0


def allcore_threads(hc) -> int:
    """Every physical core this process may run on (BASELINE.md:51: "all host
    cores of the GPU box")."""
    return max(1, min(hc["physical_cores"] or hc["affinity"], hc["affinity"]))


def cpu_baseline(I1, I2, opts, engine="mixture", label="", budget_s: float = 6.0, split: int | None = None,
                 precision: str = "fp64"):
    """The CPU paths on this host's cores, each on a bounded sample of the
    same workload from the same seeded init:
      * the literal C fp64 restatement of the engine loop (oracle/gqmap_oracle.c,
        OpenMP over rows) on this process's CPU share (`value`), on one
        thread, and on every physical core (`value_allcores`);
      * the CPU model of the kernel arithmetic (oracle/gqmap_emul.cpp) -- the
        CPU path the GPU matches bit for bit -- on the same share
        (`value_emul`) and on every physical core."""
    from gqmap_opticalflow_amd import gauss_hermite, initial_state
    from oracle import oracle
    hc = host_cpus()
    Mo, No = I1.shape
    M, N = (Mo // 4, No // 4) if engine == "super" else (Mo, No)
    o = dict(opts, engine=engine)
    X, W = gauss_hermite(int(opts["K"]))
    allc = allcore_threads(hc)

    def leg(kind, threads):
        st0 = initial_state(o, M, N, seed=0, engine=engine)
        st = oracle.State(st0.muu, st0.muv, st0.sigu, st0.sigv, st0.pn, st0.rou, st0.w, st0.alpha)
        it, T = [1], [st0.T]

        def run_n(n):
            if kind == "literal":
                done, _, T[0] = oracle.run(o, I1, I2, st, it[0], n, T=T[0], nthreads=threads)
            else:
                done, _, T[0] = oracle.emu_run(o, I1, I2, st, it[0], n, X, W, T=T[0], nthreads=threads,
                                               fp32=precision == "fp32", split=split)
            it[0] += done
            return done
        n, t = _timed_leg(run_n, budget_s)
        return Mo * No * n / t / 1e9, n, t

    v_sh, n_sh, t_sh = leg("literal", hc["threads"])
    v_1, n_1, t_1 = leg("literal", 1)
    v_all, n_all, t_all = leg("literal", allc)
    v_em, n_em, t_em = leg("emul", hc["threads"])
    v_ema, n_ema, t_ema = leg("emul", allc)
    return {"value": v_sh, "unit": "Gpixel-iter/s", "cores": hc["threads"],
            "kind": "port", "value_1thread": v_1, "value_allcores": v_all, "cores_allcores": allc,
            "value_emul": v_em, "value_emul_allcores": v_ema,
            "nproc": hc["nproc"], "affinity_cpus": hc["affinity"], "physical_cores": hc["physical_cores"],
            "cgroup_cpu_quota": hc["cpu_quota"],
            "allcores_note": "the all-physical-core legs oversubscribe when the box's cgroup grants fewer CPUs than "
                             "there are cores (cgroup_cpu_quota; OMP_NUM_THREADS names the share): `value` is the "
                             "share's figure",
            "sample": f"{label} {No}x{Mo} ({engine}, L={opts['L']} K={opts['K']}), seeded init, iterations from 1: "
                      f"literal restatement oracle/gqmap_oracle.c fp64 -- {n_sh} its on {hc['threads']} OpenMP "
                      f"threads in {t_sh:.1f}s (the process's CPU share: nproc {hc['nproc']}, affinity "
                      f"{hc['affinity']}, OMP_NUM_THREADS {os.environ.get('OMP_NUM_THREADS', 'unset')}), {n_1} on "
                      f"1 thread in {t_1:.1f}s, {n_all} on {allc} threads (all physical cores) in {t_all:.1f}s; "
                      f"CPU model of the kernel arithmetic oracle/gqmap_emul.cpp {precision} (bit-identical to the "
                      f"GPU) -- {n_em} its on {hc['threads']} threads in {t_em:.1f}s, {n_ema} on {allc} in "
                      f"{t_ema:.1f}s"}


def _pix_stats(a, b, o):
    """Pixels whose flow differs by more than 1e-9 (either component), and
    pixels whose mean sits on OPPOSITE clamp bounds of
    gqmap_gpu_mixture.m:41-42 in the two flows (|du| = maxu - minu or
    |dv| = maxv - minv)."""
    du, dv = np.abs(a[:, :, 0] - b[:, :, 0]), np.abs(a[:, :, 1] - b[:, :, 1])
    diff = int(((du > 1e-9) | (dv > 1e-9)).sum())
    flip = int(((du == o["maxu"] - o["minu"]) | (dv == o["maxv"] - o["minv"])).sum())
    return diff, flip


def _first_flip(flips):
    return next((i + 1 for i, f in enumerate(flips) if f > 0), None)


def parity_gate(r, engine, steps, precision, split, seed):
    """The north-star gate (BASELINE.md:64-65), after the timed region: the
    same `steps` iterations from the same seeded init on the CPU -- the CPU
    model of the kernel arithmetic (oracle/gqmap_emul.cpp, must match the GPU
    bit for bit: aepe_delta_emul == 0) and the literal restatement of the
    reference (oracle/gqmap_oracle.c: aepe_delta_literal against the 1e-4
    gate) -- then AEPE (gqmap_gpu_mixture.m:63-64) and flowToColor
    (gqmap_gpu_mixture.m:60; uint8 pixels that differ) of each CPU flow
    against the GPU's.

    Single-Gaussian mixture (C2) adds two records:
      * `divergence`: the literal restatement run against ITSELF with mu_u
        perturbed by +-1e-13 (aepe_spread_literal = the larger |AEPE delta|),
        and per iteration (the first TRACK_ITS) the pixels whose flow differs
        by > 1e-9 and the pixels on opposite clamp bounds, for GPU vs
        literal and literal vs perturbed literal, with the first iteration a
        bound flip appears in each;
      * `literal_engine`: the literal-order engine's flow (arith="literal")
        against the literal restatement run with the engine's Gauss-Hermite
        rule -- bit-identical (aepe_delta_literal 0.0, colour mismatch 0)."""
    from gqmap_opticalflow_amd import aepe, flow_to_color, gauss_hermite, initial_state
    from oracle import oracle
    I1, I2, opts, mp_gpu, flo, unk = r["I1"], r["I2"], r["opts"], r["map"], r["flo"], r["unk"]
    Mo, No = I1.shape
    sup = engine == "super"
    M, N = (Mo // 4, No // 4) if sup else (Mo, No)
    o = dict(opts, engine=engine)
    L = int(o["L"])
    X, W = gauss_hermite(int(o["K"]))
    threads = host_cpus()["threads"]
    up = (lambda f: np.repeat(np.repeat(f, 4, axis=0), 4, axis=1)) if sup else (lambda f: f)
    crop = 4 if sup else 1

    def cpu_map(st, det_exp):
        if L == 1:
            return np.stack([st.muu[:, :, 0], st.muv[:, :, 0]], axis=2)
        return oracle.get_map(st.alpha, st.muu, st.sigu, st.muv, st.sigv, nthreads=threads, det_exp=det_exp)

    def colour(f):
        f = up(f)
        return f[4:-4, 4:-4] if sup else f

    def seeded(pert=0.0):
        st0 = initial_state(o, M, N, seed=seed, engine=engine)
        return oracle.State(st0.muu + pert, st0.muv, st0.sigu, st0.sigv, st0.pn, st0.rou, st0.w, st0.alpha), st0.T

    img_gpu = flow_to_color(colour(mp_gpu))[0]
    a_gpu = aepe(flo, up(mp_gpu), unk, crop)
    out = {"its": steps, "threads": threads, "gate": 1e-4, "aepe_gpu": a_gpu}
    stepped = engine == "mixture" and L == 1 and r.get("maps_it") is not None
    finals = {}
    if stepped:
        # the literal restatement one iteration at a time (same arithmetic as
        # one call): unperturbed, mu_u +- 1e-13, and with the engine's rule
        t0 = time.perf_counter()
        runs = {"lit": seeded(), "lit_p": seeded(1e-13), "lit_m": seeded(-1e-13)}
        if r.get("literal") is not None and "map" in r["literal"]:
            runs["lit_rule"] = seeded()
        maps_it = r["maps_it"]
        traj = {k: {"diff": [], "flip": []} for k in ("gpu_vs_literal", "literal_vs_literal+1e-13",
                                                       "literal_vs_literal-1e-13")}
        for it in range(1, steps + 1):
            for k, (st, T) in runs.items():
                kw = dict(X=X, W=W) if k == "lit_rule" else {}
                oracle.run(o, I1, I2, st, it, 1, T=T, nthreads=threads, **kw)
            if it <= len(maps_it):
                lm = cpu_map(runs["lit"][0], False)
                for key, other in (("gpu_vs_literal", maps_it[it - 1]),
                                   ("literal_vs_literal+1e-13", cpu_map(runs["lit_p"][0], False)),
                                   ("literal_vs_literal-1e-13", cpu_map(runs["lit_m"][0], False))):
                    d, f = _pix_stats(other, lm, o)
                    traj[key]["diff"].append(d)
                    traj[key]["flip"].append(f)
        finals["literal"] = runs["lit"][0]
        a_lit = aepe(flo, cpu_map(runs["lit"][0], False), unk, crop)
        a_p = aepe(flo, cpu_map(runs["lit_p"][0], False), unk, crop)
        a_m = aepe(flo, cpu_map(runs["lit_m"][0], False), unk, crop)
        for v in traj.values():
            v["first_flip_iteration"] = _first_flip(v["flip"])
        out["divergence"] = {
            "tracked_iterations": len(maps_it), "diff_threshold": 1e-9,
            "flip": "pixels whose mean sits on opposite clamp bounds (|dmu_u| = maxu-minu or |dmu_v| = maxv-minv, "
                    "gqmap_gpu_mixture.m:41-42) in the two flows",
            "aepe_literal": a_lit, "aepe_literal_plus_1e-13": a_p, "aepe_literal_minus_1e-13": a_m,
            "trajectories": traj, "cpu_s": time.perf_counter() - t0}
        out["aepe_spread_literal"] = max(abs(a_p - a_lit), abs(a_m - a_lit))
        if "lit_rule" in runs:
            lm = cpu_map(runs["lit_rule"][0], False)
            lg = r["literal"]["map"]
            a_lg, a_lr = aepe(flo, lg, unk, crop), aepe(flo, lm, unk, crop)
            out["literal_engine"] = {
                "aepe_gpu": a_lg, "aepe_cpu_literal": a_lr, "aepe_delta_literal": a_lg - a_lr,
                "flow_bit_exact": bool(np.array_equal(lg, lm)),
                "flow_max_abs_diff": float(np.max(np.abs(lg - lm))),
                "colour_mismatch_literal": int(np.any(oracle.flow_to_color(lm)[0] != flow_to_color(lg)[0],
                                                      axis=2).sum()),
                "note": "GPU arith=literal vs oracle/gqmap_oracle.c with the engine's Gauss-Hermite rule (the "
                        "restatement's own eig rule differs by a few ulps: aepe_delta_literal above uses it)"}
    for kind in ("emul", "literal"):
        t0 = time.perf_counter()
        if kind in finals:
            st, done = finals[kind], steps
        else:
            st, T0 = seeded()
            if kind == "emul":
                done, _, _ = oracle.emu_run(o, I1, I2, st, 1, steps, X, W, T=T0, nthreads=threads,
                                            fp32=precision == "fp32", split=split)
            else:
                done, _, _ = oracle.run(o, I1, I2, st, 1, steps, T=T0, nthreads=threads)
        mp = cpu_map(st, det_exp=kind == "emul")
        a = aepe(flo, up(mp), unk, crop)
        img = oracle.flow_to_color(colour(mp))[0]
        out[f"aepe_cpu_{kind}"] = a
        out[f"aepe_delta_{kind}"] = a_gpu - a
        out[f"colour_mismatch_{kind}"] = int(np.any(img != img_gpu, axis=2).sum())
        out[f"flow_max_abs_diff_{kind}"] = float(np.max(np.abs(mp - mp_gpu)))
        out[f"cpu_s_{kind}"] = time.perf_counter() - t0
        if done != steps:
            out[f"error_{kind}"] = f"stopped after {done}/{steps}"
    if "map1" in r:  # per-step agreement: iteration 1 alone, GPU vs the literal restatement
        st, T0 = seeded()
        oracle.run(o, I1, I2, st, 1, 1, T=T0, nthreads=threads)
        mp1 = cpu_map(st, det_exp=False)
        out["it1_flow_max_abs_diff_literal"] = float(np.max(np.abs(mp1 - r["map1"])))
        out["it1_aepe_delta_literal"] = aepe(flo, up(r["map1"]), unk, crop) - aepe(flo, up(mp1), unk, crop)
    out["flow_bit_exact_emul"] = out["flow_max_abs_diff_emul"] == 0.0
    out["gate_pass_literal"] = abs(out["aepe_delta_literal"]) <= 1e-4
    out["colour_pixels"] = int(img_gpu.shape[0] * img_gpu.shape[1])
    out["colour_note"] = ("flowToColor scales every pixel by the frame's largest flow magnitude "
                          "(flowToColor.m:66-70): one differing pixel can change the whole encoding")
    out["note"] = ("emul: the CPU model sharing the kernel's arithmetic spec (gqmap_math.h) -- bit-exact at any "
                   "number of iterations; literal: the fp64 restatement of the MATLAB, which differs by a rounding "
                   "or two per operation -- the solver's transient is chaotic, so that difference grows with the "
                   "iteration count (DESIGN.md 2; divergence: the same growth between the restatement and itself "
                   "under a 1e-13 perturbation); literal_engine: the engine run in the MATLAB source's expression "
                   "order, non-fused IEEE (arith=literal)")
    return out


def traffic_per_launch(precision: str, config: str):
    """HBM bytes per k_iter launch from the committed rocprofv3 FETCH_SIZE /
    WRITE_SIZE passes (scripts/profile_round.sh -> profiles/traffic_*.json):
    counter collection needs its own profiler runs, so it is not measured
    inside the timed bench."""
    tfile = os.path.join(ROOT, "profiles", f"traffic_{config}_{precision}.json")
    if os.path.exists(tfile):
        return json.load(open(tfile)).get("hbm_bytes_per_launch")
    return None


def traffic_unit(precision: str, config: str):
    tfile = os.path.join(ROOT, "profiles", f"traffic_{config}_{precision}.json")
    if not os.path.exists(tfile):
        return None
    return json.load(open(tfile)).get("unit", "HBM bytes per k_iter launch (one iteration)")


def traffic_source(precision: str, config: str):
    tfile = os.path.join(ROOT, "profiles", f"traffic_{config}_{precision}.json")
    if not os.path.exists(tfile):
        return None
    d = json.load(open(tfile))
    return f"profiles/traffic_{config}_{precision}.json ({d.get('source', 'rocprofv3 FETCH_SIZE+WRITE_SIZE passes')})"


def roofline(engine, L, K, nodes, precision, kernel_avg_s, config, kernel_name):
    S = 8 if precision == "fp64" else 4
    fl = algorithmic_flops_per_node(engine, L, K) * nodes
    by = algorithmic_bytes_per_node(engine, L, S) * nodes
    ach = fl / kernel_avg_s / 1e12
    peak = PEAK_TFLOPS[precision]
    return {"bound": "valu", "achieved": ach, "peak": peak, "unit": "TFLOP/s", "frac": ach / peak,
            "traffic": traffic_per_launch(precision, config), "traffic_source": traffic_source(precision, config),
            "traffic_unit": traffic_unit(precision, config),
            "kernel": kernel_name,
            "kernel_avg_us": kernel_avg_s * 1e6, "flops_per_launch": fl,
            "algorithmic_bytes_per_launch": by, "hbm_algorithmic_GBps": by / kernel_avg_s / 1e9,
            "hbm_frac": by / kernel_avg_s / 1e9 / PEAK_HBM_GBPS}


# ---------------------------------------------------------------------------
def settle_clocks(run_chunk, chunk: int, min_s: float = 0.05, max_s: float = 1.0, tol: float = 0.01,
                  fixed_chunks: int | None = None):
    """Untimed clock settling before the timed region.  The MI355X ramps its
    clocks over the first ~25 ms of sustained load: successive 20-iteration
    C2 runs from the same state take 167, 163, 158, ... 147 us per iteration
    and return to ~173 after 1 s idle (scripts/clock_ramp.py,
    profiles/r04_clock_ramp.txt) -- a 20-step window (3 ms) started cold
    measures the ramp, not the kernel.  run_chunk() runs `chunk` iterations of
    the configuration's own hot path from its initial state; chunks repeat
    until two successive ones agree within tol (at least min_s, at most
    max_s), or exactly fixed_chunks times (ranks that exchange data every
    iteration must run the same count).  The timed steps are unchanged:
    iterations 1..steps from the seeded initial state."""
    t_start = time.perf_counter()
    times = []
    while True:
        t0 = time.perf_counter()
        run_chunk()
        times.append(time.perf_counter() - t0)
        el = time.perf_counter() - t_start
        if fixed_chunks is not None:
            if len(times) >= fixed_chunks:
                break
        elif el >= max_s or (el >= min_s and len(times) >= 2 and abs(times[-1] - times[-2]) <= tol * times[-2]):
            break
    return {"iterations": chunk * len(times), "seconds": round(el, 4),
            "first_chunk_us_per_it": times[0] / chunk * 1e6, "last_chunk_us_per_it": times[-1] / chunk * 1e6,
            "note": "untimed: the hot path run until the GPU clocks settle (bench.settle_clocks); the timed "
                    "steps still start from the seeded initial state at iteration 1; cold_start_value: the same "
                    "steps timed once before settling (right after the warm-up), for the record"}


def run_engine_config(args, rank, world, local, barrier, engine, names, L, K, extra, label):
    """C2 / C4: one solve per rank (frame-parallel), steps iterations timed."""
    from gqmap_opticalflow_amd import Engine, aepe
    name = names[rank % len(names)]
    I1, I2, flo, unk, opts = gt_options(name, L, K, **extra)
    eng = Engine(opts, I1, I2, engine, args.precision, device=local)
    eng.init_state(seed=1 + rank)
    if args.warmup:
        eng.run_timed(args.warmup)
    eng.prepare()  # the replayed 50-iteration graph is captured and uploaded outside the timed region

    def chunk():
        eng.init_state(seed=rank)
        eng.run(20)
    settle = None
    if not args.no_settle:
        # the same steps timed once before settling, for the record (the
        # line's value is the settled run below)
        eng.init_state(seed=rank)
        barrier()
        t0 = time.perf_counter()
        eng.run(args.steps)
        barrier()
        cold = time.perf_counter() - t0
        settle = settle_clocks(chunk, 20)
        settle["cold_start_ms_per_step"] = cold / args.steps * 1e3
    eng.init_state(seed=rank)  # timed steps are iterations 1..steps of the solve
    barrier()
    t0 = time.perf_counter()
    done, _ = eng.run(args.steps)  # the production path (gqmap_run: graph replay, no instrumentation)
    barrier()
    elapsed = time.perf_counter() - t0
    if done != args.steps:
        raise RuntimeError(f"rank {rank}: solver stopped after {done}/{args.steps} iterations")
    mp = eng.map()
    # k_iter durations: the same iterations replayed from the same initial
    # state with a HIP event pair around every launch on the engine's stream
    # (bit-identical work -- checked below; the event markers add a few us
    # between launches, which is why the timed region above runs without them)
    eng.init_state(seed=rank)
    done2, total_ms, kernel_ms = eng.run_timed(args.steps)
    if done2 != args.steps or not np.array_equal(eng.map(), mp):
        raise RuntimeError(f"rank {rank}: the instrumented replay differs from the timed run")
    eng.init_state(seed=rank)  # iteration 1 alone (the parity gate's per-step agreement)
    eng.run(1)
    mp1 = eng.map()
    # the parity gate compares the GPU flow after gate_its iterations with
    # the CPU paths' (all the timed steps, unless the CPU would take minutes:
    # the super engine's CPU model runs ~1 s per C4 iteration)
    gate_its = min(args.steps, args.parity_steps or (args.steps if engine != "super" else 20))
    mpg = mp
    if gate_its != args.steps:
        eng.init_state(seed=rank)
        eng.run(gate_its)
        mpg = eng.map()
    if engine == "super":
        flow = np.repeat(np.repeat(mp, 4, axis=0), 4, axis=1)
        a = aepe(flo, flow, unk, 4)
    else:
        a = aepe(flo, mp, unk)
    nodes = eng.M * eng.N
    split = eng.info().split
    dataflow = eng.dataflow()
    # the flow after each of the first track_its iterations (the parity
    # gate's divergence trajectory against the literal restatement)
    maps_it = []
    if rank == 0 and engine == "mixture" and L == 1 and not args.no_parity:
        eng.init_state(seed=rank)
        for _ in range(min(gate_its, TRACK_ITS)):
            eng.run(1)
            maps_it.append(eng.map())
    eng.close()
    lit = None
    if engine == "mixture" and args.precision == "fp64" and not args.no_literal:
        try:
            lit = literal_engine_leg(args, rank, opts, I1, I2, flo, unk, gate_its, local)
        except Exception as e:  # reported in the line; the headline value stands
            lit = {"error": f"{type(e).__name__}: {e}"[:300]}
    Mo, No = I1.shape
    ksuf = {"mixture": 0, "super": 1}[engine]
    R = "double" if args.precision == "fp64" else "float"
    # the padded frame's store (integer frames): binary16 column pairs for
    # the mixture engine at one lane per node (policy vv_pair), else float
    pair = (engine == "mixture" and split == 1 and "vv_pair=0" not in args.policy)
    vvt = "vvh2_t" if pair else "float"
    vvs = ("VV stored as binary16 column pairs: integer frames" if pair else
           "VV stored as float: integer frames")
    return dict(elapsed=elapsed, kernel_ms=kernel_ms, instrumented_ms=total_ms, pixels=Mo * No, nodes=nodes, aepe=a, name=name,
                settle=settle, maps_it=maps_it, literal=lit,
                I1=I1, I2=I2, opts=opts, Mo=Mo, No=No, map=mpg, gate_its=gate_its, map1=mp1, flo=flo, unk=unk, split=split, seed=rank,
                kernel=(f"gq::k_iter_flow<{R},{vvt},{ksuf},1> (dataflow launch: one per 50-iteration chunk, the "
                        f"per-iteration average; {vvs})" if dataflow else
                        f"gq::k_iter<{R},{vvt},{ksuf},Q> ({vvs})"),
                dataflow=dataflow,
                workload=f"{label}: {name} {No}x{Mo} {engine} L={L} K={K} its={args.steps} "
                         f"(one step = one full-frame iteration)")


TRACK_ITS = 60  # iterations of the per-iteration divergence record (parity gate)


def literal_engine_leg(args, rank, opts, I1, I2, flo, unk, gate_its, device):
    """The literal-order engine (options arith="literal": every expression of
    gqmap_gpu_mixture.m:87-182 in MATLAB's expression order, non-fused IEEE, k_iter_lit) on
    the same pair, seed and steps: timed like the headline (settled clocks,
    gqmap_run graph replay), its k_iter_lit mean from an instrumented replay,
    and its flow after gate_its iterations for the parity gate (bit-identical
    to the literal restatement with the same Gauss-Hermite rule)."""
    from gqmap_opticalflow_amd import Engine, aepe
    eng = Engine(dict(opts, arith="literal"), I1, I2, "mixture", "fp64", device=device)
    try:
        eng.init_state(seed=rank)
        if args.warmup:
            eng.run(args.warmup)
        eng.prepare()

        def chunk():
            eng.init_state(seed=rank)
            eng.run(20)
        if not args.no_settle:
            settle_clocks(chunk, 20)
        eng.init_state(seed=rank)
        eng.synchronize()
        # rank-local timing (the leg is reported from rank 0): no collective
        # here, so a rank whose leg fails cannot leave the others waiting
        t0 = time.perf_counter()
        done, _ = eng.run(args.steps)
        eng.synchronize()
        elapsed = time.perf_counter() - t0
        mp = eng.map()
        eng.init_state(seed=rank)
        done2, total_ms, kernel_ms = eng.run_timed(args.steps)
        replay_same = done2 == done and np.array_equal(eng.map(), mp)
        mpg = mp
        if gate_its != args.steps:
            eng.init_state(seed=rank)
            eng.run(gate_its)
            mpg = eng.map()
        Mo, No = I1.shape
        return {"value": Mo * No * done / elapsed / 1e9, "unit": "Gpixel-iter/s", "its": done,
                "ms_per_step": elapsed / max(done, 1) * 1e3, "k_iter_us": kernel_ms / max(done, 1) * 1e3,
                "instrumented_replay_bit_exact": bool(replay_same), "aepe_gpu": aepe(flo, mp, unk),
                "kernel": "gq::k_iter_lit<float,false> (literal order, fp64 arithmetic, VV stored as float)",
                "map": mpg}
    finally:
        eng.close()


def run_c3(args, rank, world, local, barrier):
    from gqmap_opticalflow_amd import C3_SCALES, Pyramid, aepe, ctf_options
    name = PAIRS_480[rank % len(PAIRS_480)]
    I1, I2, flo, unk, o = gt_options(name, 1, 11)
    opts = ctf_options(its=args.steps, minu=o["minu"], maxu=o["maxu"], minv=o["minv"], maxv=o["maxv"])
    p = Pyramid(opts, C3_SCALES, args.precision, device=local)
    p.set_images(I1, I2)
    if args.warmup:
        p.run(seed=100 + rank)
    barrier()
    t0 = time.perf_counter()
    flow, its, ms = p.run(seed=rank)
    barrier()
    elapsed = time.perf_counter() - t0
    px = sum(p.level(l)["I2"].size * its[l] for l in range(len(C3_SCALES)))
    a = aepe(flo, flow, unk)
    top = p.level(len(C3_SCALES) - 1)
    p.close()
    # the dominant (full-resolution) level's k_iter on its own: the same
    # frames (the level's warped I1 and I2) and options in a single-level
    # context, every launch bracketed by HIP events (gqmap_run_timed)
    dom = None
    if rank == 0:
        from gqmap_opticalflow_amd import Engine
        with Engine(opts, top["I1w"], top["I2"], "ctf", args.precision, device=local) as e:
            e.init_state(seed=rank + len(C3_SCALES) - 1)
            e.run_timed(min(args.steps, 20))
            e.init_state(seed=rank + len(C3_SCALES) - 1)
            done, total_ms, kernel_ms = e.run_timed(args.steps)
            M, N = top["I2"].shape
            dom = dict(level=f"{N}x{M}", its=done, kernel_avg_s=kernel_ms / max(done, 1) / 1e3, nodes=M * N,
                       split=e.info().split)
    Mo, No = I1.shape
    return dict(elapsed=elapsed, pix_its=px, aepe=a, name=name, I1=I1, I2=I2, opts=dict(opts, engine="ctf"),
                Mo=Mo, No=No, its=its, flo=flo, unk=unk, seed=rank, dominant=dom,
                workload=f"C3: {name} {No}x{Mo} coarse-to-fine, 5 levels 1/16..1 (30x40..480x640), "
                         f"gqmap_ctf K=11, {args.steps} its/level, device imresize/interp2/fillmissing; "
                         f"value counts sum over levels of level pixels x its")


def parity_gate_c3(r, precision, its=12):
    """The C3 pipeline's parity gate, after the timed region: the device
    pyramid (5 levels, `its` iterations per level, the timed run's seed)
    against the CPU pipeline (oracle.ctf_pipeline: the restated imresize /
    interp2 / fillmissing plumbing around each level's solver) with the CPU
    model of the kernel arithmetic (emul: bit-exact expected) and with the
    literal fp64 restatement (literal: a rounding or two per operation,
    DESIGN.md 2), from the same seeded per-level initial states
    (tests/test_gpu_pyramid.py at 12 iterations per level)."""
    from gqmap_opticalflow_amd import C3_SCALES, Pyramid, aepe, gauss_hermite, initial_state
    from oracle import oracle
    opts = dict(r["opts"], its=its)
    opts.pop("engine", None)
    seed = r["seed"]
    hc = host_cpus()
    t0 = time.perf_counter()
    with Pyramid(opts, C3_SCALES, precision) as p:
        p.set_images(r["I1"], r["I2"])
        flow, lits, _ = p.run(seed=seed)
    X, W = gauss_hermite(int(opts["K"]))

    def init_fn(l, lo, M, N):
        st = initial_state(lo, M, N, seed=seed + l, engine="ctf")
        return oracle.State(st.muu, st.muv, st.sigu, st.sigv, st.pn, st.rou, st.w, st.alpha)

    out = {"its_per_level": its, "levels": len(C3_SCALES), "aepe_gpu": aepe(r["flo"], flow, r["unk"])}
    for solver in ("emu", "literal"):
        t1 = time.perf_counter()
        warp, _ = oracle.ctf_pipeline(opts, r["I1"], r["I2"], C3_SCALES, init_fn, solver=solver, X=X, W=W,
                                      nthreads=hc["threads"], fp32=precision == "fp32")
        k = "emul" if solver == "emu" else "literal"
        out[f"aepe_cpu_{k}"] = aepe(r["flo"], warp, r["unk"])
        out[f"aepe_delta_{k}"] = out["aepe_gpu"] - out[f"aepe_cpu_{k}"]
        out[f"flow_bit_exact_{k}"] = bool(np.array_equal(flow, warp))
        out[f"flow_max_abs_diff_{k}"] = float(np.max(np.abs(flow - warp)))
        out[f"cpu_s_{k}"] = time.perf_counter() - t1
    out["seconds"] = time.perf_counter() - t0
    out["note"] = ("emul: CPU pipeline with the CPU model of the kernel arithmetic (gqmap_math.h) -- bit-exact; "
                   "literal: the same pipeline with the fp64 restatement of legacy/gqmap_ctf.m, a rounding or two "
                   "per operation away, amplified by the solver's chaotic transient (DESIGN.md 2)")
    return out


def run_c1(args, rank, world, local, barrier):
    """legacy/gqmap_cpu.m on the GT flow of a 584x388 pair (unknowns zeroed).
    Timed: gqmap_cpu_run_device on the flow already resident in HBM (the
    bench contract's value); the same call on host arrays (PCIe copies in and
    out) is timed after it and reported beside it, never as the value."""
    import torch
    from gqmap_opticalflow_amd import flow_to_color, flowio, gqmap_cpu, gqmap_cpu_device
    name = PAIRS[(rank + 1) % len(PAIRS)] if world > 1 else "Dimetrodon"
    gt = flowio.load_pair(name)[2]
    _, flo, _, unk = flow_to_color(gt, device=local)
    o = dict(its=args.steps, K=9)
    dev = torch.device("cuda", local)
    flo_d = torch.from_numpy(np.asfortranarray(flo)).to(dev)  # column-major M x N x 2, resident
    # warm-up: the same call (its included) until the wall clock settles --
    # the second call of a fresh process measured 33 ms against 7.1 ms from the
    # third on (scripts/c1_timing.py: first-use costs outside the kernels)
    for _ in range(min(args.warmup, 3)):
        gqmap_cpu_device(o, flo_d, seed=1)
    settle = None if args.no_settle else settle_clocks(lambda: gqmap_cpu_device(o, flo_d, seed=1), args.steps)
    torch.cuda.synchronize(dev)
    barrier()
    t0 = time.perf_counter()
    mu_d, _, _, tr = gqmap_cpu_device(o, flo_d, seed=0, return_trace=True)
    torch.cuda.synchronize(dev)
    barrier()
    elapsed = time.perf_counter() - t0
    mu = np.asfortranarray(mu_d.cpu().numpy())
    # the host-array call (copies included), same seed: bit-identical result
    gqmap_cpu(o, flo, seed=1, device=local)
    t1 = time.perf_counter()
    mu_h = gqmap_cpu(o, flo, seed=0, device=local)[0]
    host_s = time.perf_counter() - t1
    M, N, _ = flo.shape
    err = float(np.sqrt(((mu - flo) ** 2).sum(axis=2))[~unk].mean())
    return dict(elapsed=elapsed, pixels=M * N, nodes=M * N, aepe=err, flow=flo, unk=unk, mu=mu, opts=o, Mo=M, No=N,
                its=tr.shape[0], settle=settle,
                host_arrays={"value": M * N * tr.shape[0] / host_s / 1e9, "unit": "Gpixel-iter/s",
                             "ms_per_step": host_s / tr.shape[0] * 1e3,
                             "same_bits": bool(np.array_equal(mu_h, mu)),
                             "note": "gqmap_cpu_run on host arrays: the call's wall clock including the pageable "
                                     "host<->device copies (PCIe-inclusive rate; not the value)"},
                workload=f"C1: {name} {N}x{M} legacy/gqmap_cpu.m flow denoising (input = GT flow, unknowns 0), "
                         f"K=9, var=gama=1, dta=inf, {args.steps} its, sigma0 = U+2 (seed 0); flow resident in "
                         f"HBM (gqmap_cpu_run_device); aepe = mean |mu - flow|",
                value_definition="device-resident (round 5 on): the flow already in HBM, results left there -- "
                                 "not comparable with C1 values before round 5, which timed the host-array call; "
                                 "compare kernel progress across rounds with host_arrays")


def cpu_baseline_c1(flow, opts, budget_s: float = 8.0):
    """The C restatement of legacy/gqmap_cpu.m, OpenMP over rows as the
    reference's parfor (legacy/gqmap_cpu.m:17) -- all of this process's
    cores, then one thread -- on a bounded sample."""
    from gqmap_opticalflow_amd import gauss_hermite
    from oracle import oracle
    hc = host_cpus()
    M, N, _ = flow.shape
    X, W = gauss_hermite(9)
    sg0 = np.asfortranarray(np.full((M, N, 2), 2.5))
    legs = {}
    allc = allcore_threads(hc)
    for threads in (hc["threads"], 1, allc):
        def run_n(n, threads=threads):
            return oracle.cpu_run(dict(opts, its=n, min_its=10 ** 9), flow, sg0, X, W, nthreads=threads)[3].shape[0]
        legs[threads] = _timed_leg(run_n, budget_s)
    (n_all, t_all), (n_one, t_one), (n_pc, t_pc) = legs[hc["threads"]], legs[1], legs[allc]
    return {"value": M * N * n_all / t_all / 1e9, "unit": "Gpixel-iter/s", "cores": hc["threads"], "kind": "port",
            "value_1thread": M * N * n_one / t_one / 1e9, "value_allcores": M * N * n_pc / t_pc / 1e9,
            "cores_allcores": allc, "nproc": hc["nproc"], "cgroup_cpu_quota": hc["cpu_quota"],
            "affinity_cpus": hc["affinity"], "physical_cores": hc["physical_cores"],
            "sample": f"oracle/gqmap_legacy_oracle.c fp64, {N}x{M}, K=9: {n_all} iterations on {hc['threads']} "
                      f"OpenMP threads (rows, as the reference parfor) in {t_all:.1f}s, {n_one} on 1 thread "
                      f"in {t_one:.1f}s"}


def parity_gate_c1(r, steps):
    """The north-star gate on the path it names, legacy/gqmap_cpu.m (config
    C1): the C restatement (oracle/gqmap_legacy_oracle.c) from the same
    sigma0 (U + 2, the library RNG, seed 0) for the same iterations; AEPE of
    each result against the input flow (known pixels) and the uint8
    flowToColor encoding of both (mismatching pixels)."""
    from gqmap_opticalflow_amd import flow_to_color, gauss_hermite, rand_uniform
    from oracle import oracle
    flo, unk, mu = r["flow"], r["unk"], r["mu"]
    M, N, _ = flo.shape
    sg0 = np.asfortranarray(rand_uniform(0, 3, 2 * M * N).reshape((M, N, 2), order="F") + 2)
    X, W = gauss_hermite(9)
    t0 = time.perf_counter()
    mu_c, _, _, tr = oracle.cpu_run(dict(r["opts"], its=steps), flo, sg0, X, W, nthreads=host_cpus()["threads"])
    cpu_s = time.perf_counter() - t0
    err = lambda m: float(np.sqrt(((m - flo) ** 2).sum(axis=2))[~unk].mean())
    a_g, a_c = err(mu), err(mu_c)
    img_g = flow_to_color(mu)[0]
    img_c = oracle.flow_to_color(mu_c)[0]
    mism = int(np.any(img_g != img_c, axis=2).sum())
    return {"its": steps, "cpu_its": int(tr.shape[0]), "gate": 1e-4, "aepe_gpu": a_g, "aepe_cpu_literal": a_c,
            "aepe_delta_literal": a_g - a_c, "flow_max_abs_diff_literal": float(np.max(np.abs(mu - mu_c))),
            "colour_mismatch_literal": mism, "colour_pixels": M * N, "gate_pass_literal": abs(a_g - a_c) <= 1e-4,
            "cpu_s_literal": cpu_s,
            "note": "legacy/gqmap_cpu.m (the north star's named CPU path): the device engine is plain fp64 in the "
                    "restatement's operation order, so the flows are bit-identical"}


STRIP_PLANES = ("muu", "muv", "sigu", "sigv", "pn", "rou")


def gather_strips(dist, world, owned, col0, col1):
    """Every rank's owned node columns [col0, col1) of the state planes
    (STRIP_PLANES order) to rank 0: a list of (col0, col1, planes) in rank
    order there, None on the other ranks."""
    mine = (int(col0), int(col1), [np.array(p, order="F", copy=True) for p in owned])
    if dist is None or world == 1:
        return [mine]
    rank = dist.get_rank()
    parts = [None] * world if rank == 0 else None
    dist.gather_object(mine, parts, dst=0)
    return parts


def strip_parity(parts, whole, strip_trace=None, whole_trace=None, strip_done=None, whole_done=None):
    """The strips assembled into the full grid against a whole-grid solve of
    the same pair, seed and lanes per node (a Jacobi update with exact totals:
    they must agree bit for bit, gqmap_gpu_mixture.m:29-46).  whole: the
    full-grid planes in STRIP_PLANES order.  Returns the record the line
    carries (bit_exact, per-plane mismatching values, uncovered columns, the
    stop iteration of both, the trace comparison)."""
    mism = {}
    cover = np.zeros(whole[0].shape[1], dtype=int)
    for c0, c1, _ in parts:
        cover[c0:c1] += 1
    for i, name in enumerate(STRIP_PLANES):
        glob = np.zeros_like(whole[i])
        for c0, c1, owned in parts:
            glob[:, c0:c1] = owned[i]
        mism[name] = int(np.sum(glob != whole[i]))
    rec = {"bit_exact": all(v == 0 for v in mism.values()) and bool(np.all(cover == 1)),
           "mismatch": mism, "columns_not_covered_once": int(np.sum(cover != 1))}
    if strip_done is not None:
        rec["stop_iteration"] = {"strips": int(strip_done), "whole": int(whole_done)}
        rec["bit_exact"] = rec["bit_exact"] and strip_done == whole_done
    if strip_trace is not None:
        rec["trace_bit_exact"] = bool(np.array_equal(strip_trace, whole_trace))
        rec["bit_exact"] = rec["bit_exact"] and rec["trace_bit_exact"]
    return rec


def tiled_solve(args, rank, world, local, barrier, dist, I1, I2, flo, unk, opts, validate=True):
    """One frame as column-strip tiles over the ranks (gqmap_create_tile):
    RCCL ghost-column and exact-totals exchange every iteration.  Returns the
    rank's timing and its share of the AEPE sums (interior pixels)."""
    from gqmap_opticalflow_amd import Engine, comm_unique_id, strip_split
    Mo, No = I1.shape
    # lanes per node from ONE strip (the whole-grid solve with the same split
    # is bit-identical: tests/test_gpu_tiles.py)
    opts = dict(opts, split=int(opts.get("split") or strip_split(Mo, No, world)))
    eng = Engine(opts, I1, I2, "mixture", args.precision, device=local, n_tiles=world, tile=rank)
    try:
        if world > 1:
            uid = [comm_unique_id() if rank == 0 else None]
            dist.broadcast_object_list(uid, src=0)
            eng.attach_rccl(uid[0])
        eng.init_state(seed=1)
        # warm-up with single launches (fewer than a 50-iteration graph chunk):
        # the RCCL peer connections are set up before any graph capture
        eng.run(max(1, min(args.warmup, 49)))
        eng.prepare()  # the replayed graph (kernels + RCCL exchange) captured and uploaded untimed

        def chunk():
            eng.init_state(seed=0)
            eng.run(20)
        # the same count on every rank (the strips exchange every iteration)
        settle = settle_clocks(chunk, 20, fixed_chunks=8) if not args.no_settle else None
        eng.init_state(seed=0)  # timed steps are iterations 1..steps of the solve
        barrier()
        t0 = time.perf_counter()
        done, tr = eng.run(args.steps)  # production path: graph replay
        barrier()
        elapsed = time.perf_counter() - t0
        if done != args.steps:
            raise RuntimeError(f"rank {rank}: solver stopped after {done}/{args.steps} iterations")
        mp = eng.map()
        col0, col1 = eng.col0, eng.col1
        # k_iter durations: a replay of the same iterations with HIP events
        # around every iteration's k_iter launch over the strip
        eng.init_state(seed=0)
        done2, total_ms, kernel_ms = eng.run_timed(args.steps)
        if done2 != args.steps or not np.array_equal(eng.map(), mp):
            raise RuntimeError(f"rank {rank}: the instrumented replay differs from the timed run")
        sp = None
        if validate:
            # the strips' final state (the replay ends where the timed run
            # did: checked above) against a whole-grid solve on rank 0
            st = eng.get_state()
            parts = gather_strips(dist, world, [getattr(st, k)[:, col0:col1] for k in STRIP_PLANES], col0, col1)
            if rank == 0:
                with Engine(opts, I1, I2, "mixture", args.precision, device=local) as whole:
                    whole.init_state(seed=0)
                    wdone, wtr = whole.run(args.steps)
                    ws = whole.get_state()
                sp = strip_parity(parts, [getattr(ws, k) for k in STRIP_PLANES], tr, wtr, done, wdone)
                sp["reference"] = (f"whole-grid gqmap_run of the same pair, seed and lanes per node (split "
                                   f"{opts['split']}), {args.steps} iterations")
            barrier()
    finally:
        eng.close()
    Mo, No = I1.shape
    # AEPE of gqmap_gpu_mixture.m:63-64 over this rank's strip of the interior
    sl = (slice(1, Mo - 1), slice(max(col0, 1), min(col1, No - 1)))
    f = mp.copy()
    f[unk] = 0
    e = np.sqrt(((flo[sl] - f[sl]) ** 2).sum(axis=2))
    return dict(elapsed=elapsed, kernel_ms=kernel_ms, pixels=Mo * No, nodes=Mo * (col1 - col0), settle=settle,
                err_sum=float(e.sum()), err_n=int(e.size), split=opts["split"], strip_parity=sp)


def run_tiled(args, rank, world, local, barrier, dist, names, scale, label):
    """C5 (the eight pairs of legacy/optical_flow_temp.m:3 upsampled 4x) or
    the tiled C2 mode: each pair in turn split over all ranks; the timed
    region is the sum of the pairs' timed solves (frames resident in HBM)."""
    from gqmap_opticalflow_amd import flow_to_color, flowio
    tot = dict(elapsed=0.0, kernel_ms=0.0, pixels=0, nodes=0, pix_its=0, max_nodes=0)
    per_pair, ref = [], None
    for name in names:
        I1, I2, gt = flowio.load_pair_scaled(name, scale, device=local)
        _, flo, (minu, maxu, minv, maxv), unk = flow_to_color(gt, device=local)
        opts = dict(its=args.steps, K=9, L=1, temperature=0.0, drate=0.5, epsn=1e-6, lambdas=5.0, lambdad=1.0,
                    minu=minu, maxu=maxu, minv=minv, maxv=maxv)
        # the strips are checked against the whole grid on the first pair
        # (C5's 3.6 Mpx pairs: one whole-grid solve bounds the extra time)
        r = tiled_solve(args, rank, world, local, barrier, dist, I1, I2, flo, unk, opts, validate=not per_pair)
        if r["strip_parity"] is not None:
            tot["strip_parity"] = dict(r["strip_parity"], pair=name)
        Mo, No = I1.shape
        for k in ("elapsed", "kernel_ms", "pixels", "nodes"):
            tot[k] += r[k]
        tot["split"] = r["split"]
        tot.setdefault("settle", r.get("settle"))
        tot["pix_its"] += Mo * No * args.steps
        per_pair.append(dict(name=name, size=f"{No}x{Mo}", err_sum=r["err_sum"], err_n=r["err_n"],
                             elapsed=r["elapsed"]))
        if ref is None:
            ref = (I1, I2, opts)
    I1, I2, opts = ref
    desc = ", ".join(f"{p['name']} {p['size']}" for p in per_pair)
    return dict(tot, per_pair=per_pair, I1=I1, I2=I2, opts=opts, Mo=I1.shape[0], No=I1.shape[1],
                workload=f"{label}: {len(names)} pair(s) ({desc}), "
                         + (f"bicubic imresize x{scale:g} of the uint8 RGB frames then rgb2gray "
                            f"(imresize(imread(..),scale), optical_flow_temp.m:7-8), GT x{scale:g} in size and "
                            f"value; " if scale != 1 else "")
                         + f"mixture L=1 K=9, each pair as {world} column-strip tile(s) with RCCL ghost-column + "
                           f"totals exchange per iteration, Q={tot['split']} lanes per node (from one strip), "
                           f"its={args.steps} per pair, pairs run in turn")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=None)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--precision", default="fp64", choices=("fp64", "fp32"))
    ap.add_argument("--config", default="c2", choices=("c1", "c2", "c3", "c4", "c5"))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-settle", action="store_true",
                    help="time the steps without settling the GPU clocks first (settle_clocks)")
    ap.add_argument("--no-strong-scaling", action="store_true",
                    help="c2: skip the strong-scaling leg (the pair split over the ranks)")
    ap.add_argument("--parity-steps", type=int, default=0,
                    help="iterations of the parity gate (default: all timed steps; C4: 20)")
    ap.add_argument("--no-parity", action="store_true",
                    help="skip the parity gate (CPU model + literal restatement of the same steps, AEPE and "
                         "colour deltas) after the timed region")
    ap.add_argument("--no-literal", action="store_true",
                    help="c2/c4 mixture fp64: skip the literal-order engine leg (arith=literal, timed and checked "
                         "bit for bit against the literal restatement)")
    ap.add_argument("--tiled", action="store_true",
                    help="c2: strong scaling -- the RubberWhale pair split into column strips over the ranks")
    ap.add_argument("--policy", default="",
                    help="A/B only: library execution policies name=value,... (gqmap_debug_policy, e.g. flow=0 "
                         "for one launch per iteration); they never change a result")
    args = ap.parse_args()
    if args.steps is None:
        args.steps = DEFAULT_STEPS[args.config]

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    if args.policy:  # (after torch: the library must bind to torch's HIP runtime)
        from gqmap_opticalflow_amd import _lib
        for item in args.policy.split(","):
            name, _, value = item.partition("=")
            _lib.debug_policy(name.strip(), int(value))
    dist = None
    # GQMAP_BENCH_BACKEND=gloo rehearses the multi-rank harness on a box with
    # fewer GPUs than ranks (ranks then share devices round-robin); the
    # driver's runs use RCCL ("nccl") with one GPU per rank.
    backend = os.environ.get("GQMAP_BENCH_BACKEND", "nccl")
    if world > 1:
        import torch.distributed as dist
        local = local % max(1, torch.cuda.device_count())
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    else:
        torch.cuda.set_device(0)
        local = 0

    def barrier():
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()

    cfg = args.config
    tiled = cfg == "c5" or (cfg == "c2" and args.tiled)
    if tiled:
        if cfg == "c5":
            r = run_tiled(args, rank, world, local, barrier, dist, C5_PAIRS, 4.0, "C5")
        else:
            r = run_tiled(args, rank, world, local, barrier, dist, ("rubberwhale",), 1.0, "C2 tiled")
        engine, L, K = "mixture", 1, 9
    elif cfg == "c2":
        r = run_engine_config(args, rank, world, local, barrier, "mixture", PAIRS if world > 1 else PAIRS[:1],
                              1, 9, {}, "C2")
        engine, L, K = "mixture", 1, 9
    elif cfg == "c4":
        r = run_engine_config(args, rank, world, local, barrier, "super", ("Urban3", "Grove3", "Urban2", "Grove2"),
                              3, 11, dict(temperature=0.2, drate=0.75, lambdas=16.0), "C4")
        engine, L, K = "super", 3, 11
    elif cfg == "c3":
        r = run_c3(args, rank, world, local, barrier)
        engine, L, K = "ctf", 1, 11
    elif cfg == "c1":
        r = run_c1(args, rank, world, local, barrier)
        engine, L, K = "legacy", 1, 9

    elapsed = r["elapsed"]
    kernel_ms = r.get("kernel_ms", 0.0)
    if dist is not None:
        dev = "cuda" if backend == "nccl" else "cpu"
        t = torch.tensor([elapsed, kernel_ms], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, kernel_ms = t.tolist()
    if tiled:  # per pair: the ranks' strip sums -> the pair's AEPE; then the mean over pairs
        sums = [p["err_sum"] for p in r["per_pair"]] + [p["err_n"] for p in r["per_pair"]]
        if dist is not None:
            t = torch.tensor(sums, device=dev, dtype=torch.float64)
            dist.all_reduce(t)
            sums = t.tolist()
        n = len(r["per_pair"])
        for i, p in enumerate(r["per_pair"]):
            p["aepe"] = sums[i] / sums[n + i]
        r["aepe"] = float(np.mean([p["aepe"] for p in r["per_pair"]]))

    out = None
    if rank == 0:
        if cfg == "c3":
            units = r["pix_its"] * world
            parallel = f"frame-parallel x{world}"
        elif cfg == "c1":
            units = world * r["pixels"] * r["its"]
            parallel = f"frame-parallel x{world}"
        elif tiled:
            units = r["pix_its"]
            parallel = f"column-strip tiles x{world} (RCCL halo)"
        else:
            units = world * r["pixels"] * args.steps
            parallel = f"frame-parallel x{world}"
        out = {
            "metric": METRIC, "value": units / elapsed / 1e9, "unit": "Gpixel-iter/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True, "scaling": "strong" if tiled else "weak", "vs_baseline": None,
            "dtype": "f64" if args.precision == "fp64" else "f32",
            "data": "Middlebury frame10/11 + flow10.flo (real frames, in-repo data/middlebury)"
                    + ("; upsampled 4x on the device" if cfg == "c5" else ""),
            "config": {"workload": r["workload"], "engine": engine, "L": L, "K": K, "parallelism": parallel},
            "policy": args.policy or "default",
            "aepe": r["aepe"], "aepe_its": args.steps,
            "timed_region": "iterations 1..steps of the solve (gqmap_gpu_mixture.m:27-50, 69-75 on the device); "
                            "the reference loop's host evaluation block (it==1 / every 300 its: MAP, PNG, AEPE, "
                            "logP, :52-68) is outside it -- aepe is computed once after the timed steps",
        }
        if r.get("settle"):
            out["clock_settle"] = r["settle"]
            if "cold_start_ms_per_step" in r["settle"]:
                # the same steps on rank 0 timed right after the warm-up, before settling
                cs = r["settle"]["cold_start_ms_per_step"]
                out["clock_settle"]["cold_start_value"] = units / (cs * 1e-3 * args.steps) / 1e9
        if cfg == "c1":
            out["host_arrays"] = r["host_arrays"]
            out["value_definition"] = r["value_definition"]
            # per pixel: node 2 x K x 6 flop, edges 4 x K^2 x ~40 flop (legacy/gqmap_cpu.m:20-54)
            fl = (2 * K * 6 + 4 * K * K * 40) * r["pixels"] * r["its"]
            out["roofline"] = {"bound": "valu", "achieved": fl / elapsed / 1e12, "peak": PEAK_TFLOPS["fp64"],
                               "unit": "TFLOP/s", "frac": fl / elapsed / 1e12 / PEAK_TFLOPS["fp64"],
                               "traffic": traffic_per_launch("fp64", "c1"),
                               "traffic_unit": "HBM bytes per iteration (grad + update + ctl)",
                               "traffic_source": traffic_source("fp64", "c1"),
                               "kernel": "gq::k_legacy_grad + k_legacy_update + k_legacy_ctl (timed by the device call's wall "
                                         "clock)"}
        elif cfg == "c3":
            secs = elapsed
            Sb = 8 if args.precision == "fp64" else 4
            fl = algorithmic_flops_per_node("ctf", 1, K) * r["pix_its"]
            out["roofline"] = {"bound": "valu", "achieved": fl / secs / 1e12, "peak": PEAK_TFLOPS[args.precision],
                               "unit": "TFLOP/s", "frac": fl / secs / 1e12 / PEAK_TFLOPS[args.precision],
                               "traffic": traffic_per_launch(args.precision, cfg),
                               "kernel": "gq::k_iter<R,VT,2,Q> (all levels; timed by the pipeline wall clock)",
                               "traffic_source": traffic_source(args.precision, cfg),
                               "traffic_kernel": "the full-resolution level's k_iter (per launch)",
                               "algorithmic_bytes_per_node_iter": algorithmic_bytes_per_node("ctf", 1, Sb)}
            dom = r.get("dominant")
            if dom:
                # the dominant level's kernel on its own, from HIP events
                dl = roofline("ctf", 1, K, dom["nodes"], args.precision, dom["kernel_avg_s"], cfg,
                              "gq::k_iter<R,VT,2,Q> (the full-resolution level)")
                dl.update(level=dom["level"], its=dom["its"], split=dom["split"],
                          kernel_timing="HIP events around every k_iter launch (gqmap_run_timed) of a single-level "
                                        "context on the level's own frames (the pipeline's warped I1 and I2)")
                out["roofline"]["dominant_level"] = dl
            out["config"]["its_per_level"] = r["its"]
        else:
            # tiled: the kernel mean over all pairs' launches; nodes = the
            # rank's average share of a pair's grid
            nsteps = args.steps * (len(r["per_pair"]) if tiled else 1)
            kern_avg_s = kernel_ms / nsteps / 1e3
            nodes = r["nodes"] / (len(r["per_pair"]) if tiled else 1)
            out["roofline"] = roofline(engine, L, K, nodes, args.precision, kern_avg_s, cfg,
                                       r.get("kernel", "gq::k_iter"))
            if "instrumented_ms" in r:
                out["roofline"]["kernel_timing"] = (
                    ("HIP events around every dataflow launch (k_iter_flow: one launch per <= 50-iteration chunk) "
                     "in a replay of the timed iterations from the same initial state (bit-identical final state "
                     "checked), summed and divided by the iterations: kernel_avg_us is per iteration, and a "
                     "rocprofv3 duration of k_iter_flow divided by the iterations of its launch compares with it"
                     if r.get("dataflow") else
                     "HIP events around every k_iter launch in a replay of the timed iterations from the same "
                     "initial state (bit-identical final state checked)") + "; the timed region itself is gqmap_run")
                out["roofline"]["dataflow"] = bool(r.get("dataflow"))
                out["ms_per_step_instrumented"] = r["instrumented_ms"] / args.steps
        if tiled:
            out["per_pair"] = [{k: p[k] for k in ("name", "size", "aepe", "elapsed")} for p in r["per_pair"]]
            out["config"]["split"] = r["split"]
            if r.get("strip_parity"):
                out["strip_parity"] = r["strip_parity"]

    printed = []

    def emit():
        if rank == 0 and not printed:
            printed.append(1)
            print(json.dumps(out), flush=True)

    if cfg == "c2" and not tiled and not args.no_strong_scaling:
        # the headline pair split over the ranks (strong scaling).  A watchdog
        # keeps a stuck exchange from costing the whole line: after its limit
        # rank 0 prints what it has and every rank leaves.
        limit = float(os.environ.get("GQMAP_STRONG_TIMEOUT", "180"))

        def fire():
            if out is not None:
                out["strong_scaling"] = {"error": f"no result within {limit:.0f} s (watchdog)"}
            emit()
            os._exit(3)  # the line is out; a stuck exchange is still a failed run
        import threading
        wd = threading.Timer(limit, fire)
        wd.daemon = True
        wd.start()
        try:
            st = run_tiled(args, rank, world, local, barrier, dist, ("rubberwhale",), 1.0, "C2 strong scaling")
            te, tk = st["elapsed"], st["kernel_ms"]
            if dist is not None:
                t = torch.tensor([te, tk], device=dev, dtype=torch.float64)
                dist.all_reduce(t, op=dist.ReduceOp.MAX)
                te, tk = t.tolist()
            if out is not None:
                pp = st["per_pair"][0]
                out["strong_scaling"] = {
                    "value": st["pix_its"] / te / 1e9, "unit": "Gpixel-iter/s", "n_gpus": world,
                    "ms_per_step": te / args.steps * 1e3, "k_iter_us": tk / args.steps * 1e3,
                    "scaling": "strong", "split": st["split"], "parallelism": f"column-strip tiles x{world} (RCCL halo)",
                    "workload": f"rubberwhale {pp['size']} mixture L=1 K=9 its={args.steps}, one column strip per "
                                f"rank, Q={st['split']} lanes per node (from one strip)",
                    "aepe": None}
                spr = st.get("strip_parity")
                if spr:
                    out["strong_scaling"]["bit_exact"] = spr["bit_exact"]
                    out["strong_scaling"]["stop_iteration"] = spr.get("stop_iteration")
                    out["strong_scaling"]["strip_parity"] = spr
        except Exception as e:  # reported in the line; the frame-parallel value stands
            if out is not None:
                out["strong_scaling"] = {"error": f"{type(e).__name__}: {e}"[:300]}
    if rank == 0 and cfg == "c1" and not args.no_parity:
        try:
            par = parity_gate_c1(r, r["its"])
            out["parity"] = par
            for k in ("aepe_cpu_literal", "aepe_delta_literal"):
                out[k] = par[k]
            out["colour_mismatch"] = par["colour_mismatch_literal"]
        except Exception as e:
            out["parity"] = {"error": f"{type(e).__name__}: {e}"[:300]}
    if rank == 0 and cfg == "c3" and not args.no_parity:
        try:
            par = parity_gate_c3(r, args.precision, args.parity_steps or 12)
            out["parity"] = par
            for k in ("aepe_cpu_emul", "aepe_cpu_literal", "aepe_delta_emul", "aepe_delta_literal",
                      "flow_bit_exact_emul"):
                out[k] = par[k]
        except Exception as e:
            out["parity"] = {"error": f"{type(e).__name__}: {e}"[:300]}
    if rank == 0 and "map" in r and not args.no_parity:
        # the north-star parity gate on rank 0's own pair, after the timed region
        try:
            par = parity_gate(r, engine, r["gate_its"], args.precision, r["split"], r["seed"])
            out["parity"] = par
            for k in ("aepe_cpu_emul", "aepe_cpu_literal", "aepe_delta_emul", "aepe_delta_literal",
                      "aepe_spread_literal"):
                if k in par:
                    out[k] = par[k]
            if r.get("literal") is not None:
                le = {k: v for k, v in r["literal"].items() if k != "map"}
                le.update(par.get("literal_engine", {}))
                out["literal_engine"] = le
                par.pop("literal_engine", None)
            out["colour_mismatch"] = par["colour_mismatch_emul"]
            out["colour_mismatch_literal"] = par["colour_mismatch_literal"]
        except Exception as e:  # reported, never hides the measured line
            out["parity"] = {"error": f"{type(e).__name__}: {e}"[:300]}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        # the CPU baseline is a rank-0, N=1 figure (bench contract)
        if cfg == "c1":
            out["cpu_baseline"] = cpu_baseline_c1(r["flow"], r["opts"])
        else:
            lab = {"c2": "RubberWhale", "c3": "Grove3 full-resolution level", "c4": "Urban3",
                   "c5": "Urban3 x4"}[cfg]
            I1c, I2c, oc = r["I1"], r["I2"], r["opts"]
            if cfg == "c5":  # bounded sample: a 388x584 window of the upsampled frame
                I1c, I2c = (np.asfortranarray(a[600:988, 900:1484]) for a in (I1c, I2c))
            out["cpu_baseline"] = cpu_baseline(I1c, I2c, oc, engine if cfg != "c3" else "ctf", lab,
                                               split=r.get("split"), precision=args.precision)
    emit()
    if dist is not None:
        dist.destroy_process_group()
    # a tiled solve that is not bit-identical to the whole grid fails the run
    # (after the line is out)
    if out is not None:
        for rec in (out.get("strip_parity"), (out.get("strong_scaling") or {}).get("strip_parity")):
            if rec is not None and not rec["bit_exact"]:
                print("bench: column strips differ from the whole-grid solve", file=sys.stderr)
                sys.exit(4)


if __name__ == "__main__":
    main()
