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
pixels of all ranks x steps / the slowest rank's time.

The other BASELINE configs are selectable (same JSON line, their workload
named in `config`):
    --config c3   Grove3 480x640, 5-level coarse-to-fine pyramid (gqmap_ctf
                  levels + device imresize/warp/fillmissing), steps = its/level
    --config c4   Urban3 480x640, gqmap_gpuSuper_mix_entropy L=3 K=11, 1000 its
    --config c5   RubberWhale upsampled 4x (1552x2336), column-strip tiles over
                  the ranks with RCCL ghost-column exchange (strong scaling)
    --config c1   Dimetrodon 388x584 legacy/gqmap_cpu.m flow denoising, 50 its
                  (device drop-in; timed call includes its host<->device copies)
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


def cpu_baseline(I1, I2, opts, engine="mixture", label="", budget_s: float = 12.0):
    """The oracle (literal C fp64 restatement, OpenMP) on this host's cores,
    on a bounded sample of the same workload."""
    from gqmap_opticalflow_amd import initial_state
    from oracle import oracle
    threads = min(16, os.cpu_count() or 1)
    Mo, No = I1.shape
    M, N = (Mo // 4, No // 4) if engine == "super" else (Mo, No)
    o = dict(opts, engine=engine)
    st0 = initial_state(o, M, N, seed=0, engine=engine)
    st = oracle.State(st0.muu, st0.muv, st0.sigu, st0.sigv, st0.pn, st0.rou, st0.w, st0.alpha)
    t0 = time.perf_counter()
    oracle.run(o, I1, I2, st, 1, 1, nthreads=threads)
    t1 = time.perf_counter() - t0
    n = max(1, min(200, int(budget_s / max(t1, 1e-3))))
    t0 = time.perf_counter()
    done, _, _ = oracle.run(o, I1, I2, st, 2, n, nthreads=threads)
    dt = time.perf_counter() - t0
    return {"value": Mo * No * done / dt / 1e9, "unit": "Gpixel-iter/s", "cores": threads, "kind": "port",
            "sample": f"oracle/gqmap_oracle.c fp64 ({engine}), {label} {No}x{Mo}, L={opts['L']} K={opts['K']}, "
                      f"iterations 2..{done + 1} from the seeded init, {threads} OpenMP threads, {dt:.1f}s"}


def traffic_per_launch(precision: str, config: str):
    tfile = os.path.join(ROOT, "profiles", f"traffic_{config}_{precision}.json")
    if os.path.exists(tfile):
        return json.load(open(tfile)).get("hbm_bytes_per_launch")
    return None


def roofline(engine, L, K, nodes, precision, kernel_avg_s, config, kernel_name):
    S = 8 if precision == "fp64" else 4
    fl = algorithmic_flops_per_node(engine, L, K) * nodes
    by = algorithmic_bytes_per_node(engine, L, S) * nodes
    ach = fl / kernel_avg_s / 1e12
    peak = PEAK_TFLOPS[precision]
    return {"bound": "valu", "achieved": ach, "peak": peak, "unit": "TFLOP/s", "frac": ach / peak,
            "traffic": traffic_per_launch(precision, config), "kernel": kernel_name,
            "kernel_avg_us": kernel_avg_s * 1e6, "flops_per_launch": fl,
            "algorithmic_bytes_per_launch": by, "hbm_algorithmic_GBps": by / kernel_avg_s / 1e9,
            "hbm_frac": by / kernel_avg_s / 1e9 / PEAK_HBM_GBPS}


# ---------------------------------------------------------------------------
def run_engine_config(args, rank, world, local, barrier, engine, names, L, K, extra, label):
    """C2 / C4: one solve per rank (frame-parallel), steps iterations timed."""
    from gqmap_opticalflow_amd import Engine, aepe
    name = names[rank % len(names)]
    I1, I2, flo, unk, opts = gt_options(name, L, K, **extra)
    eng = Engine(opts, I1, I2, engine, args.precision, device=local)
    eng.init_state(seed=1 + rank)
    if args.warmup:
        eng.run_timed(args.warmup)
    eng.init_state(seed=rank)  # timed steps are iterations 1..steps of the solve
    barrier()
    t0 = time.perf_counter()
    done, total_ms, kernel_ms = eng.run_timed(args.steps)
    barrier()
    elapsed = time.perf_counter() - t0
    if done != args.steps:
        raise RuntimeError(f"rank {rank}: solver stopped after {done}/{args.steps} iterations")
    mp = eng.map()
    if engine == "super":
        flow = np.repeat(np.repeat(mp, 4, axis=0), 4, axis=1)
        a = aepe(flo, flow, unk, 4)
    else:
        a = aepe(flo, mp, unk)
    nodes = eng.M * eng.N
    eng.close()
    Mo, No = I1.shape
    ksuf = {"mixture": 0, "super": 1}[engine]
    R = "double" if args.precision == "fp64" else "float"
    return dict(elapsed=elapsed, kernel_ms=kernel_ms, pixels=Mo * No, nodes=nodes, aepe=a, name=name,
                I1=I1, I2=I2, opts=opts, Mo=Mo, No=No,
                kernel=f"gq::k_iter<{R},float,{ksuf},Q> (VV stored as float: integer frames)",
                workload=f"{label}: {name} {No}x{Mo} {engine} L={L} K={K} its={args.steps} "
                         f"(one step = one full-frame iteration)")


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
    p.close()
    Mo, No = I1.shape
    return dict(elapsed=elapsed, pix_its=px, aepe=a, name=name, I1=I1, I2=I2, opts=dict(opts, engine="ctf"),
                Mo=Mo, No=No, its=its,
                workload=f"C3: {name} {No}x{Mo} coarse-to-fine, 5 levels 1/16..1 (30x40..480x640), "
                         f"gqmap_ctf K=11, {args.steps} its/level, device imresize/interp2/fillmissing; "
                         f"value counts sum over levels of level pixels x its")


def run_c1(args, rank, world, local, barrier):
    """legacy/gqmap_cpu.m on the GT flow of a 584x388 pair (unknowns zeroed)."""
    from gqmap_opticalflow_amd import flow_to_color, flowio, gqmap_cpu
    name = PAIRS[(rank + 1) % len(PAIRS)] if world > 1 else "Dimetrodon"
    gt = flowio.load_pair(name)[2]
    _, flo, _, unk = flow_to_color(gt, device=local)
    o = dict(its=args.steps, K=9)
    if args.warmup:
        gqmap_cpu(dict(o, its=min(args.warmup, 5)), flo, seed=1, device=local)
    barrier()
    t0 = time.perf_counter()
    mu, sg, rou, tr = gqmap_cpu(o, flo, seed=0, device=local, return_trace=True)
    barrier()
    elapsed = time.perf_counter() - t0
    M, N, _ = flo.shape
    err = float(np.sqrt(((mu - flo) ** 2).sum(axis=2))[~unk].mean())
    return dict(elapsed=elapsed, pixels=M * N, nodes=M * N, aepe=err, flow=flo, opts=o, Mo=M, No=N, its=tr.shape[0],
                workload=f"C1: {name} {N}x{M} legacy/gqmap_cpu.m flow denoising (input = GT flow, unknowns 0), "
                         f"K=9, var=gama=1, dta=inf, {args.steps} its, sigma0 = U+2 (seed 0); value includes the "
                         f"call's host<->device copies; aepe = mean |mu - flow|")


def cpu_baseline_c1(flow, opts):
    """The C restatement of legacy/gqmap_cpu.m (single thread, as the MATLAB
    parfor would run on one worker), bounded sample."""
    from gqmap_opticalflow_amd import gauss_hermite
    from oracle import oracle
    M, N, _ = flow.shape
    X, W = gauss_hermite(9)
    sg0 = np.asfortranarray(np.full((M, N, 2), 2.5))
    t0 = time.perf_counter()
    oracle.cpu_run(dict(opts, its=1), flow, sg0, X, W)
    t1 = time.perf_counter() - t0
    n = max(1, min(opts["its"], int(10.0 / max(t1, 1e-3))))
    t0 = time.perf_counter()
    _, _, _, tr = oracle.cpu_run(dict(opts, its=n), flow, sg0, X, W)
    dt = time.perf_counter() - t0
    return {"value": M * N * tr.shape[0] / dt / 1e9, "unit": "Gpixel-iter/s", "cores": 1, "kind": "port",
            "sample": f"oracle/gqmap_legacy_oracle.c fp64, {N}x{M}, K=9, {tr.shape[0]} iterations, 1 thread, {dt:.1f}s"}


def run_c5(args, rank, world, local, barrier, dist):
    """RubberWhale bicubic-upsampled 4x (frames with the device imresize, GT
    x4 in size and value), column-strip tiles over the ranks."""
    from gqmap_opticalflow_amd import Engine, aepe, comm_unique_id, flow_to_color, flowio, imresize
    I1s, I2s, gt = flowio.load_pair("rubberwhale")
    # imresize of the uint8 frames as the drivers do (imresize(imread(..),scale),
    # optical_flowSuper.m:8-9): round half away from zero and saturate to uint8
    u8 = lambda a: np.asfortranarray(np.clip(np.sign(a) * np.floor(np.abs(a) + 0.5), 0, 255))
    I1, I2 = u8(imresize(I1s, 4.0, device=local)), u8(imresize(I2s, 4.0, device=local))
    # GT x4 in value (unknown entries stay > 1e9) and in size (nearest)
    gt4 = np.asfortranarray(np.repeat(np.repeat(gt * 4.0, 4, axis=0), 4, axis=1))
    _, flo, (minu, maxu, minv, maxv), unk = flow_to_color(gt4, device=local)
    opts = dict(its=args.steps, K=9, L=1, temperature=0.0, drate=0.5, epsn=1e-6, lambdas=5.0, lambdad=1.0,
                minu=minu, maxu=maxu, minv=minv, maxv=maxv)
    eng = Engine(opts, I1, I2, "mixture", args.precision, device=local, n_tiles=world, tile=rank)
    if world > 1:
        uid = [comm_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        eng.attach_rccl(uid[0])
    eng.init_state(seed=1)
    if args.warmup:
        eng.run(args.warmup)
    eng.init_state(seed=0)
    barrier()
    t0 = time.perf_counter()
    done, total_ms, kernel_ms = eng.run_timed(args.steps)
    barrier()
    elapsed = time.perf_counter() - t0
    mp = eng.map()
    col0, col1 = eng.col0, eng.col1
    eng.close()
    Mo, No = I1.shape
    # AEPE over this rank's strip (interior), combined on rank 0 as a pixel-weighted mean
    sl = (slice(1, Mo - 1), slice(max(col0, 1), min(col1, No - 1)))
    f = mp.copy()
    f[unk] = 0
    e = np.sqrt(((flo[sl] - f[sl]) ** 2).sum(axis=2))
    return dict(elapsed=elapsed, kernel_ms=kernel_ms, pixels=Mo * No, nodes=Mo * (col1 - col0),
                err_sum=float(e.sum()), err_n=int(e.size), Mo=Mo, No=No, I1=I1, I2=I2, opts=opts,
                workload=f"C5: RubberWhale upsampled 4x ({No}x{Mo}, bicubic imresize, uint8-rounded as "
                         f"imresize(imread(..)) gives), mixture L=1 K=9, "
                         f"{world} column-strip tile(s), RCCL ghost-column + totals exchange per iteration, "
                         f"its={args.steps}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=None)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--precision", default="fp64", choices=("fp64", "fp32"))
    ap.add_argument("--config", default="c2", choices=("c1", "c2", "c3", "c4", "c5"))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()
    if args.steps is None:
        args.steps = DEFAULT_STEPS[args.config]

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
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
    if cfg == "c2":
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
    else:
        r = run_c5(args, rank, world, local, barrier, dist)
        engine, L, K = "mixture", 1, 9

    elapsed = r["elapsed"]
    kernel_ms = r.get("kernel_ms", 0.0)
    if dist is not None:
        dev = "cuda" if backend == "nccl" else "cpu"
        t = torch.tensor([elapsed, kernel_ms], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, kernel_ms = t.tolist()
        if cfg == "c5":
            s = torch.tensor([r["err_sum"], r["err_n"]], device=dev, dtype=torch.float64)
            dist.all_reduce(s)
            r["aepe"] = s[0].item() / s[1].item()
    elif cfg == "c5":
        r["aepe"] = r["err_sum"] / r["err_n"]

    if rank == 0:
        if cfg == "c3":
            units = r["pix_its"] * world
            parallel = f"frame-parallel x{world}"
        elif cfg == "c1":
            units = world * r["pixels"] * r["its"]
            parallel = f"frame-parallel x{world}"
        elif cfg == "c5":
            units = r["pixels"] * args.steps
            parallel = f"column-strip tiles x{world} (RCCL halo)"
        else:
            units = world * r["pixels"] * args.steps
            parallel = f"frame-parallel x{world}"
        out = {
            "metric": METRIC, "value": units / elapsed / 1e9, "unit": "Gpixel-iter/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True, "scaling": "strong" if cfg == "c5" else "weak", "vs_baseline": None,
            "dtype": "f64" if args.precision == "fp64" else "f32",
            "data": "Middlebury frame10/11 + flow10.flo (real frames, in-repo data/middlebury)"
                    + ("; upsampled 4x on the device" if cfg == "c5" else ""),
            "config": {"workload": r["workload"], "engine": engine, "L": L, "K": K, "parallelism": parallel},
            "aepe": r["aepe"], "aepe_its": args.steps,
        }
        if cfg == "c1":
            # per pixel: node 2 x K x 6 flop, edges 4 x K^2 x ~40 flop (legacy/gqmap_cpu.m:20-54)
            fl = (2 * K * 6 + 4 * K * K * 40) * r["pixels"] * r["its"]
            out["roofline"] = {"bound": "valu", "achieved": fl / elapsed / 1e12, "peak": PEAK_TFLOPS["fp64"],
                               "unit": "TFLOP/s", "frac": fl / elapsed / 1e12 / PEAK_TFLOPS["fp64"], "traffic": None,
                               "kernel": "gq::k_legacy_grad + k_legacy_update (timed by the call's wall clock)"}
        elif cfg == "c3":
            secs = elapsed
            Sb = 8 if args.precision == "fp64" else 4
            fl = algorithmic_flops_per_node("ctf", 1, K) * r["pix_its"]
            out["roofline"] = {"bound": "valu", "achieved": fl / secs / 1e12, "peak": PEAK_TFLOPS[args.precision],
                               "unit": "TFLOP/s", "frac": fl / secs / 1e12 / PEAK_TFLOPS[args.precision],
                               "traffic": traffic_per_launch(args.precision, cfg),
                               "kernel": "gq::k_iter<R,VT,2,Q> (all levels; timed by the pipeline wall clock)",
                               "algorithmic_bytes_per_node_iter": algorithmic_bytes_per_node("ctf", 1, Sb)}
            out["config"]["its_per_level"] = r["its"]
        else:
            kern_avg_s = kernel_ms / args.steps / 1e3
            nodes = r["nodes"]
            out["roofline"] = roofline(engine, L, K, nodes, args.precision, kern_avg_s, cfg,
                                       r.get("kernel", "gq::k_iter"))
        if not args.no_cpu_baseline and cfg == "c1":
            out["cpu_baseline"] = cpu_baseline_c1(r["flow"], r["opts"])
        elif not args.no_cpu_baseline:
            lab = {"c2": "RubberWhale", "c3": "Grove3 full-resolution level", "c4": "Urban3",
                   "c5": "RubberWhale x4"}[cfg]
            I1c, I2c, oc = r["I1"], r["I2"], r["opts"]
            if cfg == "c5":  # bounded sample: a 388x584 window of the upsampled frame
                I1c, I2c = (np.asfortranarray(a[600:988, 900:1484]) for a in (I1c, I2c))
            out["cpu_baseline"] = cpu_baseline(I1c, I2c, oc, engine, lab)
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
