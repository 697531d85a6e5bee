"""Headline benchmark (BASELINE.json): Gpixel-iterations/s + AEPE vs the .flo
ground truth on the Middlebury 584x388 pair, 1/2/4/8 GPUs.

Workload (BASELINE config C2): RubberWhale 388x584, gqmap_gpu_mixture
(single-scale mixture QGMAP), L=1, K=9, 500 iterations, lambda_s=5,
lambda_d=1, eps=1e-6, T=0 (optical_flow.m:16-23 with L=1).  One "step" is one
iteration of the hot path over the whole frame (gqmap_gpu_mixture.m:27-75);
frames and state are resident in HBM before the timed region.

    python bench.py [--steps 500] [--warmup 20] [--precision fp64|fp32]
    python -m torch.distributed.run --nproc-per-node N bench.py --gpus N

Multi-GPU is frame-parallel (weak scaling): every rank solves its own
584x388 pair on its own GPU, no data-path collective; `value` is the pixels
of all ranks x steps / the slowest rank's time.  Rank 0 prints one JSON line.
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
PEAK_TFLOPS = {"fp64": 78.6, "fp32": 157.3}   # MI355X vector peaks (MI355X_MICROARCH.md)
PEAK_HBM_GBPS = 8000.0
PAIRS = ("rubberwhale", "Dimetrodon", "Hydrangea")  # the 584x388 Middlebury pairs


def algorithmic_flops_per_pixel(L: int, K: int) -> int:
    # F_pix = L*K^2*(128 + 4*41) for the single-scale engine
    return 292 * L * K * K


def algorithmic_bytes_per_pixel(L: int, S: int) -> int:
    # state (9 values/component) read + write, I1 and I2 once
    return (18 * L + 2) * S


def setup_problem(name: str, L: int, K: int):
    from gqmap_opticalflow_amd import flow_to_color, flowio
    I1, I2, gt = flowio.load_pair(name)
    _, flo, (minu, maxu, minv, maxv), unk = flow_to_color(gt)
    opts = dict(trueFlow=flo, unknownIdx=unk, its=500, K=K, L=L, temperature=0.0, drate=0.5,
                epsn=0.001 ** 2, lambdas=5.0, lambdad=1.0, minu=minu, maxu=maxu, minv=minv, maxv=maxv)
    return I1, I2, flo, unk, opts


def cpu_baseline(I1, I2, opts, budget_s: float = 12.0):
    """The oracle (C fp64 restatement, OpenMP) on this host: bounded sample."""
    from gqmap_opticalflow_amd import initial_state
    from oracle import oracle
    threads = min(16, os.cpu_count() or 1)
    M, N = I1.shape
    st0 = initial_state(opts, M, N, seed=0)
    st = oracle.State(st0.muu, st0.muv, st0.sigu, st0.sigv, st0.pn, st0.rou, st0.w, st0.alpha)
    t0 = time.perf_counter()
    oracle.run(opts, I1, I2, st, 1, 1, nthreads=threads)
    t1 = time.perf_counter() - t0
    n = max(1, min(200, int(budget_s / max(t1, 1e-3))))
    t0 = time.perf_counter()
    done, _, _ = oracle.run(opts, I1, I2, st, 2, n, nthreads=threads)
    dt = time.perf_counter() - t0
    return {"value": M * N * done / dt / 1e9, "unit": "Gpixel-iter/s", "cores": threads,
            "kind": "port",
            "sample": f"oracle/gqmap_oracle.c fp64, RubberWhale {N}x{M}, L={opts['L']} K={opts['K']}, "
                      f"iterations 2..{done + 1} from the seeded init, {threads} OpenMP threads, {dt:.1f}s"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=500)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--precision", default="fp64", choices=("fp64", "fp32"))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)

    def barrier():
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()

    from gqmap_opticalflow_amd import Engine, aepe
    L, K = 1, 9
    pair = PAIRS[rank % len(PAIRS)] if world > 1 else PAIRS[0]
    I1, I2, flo, unk, opts = setup_problem(pair, L, K)
    M, N = I1.shape
    eng = Engine(opts, I1, I2, "mixture", args.precision, device=local if world > 1 else 0)
    # warmup on a throw-away state, then re-initialise so the timed steps are
    # iterations 1..steps of the C2 solve
    eng.init_state(seed=1 + rank)
    if args.warmup:
        eng.run_timed(args.warmup)
    eng.init_state(seed=rank)

    barrier()
    t0 = time.perf_counter()
    done, total_ms, kernel_ms = eng.run_timed(args.steps)
    barrier()
    elapsed = time.perf_counter() - t0
    if done != args.steps:
        raise RuntimeError(f"rank {rank}: solver stopped after {done}/{args.steps} iterations")

    if dist is not None:
        t = torch.tensor([elapsed, kernel_ms], device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, kernel_ms_max = t.tolist()
    a = aepe(flo, eng.map(), unk)
    eng.close()

    if rank == 0:
        px = M * N
        value = world * px * args.steps / elapsed / 1e9
        kern_avg_s = kernel_ms / args.steps / 1e3
        S = 8 if args.precision == "fp64" else 4
        fl = algorithmic_flops_per_pixel(L, K) * px
        by = algorithmic_bytes_per_pixel(L, S) * px
        ach = fl / kern_avg_s / 1e12
        peak = PEAK_TFLOPS[args.precision]
        traffic = None
        tfile = os.path.join(ROOT, "profiles", f"traffic_{args.precision}.json")
        if os.path.exists(tfile):
            traffic = json.load(open(tfile)).get("hbm_bytes_per_launch")
        out = {
            "metric": METRIC, "value": value, "unit": "Gpixel-iter/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "f64" if args.precision == "fp64" else "f32",
            "data": "Middlebury RubberWhale frame10/11 + flow10.flo (real frames, in-repo data/)",
            "config": {"workload": f"C2: RubberWhale {N}x{M} gqmap_gpu_mixture L={L} K={K} "
                                   f"its={args.steps} (one step = one full-frame iteration)",
                       "engine": "mixture", "L": L, "K": K, "pixels_per_gpu": px,
                       "parallelism": f"frame-parallel x{world}"},
            "aepe": a, "aepe_its": args.steps,
            "roofline": {"bound": "valu", "achieved": ach, "peak": peak, "unit": "TFLOP/s",
                         "frac": ach / peak, "traffic": traffic,
                         "kernel": "gq::k_iter<%s,false>" % ("double" if S == 8 else "float"),
                         "kernel_avg_us": kern_avg_s * 1e6, "flops_per_launch": fl,
                         "algorithmic_bytes_per_launch": by,
                         "hbm_algorithmic_GBps": by / kern_avg_s / 1e9,
                         "hbm_frac": by / kern_avg_s / 1e9 / PEAK_HBM_GBPS},
        }
        if not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(I1, I2, opts)
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
