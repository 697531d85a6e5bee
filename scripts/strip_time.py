"""Per-iteration time of one rank's share of the strong-scaling layout on one
GPU: a 388 x (584/n) column strip of RubberWhale (+ the ghost columns'
width) at the per-strip lanes per node, (a) as a plain fused context and
(b) behind a one-rank RCCL communicator (the boundary / interior launches,
k_reduce_local, all-gather of totals, finalize -- everything of a tiled
iteration except the cross-GPU transfer).  usage: strip_time.py [n] [its]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from gqmap_opticalflow_amd import Engine, comm_unique_id, flow_to_color, flowio, strip_split  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 8
its = int(sys.argv[2]) if len(sys.argv) > 2 else 200
I1, I2, gt = flowio.load_pair("rubberwhale")
Mo, No = I1.shape
w = -(-No // n) + (2 if n > 1 else 0)
I1, I2, gt = (np.asfortranarray(a[:, :w]) for a in (I1, I2, gt))
_, _, (minu, maxu, minv, maxv), _ = flow_to_color(gt)
q = strip_split(Mo, No, n)
o = dict(K=9, L=1, temperature=0.0, drate=0.5, epsn=1e-6, lambdad=1.0, lambdas=5.0, minu=minu, maxu=maxu,
         minv=minv, maxv=maxv, split=q)
for mode in ("fused", "rccl1"):
    with Engine(o, I1, I2, n_tiles=1, tile=0) as e:
        if mode == "rccl1":
            e.attach_rccl(comm_unique_id())
        e.init_state(0)
        e.run(20)
        e.prepare()
        e.init_state(0)
        t0 = time.perf_counter()
        done, _ = e.run(its)
        e.synchronize()
        dt = (time.perf_counter() - t0) / done * 1e6
        e.init_state(0)
        d2, tot, ker = e.run_timed(its)
    print(f"n={n} strip {Mo}x{w} Q={q} {mode}: {dt:7.1f} us/it (graph), k_iter {ker / d2 * 1e3:7.1f} us/it", flush=True)
