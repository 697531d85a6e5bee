"""Fixed vs per-iteration wall time of gqmap_run on C2 fp64: median wall of
run(n) from the same initial state for several n (after prepare), against the
instrumented kernel mean.  usage: run_overhead.py"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from bench import gt_options  # noqa: E402
from gqmap_opticalflow_amd import Engine  # noqa: E402

I1, I2, flo, unk, o = gt_options("rubberwhale", 1, 9)
with Engine(o, I1, I2, "mixture", "fp64") as e:
    e.init_state(1)
    e.run_timed(5)
    e.prepare()
    for n in (1, 2, 4, 8, 16, 20, 32, 40, 50, 100):
        ts = []
        for r in range(7):
            e.init_state(0)
            e.synchronize()
            t0 = time.perf_counter()
            d, _ = e.run(n)
            ts.append(time.perf_counter() - t0)
        e.init_state(0)
        d2, tot, ker = e.run_timed(n)
        print(f"n={n:4d} wall median {np.median(ts) * 1e6:9.1f} us  min {min(ts) * 1e6:9.1f}  "
              f"per-it {np.median(ts) / n * 1e6:7.1f}  kernel mean {ker / d2 * 1e3:7.1f} us", flush=True)
