"""Wall per iteration of successive 20-iteration C2 fp64 runs (the driver's
window) from the same initial state, starting right after the bench's own
setup (5 warm-up iterations, graph capture), then again after 1 s idle:
separates the GPU's clock ramp from the kernel.  usage: clock_ramp.py"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from bench import gt_options  # noqa: E402
from gqmap_opticalflow_amd import Engine  # noqa: E402

I1, I2, flo, unk, o = gt_options("rubberwhale", 1, 9)
with Engine(o, I1, I2, "mixture", "fp64") as e:
    e.init_state(1)
    e.run_timed(5)
    e.prepare()
    for phase in ("after setup", "after 1 s idle", "after 1 s idle"):
        row = []
        for i in range(12):
            e.init_state(0)
            t0 = time.perf_counter()
            e.run(20)
            row.append((time.perf_counter() - t0) / 20 * 1e6)
        print(f"{phase:15s} us/it of successive run(20): " + " ".join(f"{x:6.1f}" for x in row), flush=True)
        time.sleep(1.0)
