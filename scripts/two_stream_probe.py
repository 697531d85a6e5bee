"""Does a second, independent C2 solve on its own stream fill the first one's
idle CU time inside ONE process?  Two Engine contexts (each its own
non-blocking stream), run(n) called from two threads at once (ctypes drops
the GIL), against the same contexts run one after the other.
usage: two_stream_probe.py"""
import os
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from bench import gt_options, settle_clocks  # noqa: E402
from gqmap_opticalflow_amd import Engine  # noqa: E402

I1, I2, flo, unk, o = gt_options("rubberwhale", 1, 9)
n = 100
engs = [Engine(o, I1, I2, "mixture", "fp64") for _ in range(2)]
for e in engs:
    e.init_state(1)
    e.run(5)
    e.prepare()


def chunk():
    for e in engs:
        e.init_state(0)
        e.run(20)


settle_clocks(chunk, 40)
px = I1.size
for rep in range(3):
    for e in engs:
        e.init_state(0)
    t0 = time.perf_counter()
    for e in engs:
        e.run(n)
    seq = time.perf_counter() - t0
    for e in engs:
        e.init_state(0)
    ths = [threading.Thread(target=e.run, args=(n,)) for e in engs]
    t0 = time.perf_counter()
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    par = time.perf_counter() - t0
    print(f"rep {rep}: sequential {2 * px * n / seq / 1e9:.3f} Gpix-it/s ({seq / n * 1e6 / 2:.1f} us per frame-iteration), "
          f"concurrent {2 * px * n / par / 1e9:.3f} ({par / n * 1e6 / 2:.1f})", flush=True)
for e in engs:
    e.close()
