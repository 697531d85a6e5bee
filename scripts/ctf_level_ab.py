"""C3 pyramid levels at the library's own lanes-per-node policy, for A/B of
libgqmap variants (GQMAP_LIB): k_iter us/it (HIP events, 100 its after 10)
and a checksum of the final state.  usage: ctf_level_ab.py [fp64|fp32] [scales]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import _policy  # noqa: E402  (GQMAP_POLICY="flow=1", ...)

_policy.apply()
import numpy as np  # noqa: E402

from bench import gt_options  # noqa: E402
from gqmap_opticalflow_amd import C3_SCALES, Engine, ctf_options, imresize  # noqa: E402

prec = sys.argv[1] if len(sys.argv) > 1 else "fp64"
scales = [float(x) for x in sys.argv[2].split(",")] if len(sys.argv) > 2 else C3_SCALES
I1, I2, flo, unk, o = gt_options("Grove3", 1, 11)
for s in scales:
    a, b = (np.asfortranarray(imresize(x, s)) for x in (I1, I2))
    opts = ctf_options(its=500, minu=o["minu"], maxu=o["maxu"], minv=o["minv"], maxv=o["maxv"])
    with Engine(opts, a, b, "ctf", prec) as e:
        e.init_state(0)
        e.run_timed(10)
        done, tot, ker = e.run_timed(100)
        chk = float(np.sum(e.get_state().muu))
        e.init_state(0)
        e.run(10)
        e.prepare()
        t0 = time.perf_counter()
        n, _ = e.run(100)  # production path: replayed graphs, wall clock per iteration
        e.synchronize()
        wall = (time.perf_counter() - t0) / n * 1e6
        print(f"scale {s:6.4f} {a.shape[0]:4d}x{a.shape[1]:<4d} Q={e.info().split:2d} "
              f"k_iter {ker / done * 1e3:7.1f} us/it wall {wall:7.1f} us/it chk={chk!r}", flush=True)
