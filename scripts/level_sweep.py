"""k_iter time per iteration on each C3 pyramid level (Grove3 resized, ctf
engine K=11) for lanes-per-node Q = 1, 2, 4, 16, 64 (QS=... to choose).  usage: level_sweep.py [fp64|fp32]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from bench import gt_options  # noqa: E402
from gqmap_opticalflow_amd import C3_SCALES, Engine, ctf_options, imresize  # noqa: E402

prec = sys.argv[1] if len(sys.argv) > 1 else "fp64"
I1, I2, flo, unk, o = gt_options("Grove3", 1, 11)
for s in C3_SCALES:
    a, b = (np.asfortranarray(imresize(x, s)) for x in (I1, I2))
    res = []
    for q in [int(x) for x in os.environ.get("QS", "1,2,4,16,64").split(",")]:
        opts = ctf_options(its=500, minu=o["minu"], maxu=o["maxu"], minv=o["minv"], maxv=o["maxv"], split=q)
        with Engine(opts, a, b, "ctf", prec) as e:
            e.init_state(0)
            e.run_timed(10)
            done, tot, ker = e.run_timed(100)
            res.append(f"Q={e.info().split:2d} {ker / done * 1e3:7.1f}")
    print(f"scale {s:6.4f} {a.shape[0]:4d}x{a.shape[1]:<4d} k_iter us/it: " + "  ".join(res), flush=True)
