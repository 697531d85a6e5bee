"""Profiling driver for one small grid (no torch): C3's middle pyramid levels
(Grove3 full size or resized, ctf K=11, the library's default lanes per node) or one
rank's share of the 8-way strong-scaling layout (RubberWhale 388 x 75,
mixture K=9, Q=4, as a plain fused context).  Runs `its` iterations as
replayed graphs after a warm-up.  usage: level_prof.py l480|l240|l120|l60|l30|strip2|strip4|strip8 [its] [fp64|fp32]
(GQMAP_SPLIT=q forces the lanes per node)"""
import hashlib
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import _policy  # noqa: E402

_policy.apply()
import numpy as np  # noqa: E402

from bench import gt_options  # noqa: E402
from gqmap_opticalflow_amd import Engine, ctf_options, imresize, strip_split  # noqa: E402

case = sys.argv[1] if len(sys.argv) > 1 else "l240"
its = int(sys.argv[2]) if len(sys.argv) > 2 else 50
prec = sys.argv[3] if len(sys.argv) > 3 else "fp64"
if case in ("l480", "l240", "l120", "l60", "l30"):
    I1, I2, flo, unk, o = gt_options("Grove3", 1, 11)
    s = {"l480": 1.0, "l240": 0.5, "l120": 0.25, "l60": 0.125, "l30": 0.0625}[case]
    a, b = (np.asfortranarray(imresize(x, s) if s != 1 else x) for x in (I1, I2))
    opts = ctf_options(its=500, minu=o["minu"], maxu=o["maxu"], minv=o["minv"], maxv=o["maxv"])
    if os.environ.get("GQMAP_SPLIT"):
        opts["split"] = int(os.environ["GQMAP_SPLIT"])
    eng = Engine(opts, a, b, "ctf", prec)
else:  # stripN: one rank's column strip of the N-way layout (+2 ghost columns)
    nt = int(case[5:] or 8)
    I1, I2, flo, unk, o = gt_options("rubberwhale", 1, 9)
    w = -(-I1.shape[1] // nt) + 2
    a, b = (np.asfortranarray(x[:, :w]) for x in (I1, I2))
    q = int(os.environ.get("GQMAP_SPLIT") or strip_split(I1.shape[0], I1.shape[1], nt))
    eng = Engine(dict(o, split=q), a, b, "mixture", prec)
with eng:
    eng.init_state(0)
    eng.run(100)
    eng.init_state(0)
    done, tot, ker = eng.run_timed(its)
    eng.init_state(0)
    eng.run(its)  # the production path (graph replay; persistent on the smallest levels), first run builds it
    eng.init_state(0)
    t0 = time.perf_counter()
    eng.run(its)
    eng.synchronize()
    wall = (time.perf_counter() - t0) / its * 1e6
    chk = hashlib.sha1(np.ascontiguousarray(eng.map()).tobytes()).hexdigest()[:12]  # same bits across variants
    print(f"{case} {a.shape[0]}x{a.shape[1]} {prec} Q={eng.info().split}: k_iter {ker / done * 1e3:.1f} us/it "
          f"run {wall:.1f} us/it "
          f"chk={chk}")
