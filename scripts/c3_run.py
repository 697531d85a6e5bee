"""C3 (Grove3 480x640, 5-level coarse-to-fine) timing + AEPE on the device.
usage: python scripts/c3_run.py [its_per_level] [precision] [reps]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from gqmap_opticalflow_amd import C3_SCALES, Pyramid, aepe, ctf_options, flow_to_color, flowio  # noqa: E402

its = int(sys.argv[1]) if len(sys.argv) > 1 else 500
prec = sys.argv[2] if len(sys.argv) > 2 else "fp64"
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 2
I1, I2, gt = flowio.load_pair("Grove3")
_, flo, (minu, maxu, minv, maxv), unk = flow_to_color(gt)
opts = ctf_options(its=its, minu=minu, maxu=maxu, minv=minv, maxv=maxv)
with Pyramid(opts, C3_SCALES, prec) as p:
    p.set_images(I1, I2)
    for r in range(reps):
        flow, done, ms = p.run(seed=r)
        px = sum(p.level(l)["I2"].size * done[l] for l in range(len(C3_SCALES)))
        print(f"rep {r}: its/level {done}  {ms:.1f} ms  {px / ms / 1e6:.4f} Gpix-it/s  "
              f"AEPE {aepe(flo, flow, unk):.4f}", flush=True)
