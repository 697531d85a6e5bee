"""k_iter time vs grid size (tail / occupancy effects).  usage: size_sweep.py [fp64|fp32]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from gqmap_opticalflow_amd import Engine, flow_to_color, flowio, imresize  # noqa: E402

prec = sys.argv[1] if len(sys.argv) > 1 else "fp64"
I1, I2, gt = flowio.load_pair("rubberwhale")
I1b, I2b = np.round(imresize(I1, 3.0)), np.round(imresize(I2, 3.0))  # integer frames, 1164x1752
_, _, (minu, maxu, minv, maxv), _ = flow_to_color(gt)
o = dict(K=9, L=1, temperature=0.0, epsn=1e-6, lambdas=5.0, lambdad=1.0, minu=minu, maxu=maxu, minv=minv, maxv=maxv)
for (M, N) in [(256, 256), (384, 512), (388, 584), (400, 608), (512, 512), (512, 768), (768, 1024), (1024, 1536)]:
    a, b = np.asfortranarray(I1b[:M, :N]), np.asfortranarray(I2b[:M, :N])
    with Engine(o, a, b, "mixture", prec) as e:
        e.init_state(0)
        e.run_timed(5)
        done, tot, ker = e.run_timed(40)
        blocks = ((M + 15) // 16) * ((N + 15) // 16)
        us = ker / 40 * 1e3
        print(f"{M:5d}x{N:<5d} blocks {blocks:5d}  k_iter {us:8.1f} us  {M * N / us / 1e3:.3f} Gnode-it/s  "
              f"{us / blocks * 768:.1f} us per 768 blocks", flush=True)
