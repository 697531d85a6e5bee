"""k_iter us/it of one large frame (C5 unit: a Middlebury pair upsampled 4x)
and C2, for the tile order the environment selects (GQMAP_TILE_STRIP).
usage: python scripts/order_ab.py [pair] [scale] [its]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from gqmap_opticalflow_amd import Engine, flow_to_color, flowio  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "rubberwhale"
scale = float(sys.argv[2]) if len(sys.argv) > 2 else 4.0
its = int(sys.argv[3]) if len(sys.argv) > 3 else 20
I1, I2, gt = flowio.load_pair_scaled(name, scale)
_, flo, (minu, maxu, minv, maxv), unk = flow_to_color(gt)
o = dict(K=9, L=1, temperature=0.0, drate=0.5, epsn=1e-6, lambdad=1.0, lambdas=5.0,
         minu=minu, maxu=maxu, minv=minv, maxv=maxv)
with Engine(o, I1, I2) as e:
    e.init_state(0)
    e.run_timed(3)
    out = []
    for start in (3, 100):
        if start > 3 + its:
            e.run(start - 3 - its)
        done, tot, ker = e.run_timed(its)
        out.append(f"{ker / done * 1e3:8.1f}")
    chk = float(np.sum(e.get_state().muu))
print(f"strip={os.environ.get('GQMAP_TILE_STRIP', '-')} {name} x{scale:g} {I1.shape} k_iter us/it "
      + " | ".join(out) + f" chk={chk!r}", flush=True)
