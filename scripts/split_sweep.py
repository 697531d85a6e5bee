"""k_iter time vs lanes-per-node Q at several grid sizes.  usage: split_sweep.py [fp64|fp32] [mixture|super]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from gqmap_opticalflow_amd import Engine, flow_to_color, flowio, imresize  # noqa: E402

prec = sys.argv[1] if len(sys.argv) > 1 else "fp64"
eng = sys.argv[2] if len(sys.argv) > 2 else "mixture"
I1, I2, gt = flowio.load_pair("rubberwhale")
I1b, I2b = np.round(imresize(I1, 3.0)), np.round(imresize(I2, 3.0))
_, _, (minu, maxu, minv, maxv), _ = flow_to_color(gt)
K, L = (11, 3) if eng == "super" else (9, 1)
o = dict(K=K, L=L, temperature=0.2 if eng == "super" else 0.0, epsn=1e-6, lambdas=5.0, lambdad=1.0,
         minu=minu, maxu=maxu, minv=minv, maxv=maxv)
sizes = [(480, 640)] if eng == "super" else [(388, 584), (512, 768), (1024, 1536)]
for (M, N) in sizes:
    a, b = np.asfortranarray(I1b[:M, :N]), np.asfortranarray(I2b[:M, :N])
    res = []
    for q, xw in ((1, 0), (4, 0), (16, 0)):
        try:
            with Engine(dict(o, split=q), a, b, eng, prec) as e:
                if e.info().split != q:
                    continue
                e.init_state(0)
                e.run_timed(5)
                done, tot, ker = e.run_timed(40)
                res.append(f"Q={q}{'w' if xw else ''}: {ker / 40 * 1e3:7.1f} us")
        except Exception as ex:  # noqa: BLE001
            res.append(f"Q={q}: {ex}")
    print(f"{eng} {prec} {M}x{N}: " + "  ".join(res), flush=True)
