"""Wall clock per iteration of the C3 small pyramid levels on the production
path (prepared graph, 100 iterations after 10), for A/B of libgqmap builds
(GQMAP_LIB) and GQMAP_NO_PERSIST.  Timing only: the variants built with the
GQ_PERSIST_* experiment switches do not produce valid results.
usage: [SPLIT=q] persist_ab.py [fp64|fp32] [scales]  (SPLIT=-1: role split)"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from bench import gt_options  # noqa: E402
from gqmap_opticalflow_amd import Engine, ctf_options, imresize  # noqa: E402

prec = sys.argv[1] if len(sys.argv) > 1 else "fp64"
scales = [float(x) for x in sys.argv[2].split(",")] if len(sys.argv) > 2 else [0.0625, 0.125, 0.25]
lab = os.path.basename(os.environ.get("GQMAP_LIB", "libgqmap.so")) + (" no-persist" if os.environ.get("GQMAP_NO_PERSIST") else "") \
    + (" split=" + os.environ["SPLIT"] if os.environ.get("SPLIT") else "")
I1, I2, flo, unk, o = gt_options("Grove3", 1, 11)
for s in scales:
    a, b = (np.asfortranarray(imresize(x, s)) for x in (I1, I2))
    opts = ctf_options(its=500, minu=o["minu"], maxu=o["maxu"], minv=o["minv"], maxv=o["maxv"],
                       split=int(os.environ.get("SPLIT", "0")))
    with Engine(opts, a, b, "ctf", prec) as e:
        best = 1e9
        for rep in range(3):
            e.init_state(0)
            e.run(10)
            e.prepare()
            e.synchronize()
            t0 = time.perf_counter()
            e.run(100)
            e.synchronize()
            best = min(best, (time.perf_counter() - t0) / 100 * 1e6)
        print(f"{lab:28s} {a.shape[0]:4d}x{a.shape[1]:<4d} Q={e.info().split:2d} wall {best:7.1f} us/it", flush=True)
