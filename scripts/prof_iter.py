"""Profiling driver: C2 (RubberWhale 388x584, mixture, L=1, K=9) iterations,
no torch.  Usage: python scripts/prof_iter.py [its] [fp64|fp32] [mixture|super]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import _policy  # noqa: E402

_policy.apply()
from bench import setup_problem  # noqa: E402
from gqmap_opticalflow_amd import Engine  # noqa: E402

its = int(sys.argv[1]) if len(sys.argv) > 1 else 20
prec = sys.argv[2] if len(sys.argv) > 2 else "fp64"
engine = sys.argv[3] if len(sys.argv) > 3 else "mixture"
if engine == "super":
    I1, I2, flo, unk, o = setup_problem("Urban3", 3, 11)
    o.update(temperature=0.2, drate=0.75, lambdas=16.0)
elif os.environ.get("GQMAP_SCALE"):  # a C5 frame: RubberWhale upsampled (optical_flow_temp.m:7-8)
    from gqmap_opticalflow_amd import flow_to_color, flowio
    I1, I2, gt = flowio.load_pair_scaled("rubberwhale", float(os.environ["GQMAP_SCALE"]))
    _, flo, (minu, maxu, minv, maxv), unk = flow_to_color(gt)
    o = dict(K=9, L=1, temperature=0.0, drate=0.5, epsn=1e-6, lambdas=5.0, lambdad=1.0,
             minu=minu, maxu=maxu, minv=minv, maxv=maxv)
else:
    I1, I2, flo, unk, o = setup_problem("rubberwhale", 1, 9)
if os.environ.get("GQMAP_SPLIT"):
    o["split"] = int(os.environ["GQMAP_SPLIT"])
if os.environ.get("GQMAP_ARITH"):  # "literal": the literal-order engine
    o["arith"] = os.environ["GQMAP_ARITH"]
with Engine(o, I1, I2, engine, prec) as eng:
    eng.init_state(0)
    done, tot, ker = eng.run_timed(its)
    eng.init_state(0)  # same iterations as the timed pass; first run builds the graph
    t = time.perf_counter()
    eng.run(its)
    dt0 = time.perf_counter() - t
    eng.init_state(0)
    t = time.perf_counter()
    _, tr = eng.run(its)
    eng.synchronize()
    dt = time.perf_counter() - t
    chk = f"{tr[-1, 0]:.17g}"
print(f"{engine} {prec}: {done} its, events total {tot:.3f} ms, k_iter sum {ker:.3f} ms "
      f"({ker / its * 1e3:.1f} us/it); graph run {dt / its * 1e6:.1f} us/it chk={chk} "
      f"(first run incl. graph build {dt0 * 1e3:.1f} ms)")
