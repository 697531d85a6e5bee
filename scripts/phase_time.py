"""k_iter time per iteration in three phases of a C2 solve (early: random
init, middle, late: smoothed state), for the library GQMAP_LIB points at.
Usage: python scripts/phase_time.py [fp64|fp32] [window] [c2|c4]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import _policy  # noqa: E402

_policy.apply()
from bench import gt_options, setup_problem  # noqa: E402
from gqmap_opticalflow_amd import Engine  # noqa: E402

prec = sys.argv[1] if len(sys.argv) > 1 else "fp64"
win = int(sys.argv[2]) if len(sys.argv) > 2 else 20
cfg = sys.argv[3] if len(sys.argv) > 3 else "c2"
if cfg == "c4":
    I1, I2, flo, unk, o = gt_options("Urban3", 3, 11, temperature=0.2, drate=0.75, lambdas=16.0)
    engine = "super"
else:
    I1, I2, flo, unk, o = setup_problem("rubberwhale", 1, 9)
    engine = "mixture"
if os.environ.get("GQMAP_SPLIT"):
    o["split"] = int(os.environ["GQMAP_SPLIT"])
out = []
with Engine(o, I1, I2, engine, prec) as eng:
    eng.init_state(0)
    eng.run_timed(2)  # graph build / warm-up (iterations 1-2)
    pos = 2
    for start in (2, 250, 480):
        if start > pos:
            eng.run(start - pos)
        done, tot, ker = eng.run_timed(win)
        pos = start + win
        out.append(f"it{start}-{start + win}: {ker / win * 1e3:.1f}")
    _, tr = eng.run(1)
print(f"{os.path.basename(os.environ.get('GQMAP_LIB', 'libgqmap.so'))} {cfg} {prec} split={o.get('split', 0)} k_iter us/it " + " | ".join(out)
      + f" chk={tr[-1, 0]:.12g}", flush=True)
