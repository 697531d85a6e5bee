"""Where does a captured banded graph fail?  Step by step with faulthandler."""
import faulthandler
import sys

faulthandler.enable()
sys.path.insert(0, ".")
from bench import gt_options  # noqa: E402
from gqmap_opticalflow_amd import Engine  # noqa: E402

I1, I2, flo, unk, o = gt_options("rubberwhale", 1, 9)
with Engine(o, I1, I2, "mixture", "fp64") as e:
    e.init_state(0)
    for n in (1, 2, 4, 50):
        print("run", n, flush=True)
        d, tr = e.run(n)
        print("  done", d, tr[-1], flush=True)
