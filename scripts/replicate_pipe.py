import os, sys
sys.path.insert(0, '/root/repo') if os.path.exists('/root/repo') else None
sys.path.insert(0, os.getcwd())
import numpy as np
from bench import setup_problem
from gqmap_opticalflow_amd import Engine
I1, I2, flo, unk, o = setup_problem("rubberwhale", 1, 9)
for (r, c) in [(1, 1), (2, 2), (4, 2)]:
    a, b = np.asfortranarray(np.tile(I1, (r, c))), np.asfortranarray(np.tile(I2, (r, c)))
    out = []
    for pipe in ("0", "1"):
        os.environ["GQMAP_PIPE"] = pipe
        with Engine(o, a, b, "mixture", "fp64") as e:
            e.init_state(0)
            e.run_timed(5)
            done, tot, ker = e.run_timed(40)
            out.append(f"pipe={pipe} {ker / 40 * 1e3 / (r * c):7.1f} us/frame")
    print(f"{r}x{c}", "  ".join(out), flush=True)
