"""k_iter time when the C2 frame pair is replicated r x c times (same
statistics, more tiles): how far a single-frame launch is from the
throughput of a long grid.  usage: replicate_sweep.py [fp64|fp32]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from bench import setup_problem  # noqa: E402
from gqmap_opticalflow_amd import Engine  # noqa: E402

prec = sys.argv[1] if len(sys.argv) > 1 else "fp64"
I1, I2, flo, unk, o = setup_problem("rubberwhale", 1, 9)
for (r, c) in [(1, 1), (2, 1), (1, 2), (2, 2), (4, 2)]:
    a, b = np.asfortranarray(np.tile(I1, (r, c))), np.asfortranarray(np.tile(I2, (r, c)))
    M, N = a.shape
    with Engine(o, a, b, "mixture", prec) as e:
        e.init_state(0)
        e.run_timed(5)
        done, tot, ker = e.run_timed(40)
        blocks = ((M + 15) // 16) * ((N + 15) // 16)
        us = ker / 40 * 1e3
        print(f"{r}x{c} {M:5d}x{N:<5d} blocks {blocks:5d}  k_iter {us:8.1f} us  {M * N / us / 1e3:.3f} Gnode-it/s  "
              f"{us / (r * c):.1f} us per frame", flush=True)
