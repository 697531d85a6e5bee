"""The (pair, seed) solves the multi-GPU C2 bench gives ranks 0..7
(PAIRS[rank % 3], init seed = rank): each must run all 500 iterations
(bench.py raises if the stop rule fires early).  One process, one GPU."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import PAIRS, gt_options  # noqa: E402
from gqmap_opticalflow_amd import Engine  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 500
bad = 0
for rank in range(8):
    name = PAIRS[rank % len(PAIRS)]
    I1, I2, flo, unk, opts = gt_options(name, 1, 9)
    with Engine(opts, I1, I2, "mixture", "fp64") as eng:
        eng.init_state(seed=rank)
        done, tr = eng.run(steps)
        print(f"rank {rank} {name:12s} seed {rank}: {done}/{steps} iterations, last ptdmu {tr[-1, 1]:.3e}", flush=True)
        bad += done != steps
sys.exit(1 if bad else 0)
