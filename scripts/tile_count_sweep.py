"""C2 kernel time against the number of 16x16 tiles: crops of the
RubberWhale pair whose tile count is below, at and above the 768 workgroups
resident at 3 per CU (the second-round question of DESIGN.md 8).  Prints
k_iter us/it (HIP events, iterations 101-120 of the solve) and us per
1000 nodes.  usage: tile_count_sweep.py [fp64|fp32]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from bench import gt_options  # noqa: E402
from gqmap_opticalflow_amd import Engine  # noqa: E402

prec = sys.argv[1] if len(sys.argv) > 1 else "fp64"
I1, I2, flo, unk, o = gt_options("rubberwhale", 1, 9)
for M, N in ((256, 512), (320, 512), (352, 544), (384, 512), (384, 528), (384, 560), (388, 584), (384, 592),
             (384, 640)):
    a, b = (np.asfortranarray(x[:M, :N]) for x in (I1, I2))
    if N > I1.shape[1]:
        a, b = (np.asfortranarray(np.pad(x[:M], ((0, 0), (0, N - x.shape[1])), mode="reflect")) for x in (I1, I2))
    with Engine(dict(o, split=1), a, b, "mixture", prec) as e:
        e.init_state(0)
        e.run(100)
        done, tot, ker = e.run_timed(20)
    tiles = -(-M // 16) * -(-N // 16)
    us = ker / done * 1e3
    print(f"{M}x{N} tiles {tiles:4d} ({tiles / 768:.2f} x 768) k_iter {us:7.1f} us/it  "
          f"{us / (M * N) * 1e3:.3f} us/knode  {us / tiles * 1e3:.1f} ns/tile", flush=True)
