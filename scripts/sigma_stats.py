"""Spread of the quadrature sample offsets over a C2 solve: how far from its
node does each node sample VV (|mu| + 4.5 sigma), per iteration checkpoint."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from bench import setup_problem  # noqa: E402
from gqmap_opticalflow_amd import Engine  # noqa: E402

I1, I2, flo, unk, o = setup_problem("rubberwhale", 1, 9)
with Engine(o, I1, I2) as e:
    e.init_state(0)
    done = 0
    for target in (0, 1, 10, 50, 100, 200, 300, 500):
        if target > done:
            e.run(target - done)
            done = target
        st = e.get_state()
        for name, mu, sg in (("u", st.muu, st.sigu), ("v", st.muv, st.sigv)):
            r = np.abs(mu) + 4.5 * sg
            print(f"it {done:4d} {name}: sigma p50 {np.median(sg):6.2f} p99 {np.percentile(sg, 99):6.2f} "
                  f"| reach p50 {np.median(r):6.2f} p90 {np.percentile(r, 90):6.2f} p99 {np.percentile(r, 99):6.2f} "
                  f"frac<=8: {(r <= 8).mean():.3f} frac<=12: {(r <= 12).mean():.3f}", flush=True)
