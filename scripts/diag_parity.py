"""Diagnostics: where does the HIP iteration diverge from the oracle?"""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from gqmap_opticalflow_amd import Engine, State
from oracle import oracle
from tests import _golden as G

np.set_printoptions(linewidth=200, precision=4)
for name in G.CASES:
    d = G.load(name)
    o = d["opts"]
    for prec in ("fp64",):
        with Engine(o, d["I1"], d["I2"], o.get("engine", "mixture"), prec) as eng:
            eng.set_state(State(**G.state(d), it=1, T=o["temperature"]))
            done, tr = eng.run(1)
            st = eng.get_state()
        ost = oracle.State(*G.state(d).values())
        _, otr, _ = oracle.run(o, d["I1"], d["I2"], ost, 1, 1)
        print(f"== {name} {prec}: trace gpu {tr[0]} oracle {otr[0]}")
        for k, a in zip(G.STATE_KEYS, ost.arrays()):
            g = getattr(st, k)
            diff = np.abs(g - a)
            bad = np.argwhere(~(diff <= 1e-8))
            print(f"  {k}: maxdiff {np.nanmax(diff) if diff.size else 0:.3e} nbad {len(bad)} nan {np.isnan(g).sum()} first {bad[:6].tolist()}")
        # gradient-level view: state delta / step
        step = o.get("step0", 0.1) / (1 + 1 / o.get("step_decay", 8000.0))
        i0 = G.state(d)
        gm = (st.muu - i0["muu"]) / step
        om = (ost.muu - i0["muu"]) / step
        print("  dmuu gpu[:6,:6,0]\n", gm[:6, :6, 0], "\n  oracle\n", om[:6, :6, 0])
