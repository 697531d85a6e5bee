import sys, numpy as np
sys.path.insert(0, '.')
from tests import test_gpu_parity as T
from tests import _golden as G
from gqmap_opticalflow_amd import Engine
from oracle import oracle
prec = sys.argv[1] if len(sys.argv) > 1 else "fp64"
I1, I2, _, _, o, st = T._reference_init_case("rubberwhale", 96, 128, 150, 200, L=1, K=11, engine="ctf",
                                             alpha_start=10, t_decay_every=20, split=1)
ost = T._oracle_state(st)
X, W = T._gh(11)
with Engine(o, I1, I2, "ctf", prec) as eng:
    eng.set_state(st)
    Tt = st.T
    for it in range(1, 41):
        _, tr = eng.run(1)
        _, etr, Tt = oracle.emu_run(o, I1, I2, ost, it, 1, X, W, T=Tt, nthreads=8, fp32=prec == "fp32", split=1)
        g = eng.get_state()
        bad = []
        for k, a in zip(G.STATE_KEYS, ost.arrays()):
            b = getattr(g, k)
            nd = np.argwhere(b != a)
            if len(nd):
                bad.append((k, len(nd), nd[:3].tolist(), np.abs(b - a).max()))
        if bad or not np.array_equal(tr, etr):
            print("iteration", it, tr, etr, bad)
            break
    else:
        print("all 40 equal")
