"""Per-workgroup timeline of two consecutive k_iter launches (iterations 20
and 21) from a GQ_TIMELINE=20 debug build: per block the start, the end of
phase 0 (wave 0), both phases done, components done, partials stored and, for
the last block, the finalize; plus the gap between the two launches.
Usage: GQMAP_LIB=.../libgqmap_tl.so python scripts/timeline.py [fp64|fp32] [c2|ctf:<scale>]"""
import ctypes as C
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import gt_options, setup_problem  # noqa: E402
from gqmap_opticalflow_amd import Engine, ctf_options, imresize  # noqa: E402
from gqmap_opticalflow_amd import _lib  # noqa: E402

prec = sys.argv[1] if len(sys.argv) > 1 else "fp64"
cfg = sys.argv[2] if len(sys.argv) > 2 else "c2"
if cfg == "c2":
    I1, I2, flo, unk, o = setup_problem("rubberwhale", 1, 9)
    engine = "mixture"
else:
    s = float(cfg.split(":")[1])
    I1, I2, flo, unk, g = gt_options("Grove3", 1, 11)
    I1, I2 = (np.asfortranarray(imresize(x, s)) for x in (I1, I2))
    o = ctf_options(its=500, minu=g["minu"], maxu=g["maxu"], minv=g["minv"], maxv=g["maxv"])
    if os.environ.get("GQMAP_SPLIT"):
        o["split"] = int(os.environ["GQMAP_SPLIT"])
    engine = "ctf"
NB = 8192
with Engine(o, I1, I2, engine, prec) as eng:
    eng.init_state(0)
    eng.run(25)
    info = eng.info()
    buf = (C.c_ulonglong * (32 * NB))()
    lib = C.CDLL(_lib.LIB_PATH)
    assert lib.gqmap_debug_timeline(buf, NB) == 0
a = np.frombuffer(buf, dtype=np.uint64).reshape(NB, 2, 16).astype(np.int64)
nb = int((a[:, 0, 0] > 0).sum())
a = a[:nb]
t0 = a[:, 0, 0].min()
us = lambda x: (x - t0) / 100.0  # noqa: E731  (100 MHz)
print(f"{prec} {cfg} {I1.shape} split={info.split}: {nb} blocks")
for d in (0, 1):
    st, p0, p1, p2, en = (us(a[:, d, k]) for k in (0, 1, 2, 3, 4))
    fin = a[:, d, 7]
    lastb = int(np.argmax(fin))
    fe = us(fin[lastb])
    print(f" launch {d}: start min {st.min():7.1f} max {st.max():7.1f} | phase0(w0) med {np.median(p0 - st):6.1f} | "
          f"phases med {np.median(p1 - st):6.1f} max {np.max(p1 - st):6.1f} | comps med {np.median(p2 - st):6.1f} | "
          f"stored med {np.median(en - st):6.1f} max end {en.max():7.1f} | last block {lastb} fin start "
          f"{en[lastb]:7.1f} done {fe:7.1f} ({fe - en[lastb]:.1f}: ticket {us(a[lastb, d, 8]) - en[lastb]:.1f} "
          f"reduce {us(a[lastb, d, 9]) - us(a[lastb, d, 8]):.1f} apply {fe - us(a[lastb, d, 9]):.1f})")
print(f" launch gap: last finalize of launch 0 -> first start of launch 1: "
      f"{us(a[:, 1, 0].min()) - us(a[:, 0, 7].max()):.1f} us; period {us(a[:, 1, 0].min()) - us(a[:, 0, 0].min()):.1f} us")
if nb > 768:
    d = 0
    st, en = us(a[:, d, 0]), us(a[:, d, 4])
    order = np.argsort(st)
    first, late = order[:768], order[768:]
    print(f" first 768 blocks dur med {np.median(en[first] - st[first]):.1f}; late {len(late)}: start med "
          f"{np.median(st[late]):.1f} dur med {np.median(en[late] - st[late]):.1f} end max {en[late].max():.1f}")
np.save(os.path.join(os.environ.get("GRAFT_REPO_ROOT", "."), "gpurun_out",
                     f"timeline_{prec}_{cfg.replace(':', '_')}.npy"), a)
