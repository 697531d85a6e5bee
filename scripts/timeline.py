"""Per-workgroup timeline of one k_iter launch (iteration 20 of C2) from a
GQ_TIMELINE=20 debug build: start/end per block, CU and XCD, summarised as
rounds of resident tiles.  Usage: GQMAP_LIB=.../libgqmap_tl.so python scripts/timeline.py [fp64|fp32]"""
import ctypes as C
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import setup_problem  # noqa: E402
from gqmap_opticalflow_amd import Engine  # noqa: E402
from gqmap_opticalflow_amd import _lib  # noqa: E402

prec = sys.argv[1] if len(sys.argv) > 1 else "fp64"
I1, I2, flo, unk, o = setup_problem("rubberwhale", 1, 9)
with Engine(o, I1, I2, "mixture", prec) as eng:
    eng.init_state(0)
    eng.run(25)
    nb = 925
    buf = (C.c_ulonglong * (4 * nb))()
    lib = C.CDLL(_lib.LIB_PATH)
    assert lib.gqmap_debug_timeline(buf, nb) == 0
a = np.frombuffer(buf, dtype=np.uint64).reshape(nb, 4).astype(np.int64)
t0 = a[:, 0].min()
st = (a[:, 0] - t0) / 100.0  # us (100 MHz)
en = (a[:, 1] - t0) / 100.0
hw = a[:, 2]
cu = (hw >> 8) & 0xF
sh = (hw >> 12) & 1
se = (hw >> 13) & 0x7
xcc = a[:, 3] & 0xF
dur = en - st
print(f"{prec}: launch span {en.max():.1f} us; block duration min {dur.min():.1f} med {np.median(dur):.1f} "
      f"max {dur.max():.1f}")
order = np.argsort(st)
for q in (0, 100, 300, 500, 700, 767, 768, 800, 850, 900, 924):
    b = order[q]
    print(f"  start-rank {q:4d}: block {b:4d} start {st[b]:7.1f} end {en[b]:7.1f} dur {dur[b]:6.1f} "
          f"xcc {xcc[b]} se {se[b]} cu {cu[b]}")
first = order[:768]
late = order[768:]
print(f"first 768 blocks: start max {st[first].max():.1f}, end min {en[first].min():.1f} med {np.median(en[first]):.1f} "
      f"max {en[first].max():.1f}, dur med {np.median(dur[first]):.1f}")
print(f"late {len(late)} blocks: start min {st[late].min():.1f} med {np.median(st[late]):.1f}, dur med "
      f"{np.median(dur[late]):.1f} max {dur[late].max():.1f}, end max {en[late].max():.1f}")
# concurrency profile: resident blocks over time
ts = np.linspace(0, en.max(), 21)
print("resident blocks: " + " ".join(f"{int(((st <= t) & (en > t)).sum())}" for t in ts))
np.save(os.path.join(os.environ.get("GRAFT_REPO_ROOT", "."), "gpurun_out", f"timeline_{prec}.npy"), a)
