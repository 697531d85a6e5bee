"""Dataflow-launch timeline (a GQ_FLOW_TL=1 build in build/var, GQMAP_LIB):
C2 fp64, one 20-iteration k_iter_flow launch from the seeded state after a
warm-up; per item (iteration, tile) the claim, the end of its dependency
wait and its end (s_memrealtime, 100 MHz).  Prints where the workgroups'
time goes: waiting for a neighbour / the finalize gate, working, and the
gap between an item's end and the next claim; and per iteration the span.
usage: GQMAP_LIB=.../libgqmap_tl.so python3 scripts/flow_timeline.py"""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from bench import setup_problem  # noqa: E402
from gqmap_opticalflow_amd import Engine, _lib  # noqa: E402

ITS = 20
I1, I2, flo, unk, o = setup_problem("rubberwhale", 1, 9)
lib = _lib.load()
f = lib.gqmap_debug_flow_timeline
f.restype = C.c_int
f.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
with Engine(o, I1, I2) as e:
    assert e.dataflow()
    for _ in range(30):  # settle the clocks
        e.init_state(0)
        e.run(ITS)
    ntiles = -(-e.M // 16) * -(-e.N // 16)
    e.init_state(0)
    e.run(ITS)  # one dispatch of ITS iterations from iteration 1
    n = ITS * ntiles * 4
    buf = (C.c_ulonglong * n)()
    assert f(buf, n) == n
tl = np.frombuffer(buf, dtype=np.uint64).reshape(ITS, ntiles, 4).astype(np.int64)
os.makedirs("gpurun_out", exist_ok=True)
np.savez_compressed(os.environ.get("FLOW_TL_OUT", "gpurun_out/flow_tl.npz"), tl=tl, tiles_m=-(-e.M // 16))
t0 = tl[:, :, 0].min()
claim, go, end = [(tl[:, :, k] - t0) / 100.0 for k in range(3)]
wait = go - claim
work = end - go
print(f"C2 fp64, one k_iter_flow dispatch of {ITS} iterations, {ntiles} tiles per iteration (times in us)")
print(f"launch span {end.max():.1f} us = {end.max() / ITS:.1f} us per iteration")
print(f"item work   mean {work.mean():.1f}  median {np.median(work):.1f}  p10 {np.percentile(work, 10):.1f}  p90 {np.percentile(work, 90):.1f}")
print(f"dep wait    mean {wait.mean():.2f}  median {np.median(wait):.2f}  p90 {np.percentile(wait, 90):.2f}  max {wait.max():.1f}  "
      f"share of item time {wait.sum() / (wait.sum() + work.sum()):.3f}")
# per workgroup slot: the gap between an item's end and the next item's claim
# needs the workgroup identity -- HW_ID (CU, SIMD, wave slot) + XCC_ID
hw = tl[:, :, 3]
order = np.argsort(claim.ravel())
slots = {}
gaps = []
for idx in order:
    h = int(hw.ravel()[idx])
    c, e_ = claim.ravel()[idx], end.ravel()[idx]
    if h in slots:
        gaps.append(c - slots[h])
    slots[h] = e_
gaps = np.array(gaps)
print(f"end -> next claim (same wave slot): mean {gaps.mean():.2f}  median {np.median(gaps):.2f}  p90 {np.percentile(gaps, 90):.2f}  "
      f"({len(slots)} slots)")
for j in range(ITS):
    print(f"iteration {j:2d}: first claim {claim[j].min():8.1f}  last end {end[j].max():8.1f}  "
          f"wait mean {wait[j].mean():5.2f}  work mean {work[j].mean():6.1f}")

# which dependency released each waiting item: the latest end among the
# tile's own and its four neighbours' iteration j - 1 items, or the
# finalize gate (iteration j - 2's last end); cross-band = a neighbour in
# another XCD's band (bands: contiguous tile ranges, k_iter_flow)
TM = -(-e.M // 16)
band = np.zeros(ntiles, dtype=int)
s0 = 0
for y in range(8):
    nb = (ntiles - y + 7) >> 3
    band[s0:s0 + nb] = y
    s0 += nb
kinds = {"self": 0, "in-band nb": 0, "cross-band nb": 0, "finalize": 0, "none (<1us)": 0}
wsum = dict.fromkeys(kinds, 0.0)
for j in range(1, ITS):
    fin = end[j - 2].max() if j >= 2 else -1e9
    for t in range(ntiles):
        w = wait[j, t]
        tm = t % TM
        deps = [(t, "self")]
        if tm > 0: deps.append((t - 1, None))
        if tm < TM - 1 and t + 1 < ntiles: deps.append((t + 1, None))
        if t >= TM: deps.append((t - TM, None))
        if t + TM < ntiles: deps.append((t + TM, None))
        last, kind = -1e9, None
        for d, k in deps:
            if end[j - 1, d] > last:
                last = end[j - 1, d]
                kind = k or ("in-band nb" if band[d] == band[t] else "cross-band nb")
        if fin > last:
            last, kind = fin, "finalize"
        if w < 1.0:
            kind = "none (<1us)"
        kinds[kind] += 1
        wsum[kind] += w
print("released by: " + ", ".join(f"{k} {kinds[k]} items / {wsum[k] / max(1, (ITS - 1) * ntiles):.2f} us mean"
                                  for k in kinds))
xc = (hw >> 32) & 0xF
for x in range(8):
    m = xc == x
    print(f"XCC {x}: items {m.sum():5d}  work mean {work[m].mean():6.1f}  wait mean {wait[m].mean():6.2f}")
for y in range(8):
    m = np.broadcast_to(band == y, wait.shape)
    print(f"band {y}: work mean {work[m].mean():6.1f}  wait mean {wait[m].mean():6.2f}")
