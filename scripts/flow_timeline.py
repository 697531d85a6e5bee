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
