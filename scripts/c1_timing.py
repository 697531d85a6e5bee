"""C1 call anatomy: wall clock of repeated gqmap_cpu calls (Dimetrodon GT,
50 its) and of the pieces around the C-ABI call."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import ctypes as C  # noqa: E402

import numpy as np  # noqa: E402

from gqmap_opticalflow_amd import _lib, flow_to_color, flowio, gqmap_cpu  # noqa: E402
from gqmap_opticalflow_amd.legacy import cpu_options  # noqa: E402

gt = flowio.load_pair("Dimetrodon")[2]
_, flo, _, unk = flow_to_color(gt)
for i in range(6):
    t = time.perf_counter()
    gqmap_cpu(dict(its=50, K=9), flo, seed=0)
    print(f"call {i}: {1e3 * (time.perf_counter() - t):.2f} ms", flush=True)
lib = _lib.load()
M, N, _ = flo.shape
o = cpu_options(dict(its=50, K=9))
mu = np.zeros((M, N, 2), order="F"); sg = np.zeros((M, N, 2), order="F"); rou = np.zeros((M, N, 2, 2), order="F")
tr = np.zeros((50, 3)); done = C.c_int(0)
f = np.asfortranarray(flo)
for i in range(3):
    t = time.perf_counter()
    lib.gqmap_cpu_run(C.byref(o), _lib.dptr(f), M, N, None, C.c_uint64(0), _lib.dptr(mu), _lib.dptr(sg),
                      _lib.dptr(rou), _lib.dptr(tr), C.byref(done), 0)
    print(f"raw ABI call {i}: {1e3 * (time.perf_counter() - t):.2f} ms", flush=True)
