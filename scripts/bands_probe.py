"""C2 fp64 wall per iteration with the banded pipeline (GQMAP_BANDS=B, read
once per process: one subprocess per B) against one launch per iteration,
after clock settling: run(20) from the seeded state (the driver's window) and
run(100).  usage: bands_probe.py [B,B,...]"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CODE = r'''
import sys, time
sys.path.insert(0, ".")
from bench import gt_options, settle_clocks
from gqmap_opticalflow_amd import Engine
I1, I2, flo, unk, o = gt_options("rubberwhale", 1, 9)
with Engine(o, I1, I2, "mixture", sys.argv[1]) as e:
    e.init_state(1); e.run(5); e.prepare()
    def chunk():
        e.init_state(0); e.run(20)
    settle_clocks(chunk, 20)
    res = []
    for n in (20, 100):
        best = 1e9
        for r in range(5):
            e.init_state(0)
            t0 = time.perf_counter(); d, _ = e.run(n); dt = time.perf_counter() - t0
            assert d == n
            best = min(best, dt / n * 1e6)
        res.append(best)
    e.init_state(0); e.run(100); mp = e.map()
    print(f"{res[0]:.1f} {res[1]:.1f} chk={float(mp.sum())!r}")
'''
bands = sys.argv[1].split(",") if len(sys.argv) > 1 else ["0", "3", "4", "6", "8"]
for prec in ("fp64", "fp32"):
    for rep in range(2):
        for b in bands:
            env = {k: v for k, v in os.environ.items() if k != "GQMAP_BANDS"}
            if b != "0":
                env["GQMAP_BANDS"] = b
            out = subprocess.run([sys.executable, "-c", CODE, prec], cwd=ROOT, env=env, capture_output=True,
                                 text=True, timeout=300)
            if out.returncode != 0:
                print(f"{prec} B={b} FAILED rc={out.returncode} {out.stdout[-500:]} {out.stderr[-1500:]}", flush=True)
                sys.exit(1)
            a, bb, chk = out.stdout.split()
            print(f"{prec} rep {rep} B={b}: run(20) {a} us/it, run(100) {bb} us/it, {chk}", flush=True)
