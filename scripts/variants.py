"""Interleaved timing of libgqmap variants (build/var/libgqmap_*.so), one
subprocess per (variant, round) on the same GPU.  Prints median/min us/it of
the fused iteration kernel and checks every variant reaches the same state."""
import glob
import os
import re
import statistics
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
its = sys.argv[1] if len(sys.argv) > 1 else "100"
precs = sys.argv[2].split(",") if len(sys.argv) > 2 else ["fp64"]
engine = sys.argv[3] if len(sys.argv) > 3 else "mixture"
rounds = int(os.environ.get("ROUNDS", "3"))
libs = sorted(glob.glob(os.path.join(ROOT, "gqmap-opticalflow_amd", "build", "var", "libgqmap_*.so")))
res = {}
for r in range(rounds):
    for lib in libs:
        name = os.path.basename(lib)[9:-3]
        for prec in precs:
            env = dict(os.environ, GQMAP_LIB=lib)
            out = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "prof_iter.py"), its, prec,
                                  engine], env=env, capture_output=True, text=True, timeout=300)
            m = re.search(r"\(([\d.]+) us/it\); graph run ([\d.]+) us/it.*chk=(\S+)", out.stdout)
            if not m:
                print(name, prec, "FAILED", out.stdout[-500:], out.stderr[-2000:], flush=True)
                continue
            res.setdefault((name, prec), []).append((float(m.group(1)), float(m.group(2)), m.group(3)))
for (name, prec), v in sorted(res.items()):
    k = [a for a, _, _ in v]; g = [b for _, b, _ in v]
    print(f"{name:>10s} {prec}: kernel med {statistics.median(k):8.1f} min {min(k):8.1f} us | "
          f"graph med {statistics.median(g):8.1f} us | chk {sorted(set(c for *_, c in v))}")
