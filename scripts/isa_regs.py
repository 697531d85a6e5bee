"""Per-kernel register / spill / scratch / LDS summary of a gfx950 ISA listing
(hipcc --cuda-device-only -S): python3 scripts/isa_regs.py build/gqmap_engine.s [filter]"""
import re
import subprocess
import sys

path = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else ""
txt = open(path).read()
meta = txt[txt.find("amdhsa.kernels:"):]
rows = []
for blk in re.split(r"\n  - ", meta)[1:]:
    d = dict(re.findall(r"\.(\w+):\s+(\S+)", blk))
    if "name" not in d or flt not in d["name"]:
        continue
    try:
        nm = subprocess.run(["c++filt"], input=d["name"], capture_output=True, text=True).stdout.strip()
    except OSError:
        nm = d["name"]
    rows.append((nm.replace("gq::", "").split("(")[0], d.get("vgpr_count"), d.get("agpr_count"), d.get("sgpr_count"),
                 d.get("sgpr_spill_count"), d.get("vgpr_spill_count"), d.get("private_segment_fixed_size"),
                 d.get("group_segment_fixed_size")))
print(f"{'kernel':50s} {'vgpr':>5s} {'agpr':>5s} {'sgpr':>5s} {'sspill':>6s} {'vspill':>6s} {'scratch':>7s} {'lds':>6s}")
for r in rows:
    print(f"{r[0]:50s} " + " ".join(f"{str(x):>5s}" if i < 3 else f"{str(x):>6s}" for i, x in enumerate(r[1:])))
