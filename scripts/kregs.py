"""VGPRs / AGPRs / scratch bytes of the kernels matching a pattern in a built
library (default: the literal kernel), from the gfx950 code object notes.
usage: python3 scripts/kregs.py LIB.so [regex]"""
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
lib = sys.argv[1]
pat = re.compile(sys.argv[2] if len(sys.argv) > 2 else "k_iter_lit")
with tempfile.TemporaryDirectory() as t:
    fat, co = os.path.join(t, "f.bin"), os.path.join(t, "co.elf")
    subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fat}", lib, os.path.join(t, "x.so")],
                   check=True, capture_output=True)
    subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={fat}",
                    "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], check=True, capture_output=True)
    notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], check=True, capture_output=True, text=True).stdout
for block in re.split(r"\n  - ", notes):
    name = re.search(r"\n\s*\.name:\s+(\S+)", "\n" + block)
    v = re.search(r"\.vgpr_count:\s+(\d+)", block)
    sc = re.search(r"\.private_segment_fixed_size:\s+(\d+)", block)
    if name and v and pat.search(name.group(1)):
        print(f"{name.group(1)[:70]:70s} vgpr {v.group(1)} scratch {sc.group(1) if sc else 0}")
