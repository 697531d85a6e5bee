"""Waves-per-SIMD guard on the built library (no GPU): the headline kernels
sit on register thresholds (MI355X: <= 128 VGPRs -> 4 waves per SIMD, <= 168
-> 3, <= 256 -> 2).  Round 4 measured what crossing one costs: two extra
VGPRs on the C2 fp64 kernel (168 -> 170, 3 -> 2 waves) made it 9% slower
(profiles/r04_banded_pipeline.txt).  Reads .vgpr_count / .agpr_count from
the gfx950 code object's metadata in gqmap-opticalflow_amd/libgqmap.so."""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "gqmap-opticalflow_amd", "libgqmap.so")
LLVM = "/opt/rocm/lib/llvm/bin"

# kernel (mangled) -> max VGPRs (agpr 0): C2 fp64 (3 waves), C2 fp32 (4), C3's
# full level (3), its 240x320 level and C4 (2, no accumulation registers), the
# dataflow launches (2)
LIMITS = {
    "_ZN2gq6k_iterIdfLi0ELi1ELb0EEEvNS_10IterParamsIT_T0_EE": 168,
    "_ZN2gq6k_iterIdfLi0ELi1ELb1EEEvNS_10IterParamsIT_T0_EE": 168,
    "_ZN2gq6k_iterIffLi0ELi1ELb0EEEvNS_10IterParamsIT_T0_EE": 128,
    "_ZN2gq6k_iterIdfLi2ELi1ELb0EEEvNS_10IterParamsIT_T0_EE": 168,
    # the non-temporal-store variants the large frames run by default (state
    # > 32 MiB: C5, the full ctf levels of large pyramids)
    "_ZN2gq6k_iterIdfLi2ELi1ELb1EEEvNS_10IterParamsIT_T0_EE": 168,
    "_ZN2gq6k_iterIddLi2ELi1ELb1EEEvNS_10IterParamsIT_T0_EE": 168,
    "_ZN2gq6k_iterIddLi0ELi1ELb1EEEvNS_10IterParamsIT_T0_EE": 168,
    "_ZN2gq6k_iterIddLi2ELi2ELb0EEEvNS_10IterParamsIT_T0_EE": 256,
    "_ZN2gq6k_iterIdfLi1ELi4ELb0EEEvNS_10IterParamsIT_T0_EE": 256,
    # C3's 120x160 level (Q=4; 257 registers = 1 wave: 47.6 -> 72.5 us,
    # profiles/r05_node_pair_ab.txt) and the strong-scaling strips (mixture Q=2)
    "_ZN2gq6k_iterIddLi2ELi4ELb0EEEvNS_10IterParamsIT_T0_EE": 256,
    "_ZN2gq6k_iterIdfLi0ELi2ELb0EEEvNS_10IterParamsIT_T0_EE": 256,
    # the literal-order engine on integer frames (arith = literal, C2's
    # parity-carrying arithmetic), plain and non-temporal stores: 3 waves
    "_ZN2gq10k_iter_litIfLb0EEEvNS_10IterParamsIdT_EE": 168,
    "_ZN2gq10k_iter_litIfLb1EEEvNS_10IterParamsIdT_EE": 168,
    # the dataflow launches (k_iter_flow): 2 waves per SIMD, no spills -- C2
    # fp64 fast and literal-order, the C3 480x640 level
    "_ZN2gq11k_iter_flowIdfLi0ELi1ELb0ELi0EEEvNS_10IterParamsIT_T0_EEiPjiPKNS_3CtlE": 256,
    "_ZN2gq11k_iter_flowIdfLi0ELi1ELb1ELi0EEEvNS_10IterParamsIT_T0_EEiPjiPKNS_3CtlE": 256,
    "_ZN2gq11k_iter_flowIdfLi2ELi1ELb0ELi0EEEvNS_10IterParamsIT_T0_EEiPjiPKNS_3CtlE": 256,
    # C2 fp64 with the padded frame as binary16 column pairs (policy vv_pair,
    # the default on integer frames): per launch (3 waves) and as items (2)
    "_ZN2gq6k_iterIdNS_6vvh2_tELi0ELi1ELb0EEEvNS_10IterParamsIT_T0_EE": 168,
    "_ZN2gq11k_iter_flowIdNS_6vvh2_tELi0ELi1ELb0ELi0EEEvNS_10IterParamsIT_T0_EEiPjiPKNS_3CtlE": 256,
    "_ZN2gq6k_iterIfNS_6vvh2_tELi0ELi1ELb0EEEvNS_10IterParamsIT_T0_EE": 128,  # C2 fp32 (4 waves)
}
# kernels that must run without a private (scratch) segment: the C2 kernels
# of the fast arithmetic; the literal kernel is held to 3 waves by its launch
# bound (GQ_LIT_WAVES) and may spill a few registers there -- measured faster
# than the 174-VGPR, 2-wave allocation (profiles/r06_lit_mirror_ab.txt) --
# but not more than SCRATCH_MAX bytes
NO_SCRATCH = (
    "_ZN2gq6k_iterIdfLi0ELi1ELb0EEEvNS_10IterParamsIT_T0_EE",
    "_ZN2gq6k_iterIffLi0ELi1ELb0EEEvNS_10IterParamsIT_T0_EE",
    "_ZN2gq11k_iter_flowIdfLi0ELi1ELb0ELi0EEEvNS_10IterParamsIT_T0_EEiPjiPKNS_3CtlE",
    "_ZN2gq11k_iter_flowIdfLi0ELi1ELb1ELi0EEEvNS_10IterParamsIT_T0_EEiPjiPKNS_3CtlE",
    "_ZN2gq6k_iterIdNS_6vvh2_tELi0ELi1ELb0EEEvNS_10IterParamsIT_T0_EE",
    "_ZN2gq11k_iter_flowIdNS_6vvh2_tELi0ELi1ELb0ELi0EEEvNS_10IterParamsIT_T0_EEiPjiPKNS_3CtlE",
    "_ZN2gq6k_iterIfNS_6vvh2_tELi0ELi1ELb0EEEvNS_10IterParamsIT_T0_EE",
)
SCRATCH_MAX = {
    "_ZN2gq10k_iter_litIfLb0EEEvNS_10IterParamsIdT_EE": 128,
    "_ZN2gq10k_iter_litIfLb1EEEvNS_10IterParamsIdT_EE": 128,
}


def _kernel_registers(tmp):
    fat = os.path.join(tmp, "fatbin.bin")
    co = os.path.join(tmp, "co.elf")
    subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fat}", LIB, os.path.join(tmp, "x.so")],
                   check=True, capture_output=True)
    subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={fat}",
                    "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], check=True, capture_output=True)
    notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], check=True, capture_output=True,
                           text=True).stdout
    regs = {}
    for block in re.split(r"\n  - ", notes):
        name = re.search(r"\n\s*\.name:\s+(\S+)", "\n" + block)
        v = re.search(r"\.vgpr_count:\s+(\d+)", block)
        a = re.search(r"\.agpr_count:\s+(\d+)", block)
        sc = re.search(r"\.private_segment_fixed_size:\s+(\d+)", block)
        if name and v:
            regs[name.group(1)] = (int(v.group(1)), int(a.group(1)) if a else 0, int(sc.group(1)) if sc else 0)
    return regs


@pytest.mark.skipif(not os.path.exists(LIB) or not shutil.which(f"{LLVM}/llvm-readelf"),
                    reason="library or ROCm LLVM tools absent")
def test_headline_kernels_keep_their_waves(tmp_path):
    regs = _kernel_registers(str(tmp_path))
    for name, limit in LIMITS.items():
        assert name in regs, name
        v, a, _ = regs[name]
        assert v <= limit and a == 0, f"{name}: {v} VGPRs + {a} AGPRs > {limit}"
    for name in NO_SCRATCH:
        assert regs[name][2] == 0, f"{name}: {regs[name][2]} bytes of scratch"
    for name, mx in SCRATCH_MAX.items():
        assert regs[name][2] <= mx, f"{name}: {regs[name][2]} bytes of scratch > {mx}"
