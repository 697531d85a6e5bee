"""Which HIP runtime and which RCCL a process that imports torch first (as
bench.py and this suite do, tests/conftest.py) actually maps.

libgqmap.so is linked against libamdhip64.so.7 (RUNPATH /opt/rocm) and
dlopens librccl.so.1; the torch wheel bundles libamdhip64.so and librccl.so
whose SONAMEs are libamdhip64.so.7 and librccl.so.1.  When torch is loaded
first the dynamic loader satisfies both names with torch's copies, so the
process holds ONE HIP runtime and ONE RCCL ("PyTorch in the
same process").  The mapped paths are printed for the record."""
import pytest

pytestmark = pytest.mark.gpu


def _mapped(tag):
    paths = set()
    with open("/proc/self/maps") as f:
        for line in f:
            parts = line.split()
            if len(parts) >= 6 and tag in parts[-1]:
                paths.add(parts[-1])
    return sorted(paths)


def test_one_hip_runtime_and_one_rccl_after_torch():
    import torch
    assert torch.cuda.is_available()
    from gqmap_opticalflow_amd import comm_unique_id, _lib
    _lib.load()
    comm_unique_id()  # resolves RCCL (gqmap_engine.hip rccl(): dlopen librccl.so.1)
    hip, rccl, hsa = _mapped("libamdhip64"), _mapped("librccl"), _mapped("libhsa-runtime64")
    print("libamdhip64:", hip)
    print("librccl:", rccl)
    print("libhsa-runtime64:", hsa)
    assert len(hip) == 1, hip
    assert len(rccl) == 1, rccl
    assert len(hsa) == 1, hsa
