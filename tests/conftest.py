import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")


@pytest.fixture(scope="session")
def oracle_lib():
    from oracle import oracle
    oracle.lib()
    return oracle


@pytest.fixture(scope="session", autouse=True)
def _torch_hip_runtime_first(request):
    """GPU runs: torch is loaded and torch.cuda initialised before any test
    calls the library, as in bench.py.  Loaded after torch, libgqmap.so binds
    to torch's bundled libamdhip64 / librccl (their SONAMEs match the names
    the library asks for): one HIP runtime in the process
    (tests/test_gpu_runtime.py).  In the other order two runtimes load and
    torch reports "No HIP GPUs are available".  The device-array tests need
    torch tensors."""
    if any(item.get_closest_marker("gpu") for item in request.session.items):
        import torch
        if torch.cuda.is_available():
            torch.cuda.init()
    yield
