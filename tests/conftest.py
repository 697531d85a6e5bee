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
    """GPU runs: PyTorch bundles its own HIP/HSA runtime beside the /opt/rocm
    one libgqmap.so links; in one process the two coexist only when torch's
    initialises first (the other order leaves torch with "No HIP GPUs are
    available"), as in bench.py.  The device-array tests need torch tensors,
    so torch.cuda is initialised before any test calls the library."""
    if any(item.get_closest_marker("gpu") for item in request.session.items):
        import torch
        if torch.cuda.is_available():
            torch.cuda.init()
    yield
