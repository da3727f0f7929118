import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run on the GPU box via gpurun)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


@pytest.fixture(scope="session", autouse=True)
def _torch_hip_first(request):
    """When GPU tests run, let torch's HIP runtime open the device before
    libcauseweave's does (the order bench.py uses): a test that hands torch
    tensors to the library needs both, and torch reports no device if it comes
    second."""
    if request.config.getoption("-m") and "not gpu" not in request.config.getoption("-m"):
        try:
            import torch

            if torch.cuda.is_available():
                torch.cuda.init()
        except Exception:
            pass
    yield
