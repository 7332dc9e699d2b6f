import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs on the GPU box)")
    config.addinivalue_line("markers", "slow: longer CPU test")
    # Some GPU tests hand torch-allocated device buffers to the product library
    # (strip tiles).  torch ships its own HIP runtime; if the product library's
    # runtime initialises the device first, torch's later init finds no GPU.
    # Initialise torch's first (a no-op without a GPU).
    import torch
    if torch.cuda.is_available():
        torch.cuda.init()


@pytest.fixture(scope="session")
def golden():
    return os.path.join(ROOT, "tests", "golden")
