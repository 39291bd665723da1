import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
HERE = os.path.dirname(os.path.abspath(__file__))
if HERE not in sys.path:
    sys.path.insert(0, HERE)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box)")
    config.addinivalue_line("markers", "slow: larger CPU test")
    config.addinivalue_line("markers", "fullsize: a benchmark config at full size on the GPU (minutes, ~250 GB HBM)")


@pytest.fixture(scope="session")
def gpu_available():
    import torch
    return torch.cuda.is_available()
