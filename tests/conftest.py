import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI)")


def golden(name):
    return dict(np.load(os.path.join(GOLDEN, name), allow_pickle=False))


@pytest.fixture(scope="session")
def hip_device():
    """cuda:0 with the native library loaded, or skip (gpu-marked tests only)."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU visible")
    from bnn_kfac_amd import _native
    _native.lib()  # raises loudly if libkfac_hip.so is missing
    return torch.device("cuda:0")
