import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import gravsim  # noqa: E402,F401


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device) and libgravsim_hip.so")
    config.addinivalue_line("markers", "slow: long-running test")


@pytest.fixture(scope="session")
def hip():
    """The HIP native library; GPU tests fail loudly (not skip) if it cannot be used."""
    import torch

    from gravsim.ops import _native

    assert torch.cuda.is_available(), "GPU test run without a visible HIP device"
    lib = _native.hip_lib()
    assert lib.gs_hip_device_count() > 0
    return lib
