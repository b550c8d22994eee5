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


# Knobs that change what the native stepper computes (per-rank timing emulation, probes).
# Tests set them only through monkeypatch; one left in the process environment (e.g. by a
# module imported at collection) would silently alter every later test.
_PROCESS_KNOBS = ("GRAVSIM_EMULATE_RANK", "GRAVSIM_UNIT_TRACE", "GRAVSIM_EMU_COMM",
                  "GRAVSIM_SYM_BAND_MB", "GRAVSIM_FAULT_SKIP_UNITS", "GRAVSIM_SYM_OVERLAP",
                  "GRAVSIM_FORCE_COMM", "GRAVSIM_TEST_STALL", "GRAVSIM_SYNC",
                  "GRAVSIM_SYNC_LIMIT_S", "GRAVSIM_TAIL_SPLIT", "GRAVSIM_GRAPH_STEPS", "GRAVSIM_EMU_LINKS",
                  "ROCPROF_COUNTER_COLLECTION")


@pytest.fixture(autouse=True)
def _no_stray_native_knobs():
    stray = [k for k in _PROCESS_KNOBS if k in os.environ]
    assert not stray, f"process environment carries stepper knobs {stray}"
    yield
