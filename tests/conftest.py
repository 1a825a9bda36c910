"""Shared pytest configuration: markers and paths. `-m "not gpu"` runs everywhere; `-m gpu` needs a
gfx950 device and the in-tree libfmi_dev.so."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (gfx950) and libfmi_dev.so")
    config.addinivalue_line("markers", "slow: long-running CPU test")


@pytest.fixture(scope="session")
def device():
    """Initialise device 0 once per session; the HIP path is mandatory for gpu tests (no fallback)."""
    import fmi_amd
    fmi_amd.init(0)
    yield fmi_amd
    fmi_amd.sync()
