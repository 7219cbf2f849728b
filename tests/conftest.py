"""pytest configuration: `gpu` marker, import paths, shared env/model builders."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "pupperv3-mjx_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels)")
    config.addinivalue_line("markers", "slow: long-running")


def gpu_available() -> bool:
    try:
        from pupperv3_mjx import _lib
        return _lib.load().pp3_device_count() > 0
    except Exception:
        return False


@pytest.fixture(scope="session")
def require_gpu():
    from pupperv3_mjx import _lib
    L = _lib.load()  # raises loudly if the HIP extension is missing
    if L.pp3_device_count() <= 0:
        pytest.fail("GPU test collected on a host without a visible GPU")
    return L
