import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (run with -m gpu)")
    config.addinivalue_line("markers", "slow: long-running test")


@pytest.fixture(scope="session")
def native_build():
    """Build the native artefacts once per session (CPU: shim + fakes)."""
    from vgpu.native import build
    return build.build_all(kernels=False)


@pytest.fixture(scope="session")
def gpu_build():
    from vgpu.native import build
    return build.build_all(kernels=True)
