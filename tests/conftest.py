import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device) and the built libqldpc_hip.so")


@pytest.fixture(scope="session")
def oracle():
    import oracle as _o

    _o.build()
    return _o


@pytest.fixture(scope="session")
def gpu():
    """Skip-free: GPU tests fail loudly if the native engine cannot run."""
    from qldpc_fault_tolerance_amd import _native

    _native.require_gpu()
    return _native
