import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "platform-aware-scheduling_amd"), os.path.join(ROOT, "oracle"),
          os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libpas.so's HIP kernels)")
    config.addinivalue_line("markers", "slow: larger parity cases")


@pytest.fixture(scope="session")
def oracle():
    import oracle as _oracle  # oracle/oracle.py (test infrastructure)
    _oracle.load()
    return _oracle


@pytest.fixture(scope="session")
def ctx():
    """A pas_ctx on device 0.  GPU tests fail loudly (no skip) when it cannot be created."""
    import pas_amd
    c = pas_amd.Context(0)
    yield c
    c.close()
