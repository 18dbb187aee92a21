import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle"), os.path.dirname(os.path.abspath(__file__))):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libhip_raytrace.so on the device)")


@pytest.fixture(scope="session", autouse=True)
def _built():
    """Make sure the native library and the oracle exist (build() is cheap when up to date)."""
    import __graft_entry__
    __graft_entry__.build()
