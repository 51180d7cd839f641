import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "iterative-solver_amd")
for p in (ROOT, PKG, os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device); run with -m gpu")
    config.addinivalue_line("markers", "slow: minutes of CPU work at the configs' sizes; run with ITSOLV_SLOW=1")


def pytest_collection_modifyitems(config, items):
    if os.environ.get("ITSOLV_SLOW"):
        return
    skip = pytest.mark.skip(reason="slow (minutes of CPU work at the configs' sizes): set ITSOLV_SLOW=1")
    for item in items:
        if "slow" in item.keywords:
            item.add_marker(skip)


@pytest.fixture(scope="session")
def ctx():
    """One HIP context for the whole GPU session (tests run in one process on the box)."""
    import subspace_hip as sh

    if sh.device_count() < 1:
        pytest.fail("no HIP device visible: GPU tests must run on an MI355X")
    c = sh.Context(0)
    yield c
    c.close()
