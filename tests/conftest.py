import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU")
    config.addinivalue_line("markers", "slow: long CPU test")


@pytest.fixture(scope="session")
def golden_dir():
    return GOLDEN


@pytest.fixture
def knob():
    """Set library test knobs (tsg_test_knob) for one test; every one is reset afterwards."""
    from trivy_amd import _native as N
    names = []

    def set_(name, value):
        N.knob(name, value)
        names.append(name)
    yield set_
    for n in names:
        N.knob(n, None)
