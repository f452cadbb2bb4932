import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU; run with -m gpu")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(scope="session")
def oracle():
    from oracle import refcpu
    refcpu.build()
    return refcpu


@pytest.fixture(scope="session")
def saln():
    import sequencealigning_amd as s
    from sequencealigning_amd import _lib
    _lib.lib()
    return s
