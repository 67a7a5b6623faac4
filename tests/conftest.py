import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libme_hip.so on the device)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


@pytest.fixture(scope="session")
def oracle():
    import oracle as O

    O.lib()
    return O


@pytest.fixture(scope="session")
def ctx():
    from uasl_motion_estimation_amd import _lib

    return _lib.default_context()
