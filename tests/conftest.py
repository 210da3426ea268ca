import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TESTS = os.path.dirname(os.path.abspath(__file__))
for p in (ROOT, TESTS):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 GPU (runs on the MI355X box)")
    config.addinivalue_line("markers", "slow: long-running (large corpus)")


@pytest.fixture(scope="session")
def golden():
    import golden_io
    return golden_io.load_ed25519_golden()


@pytest.fixture(scope="session")
def golden_meta():
    import golden_io
    return golden_io.golden_meta()
