import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TESTS = os.path.dirname(os.path.abspath(__file__))
for p in (ROOT, TESTS):
    if p not in sys.path:
        sys.path.insert(0, p)


# Host-code sanitizer runs (tools/asan_host.sh): load an AddressSanitizer build
# of the native host-prep extension in place of the in-tree one.
_HOSTEXT = os.environ.get("EDV_HOSTEXT_OVERRIDE")
if _HOSTEXT:
    import importlib.util
    import indy_plenum_amd  # noqa: F401  (the package only; it imports no extension)
    _spec = importlib.util.spec_from_file_location("indy_plenum_amd._edvhost", _HOSTEXT)
    _mod = importlib.util.module_from_spec(_spec)
    _spec.loader.exec_module(_mod)
    sys.modules["indy_plenum_amd._edvhost"] = _mod


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
