"""The authenticator mirror's whole suite (tests/test_authn_host.py) again with
the REAL GPU verifier behind edv.open_batch, plus batch-on-GPU vs
sequential-on-oracle equality over mixed request streams.  Reference tests
mirrored there: plenum/test/client/test_client_authn.py:39-74,
test_core_authn.py:41-151, plenum/test/test_req_authenticator.py:16-80."""
import pytest

import test_authn_host as H
from indy_plenum_amd import edv
from indy_plenum_amd.req_authenticator import ReqAuthenticator

pytestmark = pytest.mark.gpu
_REAL_OPEN = edv.open_batch


@pytest.fixture(autouse=True)
def cpu_checker(monkeypatch):
    """Same name as the host suite's fixture: counts device calls, but they go to the GPU."""
    calls = []

    def counting(items, device_mask=0):
        items = list(items)
        calls.append(len(items))
        return _REAL_OPEN(items, device_mask)
    monkeypatch.setattr(edv, "open_batch", counting)
    return calls


signer, sa, msg, signers = H.signer, H.sa, H.msg, H.signers
for _name in dir(H):
    if _name.startswith("test_"):
        globals()[_name] = getattr(H, _name)


def _sequential_on_oracle(f, monkeypatch):
    monkeypatch.setattr(edv, "open_batch", H.oracle_open_batch)
    try:
        return f()
    finally:
        monkeypatch.undo()


@pytest.mark.parametrize("seed", [11, 12])
def test_gpu_batch_equals_oracle_sequential(seed, monkeypatch):
    auth, reqs = H.make_requests(600, seed=seed)
    ra = ReqAuthenticator()
    ra.register_authenticator(auth)
    want = _sequential_on_oracle(lambda: [H.outcome(lambda r=r: ra.authenticate(r)) for r in reqs], monkeypatch)
    got = ra.authenticate_batch(reqs)
    got = [("raise", type(x).__name__, x.args) if isinstance(x, BaseException) else ("ok", x) for x in got]
    assert got == want
    assert sum(1 for o in want if o[0] == "ok") > 100


def test_gpu_whole_batch_native_path(monkeypatch):
    """CoreAuthNr.authenticate_batch through _edvhost.auth_core_batch (native
    prep, edv_verify_batch called from C++ with the GIL released) on the real
    GPU, against the sequential reference chain on the oracle."""
    auth, reqs = H.make_requests(3000, seed=41)
    want = _sequential_on_oracle(lambda: [H.outcome(lambda r=r: auth.authenticate(r)) for r in reqs], monkeypatch)
    assert edv.native_batch_enabled()     # the genuine entry point is back in place
    got = auth.authenticate_batch(reqs)
    got = [("raise", type(x).__name__, x.args) if isinstance(x, BaseException) else ("ok", x) for x in got]
    assert got == want
