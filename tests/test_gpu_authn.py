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


def test_gpu_async_submit_with_digests_and_state(monkeypatch):
    """authenticate_batch_submit on the real GPU (native prep, ONE queued
    edv_verify_digest_batch_async call, wait at result()): the sequential
    reference chain's outcomes, Request.getDigest for every request the device
    hashed, and state-backed verkeys (client_authn.py:148-160) on the same
    native path.  Several batches in flight at once (as the pool's nodes keep
    them), finished out of order."""
    import json
    from indy_plenum_amd.client_authn import nym_to_state_key
    from indy_plenum_amd.pool import cpu_digests
    auth, reqs = H.make_requests(2400, seed=43)

    class St:
        kv = {}

        def get(self, key, isCommitted=True):
            assert isCommitted is False
            return self.kv.get(key)
    st = St()
    for idr in list(auth.clients)[:5]:
        st.kv[nym_to_state_key(idr)] = json.dumps(auth.clients.pop(idr)).encode()
    auth.state = st
    want = _sequential_on_oracle(lambda: [H.outcome(lambda r=r: auth.authenticate(r)) for r in reqs], monkeypatch)
    assert edv.native_batch_enabled()
    norm = lambda res: [("raise", type(x).__name__, x.args) if isinstance(x, BaseException) else ("ok", x)
                        for x in res]
    parts = [reqs[k::4] for k in range(4)]
    pend = [auth.authenticate_batch_submit(p, digests=True) for p in parts]
    for k in (2, 0, 3, 1):
        got = norm(pend[k].result())
        assert got == want[k::4]
        hashed = 0
        for q, d in zip(parts[k], pend[k].digests()):
            if d is not None:
                hashed += 1
                assert d == cpu_digests([q])[0]
        assert hashed > 300
