"""Row f-1: the native host prep (_edvhost, csrc/edv_host.cpp) gives exactly the
results of the Python restatements of base58 1.0.0 and SigningSerializer (which
are pinned by the reference's fixtures and outputs in test_base58_serializer.py),
on fixed edge cases and on randomized inputs; anything it does not handle falls
back (NotImplemented) so the reference's exceptions are unchanged."""
import random

import numpy as np
import pytest

from indy_plenum_amd import _edvhost, base58, edv, signing_serializer
from indy_plenum_amd.signing_serializer import SigningSerializer, serialize_msg_for_signing


def test_native_module_is_loaded():
    assert base58._native is _edvhost and signing_serializer._native is _edvhost


def py_dec(v):
    try:
        return base58._b58decode_py(v)
    except Exception as ex:
        return type(ex)


def api_dec(v):
    try:
        return base58.b58decode(v)
    except Exception as ex:
        return type(ex)


def test_b58_edge_cases():
    cases = ["", "1", "11", "111z", "2", "z", "zz", " 1A ", "1A\n", "1A\x1c", "1A\t\r\x0b\x0c", "0", "O", "I",
             "l", "abc!", "é", "1é", "　", "A　", b"", b"1", b"1A \n", b"1A\x1c", b"\x00", b"zz",
             "V4SGRU86Z58d6TV7PBUe6f", "5rArie7XKukPCaEwq5XGQJnM9Fc5aZE3M9HAPVfMU2xC", 42, None, bytearray(b"1A")]
    for c in cases:
        assert api_dec(c) == py_dec(c), repr(c)
        nat = _edvhost.b58decode(c)
        if nat is not NotImplemented:
            assert nat == py_dec(c), repr(c)


def test_b58_random_roundtrip():
    r = random.Random(3)
    for _ in range(3000):
        raw = bytes([0] * r.randrange(4)) + bytes(r.getrandbits(8) for _ in range(r.randrange(0, 70)))
        enc = base58.b58encode(raw)
        assert enc == base58._b58encode_py(raw)
        assert base58.b58decode(enc) == raw == base58._b58decode_py(enc)
        s = enc.decode() + r.choice(["", " ", "\n", "  \t"])
        assert base58.b58decode(s) == base58._b58decode_py(s)
        t = "".join(r.choice("123456789ABCDEFGHJKLMNPQRSTUVWXYZabcdefghijkmnopqrstuvwxyz0OIl!")
                    for _ in range(r.randrange(0, 50)))
        assert api_dec(t) == py_dec(t)


def test_b58_decoder_lengths_around_the_fast_path_limit():
    """str inputs up to 128 characters take the allocation-free 64-bit-limb
    decoder (also used by the batch path's decode threads), longer ones the
    general one: both equal the restatement, including leading '1's and
    trailing whitespace at every length."""
    r = random.Random(17)
    alpha = "123456789ABCDEFGHJKLMNPQRSTUVWXYZabcdefghijkmnopqrstuvwxyz"
    for n in list(range(0, 140)) + [200, 300]:
        for _ in range(6):
            t = "1" * r.randrange(0, 4) + "".join(r.choice(alpha) for _ in range(n))
            t += r.choice(["", " ", "\t\n", "\x1f"])
            assert _edvhost.b58decode(t) == py_dec(t), (n, t)
    assert _edvhost.b58decode("z" * 128) == py_dec("z" * 128)
    assert _edvhost.b58decode("1" * 128) == b"\0" * 128


def _rand_obj(r, depth=0):
    k = r.randrange(9 if depth < 3 else 6)
    if k == 0:
        return r.choice(["", "a", "x|y:z", "ünï", "日本", "1,2"])
    if k == 1:
        return r.choice([0, 1, -7, 2**70, -(2**64), 10**20])
    if k == 2:
        return r.choice([0.1, 1.5, -2.0, 1e300, 1e-7, float("inf")])
    if k == 3:
        return r.choice([True, False])
    if k == 4:
        return None
    if k == 5:
        return r.choice(["NYM", "1", "~abc"])
    if k == 6:
        return [_rand_obj(r, depth + 1) for _ in range(r.randrange(4))]
    return {r.choice(["a", "b", "B", "type", "dest", "verkey", "é", "_", "10", "9", "zz"]) + str(i):
            _rand_obj(r, depth + 1) for i in range(r.randrange(5))}


def test_serializer_native_equals_restatement():
    r = random.Random(4)
    ss = SigningSerializer()
    for _ in range(4000):
        obj = {"identifier": "L5AD5g65TDQr1PPHHRoiGf", "operation": _rand_obj(r), "reqId": r.randrange(10**16),
               "extra": _rand_obj(r)}
        for ignore in (None, ["extra"], ("reqId", "extra"), {"operation"}):
            want = ss.serialize(obj, topLevelKeysToIgnore=ignore)
            assert _edvhost.serialize(obj, ignore) == want
            assert serialize_msg_for_signing(obj, topLevelKeysToIgnore=ignore) == want


def test_serializer_fallbacks_keep_reference_errors():
    ss = SigningSerializer()
    for bad in ({"a": (1, 2)}, {"a": {1: "x"}}, {"a": b"bytes"}, {"a": object()}, {1: "x", 2: "y"}):
        assert _edvhost.serialize(bad, None) is NotImplemented
        try:
            want = ss.serialize(bad)
        except Exception as ex:
            with pytest.raises(type(ex)):
                serialize_msg_for_signing(bad)
        else:
            assert serialize_msg_for_signing(bad) == want
    s = {"a": "\ud800"}  # lone surrogate: UnicodeEncodeError from the restatement
    assert _edvhost.serialize(s, None) is NotImplemented
    with pytest.raises(UnicodeEncodeError):
        serialize_msg_for_signing(s)


def test_pack_open_batch_positional_split():
    r = random.Random(5)
    items = []
    for _ in range(500):
        ls = r.choice([0, 10, 63, 64, 65, 100])
        lm = r.choice([0, 1, 20, 300])
        items.append((bytes(r.getrandbits(8) for _ in range(ls)), bytes(r.getrandbits(8) for _ in range(lm)),
                      bytes(r.getrandbits(8) for _ in range(32))))
    sigs, pks, msgs, off, idx = _edvhost.pack_open_batch(items)
    off = np.frombuffer(off, np.uint64)
    want_idx = [k for k, (s, m, _p) in enumerate(items) if len(s) + len(m) >= 64]
    assert idx == want_idx and len(off) == len(idx) + 1
    for j, k in enumerate(idx):
        s, m, p = items[k]
        sm = s + m
        assert sigs[64 * j:64 * j + 64] == sm[:64]
        assert msgs[off[j]:off[j + 1]] == sm[64:]
        assert pks[32 * j:32 * j + 32] == p
    assert len(msgs) >= off[-1] + 16
    with pytest.raises(ValueError):
        _edvhost.pack_open_batch([(b"x" * 64, b"", b"k" * 31)])
    with pytest.raises(ValueError):
        edv.open_batch([(b"x" * 64, b"", b"k" * 31)])


def test_core_fast_path_equals_python_plan(monkeypatch):
    """prep_core_batch (native) vs the Python plan vs sequential authenticate on
    every key form and failure the single-signature path can meet."""
    import test_authn_host as H
    from indy_plenum_amd import client_authn
    from indy_plenum_amd.client_authn import CoreAuthNr
    monkeypatch.setattr(edv, "open_batch", H.oracle_open_batch)
    r = random.Random(9)
    crypt = H.Signer(seed=b"C" * 32)                        # cryptonym: idr = full verkey
    full = H.Signer(identifier="V4SGRU86Z58d6TV7PBUe6f", seed=b"F" * 32)
    abbr = H.Signer(seed=b"B" * 32)
    abbr.identifier = base58.b58encode(abbr.pk[:16]).decode()
    auth = CoreAuthNr()
    auth.addIdr(crypt.identifier, "")                      # empty verkey -> the identifier itself
    auth.addIdr(full.identifier, full.verkey)
    auth.addIdr(abbr.identifier, "~" + base58.b58encode(abbr.pk[16:]).decode())
    auth.addIdr("BadAbbr1111111111111111", "~0OIl")        # invalid abbreviation
    auth.addIdr("HexKey", abbr.pk.hex())                  # hex-encoded 32-byte key
    auth.addIdr("NoKey", None)
    auth.clients["EmptyNym"] = {}
    reqs = []
    for i in range(400):
        s = r.choice([crypt, full, abbr])
        req = {"identifier": s.identifier, "reqId": i, "operation": {"type": "1", "n": i}, "protocolVersion": 2}
        kind = r.randrange(12)
        if kind == 0:
            req["identifier"] = r.choice(["BadAbbr1111111111111111", "HexKey", "NoKey", "EmptyNym", "Unknown9"])
        if kind == 1:
            req["signature"] = "0OIl"
        elif kind == 2:
            req["signature"] = ""
        elif kind == 3:
            req["identifier"] = ""
        elif kind == 4:
            req["signature"] = s.sign({**req, "reqId": -1})
        elif kind == 5:
            req["signature"] = s.sign(req) + "  "           # trailing whitespace is stripped by b58decode
        elif kind == 6:
            req["fees"] = [1, 2]                          # excluded from the signing bytes
            req["signature"] = s.sign({k: v for k, v in req.items() if k != "fees"})
        elif kind == 7:
            req["signature"] = s.sign(req)
            req["signatures"] = {"other": "x"}            # ignored when identifier + signature are set
        else:
            req["signature"] = s.sign(req)
        reqs.append(req)
    seq = [H.outcome(lambda q=q: auth.authenticate(dict(q))) for q in reqs]
    norm = lambda res: [("raise", type(x).__name__, x.args) if isinstance(x, BaseException) else ("ok", x)
                        for x in res]
    fast = norm(auth.authenticate_batch(reqs))
    assert sum(1 for x in _edvhost.prep_core_batch(reqs, auth.clients, auth.excluded_from_signing)
               if x is not None) > 150
    monkeypatch.setattr(client_authn, "_edvhost", None)
    slow = norm(auth.authenticate_batch(reqs))
    assert fast == slow == seq
    assert {o[0] if o[0] == "ok" else o[1] for o in seq} >= {"ok", "InsufficientCorrectSignatures",
                                                            "InvalidSignatureFormat", "UnknownIdentifier"}


def _oracle_verify_callback(calls):
    """An edv_verify_batch-compatible C function pointer backed by the oracle, so
    the whole-batch native path (_edvhost.auth_core_batch) runs on the CPU."""
    import ctypes
    import oracle_lib as orc
    CB = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                          ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint32)

    def fake(sigs, pks, msgs, off, n, acc, mask):
        o = np.ctypeslib.as_array((ctypes.c_uint64 * (n + 1)).from_address(off)).copy()
        res = orc.verify_batch(ctypes.string_at(sigs, 64 * n), ctypes.string_at(pks, 32 * n),
                               ctypes.string_at(msgs, int(o[-1]) + 16), o, n, 4)
        ctypes.memmove(acc, res, n)
        calls.append(n)
        return 0
    cb = CB(fake)
    return cb, ctypes.cast(cb, ctypes.c_void_p).value


@pytest.mark.parametrize("threads", [1, 4])
def test_whole_batch_native_path_equals_sequential(monkeypatch, threads):
    """_edvhost.auth_core_batch (phase A with the GIL, base58 on `threads` threads
    without it, the verify call inside) gives exactly what the reference's
    sequential authenticate gives, request by request, over a mixed stream:
    fast-path accepts and rejects, and every request it hands back to the Python
    plan (truncated signatures, multi-signature, missing fields, unknown DIDs)."""
    import test_authn_host as H
    from indy_plenum_amd.req_authenticator import ReqAuthenticator
    sa, reqs = H.make_requests(3000, seed=31)
    ra = ReqAuthenticator()
    ra.register_authenticator(sa)
    with monkeypatch.context() as m:
        m.setattr(edv, "open_batch", H.oracle_open_batch)
        want = [H.outcome(lambda r=r: sa.authenticate(r)) for r in reqs]
        want_ra = [H.outcome(lambda r=r: ra.authenticate(r)) for r in reqs]
    calls = []
    cb, addr = _oracle_verify_callback(calls)
    monkeypatch.setattr(edv, "verify_address", lambda: addr)
    monkeypatch.setattr(edv, "PREP_THREADS", threads)
    slow_calls = []
    real_open = edv.open_batch

    def counting_open(items, device_mask=0):
        items = list(items)
        slow_calls.append(len(items))
        return H.oracle_open_batch(items)
    # the slow remainder still goes through open_batch; route it to the oracle
    # without disabling the native path (which checks for the genuine entry point)
    monkeypatch.setattr(edv, "_OPEN_BATCH", counting_open)
    monkeypatch.setattr(edv, "open_batch", counting_open)
    got = sa.authenticate_batch(reqs)
    got = [("raise", type(x).__name__, x.args) if isinstance(x, BaseException) else ("ok", x) for x in got]
    assert got == want
    assert len(calls) == 1 and calls[0] > 1000      # the fast path carried most of the batch in one call
    assert len(slow_calls) == 1                       # and the remainder took one more
    got_ra = ra.authenticate_batch(reqs)
    got_ra = [("raise", type(x).__name__, x.args) if isinstance(x, BaseException) else ("ok", x) for x in got_ra]
    assert got_ra == want_ra
    monkeypatch.setattr(edv, "open_batch", real_open)


def test_native_request_digests_equal_request_get_digest(monkeypatch):
    """_edvhost.request_digests (native signingState serialization + one SHA-256
    batch call, here the kernel's SHA-256 compiled for the CPU) gives
    Request.getDigest = sha256(serialize_msg_for_signing(signingState)) for every
    request it takes, and None (Python path) for the rest; digest.request_digests
    equals the per-request reference restatement on a mixed batch."""
    import ctypes
    import hashlib
    import hostcheck_lib
    from indy_plenum_amd import digest
    hc = hostcheck_lib.load()
    addr = ctypes.cast(hc.hc_sha256_batch, ctypes.c_void_p).value
    r = random.Random(41)
    reqs = []
    for i in range(400):
        q = {"identifier": base58.b58encode(bytes(r.randrange(256) for _ in range(16))).decode(),
             "reqId": r.choice([1539648000000000 + i, None, -5, 2**70, 3.5]),
             "operation": r.choice([{"type": "1", "dest": "x" * r.randrange(40), "verkey": "~abc"},
                                    {"type": "101", "data": {"nested": [1, "two", None, True]}}, None, "op"]),
             "signature": "sig"}
        pv = r.choice([None, 2, 1, "2", "missing"])
        if pv != "missing":
            q["protocolVersion"] = pv
        if r.random() < 0.05:
            q.pop("identifier")
            q["signatures"] = {"B": "s", "A": "t"}   # identifier derived from the signatures: Python path
        if r.random() < 0.03:
            q["identifier"] = ""                      # falsy identifier: Python path
            q["signatures"] = {"C": "s"}
        reqs.append(q)
    want = [hashlib.sha256(serialize_msg_for_signing(digest.signing_state(q))).hexdigest() for q in reqs]
    got = _edvhost.request_digests(reqs, addr, 0)
    assert len(got) == len(reqs)
    handled = [k for k, d in enumerate(got) if d is not None]
    assert len(handled) > 300
    assert all(got[k] == want[k] for k in handled)
    assert all(reqs[k].get("identifier") for k in handled)

    def cpu_sha256_batch(messages, device_mask=0):
        return [hashlib.sha256(m).digest() for m in messages]
    monkeypatch.setattr(edv, "sha256_address", lambda: addr)
    monkeypatch.setattr(edv, "sha256_batch", cpu_sha256_batch)
    assert digest.request_digests(reqs) == want


class _RecordingState:
    """The reference state's get(key, isCommitted) contract; records every read."""

    def __init__(self):
        self.kv, self.reads = {}, []

    def get(self, key, isCommitted=True):
        self.reads.append(isCommitted)
        return self.kv.get(key)


@pytest.mark.parametrize("n_keys_on_device", [10**9, 1])
def test_whole_batch_native_path_with_state_verkeys(monkeypatch, n_keys_on_device):
    """SimpleAuthNr.getVerkey's second source (client_authn.py:148-160 ->
    domain_req_handler.py:158-167: the NYM under sha256(identifier) in the
    uncommitted state) on the whole-batch native path: identifiers known only
    to the state stay native (one verify call for them and the clients-map
    ones), and every outcome equals the sequential reference chain, including
    state values that are absent, empty, not JSON or not an object, and a
    clients entry that is empty (which falls through to the state)."""
    import json
    import hashlib
    import test_authn_host as H
    from indy_plenum_amd import client_authn, digest
    from indy_plenum_amd.client_authn import CoreAuthNr, nym_to_state_key
    r = random.Random(77)
    signers = [H.Signer(seed=bytes([k + 1, 7]) * 16) for k in range(10)]
    for k, s in enumerate(signers):
        if k % 3 == 1:            # abbreviated verkeys
            s.identifier = base58.b58encode(s.pk[:16]).decode()
    st = _RecordingState()
    auth = CoreAuthNr(state=st)
    for s in signers[:3]:
        auth.addIdr(s.identifier, s.verkey)
    for k, s in enumerate(signers[3:8]):
        vk = "~" + base58.b58encode(s.pk[16:]).decode() if s.identifier != s.verkey else s.verkey
        st.kv[nym_to_state_key(s.identifier)] = json.dumps({"verkey": vk, "role": None}).encode()
    auth.clients[signers[3].identifier] = {}          # falsy clients entry: the state decides
    odd = ["NotJson1", "ListNym1", "EmptyNym", "NoVerkey", "Absent99"]
    st.kv[nym_to_state_key("NotJson1")] = b"{not json"
    st.kv[nym_to_state_key("ListNym1")] = b"[1, 2]"
    st.kv[nym_to_state_key("EmptyNym")] = b"{}"
    st.kv[nym_to_state_key("NoVerkey")] = b'{"role": "0"}'
    reqs = []
    for i in range(600):
        s = r.choice(signers[:8])
        req = {"identifier": s.identifier, "reqId": i, "operation": {"type": "1", "n": i}, "protocolVersion": 2}
        kind = r.randrange(10)
        if kind == 0:
            req["identifier"] = r.choice(odd)
        if kind == 1:
            req["signature"] = s.sign({**req, "reqId": -1})
        else:
            req["signature"] = s.sign(req)
        reqs.append(req)
    with monkeypatch.context() as m:
        m.setattr(edv, "open_batch", H.oracle_open_batch)
        want = [H.outcome(lambda q=q: auth.authenticate(dict(q))) for q in reqs]
    assert st.reads and not any(st.reads)             # every state read is uncommitted
    calls = []
    cb, addr = _oracle_verify_callback(calls)
    monkeypatch.setattr(edv, "verify_address", lambda: addr)
    monkeypatch.setattr(client_authn.CoreAuthMixin, "STATE_KEYS_ON_DEVICE", n_keys_on_device)
    monkeypatch.setattr(digest, "nym_state_keys", lambda nyms, device_mask=0:
                        [hashlib.sha256(x.encode()).digest() for x in nyms])
    slow_calls = []

    def counting_open(items, device_mask=0):
        items = list(items)
        slow_calls.append(len(items))
        return H.oracle_open_batch(items)
    monkeypatch.setattr(edv, "_OPEN_BATCH", counting_open)
    monkeypatch.setattr(edv, "open_batch", counting_open)
    st.reads.clear()
    got = auth.authenticate_batch(reqs)
    got = [("raise", type(x).__name__, x.args) if isinstance(x, BaseException) else ("ok", x) for x in got]
    assert got == want
    assert not any(st.reads)
    n_odd = sum(1 for q in reqs if q["identifier"] in odd)
    # every request with a resolvable verkey went native, state-only identifiers included
    assert len(calls) == 1 and calls[0] == len(reqs) - n_odd
    assert sum(slow_calls) == 0                       # the odd ones fail before any verify
    assert {o[1] for o in got if o[0] == "raise"} >= {"UnknownIdentifier", "CouldNotAuthenticate",
                                                      "InsufficientCorrectSignatures"}


def _oracle_async_callbacks(calls):
    """edv_verify_digest_batch_async / edv_wait_async-compatible C function
    pointers backed by the oracle and hashlib: the batch is 'done' at submit,
    wait checks the ticket.  Lets the asynchronous native path run on the CPU."""
    import ctypes
    import hashlib
    import oracle_lib as orc
    SUB = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                           ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
                           ctypes.POINTER(ctypes.c_int64))
    WAIT = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_int, ctypes.c_int64)
    issued = []

    def submit(sigs, pks, msgs, off, n, acc, digests, device, ticket):
        o = np.ctypeslib.as_array((ctypes.c_uint64 * (n + 1)).from_address(off)).copy()
        blob = ctypes.string_at(msgs, int(o[-1]) + 16)
        res = orc.verify_batch(ctypes.string_at(sigs, 64 * n), ctypes.string_at(pks, 32 * n), blob, o, n, 4)
        ctypes.memmove(acc, res, n)
        if digests:
            d = b"".join(hashlib.sha256(blob[int(o[i]) - int(o[0]):int(o[i + 1]) - int(o[0])]).digest()
                         for i in range(n))
            ctypes.memmove(digests, d, 32 * n)
        calls.append((n, bool(digests)))
        ticket[0] = len(issued)
        issued.append(False)
        return 0

    def wait(device, ticket):
        if not 0 <= ticket < len(issued) or issued[ticket]:
            return -1
        issued[ticket] = True
        return 0

    def query(device, ticket):  # edv_query_async: done at submit, so handed over now
        if not 0 <= ticket < len(issued):
            return -1
        issued[ticket] = True
        return 0
    cbs = (SUB(submit), WAIT(wait), WAIT(query))
    return cbs, tuple(ctypes.cast(c, ctypes.c_void_p).value for c in cbs[:2]), issued


def _query_address(cbs):
    """edv.query_address stand-in for _oracle_async_callbacks' query callback."""
    import ctypes
    return lambda: ctypes.cast(cbs[2], ctypes.c_void_p).value


@pytest.mark.parametrize("with_state", [False, True])
def test_async_submit_finish_equals_sequential_with_digests(monkeypatch, with_state):
    """authenticate_batch_submit -> PendingAuth (native phases A/B, one queued
    device call with the request digests, finish = wait + output): the same
    per-request results as the sequential reference chain, and digests equal to
    Request.getDigest (hashlib over the reference restatement) exactly for the
    requests whose signing bytes are their signingState serialization, None for
    the rest.  Also through ReqAuthenticator and node_integration.PendingProd."""
    import json
    import test_authn_host as H
    from indy_plenum_amd import client_authn, digest
    from indy_plenum_amd.client_authn import nym_to_state_key
    from indy_plenum_amd.node_integration import PendingProd
    from indy_plenum_amd.pool import cpu_digests
    from indy_plenum_amd.req_authenticator import ReqAuthenticator
    sa, reqs = H.make_requests(1500, seed=57)
    r = random.Random(5)
    for q in reqs[::7]:
        q["extra"] = 1                               # signing bytes != signingState: no device digest
    for q in reqs[3::11]:
        if isinstance(q, dict):
            q["protocolVersion"] = None              # signingState drops it, the signing bytes keep it
    if with_state:
        st = _RecordingState()
        for idr in list(sa.clients)[:4]:             # some identifiers only in the state
            st.kv[nym_to_state_key(idr)] = json.dumps(sa.clients.pop(idr)).encode()
        sa.state = st
    with monkeypatch.context() as m:
        m.setattr(edv, "open_batch", H.oracle_open_batch)
        want = [H.outcome(lambda q=q: sa.authenticate(q)) for q in reqs]
    calls = []
    cbs, addrs, issued = _oracle_async_callbacks(calls)
    monkeypatch.setattr(edv, "async_addresses", lambda: addrs)
    monkeypatch.setattr(edv, "BATCH_DEVICE", 0)
    monkeypatch.setattr(edv, "verify_address", lambda: addrs[0])
    monkeypatch.setattr(client_authn.CoreAuthMixin, "STATE_KEYS_ON_DEVICE", 10**9)

    def counting_open(items, device_mask=0):
        return H.oracle_open_batch(list(items))
    monkeypatch.setattr(edv, "_OPEN_BATCH", counting_open)
    monkeypatch.setattr(edv, "open_batch", counting_open)
    norm = lambda res: [("raise", type(x).__name__, x.args) if isinstance(x, BaseException) else ("ok", x)
                        for x in res]
    if with_state:  # requests as the Node sees them: decoded from JSON, keys not interned
        reqs = [json.loads(json.dumps(q)) if isinstance(q, dict) else q for q in reqs]
    p = sa.authenticate_batch_submit(reqs, digests=True)
    assert len(calls) == 1 and calls[0][1] and issued == [False]   # queued, not waited for
    assert norm(p.result()) == want and issued == [True]
    digs = p.digests()
    ref = cpu_digests([q for q in reqs if isinstance(q, dict) and q.get("identifier")])
    got_some = 0
    it = iter(ref)
    for q, d in zip(reqs, digs):
        if not (isinstance(q, dict) and q.get("identifier")):
            assert d is None
            continue
        x = next(it)
        if d is not None:
            got_some += 1
            assert d == x
            assert "extra" not in q and q.get("protocolVersion", 0) is not None
    assert got_some > 500
    # through ReqAuthenticator (single stock authenticator) and PendingProd
    ra = ReqAuthenticator()
    ra.register_authenticator(sa)
    with monkeypatch.context() as m:
        m.setattr(edv, "open_batch", H.oracle_open_batch)
        want_ra = [H.outcome(lambda q=q: ra.authenticate(q)) for q in reqs]
    pr = ra.authenticate_batch_submit(reqs, digests=True)
    assert norm(pr.result()) == want_ra
    # requests ReqAuthenticator hands to the authenticator get the same digests; the
    # others (queries, unknown types: never submitted) get None
    assert all(d is None or d == e for d, e in zip(pr.digests(), digs))
    assert sum(d is not None for d in pr.digests()) > 400
    good = [q for q in reqs if isinstance(q, dict) and q.get("identifier")]
    props = [({"op": "PROPAGATE", "request": q}, "Beta") for q in good[:300]]
    clients = [(q, "client") for q in good[300:]]
    seen = []
    pp = PendingProd(ra, clients, props, digests=True)
    assert pp.digests(cpu_digests) == cpu_digests(good)      # device digests + the digest_fn rest
    pp.finish(lambda m, f, o: seen.append(("c", o)), lambda m, f, o: seen.append(("p", o)))
    with monkeypatch.context() as m:
        m.setattr(edv, "open_batch", H.oracle_open_batch)
        want_pp = [H.outcome(lambda q=q: ra.authenticate(q)) for q in good]
    assert norm([x for _k, x in seen]) == want_pp
    # a handle dropped unfinished is waited for (no stray batch left in flight)
    n_before = len(issued)
    sa.authenticate_batch_submit(reqs[:50], digests=False)
    import gc as _gc
    _gc.collect()
    assert len(issued) == n_before + 1 and issued[-1] is True


def test_native_state_nyms_equals_restatement():
    """_edvhost.state_nyms (CPU SHA-256 state keys, the flat-JSON fast read,
    json.loads for everything else) against the Python restatement
    (CoreAuthNr._state_nyms_py) on the values a state can hold: plain objects,
    duplicate keys, escapes, nesting, numbers of every JSON form, non-JSON
    (NaN, trailing garbage, single quotes), non-ASCII, invalid UTF-8, str and
    bytearray values, empty and falsy values, and clients entries that are
    present, empty or falsy."""
    import json
    from indy_plenum_amd.client_authn import CoreAuthNr, nym_to_state_key
    values = [
        b'{"verkey": "~abc", "role": null}', b'{"verkey":"~a","verkey":"~b"}', b'{"verkey":"~a","verkey":null}',
        b'{"verkey": null}', b'{"role": "0"}', b'{}', b' { "verkey" : "Full32ByteKeyXXXXXXXXXXXXXXXXXXXXX" } \n',
        b'{"verkey":"~a","seqNo":12,"txnTime":1.5e9,"x":-0.25E-3,"t":true,"f":false}',
        b'{"verkey":"~a","n":01}', b'{"verkey":"~a","n":1.}', b'{"verkey":"~a","n":NaN}', b'{"verkey":"~a"} x',
        b"{'verkey':'~a'}", b'{"verk\\u0065y":"~esc"}', b'{"verkey":"~a\\n"}', b'{"verkey":"~a","o":{"k":1}}',
        b'{"verkey":"~a","l":[1,2]}', '{"verkey":"~ünï"}'.encode(), b'{"verkey":"\xff"}', b'[1,2]', b'"str"',
        b'', None, '{"verkey":"~strval"}', bytearray(b'{"verkey":"~ba"}'), b'{"verkey":"~a",}', b'{,}',
        b'{"verkey":"~tab\there"}', b'  ', b'{"verkey":"~a"}\x00',
    ]
    st = _RecordingState()
    reqs, clients = [], {}
    for k, v in enumerate(values):
        idr = "Idr%02d" % k
        if v is not None:
            st.kv[nym_to_state_key(idr)] = v
        reqs.append({"identifier": idr, "reqId": k})
    clients["Idr00"] = {"verkey": "~inmem"}          # answered from the clients map: no state read
    clients["Idr01"] = {}                              # falsy: the state decides
    clients["Idr02"] = None
    reqs += [{"identifier": "Idr03"}, "notadict", {"identifier": ""}, {"identifier": 5}, {"reqId": 1}]
    auth = CoreAuthNr(state=st)
    auth.clients = clients
    py = auth._state_nyms_py(reqs) or {}
    reads_py = list(st.reads)
    st.reads.clear()
    nat = auth._state_nyms(reqs) or {}
    assert st.reads == reads_py and not any(st.reads)  # the same reads, uncommitted, deduplicated

    def view(d):
        return {i: v.get("verkey") for i, v in d.items() if isinstance(v.get("verkey"), str)}
    assert view(nat) == view(py)
    assert set(nat) <= set(py)
    assert view(py)["Idr06"] == "Full32ByteKeyXXXXXXXXXXXXXXXXXXXXX" and view(py)["Idr01"] == "~b"
    assert "Idr00" not in py and "Idr13" in view(py)   # escaped key: json.loads path


def test_native_req_auth_routing_edge_cases(monkeypatch):
    """ReqAuthenticator.authenticate_batch_submit on the native path
    (_edvhost.req_auth_submit / req_auth_finish) for the requests whose txn
    type the reference reads unusually: no operation, an operation that is not
    a dict, an unhashable or integer type, a request that is not a dict, a dict
    subclass -- each must give exactly what ReqAuthenticator.authenticate gives."""
    import test_authn_host as H
    from indy_plenum_amd.req_authenticator import ReqAuthenticator
    sa, reqs = H.make_requests(400, seed=61)
    s0 = next(q for q in reqs if isinstance(q, dict) and q.get("signature") and q["operation"]["type"] == "1")

    class D(dict):
        pass
    odd = [{k: v for k, v in s0.items() if k != "operation"},
           {**s0, "operation": ["type", "1"]},
           {**s0, "operation": {"type": ["1"]}},
           {**s0, "operation": {"type": 1}},
           {**s0, "operation": {"dest": "x"}},
           {**s0, "operation": None},
           D(s0), ["not", "a", "dict"], None, {**s0, "operation": {"type": "3"}}]
    reqs = reqs[:200] + odd + reqs[200:]
    ra = ReqAuthenticator()
    ra.register_authenticator(sa)
    with monkeypatch.context() as m:
        m.setattr(edv, "open_batch", H.oracle_open_batch)
        want = [H.outcome(lambda q=q: ra.authenticate(q)) for q in reqs]
    calls = []
    cbs, addrs, issued = _oracle_async_callbacks(calls)
    monkeypatch.setattr(edv, "async_addresses", lambda: addrs)
    monkeypatch.setattr(edv, "BATCH_DEVICE", 0)
    monkeypatch.setattr(edv, "verify_address", lambda: addrs[0])
    monkeypatch.setattr(edv, "_OPEN_BATCH", H.oracle_open_batch)
    monkeypatch.setattr(edv, "open_batch", H.oracle_open_batch)
    p = ra.authenticate_batch_submit(reqs, digests=True)
    assert len(calls) == 1                              # the native path queued one device call
    got = [("raise", type(x).__name__, x.args) if isinstance(x, BaseException) else ("ok", x) for x in p.result()]
    assert got == want
    assert {o[1] for o in want if o[0] == "raise"} >= {"NoAuthenticatorFound", "AttributeError", "TypeError"}


class _PickyState(_RecordingState):
    """A state whose read raises for one key (that request alone fails)."""

    def __init__(self, bad_key):
        super().__init__()
        self.bad_key = bad_key

    def get(self, key, isCommitted=True):
        if key == self.bad_key:
            raise KeyError("corrupt node")
        return super().get(key, isCommitted)


@pytest.mark.parametrize("native", [True, False])
def test_state_nyms_one_bad_identifier_fails_alone(monkeypatch, native):
    """An identifier with a lone surrogate (valid json.loads output that cannot be
    UTF-8 encoded) and an identifier whose state read raises, mixed into a batch
    of good state-backed requests: every request gets exactly what the sequential
    reference chain gives it -- the two odd ones their own exception, the rest
    their identifiers -- instead of one exception failing the whole batch
    (client_authn.py:148-160 -> domain_req_handler.py:158-167 per request)."""
    import json
    import hashlib
    import test_authn_host as H
    from indy_plenum_amd import client_authn, digest
    from indy_plenum_amd.client_authn import CoreAuthNr, nym_to_state_key
    signers = [H.Signer(seed=bytes([k + 9, 3]) * 16) for k in range(6)]
    st = _PickyState(nym_to_state_key("BadRead1"))
    auth = CoreAuthNr(state=st)
    for s in signers:
        st.kv[nym_to_state_key(s.identifier)] = json.dumps({"verkey": s.verkey, "role": None}).encode()
    reqs = []
    for i in range(60):
        s = signers[i % len(signers)]
        req = {"identifier": s.identifier, "reqId": i, "operation": {"type": "1", "n": i}, "protocolVersion": 2}
        req["signature"] = s.sign(req)
        reqs.append(req)
    reqs[7] = {**reqs[7], "identifier": "Sur\ud800rogate"}
    reqs[23] = {**reqs[23], "identifier": "BadRead1"}
    with monkeypatch.context() as m:
        m.setattr(edv, "open_batch", H.oracle_open_batch)
        want = [H.outcome(lambda q=q: auth.authenticate(dict(q))) for q in reqs]
    assert want[7][0] == "raise" and want[7][1] == "UnicodeEncodeError"
    assert want[23][0] == "raise" and want[23][1] == "KeyError"
    assert sum(w[0] == "ok" for w in want) == 58
    if not native:
        monkeypatch.setattr(client_authn, "_edvhost", None)
    py = auth._state_nyms_py(reqs)
    assert len(py) == len(signers)
    calls = []
    cb, addr = _oracle_verify_callback(calls)
    monkeypatch.setattr(edv, "verify_address", lambda: addr)
    monkeypatch.setattr(client_authn.CoreAuthMixin, "STATE_KEYS_ON_DEVICE", 1)
    monkeypatch.setattr(digest, "nym_state_keys", lambda nyms, device_mask=0:
                        [hashlib.sha256(x.encode()).digest() for x in nyms])
    monkeypatch.setattr(edv, "_OPEN_BATCH", H.oracle_open_batch)
    monkeypatch.setattr(edv, "open_batch", H.oracle_open_batch)
    got = auth.authenticate_batch(reqs)
    got = [("raise", type(x).__name__, x.args) if isinstance(x, BaseException) else ("ok", x) for x in got]
    assert got == want


def test_failed_async_wait_stays_failed(monkeypatch):
    """when the device wait of a submitted batch fails, result()
    raises, and so does every later result()/digests() call -- the verdict bytes
    in the (reused) arena are never read as verdicts -- and the arena is not
    handed to the next batch.  The next batch still gets its own verdicts."""
    import ctypes
    import test_authn_host as H
    from indy_plenum_amd import client_authn
    sa, reqs = H.make_requests(300, seed=91)
    with monkeypatch.context() as m:
        m.setattr(edv, "open_batch", H.oracle_open_batch)
        want = [H.outcome(lambda q=q: sa.authenticate(q)) for q in reqs]
    calls = []
    cbs, addrs, issued = _oracle_async_callbacks(calls)
    WAIT = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_int, ctypes.c_int64)
    fail = {"on": True}

    def bad_wait(device, ticket):
        return -3 if fail["on"] else cbs[1](device, ticket)
    bw = WAIT(bad_wait)
    monkeypatch.setattr(edv, "async_addresses", lambda: (addrs[0], ctypes.cast(bw, ctypes.c_void_p).value))
    monkeypatch.setattr(edv, "BATCH_DEVICE", 0)
    monkeypatch.setattr(edv, "verify_address", lambda: addrs[0])
    monkeypatch.setattr(client_authn.CoreAuthMixin, "STATE_KEYS_ON_DEVICE", 10**9)
    monkeypatch.setattr(edv, "_OPEN_BATCH", H.oracle_open_batch)
    monkeypatch.setattr(edv, "open_batch", H.oracle_open_batch)
    p = sa.authenticate_batch_submit(reqs, digests=True)
    for _ in range(3):
        with pytest.raises(RuntimeError, match="edv_wait_async"):
            p.result()
    with pytest.raises(RuntimeError):
        p.digests()
    del p
    fail["on"] = False
    p2 = sa.authenticate_batch_submit(reqs, digests=False)
    got = [("raise", type(x).__name__, x.args) if isinstance(x, BaseException) else ("ok", x) for x in p2.result()]
    assert got == want


def test_batch_ready_queries_without_waiting(monkeypatch):
    """PendingAuth.ready() / PendingProd.ready() through _edvhost.batch_ready and
    an edv_query_async-compatible callback: False while the query answers
    EDV_PENDING (and no wait happens), True once it answers 0 -- after which
    result() hands the verdicts over without calling the wait at all, with the
    same results as the sequential chain; a failed query makes ready() True and
    result() raise, for good.  Both submit paths (CoreAuthNr and the native
    ReqAuthenticator one) carry it."""
    import ctypes
    import test_authn_host as H
    from indy_plenum_amd import client_authn
    from indy_plenum_amd.node_integration import PendingProd
    from indy_plenum_amd.req_authenticator import ReqAuthenticator
    sa, reqs = H.make_requests(400, seed=93)
    with monkeypatch.context() as m:
        m.setattr(edv, "open_batch", H.oracle_open_batch)
        want = [H.outcome(lambda q=q: sa.authenticate(q)) for q in reqs]
    calls = []
    cbs, addrs, issued = _oracle_async_callbacks(calls)
    QUERY = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_int, ctypes.c_int64)
    state = {"answer": 1, "queries": 0}

    def query(device, ticket):
        state["queries"] += 1
        if state["answer"] == 0:
            issued[ticket] = True       # handed over by the query, as edv_query_async does
        return state["answer"]
    qf = QUERY(query)
    monkeypatch.setattr(edv, "async_addresses", lambda: addrs)
    monkeypatch.setattr(edv, "query_address", lambda: ctypes.cast(qf, ctypes.c_void_p).value)
    monkeypatch.setattr(edv, "BATCH_DEVICE", 0)
    monkeypatch.setattr(edv, "verify_address", lambda: addrs[0])
    monkeypatch.setattr(client_authn.CoreAuthMixin, "STATE_KEYS_ON_DEVICE", 10**9)
    monkeypatch.setattr(edv, "_OPEN_BATCH", H.oracle_open_batch)
    monkeypatch.setattr(edv, "open_batch", H.oracle_open_batch)
    norm = lambda res: [("raise", type(x).__name__, x.args) if isinstance(x, BaseException) else ("ok", x)
                        for x in res]
    ra = ReqAuthenticator()
    ra.register_authenticator(sa)
    with monkeypatch.context() as m:
        m.setattr(edv, "open_batch", H.oracle_open_batch)
        want_ra = [H.outcome(lambda q=q: ra.authenticate(q)) for q in reqs]
    for submit, expect in ((lambda: sa.authenticate_batch_submit(reqs, digests=True), want),
                           (lambda: ra.authenticate_batch_submit(reqs, digests=True), want_ra)):
        state.update(answer=1, queries=0)
        p = submit()
        t = len(issued) - 1
        assert not p.ready() and not p.ready() and state["queries"] == 2 and issued[t] is False
        state["answer"] = 0
        assert p.ready() and issued[t] is True
        assert p.ready() and state["queries"] == 3        # settled: no further query
        assert norm(p.result()) == expect                 # the wait callback was not called again
    # PendingProd: ready() follows the batch
    good = [q for q in reqs if isinstance(q, dict) and q.get("identifier")]
    state.update(answer=1, queries=0)
    pp = PendingProd(ra, [(q, "client") for q in good], [], digests=True)
    assert not pp.ready()
    state["answer"] = 0
    assert pp.ready()
    seen = []
    pp.finish(lambda m, f, o: seen.append(o), lambda m, f, o: seen.append(o))
    assert len(seen) == len(good)
    assert PendingProd(ra, [], []).ready()                # nothing submitted
    # a failed query: ready, and the result raises every time
    state.update(answer=-3)
    p = sa.authenticate_batch_submit(reqs, digests=False)
    assert p.ready()
    for _ in range(2):
        with pytest.raises(RuntimeError, match="failed earlier"):
            p.result()


def test_open_verify_packs_and_reports_device_errors():
    """_edvhost.open_verify (edv.open_batch's one native call): the positional
    sig || msg split of crypto_sign_open before the device call, a list of
    verdicts with False wherever sm is shorter than 64 bytes, and the C-ABI's
    error code handed back as an int (edv.open_batch raises on it).  Driven
    through a C callback standing in for edv_verify_batch (CPU only)."""
    import ctypes
    from indy_plenum_amd import _edvhost
    seen = []
    VER = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                           ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint32)

    def verify(sigs, pks, msgs, off, n, acc, mask):
        o = np.ctypeslib.as_array((ctypes.c_uint64 * (n + 1)).from_address(off)).copy()
        seen.append((ctypes.string_at(sigs, 64 * n), ctypes.string_at(pks, 32 * n),
                     ctypes.string_at(msgs, int(o[-1])), o.tolist(), mask))
        ctypes.memmove(acc, bytes([1, 0, 1][:n]) + bytes(max(0, n - 3)), n)
        return 0
    cb = VER(verify)
    addr = ctypes.cast(cb, ctypes.c_void_p).value
    pk = bytes(range(32))
    items = [(b"\x01" * 64, b"hello", pk),        # plain: sig 64 B
             (b"\x02" * 10, b"\x03" * 20, pk),     # sm < 64: rejected without a device call
             (b"\x04" * 70, b"tail", pk),          # 70-byte "signature": sm[:64], sm[64:]
             (b"\x05" * 64, b"", pk)]
    out = _edvhost.open_verify(items, addr, 3)
    assert out == [True, False, False, True]
    assert len(seen) == 1
    sigs, pks, msgs, off, mask = seen[0]
    assert sigs == b"\x01" * 64 + b"\x04" * 64 + b"\x05" * 64 and pks == pk * 3 and mask == 3
    assert msgs == b"hello" + b"\x04" * 6 + b"tail" and off == [0, 5, 15, 15]
    FAIL = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                            ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint32)(lambda *a: -3)
    assert _edvhost.open_verify(items[:1], ctypes.cast(FAIL, ctypes.c_void_p).value, 0) == -3
    assert _edvhost.open_verify([(b"\x01" * 3, b"", pk)], addr, 0) == [False]   # nothing reaches the device
    with pytest.raises(ValueError):
        _edvhost.open_verify([(b"\x01" * 64, b"", b"\x00" * 31)], addr, 0)
    with pytest.raises(TypeError):
        _edvhost.open_verify([(bytearray(64), b"", pk)], addr, 0)
