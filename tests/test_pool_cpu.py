"""Row f-2 harness logic on CPU: a 4-node pool (Alpha..Delta) under a small
client flood orders every valid request exactly once on every node and NACKs
the invalid ones, with one-message-at-a-time verification (the reference's
verifySignature loop) and with prod-batched authenticate_batch (one device call
per prod); the device call is the oracle here (the GPU run is in
tests/test_gpu_authn.py / tools/bench_pool.py)."""
import random

import pytest

import test_authn_host as H
from indy_plenum_amd import edv
from indy_plenum_amd.client_authn import CoreAuthNr
from indy_plenum_amd.pool import Pool, cpu_digests
from indy_plenum_amd.req_authenticator import ReqAuthenticator


def flood(n_valid=60, n_bad_sig=10, n_unknown=5, seed=3):
    r = random.Random(seed)
    signers = [H.Signer(seed=bytes([k + 1]) * 32) for k in range(6)]
    reqs, valid = [], []
    for i in range(n_valid + n_bad_sig + n_unknown):
        s = r.choice(signers)
        req = {"identifier": s.identifier, "reqId": 1539648000000000 + i, "protocolVersion": 2,
               "operation": {"type": "1", "dest": "D%d" % i}}
        if i < n_valid:
            req["signature"] = s.sign(req)
            valid.append(req)
        elif i < n_valid + n_bad_sig:
            req["signature"] = s.sign({**req, "reqId": 7})
        else:
            req["identifier"] = "Unknown%d" % i
            req["signature"] = s.sign(req)
        reqs.append(req)
    r.shuffle(reqs)
    return signers, reqs, valid


def factory(signers):
    def make(_name):
        a = CoreAuthNr()
        for s in signers:
            a.addIdr(s.identifier, s.verkey)
        ra = ReqAuthenticator()
        ra.register_authenticator(a)
        return ra
    return make


@pytest.mark.parametrize("batched,overlap", [(False, False), (True, False), (True, True)])
def test_pool_orders_every_valid_request_once(batched, overlap, monkeypatch):
    calls = []

    def oracle(items, device_mask=0):
        items = list(items)
        calls.append(len(items))
        return H.oracle_open_batch(items)
    monkeypatch.setattr(edv, "open_batch", oracle)
    signers, reqs, valid = flood()
    pool = Pool(factory(signers), n=4, batched=batched, digest_fn=cpu_digests, overlap=overlap, client_quota=16,
                max_batch=7)
    pool.submit(reqs)
    try:
        wall = pool.run(len(valid))
    finally:
        pool.close()
    st = pool.stats(wall, len(valid))
    assert st["ordered_per_node"] == [len(valid)] * 4
    assert st["nacks_per_node"] == [len(reqs) - len(valid)] * 4
    assert st["bad_propagates"] == 0
    keys = [nd.ordered_keys for nd in pool.nodes.values()]
    assert all(k == keys[0] for k in keys) and keys[0] == set(cpu_digests(valid))
    # every node verifies every request once from the client and once per peer's PROPAGATE
    assert st["verifies"] == 4 * len(reqs) + 4 * 3 * len(valid)
    if batched:
        assert st["auth_calls"] < st["verifies"] / 4   # one authenticate_batch per prod


@pytest.mark.parametrize("batched,overlap", [(False, False), (True, False), (True, True)])
def test_pool_stall_raises(batched, overlap, monkeypatch):
    """A pool asked to order more requests than it was given stops with
    RuntimeError after max_idle_rounds idle rounds instead of spinning."""
    monkeypatch.setattr(edv, "open_batch", lambda items, device_mask=0: H.oracle_open_batch(list(items)))
    signers, reqs, valid = flood(n_valid=12, n_bad_sig=3, n_unknown=1, seed=9)
    pool = Pool(factory(signers), n=4, batched=batched, digest_fn=cpu_digests, overlap=overlap, client_quota=16)
    pool.submit(reqs)
    try:
        with pytest.raises(RuntimeError, match="stalled"):
            pool.run(len(valid) + 1, max_idle_rounds=5)
        # nothing is left in flight and every valid request was still ordered once
        assert all(nd._pending is None for nd in pool.nodes.values())
        assert [nd.ordered for nd in pool.nodes.values()] == [len(valid)] * 4
    finally:
        pool.close()


def test_pool_run_ending_with_batches_in_flight(monkeypatch):
    """overlap=True: a run that reaches its target while nodes still hold a
    submitted prod hands those verdicts over in drain() (each message once),
    and the pool then goes on to order the rest."""
    monkeypatch.setattr(edv, "open_batch", lambda items, device_mask=0: H.oracle_open_batch(list(items)))
    signers, reqs, valid = flood()
    pool = Pool(factory(signers), n=4, batched=True, digest_fn=cpu_digests, overlap=True, client_quota=16,
                max_batch=7)
    pool.submit(reqs)
    try:
        pool.run(5)
        assert all(nd._pending is None for nd in pool.nodes.values())
        wall = pool.run(len(valid))
    finally:
        pool.close()
    st = pool.stats(wall, len(valid))
    assert st["ordered_per_node"] == [len(valid)] * 4
    assert st["nacks_per_node"] == [len(reqs) - len(valid)] * 4
    assert st["verifies"] == 4 * len(reqs) + 4 * 3 * len(valid)


@pytest.mark.parametrize("handover", ["early", "next"])
def test_pool_overlap_on_the_native_async_path(monkeypatch, handover):
    """overlap=True through the real native asynchronous path (auth_core_submit /
    auth_core_finish, device digests) with the device calls answered by the
    oracle and hashlib: the same ordered set and NACKs as the reference flow,
    whether a prod's batch is handed over at the end of the same prod (the
    stand-in is done at once, so every prod that submits does) or at the next."""
    from test_host_native import _oracle_async_callbacks, _query_address
    calls = []
    cbs, addrs, issued = _oracle_async_callbacks(calls)
    monkeypatch.setattr(edv, "async_addresses", lambda: addrs)
    monkeypatch.setattr(edv, "query_address", _query_address(cbs))
    monkeypatch.setattr(edv, "BATCH_DEVICE", 0)
    monkeypatch.setattr(edv, "verify_address", lambda: addrs[0])
    monkeypatch.setattr(edv, "_OPEN_BATCH", H.oracle_open_batch)
    monkeypatch.setattr(edv, "open_batch", H.oracle_open_batch)
    signers, reqs, valid = flood()
    pool = Pool(factory(signers), n=4, batched=True, digest_fn=cpu_digests, overlap=True, client_quota=16,
                max_batch=7, handover=handover)
    pool.submit(reqs)
    try:
        wall = pool.run(len(valid))
    finally:
        pool.close()
    st = pool.stats(wall, len(valid))
    assert st["ordered_per_node"] == [len(valid)] * 4
    assert st["nacks_per_node"] == [len(reqs) - len(valid)] * 4
    keys = [nd.ordered_keys for nd in pool.nodes.values()]
    assert all(k == keys[0] for k in keys) and keys[0] == set(cpu_digests(valid))
    assert calls and all(d for _n, d in calls)          # every batch asked for device digests
    assert all(issued)                                  # every queued batch was handed over
    if handover == "early":
        assert st["early_handovers"] == st["auth_calls"]
    else:
        assert st["early_handovers"] == 0


@pytest.mark.parametrize("batched,overlap", [(False, False), (True, True)])
def test_pool_paced_run_records_request_latency(batched, overlap, monkeypatch):
    """run_paced offers the requests at a fixed rate and still orders every valid
    one exactly once; every ordered (request, node) pair gets one Monitor
    latency (forwarded -> ordered), one receipt latency and one submission
    latency, each ordered receipt >= forwarded (a node forwards only requests it
    has read) and submission >= receipt."""
    monkeypatch.setattr(edv, "open_batch", lambda items, device_mask=0: H.oracle_open_batch(list(items)))
    signers, reqs, valid = flood(n_valid=40, n_bad_sig=6, n_unknown=2, seed=11)
    pool = Pool(factory(signers), n=4, batched=batched, digest_fn=cpu_digests, overlap=overlap, client_quota=16,
                max_batch=7)
    try:
        # every request is offered; the run stops once every valid one is ordered
        wall = pool.run_paced(reqs, rate=2000.0, expect=len(valid))
    finally:
        pool.close()
    st = pool.stats(wall, len(valid))
    assert st["ordered_per_node"] == [len(valid)] * 4
    lat = st["latency_ms"]
    for kind in ("monitor", "receipt", "submit"):
        assert lat[kind]["samples"] == 4 * len(valid), kind
        assert 0 <= lat[kind]["p50"] <= lat[kind]["p99"] <= lat[kind]["max"]
    assert lat["receipt"]["mean"] >= lat["monitor"]["mean"]
    assert lat["submit"]["mean"] >= lat["receipt"]["mean"]


@pytest.mark.parametrize("mode", ["sequential", "batched", "overlap_native"])
def test_pool_node_altering_propagates_is_suspected(mode, monkeypatch):
    """The reference's signing test (plenum/test/signing/test_signing.py:30-77:
    evil Alpha with changesRequest, malicious_behaviors_node.py:31-44): every
    PROPAGATE Alpha sends carries its request with a random "amount" in the
    operation.  Each good node authenticates those as
    InsufficientCorrectSignatures(0, 1), suspects Alpha with exactly that reason
    and does not count its vote; every valid request is still ordered on every
    node (the honest nodes' f + 1 PROPAGATEs), and Alpha suspects no one -- one
    message at a time, batched per prod, and overlapped through the native
    asynchronous path (early hand-over)."""
    from indy_plenum_amd.exceptions import InsufficientCorrectSignatures
    monkeypatch.setattr(edv, "open_batch", lambda items, device_mask=0: H.oracle_open_batch(list(items)))
    if mode == "overlap_native":
        from test_host_native import _oracle_async_callbacks, _query_address
        cbs, addrs, _issued = _oracle_async_callbacks([])
        monkeypatch.setattr(edv, "async_addresses", lambda: addrs)
        monkeypatch.setattr(edv, "query_address", _query_address(cbs))
        monkeypatch.setattr(edv, "BATCH_DEVICE", 0)
        monkeypatch.setattr(edv, "verify_address", lambda: addrs[0])
        monkeypatch.setattr(edv, "_OPEN_BATCH", H.oracle_open_batch)
    signers, reqs, valid = flood(n_valid=40, n_bad_sig=6, n_unknown=2, seed=21)
    pool = Pool(factory(signers), n=4, batched=mode != "sequential", digest_fn=cpu_digests,
                overlap=mode == "overlap_native", client_quota=16, max_batch=7, alters_propagates={"Alpha"})
    pool.submit(reqs)
    try:
        wall = pool.run(len(valid))
        for _ in range(20):                                 # let the last PROPAGATEs in flight arrive
            for nd in pool.nodes.values():
                nd.prod(pool)
        pool.drain()
    finally:
        pool.close()
    st = pool.stats(wall, len(valid))
    assert st["ordered_per_node"] == [len(valid)] * 4
    assert st["nacks_per_node"] == [len(reqs) - len(valid)] * 4
    keys = [nd.ordered_keys for nd in pool.nodes.values()]
    assert all(k == keys[0] for k in keys) and keys[0] == set(cpu_digests(valid))
    reason = InsufficientCorrectSignatures.reason.format(0, 1)
    for nd in pool.nodes.values():
        if nd.name == "Alpha":
            assert nd.suspicions == []
        else:   # one altered PROPAGATE per valid request, all from Alpha, all for that reason
            assert nd.suspicions == [("Alpha", reason)] * len(valid), nd.name
    assert st["bad_propagates"] == 3 * len(valid)
