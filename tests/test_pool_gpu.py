"""Config C5 / row f-2 on the GPU: the 4-node pool harness (Alpha..Delta,
indy-plenum_amd/pool.py) under a client flood with the REAL gfx950 verifier
behind ReqAuthenticator.authenticate_batch (one device call per prod) and GPU
request digests, against the reference's message flow run on the CPU (one
verifySignature per message, the oracle in place of libsodium, hashlib
digests).  Every node must order the same valid set and NACK the same requests.

Reference flow: plenum/server/node.py:1553-1622 (PROPAGATE validation),
:1646-1786 (client REQUEST), :2575-2599 (verifySignature); pool fixture
plenum/test/conftest.py:847-871 (txnPoolNodeSet, 4 nodes in one process).
"""
import pytest

import test_authn_host as H
from test_pool_cpu import factory, flood
from indy_plenum_amd import digest, edv
from indy_plenum_amd.pool import Pool, cpu_digests

pytestmark = pytest.mark.gpu


def _run(signers, reqs, valid, batched, digest_fn, overlap=False):
    pool = Pool(factory(signers), n=4, batched=batched, digest_fn=digest_fn, overlap=overlap, client_quota=50,
                max_batch=40)
    pool.submit(reqs)
    try:
        wall = pool.run(len(valid))
    finally:
        pool.close()
    st = pool.stats(wall, len(valid))
    st["ordered_keys"] = [sorted(nd.ordered_keys) for nd in pool.nodes.values()]
    return st


@pytest.mark.parametrize("overlap", [False, True])
def test_pool_c5_gpu_batched_equals_reference_flow(monkeypatch, overlap):
    assert edv.device_count() >= 1
    signers, reqs, valid = flood(n_valid=400, n_bad_sig=40, n_unknown=20, seed=55)
    with monkeypatch.context() as m:
        m.setattr(edv, "open_batch", H.oracle_open_batch)
        ref = _run(signers, reqs, valid, batched=False, digest_fn=cpu_digests)
    gpu = _run(signers, reqs, valid, batched=True, digest_fn=digest.request_digests, overlap=overlap)
    assert gpu["ordered_per_node"] == ref["ordered_per_node"] == [len(valid)] * 4
    assert gpu["nacks_per_node"] == ref["nacks_per_node"] == [len(reqs) - len(valid)] * 4
    assert gpu["bad_propagates"] == ref["bad_propagates"] == 0
    assert gpu["ordered_keys"] == ref["ordered_keys"]
    assert set(gpu["ordered_keys"][0]) == set(cpu_digests(valid))
    assert gpu["verifies"] == ref["verifies"] == 4 * len(reqs) + 4 * 3 * len(valid)
    assert gpu["auth_calls"] < ref["auth_calls"] / 10    # one authenticate_batch per prod


def _sodium():
    import ctypes
    for path in ("/opt/conda/lib/libsodium.so.23", "libsodium.so.23", "libsodium.so"):
        try:
            lib = ctypes.CDLL(path)
        except OSError:
            continue
        lib.sodium_init()
        return lib
    return None


def _sodium_open_batch(lib):
    """crypto_sign_open(sig + msg, pk) on libsodium 1.0.18 itself (the library
    the oracle is pinned to), same contract as edv.open_batch."""
    import ctypes

    def run(items, device_mask=0):
        out = []
        for s, m, p in items:
            sm = bytes(s) + bytes(m)
            buf = ctypes.create_string_buffer(len(sm))
            mlen = ctypes.c_ulonglong(0)
            out.append(lib.crypto_sign_open(buf, ctypes.byref(mlen), sm, ctypes.c_ulonglong(len(sm)), bytes(p)) == 0)
        return out
    return run


@pytest.mark.parametrize("overlap", [False, True])
def test_pool_c5_gpu_large_flood_equals_reference_flow(monkeypatch, overlap):
    """The same check on a flood ten times larger (3,250 requests, 52,000
    verifies per run), the reference flow's verifies on libsodium itself."""
    lib = _sodium()
    if lib is None:
        pytest.skip("libsodium not present")
    assert edv.device_count() >= 1
    signers, reqs, valid = flood(n_valid=3000, n_bad_sig=200, n_unknown=50, seed=56)
    with monkeypatch.context() as m:
        m.setattr(edv, "open_batch", _sodium_open_batch(lib))
        ref = _run(signers, reqs, valid, batched=False, digest_fn=cpu_digests)
    gpu = _run(signers, reqs, valid, batched=True, digest_fn=digest.request_digests, overlap=overlap)
    assert gpu["ordered_per_node"] == ref["ordered_per_node"] == [len(valid)] * 4
    assert gpu["nacks_per_node"] == ref["nacks_per_node"] == [len(reqs) - len(valid)] * 4
    assert gpu["bad_propagates"] == ref["bad_propagates"] == 0
    assert gpu["ordered_keys"] == ref["ordered_keys"]
    assert gpu["verifies"] == ref["verifies"] == 4 * len(reqs) + 4 * 3 * len(valid)


@pytest.mark.parametrize("overlap", [False, True])
def test_pool_gpu_node_altering_propagates_is_suspected(monkeypatch, overlap):
    """The reference's signing test on the GPU path (plenum/test/signing/
    test_signing.py:30-77, changesRequest): Alpha alters the request in every
    PROPAGATE it sends; the GPU-authenticated good nodes raise
    InsufficientCorrectSignatures(0, 1) for each, suspect Alpha for that reason
    and still order every valid request -- the same ordered set, NACKs and
    suspicions as the reference flow (one verifySignature per message on the
    oracle)."""
    from indy_plenum_amd.exceptions import InsufficientCorrectSignatures
    signers, reqs, valid = flood(n_valid=300, n_bad_sig=30, n_unknown=10, seed=77)

    def run(batched, digest_fn, overlap=False):
        pool = Pool(factory(signers), n=4, batched=batched, digest_fn=digest_fn, overlap=overlap, client_quota=50,
                    max_batch=40, alters_propagates={"Alpha"})
        pool.submit(reqs)
        try:
            wall = pool.run(len(valid))
            for _ in range(20):
                for nd in pool.nodes.values():
                    nd.prod(pool)
            pool.drain()
        finally:
            pool.close()
        st = pool.stats(wall, len(valid))
        st["ordered_keys"] = [sorted(nd.ordered_keys) for nd in pool.nodes.values()]
        st["suspicions"] = {nd.name: sorted(nd.suspicions) for nd in pool.nodes.values()}
        return st
    with monkeypatch.context() as m:
        m.setattr(edv, "open_batch", H.oracle_open_batch)
        ref = run(False, cpu_digests)
    gpu = run(True, digest.request_digests, overlap)
    assert gpu["ordered_per_node"] == ref["ordered_per_node"] == [len(valid)] * 4
    assert gpu["nacks_per_node"] == ref["nacks_per_node"]
    assert gpu["ordered_keys"] == ref["ordered_keys"]
    assert set(gpu["ordered_keys"][0]) == set(cpu_digests(valid))
    reason = InsufficientCorrectSignatures.reason.format(0, 1)
    assert gpu["suspicions"] == ref["suspicions"]
    assert gpu["suspicions"]["Alpha"] == []
    for name in ("Beta", "Gamma", "Delta"):
        assert gpu["suspicions"][name] == [("Alpha", reason)] * len(valid)
