"""Rows f-1/C1: end-to-end request authentication throughput on one MI355X.

N NYM-style requests (config C1 shape: identifier = b58(pk[:16]), verkey
'~' + b58(pk[16:]) registered with the authenticator, signed over the
SigningSerializer bytes) go through CoreAuthNr.authenticate_batch: host prep
(base58, DID expansion, serialisation, packing), one GPU verify, replay.
Reported: requests/s with the native host prep (_edvhost) and with the pure
Python restatement, the phase split, and the reference's own CPU chain
(sequential authenticate per request, Python + libsodium crypto_sign_open via
ctypes, i.e. what libnacl does) timed on the same host, 1 thread like the
Node's Looper.  Keys/signatures come from the GPU batch signer.
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from indy_plenum_amd import base58, edv, signing_serializer  # noqa: E402
from indy_plenum_amd.client_authn import CoreAuthNr  # noqa: E402
from indy_plenum_amd.signing_serializer import serialize_msg_for_signing  # noqa: E402

N = int(os.environ.get("N", 10000))
rng = np.random.default_rng(0xC1)
seeds = rng.integers(0, 256, size=(N, 32), dtype=np.uint8)
off0 = np.zeros(N + 1, dtype=np.uint64)
pks, _ = edv.sign_arrays(seeds.tobytes(), b"\0" * 64, off0)
pks = np.frombuffer(pks, np.uint8).reshape(N, 32)
auth = CoreAuthNr()
reqs = []
for i in range(N):
    pk = pks[i].tobytes()
    idr = base58.b58encode(pk[:16]).decode()
    auth.addIdr(idr, "~" + base58.b58encode(pk[16:]).decode())
    reqs.append({"identifier": idr, "reqId": 1539648000000000 + i, "protocolVersion": 2,
                 "operation": {"type": "1", "dest": base58.b58encode(rng.bytes(16)).decode(),
                               "verkey": "~" + base58.b58encode(rng.bytes(16)).decode()}})
sers = [serialize_msg_for_signing(r) for r in reqs]
off = np.zeros(N + 1, dtype=np.uint64)
off[1:] = np.cumsum([len(s) for s in sers])
_, sigs = edv.sign_arrays(seeds.tobytes(), b"".join(sers) + b"\0" * 64, off)
sigs = sigs.tobytes()
for i, r in enumerate(reqs):
    r["signature"] = base58.b58encode(sigs[64 * i:64 * i + 64]).decode()


def run_batch():
    t0 = time.perf_counter()
    res = auth.authenticate_batch(reqs)
    dt = time.perf_counter() - t0
    assert all(isinstance(x, list) and x == [r["identifier"]] for x, r in zip(res, reqs))
    return dt


def phases():
    """host prep / device / replay split of one authenticate_batch call."""
    t = {}
    real = edv.open_batch

    def timed(items, device_mask=0):
        t["prep_done"] = time.perf_counter()
        out = real(items, device_mask)
        t["gpu_done"] = time.perf_counter()
        return out
    edv.open_batch = timed
    try:
        t0 = time.perf_counter()
        auth.authenticate_batch(reqs)
        t1 = time.perf_counter()
    finally:
        edv.open_batch = real
    return {"host_prep_s": t["prep_done"] - t0, "verify_call_s": t["gpu_done"] - t["prep_done"],
            "replay_s": t1 - t["gpu_done"]}


def run_req_authenticator():
    from indy_plenum_amd.req_authenticator import ReqAuthenticator
    ra = ReqAuthenticator()
    ra.register_authenticator(auth)
    t0 = time.perf_counter()
    res = ra.authenticate_batch(reqs)
    dt = time.perf_counter() - t0
    assert all(x == {r["identifier"]} for x, r in zip(res, reqs))
    return dt


run_batch()
native = min(run_batch() for _ in range(3))
native_ra = min(run_req_authenticator() for _ in range(3))
ph_native = phases()
base58._native = signing_serializer._native = None  # force the Python restatements
python_prep = min(run_batch() for _ in range(2))
ph_python = phases()

# the reference's CPU chain: Python + libsodium per request (crypto_sign_open(sig + msg, pk))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import sodium_ref  # noqa: E402
cpu = None
if sodium_ref.sodium() is not None:
    k = min(N, 3000)
    cpu_auth = CoreAuthNr()
    cpu_auth.clients = auth.clients
    t0 = time.perf_counter()
    for r in reqs[:k]:
        assert cpu_auth.authenticate(r, verifier=sodium_ref.SodiumVerifier) == [r["identifier"]]
    cpu = k / (time.perf_counter() - t0)

print(json.dumps({"metric": "authenticated NYM requests/s (CoreAuthNr.authenticate_batch, 1 GPU)", "n": N,
                  "native_prep_req_per_s": N / native,
                  "req_authenticator_native_req_per_s": N / native_ra, "python_prep_req_per_s": N / python_prep,
                  "phases_native": ph_native, "phases_python": ph_python,
                  "cpu_reference_chain_req_per_s": cpu,
                  "cpu_reference_chain": "sequential CoreAuthNr.authenticate, Python restatement + libsodium "
                                         "crypto_sign_open via ctypes, 1 thread (native base58/serializer off)"}))
