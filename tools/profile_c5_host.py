"""C5's host side on the CPU: the 4-node pool (overlap mode, the native
asynchronous authentication path) with the device calls answered at once by C
stand-ins (tools/c5_standin.c: every request accepted, request digests by the
kernel's SHA-256 compiled for the CPU, their time taken out), so what is
timed is only the host work per request: phases A-D of the native path, the
Python around it and the pool itself.  Prints the auth share of node time and,
with --profile, the cProfile top entries.  Harness only (no GPU, no verify).

  python tools/profile_c5_host.py [n_requests] [--profile]
  python tools/profile_c5_host.py --submit     (the native submission alone, by batch size)
"""
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from indy_plenum_amd import base58, edv  # noqa: E402
from indy_plenum_amd.client_authn import CoreAuthNr  # noqa: E402
from indy_plenum_amd.pool import Pool  # noqa: E402
from indy_plenum_amd.req_authenticator import ReqAuthenticator  # noqa: E402



def standin():
    """Build tools/c5_standin.c (stand-in device calls, all C) into a temp dir
    and wire the hostcheck library's SHA-256 batch into it."""
    import subprocess
    import tempfile
    out = os.path.join(tempfile.mkdtemp(prefix="c5standin"), "libc5standin.so")
    subprocess.run(["gcc", "-O2", "-shared", "-fPIC", "-o", out, os.path.join(ROOT, "tools", "c5_standin.c")],
                   check=True)
    lib = ctypes.CDLL(out)
    hc = ctypes.CDLL(os.path.join(ROOT, "indy-plenum_amd", "libedv_hostcheck.so"))
    lib.standin_set_sha256(ctypes.cast(hc.hc_sha256_batch, ctypes.c_void_p))
    lib.standin_seconds.restype = ctypes.c_double
    lib._hc = hc
    return lib


SI = standin()
ADDRS = tuple(ctypes.cast(getattr(SI, f), ctypes.c_void_p).value for f in ("standin_submit", "standin_wait"))
QUERY = ctypes.cast(SI.standin_query, ctypes.c_void_p).value


def flood(n, seed=0xC5):
    rng = np.random.default_rng(seed)
    clients, reqs = {}, []
    for i in range(n):
        pk = rng.bytes(32)
        idr = base58.b58encode(pk[:16]).decode()
        clients[idr] = "~" + base58.b58encode(pk[16:]).decode()
        reqs.append({"identifier": idr, "reqId": 1539648000000000 + i, "protocolVersion": 2,
                     "operation": {"type": "1", "dest": base58.b58encode(rng.bytes(16)).decode(),
                                   "verkey": "~" + base58.b58encode(rng.bytes(16)).decode()},
                     "signature": base58.b58encode(rng.bytes(64)).decode()})
    return clients, reqs


def factory(clients):
    def make(_name):
        a = CoreAuthNr()
        for idr, vk in clients.items():
            a.addIdr(idr, vk)
        ra = ReqAuthenticator()
        ra.register_authenticator(a)
        return ra
    return make


def run(clients, reqs):
    pool = Pool(factory(clients), n=4, batched=True, overlap=True)
    pool.submit(reqs)
    SI.standin_reset()
    try:
        wall = pool.run(len(reqs))
    finally:
        pool.close()
    st = pool.stats(wall, len(reqs))
    nodes = list(pool.nodes.values())
    cb = SI.standin_seconds()
    auth = sum(nd.auth_s for nd in nodes) - cb
    busy = sum(nd.busy_s for nd in nodes) - cb
    st["auth_share_of_node_time"] = auth / busy
    st["auth_share_excluding_gc"] = (auth - pool.gc_clock.in_auth_s) / (busy - pool.gc_clock.total_s)
    st["gc_share_of_node_time"] = pool.gc_clock.total_s / busy
    st["host_auth_us_per_verify"] = 1e6 * auth / st["verifies"]
    st["stand_in_device_s"] = cb
    st["ordered_req_per_s_one_process"] = len(reqs) / (wall - cb)
    return st


def submit_bench(batch, n=4000, reps=20):
    """The native submission alone (_edvhost.req_auth_submit + req_auth_finish)
    over warm requests in batches of `batch`: microseconds per request."""
    from indy_plenum_amd.client_authn import _edvhost
    from indy_plenum_amd.exceptions import InsufficientCorrectSignatures, NoAuthenticatorFound
    clients, reqs = flood(n)
    a = CoreAuthNr()
    for idr, vk in clients.items():
        a.addIdr(idr, vk)
    cls = type(a)
    batches = [reqs[i:i + batch] for i in range(0, n, batch)]
    best = None
    for _ in range(3):
        ts = tf = 0.0
        SI.standin_reset()
        for _ in range(reps):
            for b in batches:
                t = time.perf_counter()
                h = _edvhost.req_auth_submit(b, a.clients, a.excluded_from_signing, ADDRS[0], ADDRS[1], 0,
                                             edv.PREP_THREADS, None, True, (a.query_types, a.write_types,
                                                                            cls.action_types))
                t1 = time.perf_counter()
                _edvhost.req_auth_finish(h, NoAuthenticatorFound, InsufficientCorrectSignatures)
                tf += time.perf_counter() - t1
                ts += t1 - t
        r = {"batch": batch, "submit_us_per_req": 1e6 * (ts - SI.standin_seconds()) / (reps * n),
             "finish_us_per_req": 1e6 * tf / (reps * n)}
        if best is None or r["submit_us_per_req"] < best["submit_us_per_req"]:
            best = r
    return best


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 and sys.argv[1].isdigit() else 20000
    edv.async_addresses = lambda: ADDRS
    edv.BATCH_DEVICE = 0
    edv.verify_address = lambda: ADDRS[0]
    edv.native_batch_enabled = lambda: True
    edv.query_address = lambda: QUERY
    if "--submit" in sys.argv:
        for b in (100, 400, 1000, 4000):
            print(json.dumps(submit_bench(b)))
        return
    clients, reqs = flood(n)
    run(clients, reqs[:500])
    if "--profile" in sys.argv:
        import cProfile
        import pstats
        pr = cProfile.Profile()
        pr.enable()
        st = run(clients, reqs)
        pr.disable()
        pstats.Stats(pr).sort_stats("tottime").print_stats(25)
    else:
        t = time.perf_counter()
        st = run(clients, reqs)
        st["total_s"] = time.perf_counter() - t
    keep = ("ordered_req_per_s_one_process", "auth_share_of_node_time", "auth_share_excluding_gc",
            "gc_share_of_node_time", "host_auth_us_per_verify", "verifies",
            "auth_calls", "wall_s", "stand_in_device_s")
    print(json.dumps({k: st[k] for k in keep}))


if __name__ == "__main__":
    main()
