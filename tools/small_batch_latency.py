"""Latency of Node-sized batches (1 .. 4,096 requests of 256 B) on one MI355X
from pinned host buffers: a synchronous edv_verify_batch call, and an
edv_verify_batch_async submission + edv_wait_async.  Median of R calls;
verdicts checked.  Measurement only.  (Round 4 also timed a zero-copy input
mode, profiles/r04/small_batch_latency_s2.jsonl; it was removed.)
"""
import json
import os
import statistics
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from indy_plenum_amd import edv, workload  # noqa: E402

R = int(os.environ.get("R", 51))
sizes = [int(x) for x in os.environ.get("SIZES", "1,64,400,4096").split(",")]
big = workload.DeviceBatch(max(sizes), keep_host=True, damage_every=7)
sigs, pks, msgs, off = big.host_copy()
want = big.expected()
arrs = [sigs, pks, off, msgs]
tot = sum(a.nbytes for a in arrs) + max(sizes) + 8192
pb = edv.PinnedBuffer(tot)
views, pos = [], 0
for a in arrs:
    v = pb.array[pos:pos + a.nbytes]
    v[:] = a.view(np.uint8)
    views.append(v)
    pos += (a.nbytes + 4095) // 4096 * 4096
ps, pp, po, pm = views
po = po.view(np.uint64)
pa = pb.array[pos:pos + max(sizes)]
lib = edv.lib()


def med(f):
    ts = []
    for _ in range(R):
        t = time.perf_counter()
        f()
        ts.append(1e3 * (time.perf_counter() - t))
    return statistics.median(ts)


for n in sizes:
    o = po[:n + 1]
    if True:
        def sync():
            edv._check(lib.edv_verify_batch(ps.ctypes.data, pp.ctypes.data, pm.ctypes.data, o.ctypes.data, n,
                                            pa.ctypes.data, 1))

        def asyn():
            t = edv.verify_async(ps[:64 * n], pp[:32 * n], pm, o, pa[:n], device=0)
            edv.wait_async(t, device=0)
        pa[:] = 2
        sync()
        ok_s = bool(np.array_equal(pa[:n], want[:n]))
        pa[:] = 2
        asyn()
        ok_a = bool(np.array_equal(pa[:n], want[:n]))
        rec = {"n": n, "sync_ms": med(sync), "async_ms": med(asyn), "ok": ok_s and ok_a}
        print(json.dumps(rec), flush=True)
