"""Kernel time and synchronous call latency against batch size on one MI355X:
why edv_verify_batch splits a batch only into shards of >= 65,536 requests
(one wave per SIMD of the whole chip).  Per n: prep + main HIP-event kernel
times of one device-resident launch pair (median of 10), and the median
wall time of a synchronous edv_verify_batch call from pinned host buffers.
Measurement only."""
import json
import os
import statistics
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from indy_plenum_amd import edv, workload  # noqa: E402

sizes = [int(x) for x in os.environ.get("SIZES", "1,64,400,4096,16384,32768,65536,131072,262144").split(",")]
big = workload.DeviceBatch(max(sizes), keep_host=True)
sigs, pks, msgs, off = big.host_copy()
want = big.expected()
tot = sigs.nbytes + pks.nbytes + off.nbytes + msgs.nbytes + len(want) + 5 * 64
pb = edv.PinnedBuffer(tot)
views, pos = [], 0
for a in (sigs, pks, off, msgs, want):
    v = pb.array[pos:pos + a.nbytes]
    v[:] = a.view(np.uint8)
    views.append(v)
    pos += (a.nbytes + 63) // 64 * 64
ps, pp, po, pm, pa = views
po = po.view(np.uint64)
lib = edv.lib()
for n in sizes:
    pr, mn = [], []
    for _ in range(10):
        p, m = edv.profile_device(big.d_sigs.ptr, big.d_pks.ptr, big.d_msgs.ptr, big.d_off.ptr, n,
                                  big.d_accept.ptr, 0, 1)
        pr.append(p)
        mn.append(m)
    pa[:n] = 0
    edv._check(lib.edv_verify_batch(ps.ctypes.data, pp.ctypes.data, pm.ctypes.data, po.ctypes.data, n,
                                    pa.ctypes.data, 1))
    ok = bool(np.array_equal(pa[:n], want[:n]))
    ts = []
    for _ in range(15):
        t = time.perf_counter()
        edv._check(lib.edv_verify_batch(ps.ctypes.data, pp.ctypes.data, pm.ctypes.data, po.ctypes.data, n,
                                        pa.ctypes.data, 1))
        ts.append(1e3 * (time.perf_counter() - t))
    rec = {"n": n, "prep_ms": statistics.median(pr), "main_ms": statistics.median(mn),
           "kernels_ms": statistics.median(pr) + statistics.median(mn), "sync_call_ms": statistics.median(ts),
           "ok": ok}
    rec["kernel_verifies_per_s"] = n / (rec["kernels_ms"] * 1e-3)
    print(json.dumps(rec), flush=True)
