"""Timeline of synchronous edv_verify_batch calls on pinned host buffers (C2),
for rocprofv3 --kernel-trace --memory-copy-trace: 20 calls, 5 ms apart, so each
call's copies and kernels can be told apart in the trace.  Measurement only."""
import time

import numpy as np

import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from indy_plenum_amd import edv, workload  # noqa: E402

b = workload.DeviceBatch(65536, keep_host=True)
sigs, pks, msgs, off = b.host_copy()
n = b.n
sizes = [sigs.nbytes, pks.nbytes, off.nbytes, msgs.nbytes, n]
pb = edv.PinnedBuffer(sum(sizes) + 5 * 64)
views, pos = [], 0
for a, sz in zip((sigs, pks, off, msgs, None), sizes):
    v = pb.array[pos:pos + sz]
    if a is not None:
        v[:] = a.view(np.uint8)
    views.append(v)
    pos += (sz + 63) // 64 * 64
ps, pp, po, pm, pa = views
po = po.view(np.uint64)
lib = edv.lib()
ts = []
for k in range(25):
    t = time.perf_counter()
    edv._check(lib.edv_verify_batch(ps.ctypes.data, pp.ctypes.data, pm.ctypes.data, po.ctypes.data, n,
                                    pa.ctypes.data, 1))
    ts.append(time.perf_counter() - t)
    time.sleep(0.005)
print("call ms median", 1e3 * sorted(ts)[len(ts) // 2], "ok", bool(np.array_equal(pa, b.expected())))
