"""Synchronous edv_verify_batch on pinned host buffers at C2 (65,536 x 256 B):
one sub-batch (the default) against Q sub-batches on Q streams, plain or each
confined to its own 1/Q of the CUs (EDV_HOST_CUMASK modes 1-3, see
host_streams in csrc/edv_verify.hip), and the zero-copy form (cfg suffix :z,
EDV_ZERO_COPY: the kernels read the pinned inputs over the link, no H2D copy).  Median of R calls back to back, and of
R calls 5 ms apart (the GPU idles in between, as a Node's calls would).
Verdicts checked on every configuration.  Measurement only.(The CU-mask and zero-copy knobs were removed from the library after this
measurement, profiles/r04/e2e_sync_variants_s2.jsonl; with HEAD they are ignored.)
"""
import json
import os
import statistics
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from indy_plenum_amd import edv, workload  # noqa: E402

n = int(os.environ.get("N", 65536))
R = int(os.environ.get("R", 21))
b = workload.DeviceBatch(n, keep_host=True)
sigs, pks, msgs, off = b.host_copy()
want = b.expected()
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


def call():
    edv._check(lib.edv_verify_batch(ps.ctypes.data, pp.ctypes.data, pm.ctypes.data, po.ctypes.data, n,
                                    pa.ctypes.data, 1))


s = edv.stream(0)
dev_ms = []
for _ in range(R):
    t = time.perf_counter()
    b.verify(stream=s)
    edv.sync(0)
    dev_ms.append(1e3 * (time.perf_counter() - t))
out = {"n": n, "device_resident_ms": statistics.median(dev_ms), "configs": []}
cfgs = os.environ.get("CFGS", "1:0,1:0:z,4:0,2:1,4:1,4:2,4:3,2:3,1:0,1:0:z").split(",")
for cfg in cfgs:
    parts = cfg.split(":")
    q, m = int(parts[0]), int(parts[1])
    zc = len(parts) > 2 and parts[2] == "z"
    os.environ["EDV_HOST_STREAMS"] = str(q)
    os.environ["EDV_HOST_CUMASK"] = str(m)
    if zc:
        os.environ["EDV_ZERO_COPY"] = "1"
    else:
        os.environ.pop("EDV_ZERO_COPY", None)
    pa[:] = 0
    call()
    ok = bool(np.array_equal(pa, want))
    ts = []
    for _ in range(R):
        t = time.perf_counter()
        call()
        ts.append(1e3 * (time.perf_counter() - t))
    ts_idle = []
    for _ in range(R):
        time.sleep(0.005)
        t = time.perf_counter()
        call()
        ts_idle.append(1e3 * (time.perf_counter() - t))
    rec = {"streams": q, "cumask": m, "zero_copy": zc, "ok": ok and bool(np.array_equal(pa, want)),
           "ms": statistics.median(ts), "ms_min": min(ts), "ms_spaced": statistics.median(ts_idle)}
    out["configs"].append(rec)
    print(json.dumps(rec), flush=True)
print(json.dumps(out))
