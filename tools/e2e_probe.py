"""Host-path (edv_verify_batch on host buffers) timing breakdown on one GPU:
raw pinned H2D of the batch bytes, then the verify call from pageable and from
pinned inputs for EDV_HOST_PARTS = 1, 2, 3, 4 (split-prep parts; 1 = one
sub-batch: copy, prep, main in sequence), median of 7."""
import json
import os
import statistics
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from indy_plenum_amd import edv, workload  # noqa: E402

n = int(os.environ.get("N", 65536))
b = workload.DeviceBatch(n)
sigs, pks, msgs, off = b.host_copy()
acc = np.zeros(n, np.uint8)


def med(f, r=7):
    ts = []
    for _ in range(r):
        t0 = time.perf_counter()
        f()
        ts.append(time.perf_counter() - t0)
    return 1e3 * statistics.median(ts)


def call(s, p, m, o, a):
    edv._check(edv.lib().edv_verify_batch(s.ctypes.data, p.ctypes.data, m.ctypes.data, o.ctypes.data, n,
                                          a.ctypes.data, 1))


parts = [sigs, pks, off.view(np.uint8), msgs]
pb = edv.PinnedBuffer(sum(p.nbytes for p in parts) + 4 * 64 + n)
pos, views = 0, []
for p in parts:
    v = pb.array[pos:pos + p.nbytes]
    v[:] = p
    views.append(v)
    pos += (p.nbytes + 63) // 64 * 64
pacc = pb.array[pos:pos + n]
total = sum(p.nbytes for p in parts)
d = edv.DeviceBuffer(total)
out = {"n": n, "bytes": total,
       "raw_h2d_pinned_ms": med(lambda: edv._check(edv.lib().edv_h2d(0, d.ptr, pb.ptr, total))),
       "raw_h2d_pageable_ms": med(lambda: d.upload(np.concatenate([p.view(np.uint8) for p in parts])))}
s = edv.stream(0)
out["device_resident_ms"] = med(lambda: (b.verify(stream=s), edv.sync(0)))
for q in (1, 2, 3, 4):
    os.environ["EDV_HOST_PARTS"] = str(q)
    call(sigs, pks, msgs, off, acc)
    out["pageable_q%d_ms" % q] = med(lambda: call(sigs, pks, msgs, off, acc))
    call(views[0], views[1], views[3], views[2].view(np.uint64), pacc)
    out["pinned_q%d_ms" % q] = med(lambda: call(views[0], views[1], views[3], views[2].view(np.uint64), pacc))
    assert acc.all() and pacc.all()
print(json.dumps(out))
