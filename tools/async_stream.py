"""Back-to-back edv_verify_batch_async from pinned host buffers (the product's
stream-of-batches boundary) at C2 (65,536 x 256 B) and C4 (65,536 x 200..4,096
B, 5 % invalid): a stream of K batches, waiting one batch behind, per-batch
time as the median of R streams; EDV_ASYNC_SPLIT unset (auto: the split
pipeline from a mean of 6 SHA-512 blocks), 0 (off) and 1 (on); verdicts checked
on every stream.  Also the device-resident sequential step for reference.
Measurement only.(EDV_ASYNC_SPLIT was removed from the library after this measurement,
profiles/r04/async_stream_s13.jsonl; with HEAD all three rows take the ordinary path.)
"""
import json
import os
import statistics
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from indy_plenum_amd import edv, workload  # noqa: E402

K, R = int(os.environ.get("K", 32)), int(os.environ.get("R", 5))
dev = 0
s = edv.stream(dev)
cfgs = {"C2": dict(), "C4": dict(seed=0xC4C4, var_range=(200, 4096), damage_every=20, damage_kinds=7)}
for name, kw in cfgs.items():
    b = workload.DeviceBatch(65536, device=dev, keep_host=True, **kw)
    sigs, pks, msgs, off = b.host_copy()
    want = b.expected()
    n = b.n
    arrs = [sigs, pks, off, msgs]
    pb = edv.PinnedBuffer(sum(a.nbytes for a in arrs) + 2 * n + 8192)
    views, pos = [], 0
    for a in arrs:
        v = pb.array[pos:pos + a.nbytes]
        v[:] = a.view(np.uint8)
        views.append(v)
        pos += (a.nbytes + 63) // 64 * 64
    ps, pp, po, pm = views
    po = po.view(np.uint64)
    accs = (pb.array[pos:pos + n], pb.array[pos + n:pos + 2 * n])
    reps = []
    for _ in range(R):
        t0 = time.perf_counter()
        b.verify(stream=s)
        edv.sync(dev)
        reps.append(time.perf_counter() - t0)
    dev_ms = 1e3 * statistics.median(reps)

    def stream():
        prev = None
        for k in range(K):
            t = edv.verify_async(ps, pp, pm, po, accs[k % 2], device=dev)
            if prev is not None:
                edv.wait_async(prev, device=dev)
            prev = t
        edv.wait_async(prev, device=dev)
    for mode in (None, "0", "1"):
        if mode is None:
            os.environ.pop("EDV_ASYNC_SPLIT", None)
        else:
            os.environ["EDV_ASYNC_SPLIT"] = mode
        for a in accs:
            a[:] = 7
        stream()
        ok = all(bool(np.array_equal(a, want)) for a in accs)
        ts = []
        for _ in range(R):
            t0 = time.perf_counter()
            stream()
            ts.append((time.perf_counter() - t0) / K)
        ms = 1e3 * statistics.median(ts)
        print(json.dumps({"config": name, "async_split": mode or "auto", "ms_per_batch": ms,
                          "verifies_per_s": n / (ms * 1e-3), "device_resident_seq_ms": dev_ms,
                          "verdicts_ok": ok}), flush=True)
    pb.free()
