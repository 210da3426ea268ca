"""Synchronous edv_verify_batch from host buffers: the field-ordered path
(default for a shard of one chunk: sigs/pks/offsets copied first, the point
sides running while the messages copy, then the hash side and main) against
the one-sub-batch path (EDV_HOST_FIELDS=0: copy everything, then prep, then
main), at C2 (65,536 x 256 B) and C4 (65,536 x 200..4,096 B, 5 % invalid),
pinned and pageable inputs, back to back and 5 ms apart, interleaved over
ROUNDS.  Verdicts checked on every configuration.  Measurement only."""
import json
import os
import statistics
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from indy_plenum_amd import edv, workload  # noqa: E402

R, ROUNDS = int(os.environ.get("R", 15)), int(os.environ.get("ROUNDS", 2))
lib = edv.lib()
s = edv.stream(0)
cfgs = {"C2": dict(), "C4": dict(seed=0xC4C4, var_range=(200, 4096), damage_every=20, damage_kinds=7)}
data = {}
for name, kw in cfgs.items():
    b = workload.DeviceBatch(65536, keep_host=True, **kw)
    sigs, pks, msgs, off = b.host_copy()
    arrs = [sigs, pks, off, msgs]
    pb = edv.PinnedBuffer(sum(a.nbytes for a in arrs) + b.n + 8192)
    views, pos = [], 0
    for a in arrs:
        v = pb.array[pos:pos + a.nbytes]
        v[:] = a.view(np.uint8)
        views.append(v)
        pos += (a.nbytes + 63) // 64 * 64
    ts = []
    for _ in range(R):
        t0 = time.perf_counter()
        b.verify(stream=s)
        edv.sync(0)
        ts.append(time.perf_counter() - t0)
    data[name] = (b, (sigs, pks, msgs, off, np.zeros(b.n, np.uint8)),
                  (views[0], views[1], views[3], views[2].view(np.uint64), pb.array[pos:pos + b.n]), pb,
                  1e3 * statistics.median(ts))


def call(arrs, n):
    sg, pk, ms, of, ac = arrs
    edv._check(lib.edv_verify_batch(sg.ctypes.data, pk.ctypes.data, ms.ctypes.data, of.ctypes.data, n,
                                    ac.ctypes.data, 1))


for rnd in range(ROUNDS):
    for name, (b, page, pin, pb, dev_ms) in data.items():
        want = b.expected()
        for mem, arrs in (("pinned", pin), ("pageable", page)):
            for fields in ("1", "0"):
                os.environ["EDV_HOST_FIELDS"] = fields
                arrs[4][:] = 7
                call(arrs, b.n)
                ok = bool(np.array_equal(arrs[4], want))
                ts, tsp = [], []
                for _ in range(R):
                    t0 = time.perf_counter()
                    call(arrs, b.n)
                    ts.append(1e3 * (time.perf_counter() - t0))
                for _ in range(R):
                    time.sleep(0.005)
                    t0 = time.perf_counter()
                    call(arrs, b.n)
                    tsp.append(1e3 * (time.perf_counter() - t0))
                ok = ok and bool(np.array_equal(arrs[4], want))
                print(json.dumps({"round": rnd, "config": name, "memory": mem,
                                  "path": "fields" if fields == "1" else "one_sub_batch",
                                  "ms": statistics.median(ts), "ms_spaced": statistics.median(tsp),
                                  "device_resident_ms": dev_ms,
                                  "vs_device_resident": dev_ms / statistics.median(ts), "verdicts_ok": ok}),
                      flush=True)
