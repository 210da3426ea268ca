"""Back-to-back edv_verify_batch_async from pinned host buffers (the product's
stream-of-batches boundary) at C2 (65,536 x 256 B) and C4 (65,536 x
200..4,096 B, 5 % invalid): a stream of K batches waiting one batch behind,
per-batch time as the median of R streams, next to the device-resident
sequential step; verdicts checked on every stream (PAGEABLE=1: from the
caller's pageable numpy arrays instead).  With library paths as
arguments, each .so (EDV_LIB) runs in its own process, in the order given
(A B A B interleaves them).  Measurement only.

  python tools/async_stream.py [lib.so ...]
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r"""
import json, os, statistics, sys, time
import numpy as np
sys.path.insert(0, os.environ["ROOT"])
from indy_plenum_amd import edv, workload
K, R = int(os.environ.get("K", 32)), int(os.environ.get("R", 5))
dev = 0
s = edv.stream(dev)
cfgs = {"C2": dict(), "C4": dict(seed=0xC4C4, var_range=(200, 4096), damage_every=20, damage_kinds=7)}
for name in os.environ.get("CFGS", "C2,C4").split(","):
    kw = cfgs[name]
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
    pageable = os.environ.get("PAGEABLE") == "1"
    if pageable:  # the caller's own (pageable) numpy buffers: staged by the library
        ps, pp, pm, po = sigs, pks, msgs, off
        accs = (np.zeros(n, np.uint8), np.zeros(n, np.uint8))
    reps = []
    for _ in range(R):
        t0 = time.perf_counter()
        for _ in range(K):
            b.verify(stream=s)
        edv.sync(dev)
        reps.append((time.perf_counter() - t0) / K)
    dev_ms = 1e3 * statistics.median(reps)

    def stream():
        prev = None
        for k in range(K):
            t = edv.verify_async(ps, pp, pm, po, accs[k % 2], device=dev)
            if prev is not None:
                edv.wait_async(prev, device=dev)
            prev = t
        edv.wait_async(prev, device=dev)
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
    print(json.dumps({"lib": os.path.basename(os.environ.get("EDV_LIB", "libedv.so")), "config": name,
                      "inputs": "pageable" if pageable else "pinned",
                      "ms_per_batch": ms, "verifies_per_s": n / (ms * 1e-3), "device_resident_seq_ms": dev_ms,
                      "async_vs_device_resident": dev_ms / ms, "verdicts_ok": ok}), flush=True)
    pb.free()
"""
libs = sys.argv[1:] or [os.path.join(ROOT, "indy-plenum_amd", "libedv.so")]
for lib in libs:
    env = dict(os.environ, EDV_LIB=os.path.abspath(lib), ROOT=ROOT)
    r = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=600)
    print(r.stdout.strip() if r.returncode == 0 else json.dumps({"lib": lib, "error": r.stderr[-800:]}), flush=True)
