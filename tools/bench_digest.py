"""Row f-3 measurement: batch SHA-256 request digests on one MI355X
(edv_sha256_batch_dev, device-resident NYM-shaped signing bytes) vs hashlib on
the host, same messages.  Prints one JSON line.

Work per message: ceil((m + 9) / 64) SHA-256 compressions; one compression is
counted as 64 rounds x 23 (Sigma1 5, Ch 3, T1 4 adds, Sigma0 5, Maj 4, 2 adds)
+ 48 schedule steps x 13 (sigma0 5, sigma1 5, 3 adds) = 2,096 INT32 ops (the
same accounting style as SURVEY.md section 8d's SHA-512 term).
"""
import hashlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from indy_plenum_amd import edv, workload  # noqa: E402

n = int(os.environ.get("N", 65536))
m = int(os.environ.get("MSG_LEN", 256))
msgs, off = workload.nym_messages(n, msg_len=m)
dm, do, dd = edv.DeviceBuffer(msgs.nbytes), edv.DeviceBuffer(off.nbytes), edv.DeviceBuffer(32 * n)
dm.upload(msgs)
do.upload(off)
for _ in range(3):
    edv.sha256_device(dm.ptr, do.ptr, n, dd.ptr)
iters = 50
s = edv.stream(0)
edv.sync(0)
t0 = time.perf_counter()
for _ in range(iters):
    edv.sha256_device(dm.ptr, do.ptr, n, dd.ptr, stream=s)
edv.sync(0)
dt = (time.perf_counter() - t0) / iters
got = dd.download(32 * n).reshape(n, 32)
k = min(n, 4096)
for i in range(k):
    assert got[i].tobytes() == hashlib.sha256(msgs[off[i]:off[i + 1]].tobytes()).digest()
blocks = (m + 9 + 63) // 64
ops = n * blocks * 2096
t1 = time.perf_counter()
reps = 0
while time.perf_counter() - t1 < 3.0:
    for i in range(n):
        hashlib.sha256(msgs[off[i]:off[i + 1]].tobytes()).digest()
    reps += 1
cpu = reps * n / (time.perf_counter() - t1)
print(json.dumps({"metric": "request digests/s (SHA-256 of signing bytes)", "n": n, "msg_len": m,
                  "value": n / dt, "ms_per_batch": dt * 1e3,
                  "roofline": {"bound": "valu_int32", "achieved_tops": ops / dt / 1e12, "peak_tops": 39.3216,
                               "frac": ops / dt / 39.3216e12, "hbm_bytes": n * (m + 8 + 32),
                               "hbm_gbs": n * (m + 8 + 32) / dt / 1e9},
                  "cpu_baseline": {"value": cpu, "kind": "python hashlib, 1 thread (the reference's per-request call)"}}))
