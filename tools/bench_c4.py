"""Config C4: variable-length requests (200..4096 B) -- verifies/s of the
length-bucketed verify path at a few batch sizes (all-valid synthetic batch,
GPU-signed), timed like bench.py: about a second of back-to-back batches to
bring the clocks up, then 20 back-to-back launches between HIP events
(edv_time_batch_dev), then the prep/main split (edv_profile_batch_dev)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from indy_plenum_amd import edv, workload  # noqa: E402

for n in [int(x) for x in os.environ.get("SIZES", "65536,262144").split(",")]:
    b = workload.DeviceBatch(n, var_range=(200, 4096))
    b.verify()
    assert b.accept().all()
    args = (b.d_sigs.ptr, b.d_pks.ptr, b.d_msgs.ptr, b.d_off.ptr, n, b.d_accept.ptr, 0)
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 1.0:
        edv.time_device(*args, 8)
    ms = edv.time_device(*args, 20) / 20
    p, m = edv.profile_device(*args, 10)
    mean_len = float((b.host_off[1:] - b.host_off[:-1]).mean())
    print(json.dumps({"config": "C4 200..4096 B", "n": n, "mean_msg_len": mean_len, "ms_per_batch": ms,
                      "verifies_per_s": n / (ms * 1e-3), "prep_ms": p, "main_ms": m}), flush=True)
    del b
