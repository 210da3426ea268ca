"""Why is the main kernel slower at C4 than at C2?  Same profile method
(edv_profile_batch_dev, prep then main, HIP events, 10 iterations) on:
C2 (256 B), C2 with buckets forced, C4 (200..4096 B) bucketed, C4 unbucketed,
and fixed 2,143 B messages (C4's mean length, no buckets)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from indy_plenum_amd import edv, workload  # noqa: E402

n = 65536
cases = [("c2", dict(), 0), ("c2_bucketed", dict(), 1), ("c4_bucketed", dict(var_range=(200, 4096)), 1),
         ("c4_unbucketed", dict(var_range=(200, 4096)), 0), ("fixed_2143", dict(msg_len=2143), 0)]
for tag, kw, mode in cases:
    b = workload.DeviceBatch(n, **kw)
    edv.set_length_buckets(0, mode)
    b.verify()
    edv.sync(0)
    assert b.accept().all()
    p, m = edv.profile_device(b.d_sigs.ptr, b.d_pks.ptr, b.d_msgs.ptr, b.d_off.ptr, n, b.d_accept.ptr, 0, 10)
    print(json.dumps({"case": tag, "bucket_mode": mode, "prep_ms": p, "main_ms": m}), flush=True)
    del b
edv.set_length_buckets(0, 2)
