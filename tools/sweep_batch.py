"""Throughput vs batch size (occupancy) on one GPU: per-kernel HIP-event times."""
import os, sys, json
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from indy_plenum_amd import edv, workload
sizes = [int(x) for x in os.environ.get("SIZES", "16384,65536,131072,262144").split(",")]
for n in sizes:
    b = workload.DeviceBatch(n)
    b.verify()
    assert b.accept().all()
    p, m = edv.profile_device(b.d_sigs.ptr, b.d_pks.ptr, b.d_msgs.ptr, b.d_off.ptr, n, b.d_accept.ptr, 0, 5)
    print(json.dumps({"n": n, "prep_ms": p, "main_ms": m, "verifies_per_s_kernels": n / ((p + m) * 1e-3),
                      "main_only_per_s": n / (m * 1e-3)}), flush=True)
    del b
