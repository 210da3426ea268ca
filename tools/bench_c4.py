"""Config C4: variable-length requests (200..4096 B) -- prep/main kernel times
and verifies/s at a few batch sizes (all-valid synthetic batch, GPU-signed)."""
import os, sys, json
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from indy_plenum_amd import edv, workload
for n in [int(x) for x in os.environ.get("SIZES", "65536,262144").split(",")]:
    b = workload.DeviceBatch(n, var_range=(200, 4096))
    b.verify()
    assert b.accept().all()
    edv.sync(0)
    p, m = edv.profile_device(b.d_sigs.ptr, b.d_pks.ptr, b.d_msgs.ptr, b.d_off.ptr, n, b.d_accept.ptr, 0, 5)
    mean_len = float((b.host_off[1:] - b.host_off[:-1]).mean())
    print(json.dumps({"config": "C4 200..4096 B", "n": n, "mean_msg_len": mean_len, "prep_ms": p, "main_ms": m,
                      "verifies_per_s_kernels": n / ((p + m) * 1e-3)}), flush=True)
    del b
