"""A/B timing of library variants on one GPU: for each .so (EDV_LIB), in its own
process, the per-kernel HIP-event times (prep, main) at the given batch sizes and
the sequential device-resident step time at 64k (median of 5 x 20 steps).

  python tools/ab_bench.py indy-plenum_amd/libedv.so indy-plenum_amd/variants/libedv_X.so ...
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r"""
import json, os, statistics, sys, time
sys.path.insert(0, os.environ["ROOT"])
from indy_plenum_amd import edv, workload
out = {"lib": os.environ["EDV_LIB"]}
for n in [int(x) for x in os.environ.get("SIZES", "65536,262144").split(",")]:
    b = workload.DeviceBatch(n)
    b.verify()
    if os.environ.get("AB_NO_CHECK") != "1":
        assert b.accept().all()
    p, m = edv.profile_device(b.d_sigs.ptr, b.d_pks.ptr, b.d_msgs.ptr, b.d_off.ptr, n, b.d_accept.ptr, 0, 10)
    out["n%d" % n] = {"prep_ms": p, "main_ms": m}
    if n == 65536:
        s = edv.stream(0)
        for _ in range(200):
            b.verify(stream=s)
        edv.sync(0)
        reps = []
        for _ in range(5):
            t0 = time.perf_counter()
            for _ in range(20):
                b.verify(stream=s)
            edv.sync(0)
            reps.append((time.perf_counter() - t0) / 20)
        out["step_ms_64k"] = 1e3 * statistics.median(reps)
    del b
print(json.dumps(out))
"""
for lib in sys.argv[1:]:
    env = dict(os.environ, EDV_LIB=os.path.abspath(lib), ROOT=ROOT)
    r = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=300)
    print(r.stdout.strip() if r.returncode == 0 else json.dumps({"lib": lib, "error": r.stderr[-800:]}), flush=True)
