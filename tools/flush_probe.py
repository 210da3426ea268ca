"""Does the main kernel care whether its table reads come from the Infinity
Cache or from DRAM?  (measurement only.)

C2 (65,536 x 256 B, device resident): the prep -> main launch pair as the
bench runs it, against the same pair with a kernel between them that reads and
rewrites a buffer larger than the 256 MiB Infinity Cache (edv_profile_batch_dev_flush),
so main's first touch of every table line goes to DRAM.  Interleaved
repetitions; one JSON line per repetition and a summary line.  Under
rocprofv3 --pmc the counters of each kernel come per dispatch, so the same run
gives main's TCC request counts with and without the flush.

  python3 tools/flush_probe.py [--n 65536] [--flush-mib 512] [--reps 5] [--iters 10]
"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
from indy_plenum_amd import edv, workload  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=65536)
ap.add_argument("--flush-mib", type=int, default=512)
ap.add_argument("--reps", type=int, default=5)
ap.add_argument("--iters", type=int, default=10)
a = ap.parse_args()
b = workload.DeviceBatch(a.n, keep_host=False)
b.verify()
assert np.array_equal(b.accept(), b.expected())
args = (b.d_sigs.ptr, b.d_pks.ptr, b.d_msgs.ptr, b.d_off.ptr, a.n, b.d_accept.ptr, 0, a.iters)
res = {"plain": [], "flushed": []}
for r in range(a.reps):
    for mode, fb in (("plain", 0), ("flushed", a.flush_mib << 20)):
        p, f, m = edv.profile_device_flush(*args, flush_bytes=fb)
        res[mode].append((p, f, m))
        print(json.dumps({"rep": r, "mode": mode, "prep_ms": p, "flush_ms": f, "main_ms": m}), flush=True)
ok = bool(np.array_equal(b.accept(), b.expected()))
med = {k: [statistics.median(x[i] for x in v) for i in range(3)] for k, v in res.items()}
print(json.dumps({"summary": True, "n": a.n, "flush_mib": a.flush_mib, "iters": a.iters, "reps": a.reps,
                  "plain_prep_ms": med["plain"][0], "plain_main_ms": med["plain"][2],
                  "flushed_prep_ms": med["flushed"][0], "flush_ms": med["flushed"][1],
                  "flushed_main_ms": med["flushed"][2],
                  "main_flushed_over_plain": med["flushed"][2] / med["plain"][2],
                  "verdicts_ok": ok}), flush=True)
