"""Latency of one batch, batch kernels against the latency path (VERDICT r5
item 5): median wall time of edv_verify_batch on host buffers (synchronous,
the boundary a Node calls) and of a device-resident verify (inputs in HBM,
library stream, synchronised), for batch sizes from 1 to 16,384, with the
latency path off (edv_set_latency_path 0: prep + main kernels) and on (limit
8,192: one quad-kernel launch).  Verdicts checked against the construction.

  python tools/latency_paths.py [--reps 50] [--sizes 1 64 400 ...]
"""
import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402


def med(f, reps):
    for _ in range(3):
        f()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        f()
        ts.append(time.perf_counter() - t0)
    return 1e6 * statistics.median(ts)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--sizes", type=int, nargs="+", default=[1, 16, 64, 256, 400, 1024, 2048, 4096, 8192, 16384])
    a = ap.parse_args()
    from indy_plenum_amd import edv, workload
    nmax = max(a.sizes)
    b = workload.DeviceBatch(nmax, damage_every=20)
    sigs, pks, msgs, off, exp = b.host_prefix(nmax)
    for n in a.sizes:
        row = {"n": n}
        for name, limit in (("batch_kernels", 0), ("latency_path", 8192)):
            edv.set_latency_path(0, limit)
            acc = edv.verify_arrays(sigs[:64 * n], pks[:32 * n], msgs, off[:n + 1])
            assert np.array_equal(acc, exp[:n]), (n, name)
            row[name + "_host_us"] = med(lambda: edv.verify_arrays(sigs[:64 * n], pks[:32 * n], msgs, off[:n + 1]),
                                         a.reps)

            def dev():
                edv.verify_device(b.d_sigs.ptr, b.d_pks.ptr, b.d_msgs.ptr, b.d_off.ptr, n, b.d_accept.ptr, 0,
                                  flags=edv.FLAG_UNIFORM_LENGTH)
            row[name + "_device_us"] = med(dev, a.reps)
            assert np.array_equal(b.d_accept.download(n), exp[:n]), (n, name, "device")
        print(json.dumps(row), flush=True)
    edv.set_latency_path(0, edv.LATENCY_PATH_DEFAULT)


if __name__ == "__main__":
    main()
