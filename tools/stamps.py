"""Phase shares of the prep and main kernels from the diagnostic stamp build
(EDV_STAMPS: lane 0 of each wave records s_memtime at the EDV_STAMP points of
edv_verify_core.h).  Read the SHARES, not absolute lengths: the stamps' fences
forbid overlaps the real kernels have (cdna_hip_programming.md section 7,
In-kernel stamps).

  tools/build_variant.sh stamps -DEDV_STAMPS
  EDV_LIB=indy-plenum_amd/variants/libedv_stamps.so python tools/stamps.py [n]
"""
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from indy_plenum_amd import edv, workload  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
lib = edv.lib()
lib.edv_debug_set_stamps.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
waves_prep = 3 * ((n + 255) // 256) * 4
waves_main = ((n + 255) // 256) * 4
bp = edv.DeviceBuffer(8 * 16 * waves_prep)
bm = edv.DeviceBuffer(8 * 16 * waves_main)
b = workload.DeviceBatch(n)
for _ in range(20):
    b.verify()
assert b.accept().all()
zero_p = np.zeros(16 * waves_prep, np.uint64)
zero_m = np.zeros(16 * waves_main, np.uint64)
bp.upload(zero_p)
bm.upload(zero_m)
assert lib.edv_debug_set_stamps(bp.ptr, bm.ptr) == 0
b.verify()
assert lib.edv_debug_set_stamps(None, None) == 0
sp = bp.download(dtype=np.uint64).reshape(waves_prep, 16).astype(np.int64)
sm = bm.download(dtype=np.uint64).reshape(waves_main, 16).astype(np.int64)
out = {"n": n}
t0 = sp[:, 0][sp[:, 0] > 0].min()
side = (np.arange(waves_prep) // 4) % 3     # block b runs side b % 3; 4 waves per block
for s, names in ((0, ["start->hash", "sha512", "sc_reduce", "half_scalars", "sc_mul", "recode+store"]),
                 (1, ["start->point", "decompress", "table", "store/end"]),
                 (2, ["start->point", "decompress", "table", "store/end"])):
    rows = sp[side == s]
    slots = [0, 1, 2, 3, 4, 5, 15] if s == 0 else [0, 1, 2, 3, 15]
    d = np.diff(rows[:, slots], axis=1)
    tot = rows[:, 15] - rows[:, 0]
    out["prep_side%d" % s] = {"median_cycles": float(np.median(tot)),
                              "start_spread_cycles": float(np.percentile(rows[:, 0] - t0, 99)),
                              "end_p50": float(np.median(rows[:, 15] - t0)), "end_max": float((rows[:, 15] - t0).max()),
                              "shares": {nm: float(np.median(d[:, k]) / np.median(tot)) for k, nm in enumerate(names)}}
m0 = sm[:, 0].min()
pro = sm[:, 1] - sm[:, 0]
top = sm[:, 2] - sm[:, 1]
four = sm[:, 3] - sm[:, 2]
body = sm[:, 14] - sm[:, 1]
out["main"] = {"prologue_cycles_p50": float(np.median(pro)), "top_window_cycles_p50": float(np.median(top)),
               "cycles_per_window_p50": float(np.median(four) / 4), "walk_cycles_p50": float(np.median(body)),
               "epilogue_cycles_p50": float(np.median(sm[:, 15] - sm[:, 14])),
               "start_spread_p99": float(np.percentile(sm[:, 0] - m0, 99)),
               "end_p50": float(np.median(sm[:, 15] - m0)), "end_max": float((sm[:, 15] - m0).max()),
               "prologue_share": float(np.median(pro) / np.median(sm[:, 15] - sm[:, 0]))}
win = sm[:, 10] - sm[:, 5]
names = ["doublings", "fetch_A (LDS wait)", "add_A + to_p3", "fetch_R (LDS wait)", "add_R + to_p2"]
d = np.diff(sm[:, 5:11], axis=1)
out["main"]["plain_window"] = {"cycles_p50": float(np.median(win)),
                               "shares": {nm: float(np.median(d[:, k]) / np.median(win)) for k, nm in enumerate(names)}}
bw = sm[:, 13] - sm[:, 11]
out["main"]["b_window_after_doublings"] = {"add_A_R_cycles_p50": float(np.median(sm[:, 12] - sm[:, 11])),
                                          "b_adds_cycles_p50": float(np.median(sm[:, 13] - sm[:, 12])),
                                          "cycles_p50": float(np.median(bw))}
print(json.dumps(out, indent=1))
