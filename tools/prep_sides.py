"""The prep kernel's three sides timed apart on HEAD's kernels (VERDICT r5
item 4): C2's 65,536 requests (and a 2^18 chunk), hash side, A side, R side
alone, all three in one launch and the two point sides together
(edv_profile_prep_sides, libedv_measure.so), both [S]B table sets.

  python tools/prep_sides.py [--iters 10] [--n 65536 262144]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--n", type=int, nargs="+", default=[65536, 262144])
    a = ap.parse_args()
    from indy_plenum_amd import edv, workload
    for n in a.n:
        b = workload.DeviceBatch(n, keep_host=False)
        args = (b.d_sigs.ptr, b.d_pks.ptr, b.d_msgs.ptr, b.d_off.ptr, n, b.d_accept.ptr, 0)
        edv.profile_prep_sides(*args, 2)  # warm (builds the large tables at n >= 65,536)
        sides = edv.profile_prep_sides(*args, a.iters)
        prep, main = edv.profile_device(*args, a.iters)
        print(json.dumps({"n": n, "sides_ms": sides, "prep_ms": prep, "main_ms": main,
                          "tables": "large" if n >= 65536 else "compact"}), flush=True)


if __name__ == "__main__":
    main()
