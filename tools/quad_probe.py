"""Kernel-time probe of the latency path (run under rocprofv3 --kernel-trace):
for each batch size n, `iters` device-resident verifies of the first n
requests of a C2-shaped batch, each synchronised.

  python tools/quad_probe.py ITERS N [N ...]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    iters = int(sys.argv[1])
    sizes = [int(x) for x in sys.argv[2:]]
    from indy_plenum_amd import edv, workload
    b = workload.DeviceBatch(max(max(sizes), 64), keep_host=False)
    for n in sizes:
        for _ in range(iters):
            edv.verify_device(b.d_sigs.ptr, b.d_pks.ptr, b.d_msgs.ptr, b.d_off.ptr, n, b.d_accept.ptr, 0,
                              flags=edv.FLAG_UNIFORM_LENGTH)
        if os.environ.get("QUAD_PROBE_NOCHECK") != "1":  # phase probes write partial verdicts
            assert b.d_accept.download(n).all()


if __name__ == "__main__":
    main()
