"""Same-box A/B of two builds of libedv.so on the latency path: in alternating
child processes (EDV_LIB=each), the median wall time of a device-resident
verify (library stream, synchronised) of the first n requests of a C2-shaped
batch, and of one Verifier.verify; verdicts checked against the construction.
One JSON line per (round, library).

  python tools/ab_lib_latency.py LIB_A LIB_B [ROUNDS] [N ...]
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r'''
import json, statistics, sys, time
sys.path.insert(0, %r)
import numpy as np
from indy_plenum_amd import edv, workload
from indy_plenum_amd.nacl_wrappers import Verifier
sizes = %r
b = workload.DeviceBatch(max(sizes), damage_every=20)
exp = b.expected()
def med(f, reps):
    for _ in range(10):
        f()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter(); f(); ts.append(time.perf_counter() - t0)
    return round(1e6 * statistics.median(ts), 1)
out = {"lib": edv.LIB_PATH.rsplit("/", 1)[-1]}
for n in sizes:
    f = lambda: edv.verify_device(b.d_sigs.ptr, b.d_pks.ptr, b.d_msgs.ptr, b.d_off.ptr, n, b.d_accept.ptr, 0,
                                  flags=edv.FLAG_UNIFORM_LENGTH)
    out["dev_us_%%d" %% n] = med(f, 200 if n <= 4096 else 50)
    assert np.array_equal(b.d_accept.download(n), exp[:n]), n
sigs, pks, msgs, off, e = b.host_prefix(1)
v = Verifier(bytes(pks[:32]))
sig, msg = bytes(sigs[:64]), bytes(msgs[int(off[0]):int(off[1])])
assert v.verify(sig, msg) == bool(e[0])
out["verifier_verify_us"] = med(lambda: v.verify(sig, msg), 300)
print(json.dumps(out))
'''


def main():
    a, b = sys.argv[1], sys.argv[2]
    rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    sizes = [int(x) for x in sys.argv[4:]] or [1, 16, 400, 4096]
    code = CHILD % (ROOT, sizes)
    for r in range(rounds):
        for lib in (a, b):
            p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300,
                               env=dict(os.environ, EDV_LIB=os.path.abspath(lib)))
            if p.returncode != 0:
                print(json.dumps({"round": r, "lib": lib, "error": p.stderr[-1500:]}), flush=True)
                sys.exit(1)
            print(json.dumps(dict({"round": r}, **json.loads(p.stdout.strip().splitlines()[-1]))), flush=True)


if __name__ == "__main__":
    main()
