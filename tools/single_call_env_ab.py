"""One Verifier.verify (a batch of one through the latency path) under HIP
runtime wait settings, each in a fresh child process: median wall time of 300
calls after 20 warm ones, and of the device-resident call (edv.verify_device,
library stream, synchronised).  Which part of the ~20 us between the kernel
(~0.18 ms) and the call is the host's wait for the completion signal.

  python tools/single_call_env_ab.py
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
b = workload.DeviceBatch(16, damage_every=0)
sigs, pks, msgs, off, exp = b.host_prefix(1)
sig, pk, msg = bytes(sigs[:64]), bytes(pks[:32]), bytes(msgs[int(off[0]):int(off[1])])
v = Verifier(pk)
assert v.verify(sig, msg)
def med(f, reps=300):
    for _ in range(20):
        f()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter(); f(); ts.append(time.perf_counter() - t0)
    return round(1e6 * statistics.median(ts), 1)
out = {"verifier_verify_us": med(lambda: v.verify(sig, msg))}
out["device_resident_us"] = med(lambda: edv.verify_device(b.d_sigs.ptr, b.d_pks.ptr, b.d_msgs.ptr, b.d_off.ptr, 1,
                                                           b.d_accept.ptr, 0, flags=edv.FLAG_UNIFORM_LENGTH))
print(json.dumps(out))
''' % ROOT


def main():
    settings = [("default", {}), ("ROC_ACTIVE_WAIT_TIMEOUT=1000", {"ROC_ACTIVE_WAIT_TIMEOUT": "1000"}),
                ("HIP_FORCE_DEV_KERNARG=1", {"HIP_FORCE_DEV_KERNARG": "1"}),
                ("both", {"ROC_ACTIVE_WAIT_TIMEOUT": "1000", "HIP_FORCE_DEV_KERNARG": "1"})]
    for rep in range(2):
        for name, env in settings:
            r = subprocess.run([sys.executable, "-c", CHILD], capture_output=True, text=True, timeout=300,
                               env=dict(os.environ, **env))
            if r.returncode != 0:
                print(json.dumps({"setting": name, "error": r.stderr[-1500:]}), flush=True)
                continue
            print(json.dumps(dict({"rep": rep, "setting": name}, **json.loads(r.stdout.strip().splitlines()[-1]))),
                  flush=True)


if __name__ == "__main__":
    main()
