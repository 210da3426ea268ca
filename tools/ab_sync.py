"""A/B of the synchronous host-buffer call (edv_verify_batch, C2: 65,536 x
256 B) across library builds: for each .so (EDV_LIB), in its own process, the
median of R calls from pinned buffers back to back, of R calls 5 ms apart,
and of R calls from pageable numpy arrays; verdicts checked.  Libraries are
run in the order given, so A B A B interleaves them.  Measurement only.

  python tools/ab_sync.py indy-plenum_amd/libedv.so indy-plenum_amd/variants/libedv_X.so ...
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r"""
import json, os, statistics, sys, time
import numpy as np
sys.path.insert(0, os.environ["ROOT"])
from indy_plenum_amd import edv, workload
R = int(os.environ.get("R", 41))
b = workload.DeviceBatch(65536, keep_host=True, damage_every=20)
sigs, pks, msgs, off = b.host_copy()
want = b.expected()
n = b.n
sizes = [sigs.nbytes, pks.nbytes, off.nbytes, msgs.nbytes, n]
pb = edv.PinnedBuffer(sum(sizes) + 5 * 64)
views, pos = [], 0
for a, sz in zip((sigs, pks, off, msgs, None), sizes):
    v = pb.array[pos:pos + sz]
    if a is not None:
        v[:] = a.view(np.uint8)
    views.append(v)
    pos += (sz + 63) // 64 * 64
ps, pp, po, pm, pa = views
po = po.view(np.uint64)
lib = edv.lib()
acc = np.zeros(n, np.uint8)
def call(s, p, m, o, a):
    edv._check(lib.edv_verify_batch(s.ctypes.data, p.ctypes.data, m.ctypes.data, o.ctypes.data, n, a.ctypes.data, 1))
def med(f, spaced=False):
    ts = []
    for _ in range(R):
        if spaced:
            time.sleep(0.005)
        t = time.perf_counter()
        f()
        ts.append(1e3 * (time.perf_counter() - t))
    return statistics.median(ts)
for _ in range(3):
    call(ps, pp, pm, po, pa)
    call(sigs, pks, msgs, off, acc)
ok = bool(np.array_equal(pa, want)) and bool(np.array_equal(acc, want))
out = {"lib": os.path.basename(os.environ["EDV_LIB"]),
       "pinned_ms": med(lambda: call(ps, pp, pm, po, pa)),
       "pinned_spaced_ms": med(lambda: call(ps, pp, pm, po, pa), True),
       "pageable_ms": med(lambda: call(sigs, pks, msgs, off, acc))}
out["verdicts_ok"] = ok and bool(np.array_equal(pa, want)) and bool(np.array_equal(acc, want))
print(json.dumps(out))
"""
for lib in sys.argv[1:]:
    env = dict(os.environ, EDV_LIB=os.path.abspath(lib), ROOT=ROOT)
    r = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=300)
    print(r.stdout.strip() if r.returncode == 0 else json.dumps({"lib": lib, "error": r.stderr[-800:]}), flush=True)
