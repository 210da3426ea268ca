"""Live parity on the GPU box: the bench's own workloads, verified by the GPU
(C-ABI, device-resident batches) and by libsodium 1.0.18 itself on the host
(oracle/sodium_batch.c, crypto_sign_ed25519_verify_detached on 16 threads),
every verdict compared.  Complements the committed-bitmask parity of
tests/test_gpu_parity.py with fresh corpora of a different generator:

  C3  16,777,216 requests of 256 B (bench.py's C3: GPU-signed, 5 % damaged
      over four kinds), in slices of 2^20
  C4  4,194,304 requests of 200..4,096 B, 5 % damaged over seven kinds
      (small-order R, non-canonical A, small-order A included)

  python tools/parity_live_sodium.py [c3_total] [c4_total]
Prints one JSON line per workload and a summary; exit status 1 on any mismatch.
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import oracle_lib as orc  # noqa: E402  (libsodium harness: the checker)
from indy_plenum_amd import workload  # noqa: E402

SLICE = 1 << 20


def run(name, total, **kw):
    t0 = time.time()
    checked = mism = rejected = 0
    first_bad = None
    for start in range(0, total, SLICE):
        n = min(SLICE, total - start)
        b = workload.DeviceBatch(n, start=start, keep_host=True, **kw)
        b.verify()
        got = b.accept()
        sigs, pks, msgs, off = b.host_copy()
        want = orc.sodium_verify_batch(sigs, pks, msgs, off, 16)
        bad = np.nonzero(got != want)[0]
        if bad.size and first_bad is None:
            first_bad = int(start + bad[0])
        mism += int(bad.size)
        checked += n
        rejected += int(n - want.sum())
        del b
    out = {"workload": name, "requests": checked, "libsodium_rejected": rejected, "mismatches": mism,
           "first_mismatch": first_bad, "seconds": round(time.time() - t0, 1)}
    print(json.dumps(out), flush=True)
    return out


def main():
    if orc.sodium_batch() is None:
        sys.exit("libsodium not present: nothing to compare against")
    c3 = int(sys.argv[1]) if len(sys.argv) > 1 else 16777216
    c4 = int(sys.argv[2]) if len(sys.argv) > 2 else 4194304
    res = [run("C3 256 B, 5 % damaged (4 kinds)", c3, damage_every=20, damage_kinds=4),
           run("C4 200..4,096 B, 5 % damaged (7 kinds)", c4, seed=0xC4C4, var_range=(200, 4096), damage_every=20,
               damage_kinds=7)]
    total = sum(r["requests"] for r in res)
    bad = sum(r["mismatches"] for r in res)
    print(json.dumps({"summary": "GPU vs libsodium 1.0.18, live", "requests": total, "mismatches": bad}))
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
