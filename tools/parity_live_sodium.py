"""Live parity on the GPU box: the bench's own workloads, verified by the GPU
(C-ABI, device-resident batches) and by libsodium 1.0.18 itself on the host
(oracle/sodium_batch.c, crypto_sign_ed25519_verify_detached on 16 threads),
every verdict compared.  Complements the committed-bitmask parity of
tests/test_gpu_parity.py with fresh corpora of a different generator:

  C3  16,777,216 requests of 256 B (bench.py's C3: GPU-signed, 5 % damaged
      over four kinds), in slices of 2^20
  C4  4,194,304 requests of 200..4,096 B, 5 % damaged over seven kinds
      (small-order R, non-canonical A, small-order A included)

  fuzz 2,097,152 requests of 256 B with random bit flips anywhere in sig, pk
      or message, or a random R, S or A (pageable host buffers through
      edv_verify_batch, FUZZ_SLICE requests per call, default 2^18 = one chunk:
      the field-ordered path with staged message quarters)

  latency  requests sent in calls of 1..LATENCY_PATH_DEFAULT requests (random sizes), i.e.
      through the latency kernel (csrc/edv_quad.hip): half fuzzed 256-B
      requests as above, half C4-style 200..4,096-B requests, 5 % damaged
      over seven kinds

  python tools/parity_live_sodium.py [c3_total] [c4_total] [fuzz_total] [latency_total]
LIVE_SEED=k (default 0) XORs k into every corpus seed: a rerun with a new k checks
fresh keys, messages and damage instead of repeating the corpora already recorded.
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
SEED = int(os.environ.get("LIVE_SEED", "0"), 0)
BENCH_SEED = 0x5EED2025  # workload.DeviceBatch's default


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


def fuzzed(n, start, seed, rng):
    """n valid 256-B requests of the bench generator, then per request one of
    1-3 random bit flips over sig || pk || msg (45 %), a random 32-byte R, S or
    A (5 % each), or left intact -> host arrays (sigs, pks, msgs, off)."""
    b = workload.DeviceBatch(n, start=start, seed=seed, keep_host=True)
    sigs, pks, msgs, off = b.host_copy()
    del b
    sigs = sigs.reshape(n, 64).copy()
    pks = pks.reshape(n, 32).copy()
    msgs = msgs.copy()
    kind = rng.integers(0, 100, size=n)
    flip = np.nonzero(kind < 45)[0]
    for _ in range(3):
        sel = flip[rng.random(flip.size) < 0.6]
        pos = rng.integers(0, 64 + 32 + 256, size=sel.size)
        bit = (np.uint8(1) << rng.integers(0, 8, size=sel.size).astype(np.uint8))
        s_ = pos < 64
        sigs[sel[s_], pos[s_]] ^= bit[s_]
        p_ = (pos >= 64) & (pos < 96)
        pks[sel[p_], pos[p_] - 64] ^= bit[p_]
        m_ = pos >= 96
        mo = off[sel[m_]].astype(np.int64) + (pos[m_] - 96)
        msgs[mo] ^= bit[m_]
    for lo_k, hi_k, arr, a, bb in ((45, 50, sigs, 0, 32), (50, 55, sigs, 32, 64), (55, 60, pks, 0, 32)):
        sel = np.nonzero((kind >= lo_k) & (kind < hi_k))[0]
        arr[sel, a:bb] = rng.integers(0, 256, size=(sel.size, bb - a), dtype=np.uint8)
    return sigs.reshape(-1), pks.reshape(-1), msgs, off


def fuzz(total, seed=0xF022 ^ SEED):
    """Random damage anywhere (fuzzed()), verified through the C-ABI host path
    (edv_verify_batch on host buffers)."""
    from indy_plenum_amd import edv
    t0 = time.time()
    rng = np.random.default_rng(seed)
    checked = mism = rejected = 0
    first_bad = None
    fslice = int(os.environ.get("FUZZ_SLICE", 1 << 18))   # one chunk: the field-ordered synchronous path
    for start in range(0, total, fslice):
        n = min(fslice, total - start)
        sigs, pks, msgs, off = fuzzed(n, start, seed, rng)
        got = edv.verify_arrays(sigs, pks, msgs, off)
        want = orc.sodium_verify_batch(sigs, pks, msgs, off, 16)
        bad = np.nonzero(got != want)[0]
        if bad.size and first_bad is None:
            first_bad = int(start + bad[0])
        mism += int(bad.size)
        checked += n
        rejected += int(n - want.sum())
    out = {"workload": "fuzz: random bit flips over sig/pk/msg and random R, S, A (256 B)", "requests": checked,
           "libsodium_rejected": rejected, "mismatches": mism, "first_mismatch": first_bad,
           "seconds": round(time.time() - t0, 1)}
    print(json.dumps(out), flush=True)
    return out


def latency(total, seed=0x1A7E ^ SEED):
    """The latency kernel: slices of 2^18 requests (alternately fuzzed 256-B
    and C4-style 200..4,096-B with seven damage kinds) sent through
    edv_verify_batch in calls of random size 1..edv.LATENCY_PATH_DEFAULT
    (16,384: every call on the latency path), all verdicts against libsodium live."""
    from indy_plenum_amd import edv
    t0 = time.time()
    rng = np.random.default_rng(seed)
    checked = mism = rejected = calls = 0
    first_bad = None
    sl = 1 << 18
    for k, start in enumerate(range(0, total, sl)):
        n = min(sl, total - start)
        if k % 2 == 0:
            sigs, pks, msgs, off = fuzzed(n, start, seed, rng)
        else:
            b = workload.DeviceBatch(n, start=start, seed=0xC4C4 ^ SEED, keep_host=True, var_range=(200, 4096),
                                     damage_every=20, damage_kinds=7)
            sigs, pks, msgs, off = b.host_copy()
            del b
        got = np.zeros(n, np.uint8)
        lo = 0
        while lo < n:
            m = min(n - lo, int(rng.integers(1, edv.LATENCY_PATH_DEFAULT + 1)))
            o = off[lo:lo + m + 1]
            got[lo:lo + m] = edv.verify_arrays(sigs[64 * lo:64 * (lo + m)], pks[32 * lo:32 * (lo + m)], msgs, o)
            lo += m
            calls += 1
        want = orc.sodium_verify_batch(sigs, pks, msgs, off, 16)
        bad = np.nonzero(got != want)[0]
        if bad.size and first_bad is None:
            first_bad = int(start + bad[0])
        mism += int(bad.size)
        checked += n
        rejected += int(n - want.sum())
    out = {"workload": "latency path: fuzzed 256-B and C4-style 200..4,096-B requests in calls of 1..%d"
                       % edv.LATENCY_PATH_DEFAULT,
           "requests": checked, "calls": calls, "libsodium_rejected": rejected, "mismatches": mism,
           "first_mismatch": first_bad, "seconds": round(time.time() - t0, 1)}
    print(json.dumps(out), flush=True)
    return out


def main():
    if orc.sodium_batch() is None:
        sys.exit("libsodium not present: nothing to compare against")
    c3 = int(sys.argv[1]) if len(sys.argv) > 1 else 16777216
    c4 = int(sys.argv[2]) if len(sys.argv) > 2 else 4194304
    nf = int(sys.argv[3]) if len(sys.argv) > 3 else 2097152
    nl = int(sys.argv[4]) if len(sys.argv) > 4 else 1048576
    res = [run("C3 256 B, 5 % damaged (4 kinds)", c3, seed=BENCH_SEED ^ SEED, damage_every=20, damage_kinds=4),
           run("C4 200..4,096 B, 5 % damaged (7 kinds)", c4, seed=0xC4C4 ^ SEED, var_range=(200, 4096), damage_every=20,
               damage_kinds=7),
           fuzz(nf), latency(nl)]
    total = sum(r["requests"] for r in res)
    bad = sum(r["mismatches"] for r in res)
    print(json.dumps({"summary": "GPU vs libsodium 1.0.18, live", "live_seed": SEED, "requests": total, "mismatches": bad}))
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
