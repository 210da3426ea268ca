#!/usr/bin/env python3
"""libsodium 1.0.18 verdict bitmasks for the large seeded parity corpora.

The corpus is regenerated bit-identically from its seed by the oracle's
generator (oracle/ed25519_oracle.c oref_corpus_gen) on any machine; this script
(run in the build container, where libsodium is present) records per 1M-item
slice the SHA-256 of (sigs || pks || msgs) and the packed accept bits.  The GPU
box regenerates each slice, checks the hash, verifies on the GPU and compares
bits (tests/test_gpu_parity.py::test_big_corpus_parity).

  C2 shape: 10,485,760 items, 256-byte messages, 5% invalid  (>= 10M)
  C4 shape:  1,048,576 items, 200..4096-byte messages, 5% invalid
"""
import hashlib
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import oracle_lib as orc  # noqa: E402

SLICE = 1 << 20
CORPORA = {
    "c2_256B": dict(seed=0x5EED2025, mode=0, invalid_permille=50, count=10 * SLICE),
    "c4_var": dict(seed=0xC4C4, mode=1, invalid_permille=50, count=1 * SLICE),
}


def slice_hash(sigs, pks, msgs, off):
    h = hashlib.sha256()
    h.update(sigs.tobytes())
    h.update(pks.tobytes())
    h.update(msgs[:int(off[-1])].tobytes())
    return h.hexdigest()


def main():
    threads = int(os.environ.get("THREADS", os.cpu_count() or 8))
    meta = {"slice": SLICE, "verdicts_from": "libsodium " + orc.sodium_batch().sb_version().decode(),
            "generator": "oracle/ed25519_oracle.c oref_corpus_gen", "corpora": {}}
    for name, cfg in CORPORA.items():
        bits = []
        hashes, accepts = [], []
        for s in range(cfg["count"] // SLICE):
            t = time.time()
            sigs, pks, msgs, off = orc.corpus(cfg["seed"], s * SLICE, SLICE, cfg["mode"], cfg["invalid_permille"],
                                              threads)
            acc = orc.sodium_verify_batch(sigs, pks, msgs, off, threads)
            hashes.append(slice_hash(sigs, pks, msgs, off))
            accepts.append(int(acc.sum()))
            bits.append(np.packbits(acc, bitorder="little"))
            print(name, s, accepts[-1], "%.1fs" % (time.time() - t), flush=True)
        np.concatenate(bits).tofile(os.path.join(HERE, "corpus_%s.bits" % name))
        meta["corpora"][name] = dict(cfg, slice_sha256=hashes, slice_accepts=accepts)
        with open(os.path.join(HERE, "corpus_bitmask.json"), "w") as f:
            json.dump(meta, f, indent=1)


if __name__ == "__main__":
    main()
