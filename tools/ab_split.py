"""Device-resident step rate at C2 (65,536 x 256 B) and C4 (65,536 x 200..4,096 B,
5 % invalid) on one MI355X: sequential prep -> main, the two-stream pipeline
(prep of step k+1 beside main of step k), and the split pipeline
(EDV_FLAG_SPLIT_PREP: only the hash side beside the previous main kernel, the
point sides in front of this step's main).  Median of REPS x STEPS steps,
modes interleaved over ROUNDS; verdicts checked after every mode.  Measurement
only."""
import json
import os
import statistics
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from indy_plenum_amd import edv, workload  # noqa: E402

STEPS, REPS, ROUNDS = (int(os.environ.get(k, d)) for k, d in (("STEPS", 20), ("REPS", 5), ("ROUNDS", 2)))
dev = 0
s = edv.stream(dev)
CONFIGS = os.environ.get("CONFIGS", "C2,C4").split(",")
batches = {}
if "C2" in CONFIGS:
    batches["C2"] = workload.DeviceBatch(65536, device=dev)
if "C4" in CONFIGS:
    batches["C4"] = workload.DeviceBatch(65536, device=dev, seed=0xC4C4, var_range=(200, 4096), damage_every=20,
                                         damage_kinds=7, keep_host=False)
MODES = os.environ.get("MODES", "sequential,pipelined,split").split(",")
modes = {"sequential": (lambda b: b.verify(stream=s), lambda: edv.sync(dev)),
         "pipelined": (lambda b: b.submit(), lambda: edv.pipeline_sync(dev)),
         "split": (lambda b: b.submit(edv.FLAG_SPLIT_PREP), lambda: edv.pipeline_sync(dev))}
for rnd in range(ROUNDS):
    for name, b in batches.items():
        exp = b.expected()
        for mode, (step, drain) in modes.items():
            if mode not in MODES:
                continue
            for _ in range(10):
                step(b)
            drain()
            b.d_accept.upload(np.full(b.n, 7, np.uint8))
            step(b)
            drain()
            ok = bool(np.array_equal(b.accept(), exp))
            reps = []
            for _ in range(REPS):
                drain()
                t0 = time.perf_counter()
                for _ in range(STEPS):
                    step(b)
                drain()
                reps.append((time.perf_counter() - t0) / STEPS)
            ms = 1e3 * statistics.median(reps)
            print(json.dumps({"lib": os.path.basename(edv.LIB_PATH), "round": rnd, "config": name, "mode": mode, "ms_per_step": ms,
                              "verifies_per_s": b.n / (ms * 1e-3), "verdicts_ok": ok}), flush=True)
