"""A/B of bench.py's step modes on one GPU: each mode's default C2 line (no
extra legs), each in its own process, the modes interleaved `--rounds` times;
one compact JSON line per run.  Measurement only.

  python tools/ab_bench_modes.py [--rounds 2] [--modes "|--pipeline|--pipeline --split-prep"] [-- extra bench args]
"""
import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--modes", default="|--pipeline|--pipeline --split-prep")
    a, extra = ap.parse_known_args()
    extra = [x for x in extra if x != "--"]
    for _ in range(a.rounds):
        for m in a.modes.split("|"):
            cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--no-e2e", "--no-extra", "--no-cpu-baseline"]
            cmd += m.split() + extra
            r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
            if r.returncode != 0:
                print(json.dumps({"mode": m, "error": r.stderr[-600:]}), flush=True)
                sys.exit(1)
            d = json.loads(r.stdout.strip().splitlines()[-1])
            print(json.dumps({"mode": m or "sequential", "args": extra, "value": d["value"],
                              "ms_per_step": d["ms_per_step"], "frac": d["roofline"]["frac"],
                              "verdicts_as_expected": d.get("verdicts_as_expected")}), flush=True)
