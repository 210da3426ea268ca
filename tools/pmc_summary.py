"""Summarise rocprofv3 --pmc passes (FETCH_SIZE / WRITE_SIZE, one pass each) into
per-kernel HBM bytes per launch, with the gfx950 correction of
MI355X_MICROARCH.md "HBM": FETCH_SIZE reports half the bytes of wide coalesced
reads, so read bytes = 2 x FETCH_SIZE x 1024; WRITE_SIZE is exact (x 1024).
Infinity-Cache (MALL) hits are counted by these counters, not excluded.

  python tools/pmc_summary.py <pmc_dir_fetch> <pmc_dir_write> [out.json]

The summary records the SHA-256 of the kernel sources it was measured on
(bench.kernel_source_hash); bench.py reports it as roofline.traffic only while
the sources still hash the same.
"""
import collections
import csv
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import kernel_source_hash  # noqa: E402


def per_kernel(d, counter):
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(os.path.join(d, "run_counter_collection.csv"))):
        if r["Counter_Name"] != counter:
            continue
        name = r["Kernel_Name"]
        short = name.replace("(anonymous namespace)::", "").split("(")[0]
        acc[short].append(float(r["Counter_Value"]))
    return {k: (sum(v) / len(v), len(v)) for k, v in acc.items()}


def main():
    fetch = per_kernel(sys.argv[1], "FETCH_SIZE")
    write = per_kernel(sys.argv[2], "WRITE_SIZE")
    out = {"source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes) over bench.py",
           "correction": "read_bytes = 2 * FETCH_SIZE_KB * 1024 (gfx950), write_bytes = WRITE_SIZE_KB * 1024",
           "kernel_source_sha256": kernel_source_hash(),
           "bench_args": "--steps 6 --warmup 20 --no-cpu-baseline (batch 65536 x 256 B)",
           "kernels": {}}
    for k in sorted(set(fetch) | set(write)):
        f, nf = fetch.get(k, (0.0, 0))
        w, nw = write.get(k, (0.0, 0))
        out["kernels"][k] = {"fetch_size_kb": f, "write_size_kb": w, "launches": max(nf, nw),
                             "read_bytes": 2 * f * 1024, "write_bytes": w * 1024,
                             "hbm_bytes_per_launch": 2 * f * 1024 + w * 1024}
    s = json.dumps(out, indent=1)
    if len(sys.argv) > 3:
        open(sys.argv[3], "w").write(s + "\n")
    print(s)


if __name__ == "__main__":
    main()
