"""Summarise rocprofv3 --pmc passes (one counter group per pass, each pass its
own run over bench.py) into per-kernel averages per launch, plus the derived
HBM and VALU figures bench.py reports in `roofline`.

  python tools/pmc_summary.py <pmc_root_dir> [out.json]

<pmc_root_dir> holds one sub-directory per pass (p1, p2, ...), each with the
run_counter_collection.csv rocprofv3 wrote.

HBM (MI355X_MICROARCH.md "HBM"): on gfx950 FETCH_SIZE reports half the bytes of
wide coalesced reads, so read bytes = 2 x FETCH_SIZE x 1024; WRITE_SIZE is exact
(x 1024).  When the pass with the request-size counters (TCC_EA0_RDREQ_{32B,64B,
128B}_sum) is present, read bytes come from them instead (calibrated on known
byte counts for the main kernel's gather pattern, tools/ubench_gather.hip), and
the FETCH_SIZE figure is kept as a cross-check.  Infinity-Cache (MALL) hits are
counted by these counters, not excluded, so the figure is an upper bound on
DRAM traffic.

VALU: SQ_INSTS_VALU counts wave-instructions (one per wave per VALU
instruction); SQ_ACTIVE_INST_VALU counts them in quad-cycles; GRBM_GUI_ACTIVE
is summed over the 8 XCDs (MI355X_MICROARCH.md "DVFS give-back"), so the
kernel's GPU-busy cycles are GRBM_GUI_ACTIVE / 8.

The summary records the SHA-256 of the device code it was measured on
(bench.device_code_hash: the .hip_fatbin section of libedv.so); bench.py
reports its figures only while the library's device code hashes the same.
"""
import collections
import csv
import glob
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import device_code_hash  # noqa: E402

N_SIMD = 256 * 4


def short(name):
    return name.replace("(anonymous namespace)::", "").split("(")[0].split("::")[-1]


def collect(root):
    """-> {kernel: {counter: [values per launch]}}, {kernel: grid sizes}"""
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    grid = collections.defaultdict(set)
    for f in sorted(glob.glob(os.path.join(root, "*", "**", "*counter_collection.csv"), recursive=True)):
        for r in csv.DictReader(open(f)):
            k = short(r["Kernel_Name"])
            acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
            grid[k].add(int(r["Grid_Size"]))
    return acc, grid


def summarise(root):
    acc, grid = collect(root)
    out = {"source": "rocprofv3 --pmc, one counter group per pass, over bench.py --steps 6 --warmup 2",
           "correction": "read_bytes = 2 * FETCH_SIZE_KB * 1024 (gfx950), write_bytes = WRITE_SIZE_KB * 1024; "
                         "MALL (Infinity Cache) hits are included",
           "device_code_sha256": device_code_hash(),
           "kernels": {}}
    for k, cs in sorted(acc.items()):
        avg = {c: sum(v) / len(v) for c, v in cs.items()}
        d = {"launches": max(len(v) for v in cs.values()), "grid_sizes": sorted(grid[k]), "counters": avg}
        if "FETCH_SIZE" in avg or "WRITE_SIZE" in avg:
            d["read_bytes"] = 2 * avg.get("FETCH_SIZE", 0.0) * 1024
            d["write_bytes"] = avg.get("WRITE_SIZE", 0.0) * 1024
            d["hbm_bytes_per_launch"] = d["read_bytes"] + d["write_bytes"]
        if "TCC_EA0_RDREQ_128B_sum" in avg:
            # calibrated (profiles/r05/gather_calibration.json): the L2's fabric read
            # requests by size; bytes = 128 x (128-B) + 64 x (64-B) + 32 x (32-B)
            # requests, exact for a known streamed byte count and for the main
            # kernel's per-lane 160-B gather alike
            d["read_bytes_by_request_size"] = (128 * avg["TCC_EA0_RDREQ_128B_sum"]
                                               + 64 * avg.get("TCC_EA0_RDREQ_64B_sum", 0.0)
                                               + 32 * avg.get("TCC_EA0_RDREQ_32B_sum", 0.0))
            if "read_bytes" in d:
                d["read_bytes_fetch_vs_request_size"] = d["read_bytes"] / max(d["read_bytes_by_request_size"], 1.0)
                d["read_bytes"] = d["read_bytes_by_request_size"]
                d["hbm_bytes_per_launch"] = d["read_bytes"] + d["write_bytes"]
        if "SQ_INSTS_VALU" in avg and avg.get("SQ_WAVES"):
            d["valu_insts_per_wave"] = avg["SQ_INSTS_VALU"] / avg["SQ_WAVES"]
            d["salu_insts_per_wave"] = avg.get("SQ_INSTS_SALU", 0.0) / avg["SQ_WAVES"]
            d["vmem_insts_per_wave"] = avg.get("SQ_INSTS_VMEM", 0.0) / avg["SQ_WAVES"]
        if "SQ_ACTIVE_INST_VALU" in avg and "GRBM_GUI_ACTIVE" in avg:
            busy = avg["GRBM_GUI_ACTIVE"] / 8.0  # GPU-busy cycles of the kernel
            d["gpu_busy_cycles"] = busy
            # fraction of all SIMD cycles in which a VALU instruction was issuing (quad-cycle units)
            d["valu_busy"] = 4.0 * avg["SQ_ACTIVE_INST_VALU"] / (busy * N_SIMD)
        if avg.get("TCC_HIT_sum", 0.0) + avg.get("TCC_MISS_sum", 0.0) > 0:
            d["l2_hit_rate"] = avg["TCC_HIT_sum"] / (avg["TCC_HIT_sum"] + avg["TCC_MISS_sum"])
        if "SQ_WAVE_CYCLES" in avg:
            wc = avg["SQ_WAVE_CYCLES"]
            d["wave_cycle_split"] = {c: avg.get(c, 0.0) / wc for c in
                                     ("SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_ANY", "SQ_WAIT_ANY")}
        out["kernels"][k] = d
    return out


def main():
    s = json.dumps(summarise(sys.argv[1]), indent=1)
    if len(sys.argv) > 2:
        open(sys.argv[2], "w").write(s + "\n")
    print(s)


if __name__ == "__main__":
    main()
