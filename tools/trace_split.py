"""Overlap evidence from rocprofv3 traces (--kernel-trace [--memory-copy-trace]):

  split:  for tools/ab_split.py (MODES=split) -- how much of each hash-side
          prep launch (edv_prep_kernel, grid n) ran while a main kernel was
          running, and the per-class kernel durations
  fields: per synchronous call on the field-ordered path (a trace of
          synchronous calls, e.g. tools/trace_sync.py's), how long the
          point-side prep launch (grid 2n) ran before the message copy finished

  python tools/trace_split.py split|fields <trace dir> [n=65536]
Measurement only."""
import csv
import glob
import json
import os
import statistics
import sys

mode, d = sys.argv[1], sys.argv[2]
n = int(sys.argv[3]) if len(sys.argv) > 3 else 65536


def rows(pattern):
    out = []
    for f in glob.glob(os.path.join(d, "**", pattern), recursive=True):
        with open(f) as fh:
            out += list(csv.DictReader(fh))
    return out


ks = []
for r in rows("*kernel_trace.csv"):
    name, grid = r["Kernel_Name"], int(r["Grid_Size_X"])
    if "edv_prep_kernel" in name:
        cls = {n: "prep_hash", 2 * n: "prep_points", 3 * n: "prep_all"}.get(grid, "prep_other")
    elif "edv_main_kernel_prio" in name:
        cls = "main_prio"
    elif "edv_main_kernel" in name:
        cls = "main"
    else:
        continue
    ks.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), cls))
ks.sort()


def overlap(a, b, ivs):
    tot = 0
    for s, e in ivs:
        tot += max(0, min(b, e) - max(a, s))
    return tot


out = {"mode": mode, "kernels": {}}
for cls in sorted({k[2] for k in ks}):
    dur = [(e - s) / 1e6 for s, e, c in ks if c == cls]
    out["kernels"][cls] = {"launches": len(dur), "median_ms": statistics.median(dur)}
if mode == "split":
    mains = [(s, e) for s, e, c in ks if c.startswith("main")]
    pts = [(s, e) for s, e, c in ks if c == "prep_points"]
    fr = [overlap(s, e, mains) / max(1, e - s) for s, e, c in ks if c == "prep_hash"]
    fp = [overlap(s, e, pts) / max(1, e - s) for s, e, c in ks if c == "prep_hash"]
    if fr:
        out["hash_side_time_beside_a_main_kernel"] = {"median": statistics.median(fr), "min": min(fr),
                                                      "launches": len(fr)}
        out["hash_side_time_beside_a_point_side_launch"] = {"median": statistics.median(fp), "launches": len(fp)}
    # the steady state: span from one main kernel's end to the next one's
    me = sorted(e for s, e, c in ks if c.startswith("main"))
    gaps = [(b - a) / 1e6 for a, b in zip(me, me[1:]) if b - a < 5_000_000]
    if gaps:
        out["main_end_to_main_end_ms"] = statistics.median(gaps)
else:
    copies = []
    for r in rows("*memory_copy_trace.csv"):
        if "HOST_TO_DEVICE" in r["Direction"]:
            copies.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    copies.sort()
    lead = []
    for s, e, c in ks:
        if c != "prep_points":
            continue
        # copies in flight when this launch started (this call's message copy, if
        # the point sides started before it finished): how much longer they ran
        inflight = [ce - s for cs, ce in copies if cs <= s < ce]
        lead.append(max(inflight) / 1e6 if inflight else 0.0)
    if lead:
        out["points_side_ran_before_message_copy_ended_ms"] = {"median": statistics.median(lead), "max": max(lead),
                                                              "calls": len(lead)}
print(json.dumps(out, indent=1))
