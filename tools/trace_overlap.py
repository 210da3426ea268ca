"""Read a rocprofv3 --kernel-trace --memory-copy-trace run of tools/e2e_cumask.py
and describe the synchronous calls made 5 ms apart (each one an isolated cluster
of copies and kernels): per configuration (CFGS order), the call's span on the
GPU (first H2D start to last D2H end), the copy time, the union of the
verify-kernel intervals, how many kernels ran at once, and each kernel's
duration.  Measurement only.

  python tools/trace_overlap.py <trace dir> [CFGS] [R]
"""
import csv
import glob
import json
import os
import statistics
import sys

d = sys.argv[1]
cfgs = (sys.argv[2] if len(sys.argv) > 2 else "1:0,4:0,4:1,4:3").split(",")
R = int(sys.argv[3]) if len(sys.argv) > 3 else 5


def rows(pattern):
    out = []
    for f in glob.glob(os.path.join(d, "**", pattern), recursive=True):
        with open(f) as fh:
            out += list(csv.DictReader(fh))
    return out


ev = []
for r in rows("*kernel_trace.csv"):
    name = r["Kernel_Name"]
    kind = "prep" if "edv_prep_kernel" in name else ("main" if "edv_main_kernel" in name else "other")
    ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), kind, r.get("Queue_Id")))
for r in rows("*memory_copy_trace.csv"):
    kind = "h2d" if "HOST_TO_DEVICE" in r["Direction"] else ("d2h" if "DEVICE_TO_HOST" in r["Direction"] else "copy")
    ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), kind, r.get("Stream_Id")))
ev.sort()
clusters, cur, end = [], [], None
for e in ev:
    if cur and e[0] - end > 2_000_000:   # 2 ms of nothing: a new cluster
        clusters.append(cur)
        cur = []
    cur.append(e)
    end = e[1] if end is None or not cur[:-1] else max(end, e[1])
if cur:
    clusters.append(cur)


def union(iv):
    iv = sorted(iv)
    tot, s0, e0 = 0, None, None
    for s, e in iv:
        if s0 is None or s > e0:
            if s0 is not None:
                tot += e0 - s0
            s0, e0 = s, e
        else:
            e0 = max(e0, e)
    return tot + (e0 - s0 if s0 is not None else 0)


def max_concurrency(iv):
    pts = sorted([(s, 1) for s, _ in iv] + [(e, -1) for _, e in iv])
    c = m = 0
    for _, k in pts:
        c += k
        m = max(m, c)
    return m


calls = []
for c in clusters:
    ks = [e for e in c if e[2] in ("prep", "main")]
    cp = [e for e in c if e[2] in ("h2d", "d2h")]
    if len(ks) in (2, 4, 6, 8) and all(e[2] != "other" for e in c):   # zero-copy calls have no copies
        calls.append(c)
out = {"clusters": len(clusters), "isolated_calls": len(calls), "configs": []}
for k, cfg in enumerate(cfgs):
    sel = calls[k * R:(k + 1) * R]
    if not sel:
        break
    span, h2d, kern, conc, prep, main = [], [], [], [], [], []
    for c in sel:
        span.append((max(e[1] for e in c) - min(e[0] for e in c)) / 1e6)
        h2d.append(union([(e[0], e[1]) for e in c if e[2] == "h2d"]) / 1e6)
        kv = [(e[0], e[1]) for e in c if e[2] in ("prep", "main")]
        kern.append(union(kv) / 1e6)
        conc.append(max_concurrency(kv))
        prep += [(e[1] - e[0]) / 1e6 for e in c if e[2] == "prep"]
        main += [(e[1] - e[0]) / 1e6 for e in c if e[2] == "main"]
    out["configs"].append({"cfg": cfg, "calls": len(sel), "span_ms": statistics.median(span),
                           "h2d_union_ms": statistics.median(h2d), "kernel_union_ms": statistics.median(kern),
                           "max_kernels_at_once": max(conc), "prep_kernel_ms": statistics.median(prep),
                           "main_kernel_ms": statistics.median(main)})
print(json.dumps(out, indent=1))
