"""Anatomy of one synchronous edv_verify_batch call (C2: 65,536 x 256 B) from
pinned host buffers -- measurement only.

Run under rocprofv3 (kernel, memory-copy and HIP runtime traces, no counters):

  rocprofv3 --kernel-trace --memory-copy-trace --hip-runtime-trace -d OUT -o run \
      -- python3 tools/trace_sync.py --calls 20 --marks OUT/marks.json
  python3 tools/trace_sync.py --parse OUT

The first form makes `--calls` calls 5 ms apart (so each call is an isolated
cluster in the trace) and writes each call's host entry/return times
(CLOCK_MONOTONIC and CLOCK_BOOTTIME, ns).  The second lines the trace up with
them and prints, per phase, the median over the calls: host work before the
first copy, the copies, each kernel, the D2H, and the return after it.
"""
import argparse
import csv
import glob
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def run(args):
    import numpy as np
    from indy_plenum_amd import edv, workload
    b = workload.DeviceBatch(args.n, keep_host=True)
    sigs, pks, msgs, off = b.host_copy()
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
    want = b.expected()
    marks = []
    for k in range(args.calls + 3):
        t0m, t0b = time.monotonic_ns(), time.clock_gettime_ns(time.CLOCK_BOOTTIME)
        edv._check(lib.edv_verify_batch(ps.ctypes.data, pp.ctypes.data, pm.ctypes.data, po.ctypes.data, n,
                                        pa.ctypes.data, 1))
        t1m, t1b = time.monotonic_ns(), time.clock_gettime_ns(time.CLOCK_BOOTTIME)
        if not np.array_equal(pa, want):
            raise SystemExit("verdicts differ")
        if k >= 3:  # the first calls set up the context and buffers
            marks.append({"mono": [t0m, t1m], "boot": [t0b, t1b]})
        time.sleep(0.005)
    json.dump({"n": n, "calls": marks}, open(args.marks, "w"))
    ms = sorted((m["mono"][1] - m["mono"][0]) / 1e6 for m in marks)
    print(json.dumps({"calls": len(ms), "call_ms_median": ms[len(ms) // 2], "verdicts_ok": True}))


def rows(d, pattern):
    out = []
    for f in glob.glob(os.path.join(d, "**", pattern), recursive=True):
        with open(f) as fh:
            out += list(csv.DictReader(fh))
    return out


def parse(args):
    d = args.parse
    marks = json.load(open(args.marks or os.path.join(d, "marks.json")))["calls"]
    ev = []
    for r in rows(d, "*kernel_trace.csv"):
        name = r["Kernel_Name"]
        kind = "kernel:" + ("prep" if "prep_kernel" in name else "main" if "main_kernel" in name else name[:40])
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), kind, r))
    for r in rows(d, "*memory_copy_trace.csv"):
        kind = "h2d" if "HOST_TO_DEVICE" in r["Direction"] else ("d2h" if "DEVICE_TO_HOST" in r["Direction"] else "copy")
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), kind, r))
    api = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Function"]) for r in rows(d, "*hip_api_trace.csv")]
    ev.sort(key=lambda e: e[0])
    api.sort()
    # which host clock the trace uses: the one whose call windows contain the events
    clock = None
    for c in ("mono", "boot"):
        m = marks[len(marks) // 2][c]
        if any(m[0] <= e[0] <= m[1] for e in ev):
            clock = c
            break
    if clock is None:
        raise SystemExit("trace timestamps match neither CLOCK_MONOTONIC nor CLOCK_BOOTTIME")
    phases = {}

    def add(k, v):
        phases.setdefault(k, []).append(v / 1e6)

    for m in marks:
        t0, t1 = m[clock]
        es = [e for e in ev if t0 <= e[0] <= t1]
        h2d = [e for e in es if e[2] == "h2d"]
        d2h = [e for e in es if e[2] == "d2h"]
        ks = [e for e in es if e[2].startswith("kernel:")]
        if not h2d or not ks:
            continue
        add("call", t1 - t0)
        add("host_before_first_copy", h2d[0][0] - t0)
        add("h2d_span", max(e[1] for e in h2d) - h2d[0][0])
        for j, e in enumerate(h2d):
            add("h2d_%d_ms" % j, e[1] - e[0])
            add("h2d_%d_MB" % j, int(e[3].get("Size", 0) or 0))  # add() divides by 1e6
        for j, e in enumerate(ks):
            add("k%d_%s_start_after_first_copy" % (j, e[2][7:]), e[0] - h2d[0][0])
            add("k%d_%s_ms" % (j, e[2][7:]), e[1] - e[0])
        add("last_h2d_end_to_last_kernel_start", ks[-1][0] - max(e[1] for e in h2d))
        if d2h:
            add("last_kernel_end_to_d2h_start", d2h[-1][0] - ks[-1][1])
            add("d2h_ms", d2h[-1][1] - d2h[-1][0])
            add("d2h_end_to_return", t1 - d2h[-1][1])
        else:  # verdicts written zero-copy by the main kernel
            add("last_kernel_end_to_return", t1 - ks[-1][1])
        for a in api:
            if t0 <= a[0] <= t1:
                add("api:" + a[2], a[1] - a[0])
    out = {"clock": clock, "calls": len(phases.get("call", []))}
    for k, v in phases.items():
        out[k] = {"median": round(statistics.median(v), 4), "n": len(v)} if not k.startswith("api:") else \
            {"median_ms": round(statistics.median(v), 4), "per_call": round(len(v) / max(1, out["calls"]), 2),
             "sum_per_call_ms": round(sum(v) / max(1, out["calls"]), 4)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=65536)
    ap.add_argument("--calls", type=int, default=20)
    ap.add_argument("--marks", default=None)
    ap.add_argument("--parse", default=None)
    a = ap.parse_args()
    if a.parse:
        parse(a)
    else:
        a.marks = a.marks or "marks.json"
        run(a)
