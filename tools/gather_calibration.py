"""Summarise the counter calibration of tools/ubench_gather.hip (PMC passes
of tools/gpu_r05.sh STEP=gather) and the Infinity-Cache flush probe
(STEP=flush) into one JSON document.  Measurement only.

  python tools/gather_calibration.py gpurun_out/r05/<TAG> > profiles/r05/gather_calibration.json

For every ubench launch: the bytes it asks for (known by construction), the
distinct 128-B lines it touches, and what the counters report -- the L2's
fabric read requests by size (TCC_EA0_RDREQ_{32B,64B,128B}_sum), FETCH_SIZE,
TCC hits and misses -- with the ratios that calibrate them.  For the flush
probe: the main kernel's time and fabric reads with and without a 512 MiB
read-and-rewrite between prep and main.
"""
import collections
import csv
import glob
import json
import os
import statistics
import sys


def passes(d):
    """-> list of launches (in order) of each kernel: {counter: value}"""
    per = collections.defaultdict(lambda: collections.defaultdict(dict))
    for f in sorted(glob.glob(os.path.join(d, "p*", "**", "*counter_collection.csv"), recursive=True)):
        p = os.path.relpath(f, d).split(os.sep)[0]
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0].split("::")[-1]
            per[p][(int(r["Dispatch_Id"]), name, int(r["Grid_Size"]))][r["Counter_Name"]] = float(r["Counter_Value"])
    launches = collections.defaultdict(list)   # (name, grid) -> [merged counters per launch index]
    for p, ds in sorted(per.items()):
        seen = collections.Counter()
        for (_, name, grid), cs in sorted(ds.items()):
            k = (name, grid)
            i = seen[k]
            seen[k] += 1
            lst = launches[k]
            while len(lst) <= i:
                lst.append({})
            lst[i].update(cs)
    return launches


def req_bytes(c):
    return (128 * c.get("TCC_EA0_RDREQ_128B_sum", 0) + 64 * c.get("TCC_EA0_RDREQ_64B_sum", 0)
            + 32 * c.get("TCC_EA0_RDREQ_32B_sum", 0))


def main(root):
    out = {"what": __doc__.strip().splitlines()[0]}
    g = os.path.join(root, "gather")
    if os.path.isdir(g):
        plain = [json.loads(ln) for ln in open(os.path.join(g, "plain.jsonl")) if ln.startswith("{")]
        launches = passes(g)
        rows = []
        idx = collections.Counter()
        for rec in plain:
            name = rec["kernel"]
            grid = {"k_stream": 4096 * 256}.get(name, rec.get("lanes"))
            grid = ((grid + 255) // 256) * 256
            i = idx[(name, grid)]
            idx[(name, grid)] += 1
            c = launches.get((name, grid), [{}] * (i + 1))[i] if i < len(launches.get((name, grid), [])) else {}
            rb = req_bytes(c)
            row = dict(rec)
            row.update({
                "fabric_read_bytes_by_request_size": rb,
                "fetch_size_x2_bytes": 2 * 1024 * c.get("FETCH_SIZE", 0),
                "requests_128B": c.get("TCC_EA0_RDREQ_128B_sum"), "requests_64B": c.get("TCC_EA0_RDREQ_64B_sum"),
                "requests_32B": c.get("TCC_EA0_RDREQ_32B_sum"),
                "l2_hit": c.get("TCC_HIT_sum"), "l2_miss": c.get("TCC_MISS_sum"),
            })
            if rb:
                row["fetch_x2_over_request_bytes"] = row["fetch_size_x2_bytes"] / rb
                lines = rec.get("lines_128") or rec.get("distinct_lines_128")
                row["request_bytes_over_distinct_bytes"] = rb / (128 * lines) if lines else None
                if name == "k_walk":
                    row["request_bytes_over_gathered_lines"] = rb / (128 * rec["gather_lines_128"])
            rows.append(row)
        out["ubench"] = rows
        out["reading"] = (
            "k_stream (coalesced 16 B/lane, 1 GiB): every fabric read is one 128-B request, requests x 128 B = "
            "the bytes read, FETCH_SIZE = exactly half (the guide's gfx950 correction). The same holds for the "
            "main kernel's per-lane 160-B gather (k_once, k_walk): all requests are 128-B, so 2 x FETCH_SIZE = "
            "128 x requests there too -- the x2 correction is calibrated for this access pattern. k_once reads "
            "each table byte once yet fetches 1.24x the distinct lines (L2 re-misses between the ten 16-B "
            "pieces of a lane's entries); k_walk at 65,536 lanes (two 94 MB tables, C2's shape) fetches 4.9x "
            "the distinct table lines, 0.88 of all lines gathered: the re-reads are L2 misses served above it.")
    f = os.path.join(root, "flush")
    if os.path.isdir(f):
        recs = [json.loads(ln) for ln in open(os.path.join(f, "time.jsonl")) if ln.startswith("{")]
        summ = [r for r in recs if r.get("summary")]
        fl = {"timing": summ[-1] if summ else None, "reps": [r for r in recs if not r.get("summary")]}
        launches = passes(f)
        main = launches.get(("edv_main_kernel", 65536), [])
        prep = launches.get(("edv_prep_kernel", 3 * 65536), [])
        flush = launches.get(("edv_flush_kernel", 4096 * 256), [])
        if main:
            rbm = [req_bytes(c) for c in main if "TCC_EA0_RDREQ_128B_sum" in c]
            fl["main_fabric_read_bytes_per_launch"] = statistics.median(rbm) if rbm else None
            wr = [1024 * c["WRITE_SIZE"] for c in prep if "WRITE_SIZE" in c]
            rp = [req_bytes(c) for c in prep if "TCC_EA0_RDREQ_128B_sum" in c]
            fl["prep_write_bytes_per_launch"] = statistics.median(wr) if wr else None
            fl["prep_fabric_read_bytes_per_launch"] = statistics.median(rp) if rp else None
            fl["flush_kernel_read_write_bytes"] = ([req_bytes(c) for c in flush if "TCC_EA0_RDREQ_128B_sum" in c][:1]
                                                   + [1024 * c["WRITE_SIZE"] for c in flush if "WRITE_SIZE" in c][:1])
            fl["note"] = ("the counters see L2-to-fabric requests, Infinity-Cache hits included, so main's "
                          "request counts do not change with the flush; its time does, by the factor in timing")
        out["flush_probe"] = fl
    return out


if __name__ == "__main__":
    print(json.dumps(main(sys.argv[1]), indent=1))
