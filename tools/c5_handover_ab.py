"""C5 overlap mode, hand-over A/B on one box: a prod's batch handed over at the
end of the same prod when the GPU is already done (handover="early", the
default) against always at the node's next prod ("next"), interleaved with the
no-verify ceiling; ordered requests/s, auth and GC shares, how many prods
handed over early, request latency (p50).  One JSON line per run.

  python tools/c5_handover_ab.py [N] [REPS]
"""
import gc
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import bench_pool  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 20000
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    clients, reqs = bench_pool.make_flood(n)
    bench_pool.run("gpu_batched_overlap", clients, reqs[:500])
    for r in range(reps):
        for mode, ho in (("gpu_batched_overlap", "early"), ("gpu_batched_overlap", "next"),
                         ("no_verify_ceiling", "early")):
            gc.collect()
            st = bench_pool.run(mode, clients, reqs, handover=ho)
            lat = st["latency_ms"]
            print(json.dumps({"rep": r, "mode": mode, "handover": ho if mode != "no_verify_ceiling" else None,
                              "ordered_req_per_s": round(st["ordered_req_per_s_one_process"]),
                              "auth_share": round(st["auth_share_of_node_time"], 4),
                              "gc_share": round(st["gc_share_of_node_time"], 4),
                              "auth_calls": st["auth_calls"], "early_handovers": st["early_handovers"],
                              "receipt_p50_ms": round(lat["receipt"]["p50"], 3),
                              "monitor_p50_ms": round(lat["monitor"]["p50"], 3)}), flush=True)
    for ho in ("early", "next"):
        st = bench_pool.run("gpu_batched_overlap", clients, reqs[:1200], rate=400, handover=ho)
        lat = st["latency_ms"]
        print(json.dumps({"paced_400_req_s": True, "handover": ho, "early_handovers": st["early_handovers"],
                          "submit_p50_ms": round(lat["submit"]["p50"], 3), "submit_p99_ms": round(lat["submit"]["p99"], 3),
                          "receipt_p50_ms": round(lat["receipt"]["p50"], 3)}), flush=True)


if __name__ == "__main__":
    main()
