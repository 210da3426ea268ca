"""Where the C5 overlap pool spends its host time: cProfile over one
gpu_batched_overlap run (tools/bench_pool.py) after a warm-up, top functions
by own time, plus the pool's stats line.

  python tools/c5_profile.py [N] [MODE]
"""
import cProfile
import io
import json
import os
import pstats
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import bench_pool  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 20000
    mode = sys.argv[2] if len(sys.argv) > 2 else "gpu_batched_overlap"
    clients, reqs = bench_pool.make_flood(n)
    bench_pool.run(mode, clients, reqs[:500])
    st = bench_pool.run(mode, clients, reqs)
    print(json.dumps({k: st[k] for k in ("wall_s", "ordered_req_per_s_one_process", "auth_share_of_node_time",
                                         "gc_share_of_node_time", "max_node_busy_s")}))
    pr = cProfile.Profile()
    pr.enable()
    bench_pool.run(mode, clients, reqs)
    pr.disable()
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(30)
    print(s.getvalue())


if __name__ == "__main__":
    main()
