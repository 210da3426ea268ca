"""cProfile of one C5 pool run (tools/bench_pool.py) in a chosen mode:
  python tools/prof_pool.py [gpu_batched_overlap|gpu_batched|no_verify_ceiling] [N]"""
import cProfile
import io
import os
import pstats
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
sys.path.insert(0, ROOT)
import bench_pool  # noqa: E402

mode = sys.argv[1] if len(sys.argv) > 1 else "gpu_batched_overlap"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 20000
clients, reqs = bench_pool.make_flood(n)
bench_pool.run(mode, clients, reqs[:500])
pr = cProfile.Profile()
pr.enable()
st = bench_pool.run(mode, clients, reqs)
pr.disable()
s = io.StringIO()
pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(30)
print(s.getvalue())
print(st)
