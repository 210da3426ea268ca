"""Where the C5 pool's cyclic-GC time comes from: one warm run per mode
(tools/bench_pool.py), with collections counted and timed per generation and
the live GC-tracked object count sampled at each collection's start.

  python tools/c5_gc_probe.py [N] [MODE ...]
"""
import gc
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import bench_pool  # noqa: E402


class GenClock:
    def __init__(self):
        self.n = [0, 0, 0]
        self.s = [0.0, 0.0, 0.0]
        self.collected = [0, 0, 0]
        self._t = None

    def __call__(self, phase, info):
        if phase == "start":
            self._t = time.perf_counter()
        elif self._t is not None:
            g = info["generation"]
            self.n[g] += 1
            self.s[g] += time.perf_counter() - self._t
            self.collected[g] += info["collected"]
            self._t = None


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 20000
    # MODE: bench_pool mode, or gpu_batched_overlap:next / :early (the hand-over)
    modes = sys.argv[2:] or ["gpu_batched_overlap:early", "gpu_batched_overlap:next", "no_verify_ceiling"]
    clients, reqs = bench_pool.make_flood(n)
    for spec in modes:
        mode, _, ho = spec.partition(":")
        ho = ho or "early"
        bench_pool.run(mode, clients, reqs[:500], handover=ho)
        gc.collect()
        clk = GenClock()
        gc.callbacks.append(clk)
        try:
            st = bench_pool.run(mode, clients, reqs, handover=ho)
        finally:
            gc.callbacks.remove(clk)
        print(json.dumps({"mode": spec, "ordered_req_per_s": round(st["ordered_req_per_s_one_process"]),
                          "wall_s": round(st["wall_s"], 4), "gc_share": round(st["gc_share_of_node_time"], 4),
                          "auth_share": round(st["auth_share_of_node_time"], 4),
                          "collections": clk.n, "gc_s": [round(x, 4) for x in clk.s], "collected": clk.collected,
                          "thresholds": gc.get_threshold(), "tracked_after": len(gc.get_objects())}), flush=True)


if __name__ == "__main__":
    main()
