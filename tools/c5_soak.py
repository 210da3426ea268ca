"""Soak of the Node path a long-running pool exercises: the 4-node C5 pool in
overlap mode (early hand-over) run R times over the same 20,000-request flood
in one process; after each run the process's resident memory, the library's
device memory (edv.context_memory) and the ordered rate.  A leak in the native
batch handles, arenas, async slots or tickets would show as growth.

  python tools/c5_soak.py [ROUNDS] [N]
"""
import gc
import json
import os
import resource
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import bench_pool  # noqa: E402


def rss_mb():
    with open("/proc/self/status") as f:
        for line in f:
            if line.startswith("VmRSS:"):
                return int(line.split()[1]) / 1024.0
    return resource.getrusage(resource.RUSAGE_SELF).ru_maxrss / 1024.0


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 20000
    from indy_plenum_amd import edv
    clients, reqs = bench_pool.make_flood(n)
    for r in range(rounds):
        st = bench_pool.run("gpu_batched_overlap", clients, reqs)
        gc.collect()
        mem = edv.context_memory(0)
        print(json.dumps({"round": r, "ordered_req_per_s": round(st["ordered_req_per_s_one_process"]),
                          "ordered_per_node": st["ordered_per_node"], "nacks": sum(st["nacks_per_node"]),
                          "early_handovers": st["early_handovers"], "rss_mb": round(rss_mb(), 1),
                          "device_bytes": mem["total"], "async_slots_bytes": mem["async_slots"]}), flush=True)


if __name__ == "__main__":
    main()
