#!/usr/bin/env python3
"""Benchmark: Ed25519 verifies/s on MI355X for Plenum's client-request
authentication hot path (BASELINE.json metric), with the INT32-VALU roofline
fraction and the libsodium CPU baseline timed on the same box.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B] [--msg-len 256]

A "step" = one pass of the verifier (prep + main kernels) over one batch of B
synthetic signed requests resident in HBM (default B = 65,536 x 256-byte
NYM-shaped messages, distinct signers: BASELINE.json configs[1]).  The K timed
steps are enqueued back to back on the library stream, strictly in sequence
(prep, main, prep, main, ...), so the kernel durations rocprofv3 reports for the
run are the ones the roofline uses.  --pipeline times the library's two-stream
pipeline instead (prep of step k+1 beside main of step k, double-buffered
state; +1-3 %) and reports the sequential rate beside it.  With N > 1
(launched by torch.distributed.run) every rank verifies its own B-request shard
of the request index space: weak scaling, no collective on the data path; the
per-request accept bytes are checked after the timed region.

The verify inputs are produced by the product's own GPU batch signer (row f-4),
never by the oracle; only the cpu_baseline leg uses oracle/ (the libsodium
harness oracle/sodium_batch.c, i.e. the reference's own CPU path).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

from indy_plenum_amd import edv, workload  # noqa: E402

# Algorithmic INT32 work per verify:
#   W(m) = 217,600 + 5,500 * ceil((m + 81) / 128)   (3,400 GF(p) mul/sq x 64 u32 mul-adds + SHA-512 blocks)
# split by kernel: main = V8 loop + V9 encode = (2,737 + 267) x 64; prep = the rest.
MAIN_OPS = (2737 + 267) * 64


def kernel_source_hash():
    """SHA-256 over the HIP sources of libedv.so (ties a committed PMC summary to the code it measured)."""
    import hashlib
    d = os.path.join(ROOT, "indy-plenum_amd", "csrc")
    h = hashlib.sha256()
    for f in sorted(os.listdir(d)):
        if f.endswith((".hip", ".h")):
            h.update(f.encode())
            h.update(open(os.path.join(d, f), "rb").read())
    return h.hexdigest()


PMC_SUMMARY = os.path.join(ROOT, "profiles", "pmc_hbm_latest.json")


def measured_traffic(kernel, batch, msg_len):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 PMC summary
    (tools/pmc_summary.py), only if it was measured on these exact kernel sources
    at the default C2 shape; else None."""
    if batch != 65536 or msg_len != 256 or not os.path.exists(PMC_SUMMARY):
        return None, "no PMC summary for this shape"
    with open(PMC_SUMMARY) as f:
        s = json.load(f)
    if s.get("kernel_source_sha256") != kernel_source_hash():
        return None, "PMC summary is stale (kernel sources changed since it was measured)"
    k = s["kernels"].get(kernel)
    if not k:
        return None, "kernel not in PMC summary"
    return k["hbm_bytes_per_launch"], "profiles/pmc_hbm_latest.json: (2 x FETCH_SIZE + WRITE_SIZE) KiB per launch"


def w_total(m):
    return 217600 + 5500 * -(-(m + 81) // 128)


# INT32 VALU peak: 256 CUs x 64 lanes/clk (4 SIMDs at the 4-cycle VOP3 rate that
# v_mad_i64_i32 / v_mad_u64_u32 issue at, tools/ubench_valu.hip) x 2.4 GHz.
PEAK_INT32 = 256 * 64 * 2.4e9


def cpu_baseline(batch, budget_s):
    """libsodium 1.0.18 verify_detached over the same batch on the host cores."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib as orc  # the baseline leg is the only oracle/ user here
    sb = orc.sodium_batch()
    sigs, pks, msgs, off = batch.host_copy()
    if sb is None:
        return None
    ncpu = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    threads = max(1, min(16, ncpu))  # the GPU box's CPU share for one GPU is 16 threads
    acc = orc.sodium_verify_batch(sigs, pks, msgs, off, threads)  # warm + sanity
    assert acc.all()
    n = batch.n
    done, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < budget_s:
        orc.sodium_verify_batch(sigs, pks, msgs, off, threads)
        done += n
    dt = time.perf_counter() - t0
    # single-thread reference point on a smaller slice
    k = min(n, 16384)
    o1 = off[:k + 1]
    t1 = time.perf_counter()
    orc.sodium_verify_batch(sigs[:64 * k], pks[:32 * k], msgs, o1, 1)
    one = k / (time.perf_counter() - t1)
    return {"value": done / dt, "unit": "verifies/s", "cores": threads, "kind": "reference",
            "sample": "%d passes over the %d-request batch (%d B msgs): libsodium %s crypto_sign_ed25519_verify_detached "
                      "(oracle/sodium_batch.c), %d threads, %.1f s; 1 thread: %.0f verifies/s"
                      % (done // n, n, int(off[1] - off[0]), sb.sb_version().decode(), threads, dt, one)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=50, help="untimed steps first (clocks settle; ~50 ms)")
    ap.add_argument("--batch", type=int, default=65536, help="requests per GPU per step")
    ap.add_argument("--msg-len", type=int, default=256)
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--pipeline", action="store_true",
                    help="time the two-stream pipelined submission (prep of step k+1 beside main of step k)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # EDV_BENCH_ONE_DEVICE=1 (rehearsal on a 1-GPU box only): every rank uses device 0
    # and gloo, since RCCL refuses two ranks on one GPU
    one_dev = os.environ.get("EDV_BENCH_ONE_DEVICE") == "1"
    dist = None
    if world > 1:
        import torch
        import torch.distributed as tdist
        if one_dev:
            tdist.init_process_group("gloo")
        else:
            torch.cuda.set_device(local)
            tdist.init_process_group("nccl")  # RCCL over xGMI
        dist = tdist

    def barrier():
        if dist is not None:
            dist.barrier()

    def max_over_ranks(x):
        if dist is None:
            return x
        import torch
        t = torch.tensor([x], dtype=torch.float64, device="cpu" if one_dev else "cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    dev = 0 if one_dev else local
    n = args.batch
    # this rank's shard of the request index space: [rank * n, (rank + 1) * n)
    batch = workload.DeviceBatch(n, device=dev, start=rank * n, msg_len=args.msg_len)

    for _ in range(args.warmup):
        batch.verify()
        if args.pipeline:
            batch.submit()
    if args.pipeline:
        edv.pipeline_sync(dev)
    ok = batch.accept()
    assert ok.all(), "warm-up verify rejected %d valid signatures" % int((ok == 0).sum())

    # Timed region: K steps enqueued back to back (host launch latency never
    # sits between steps), closed by a device sync; with --pipeline, on the
    # library's two-stream pipeline (edv_verify_batch_dev_pipelined) instead.
    def timed(submit, drain):
        edv.sync(dev)
        drain()
        barrier()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            submit()
        drain()
        t1 = time.perf_counter()
        barrier()
        return max_over_ranks(t1 - t0)

    s = edv.stream(dev)
    seq_elapsed = timed(lambda: batch.verify(stream=s), lambda: edv.sync(dev))
    elapsed = timed(batch.submit, lambda: edv.pipeline_sync(dev)) if args.pipeline else seq_elapsed
    ms_step = 1e3 * elapsed / args.steps
    total = n * world * args.steps
    value = total / elapsed

    # per-kernel durations (HIP events on the kernels' own stream), same batch
    iters = max(3, min(args.steps, 10))
    prep_ms, main_ms = edv.profile_device(batch.d_sigs.ptr, batch.d_pks.ptr, batch.d_msgs.ptr, batch.d_off.ptr, n,
                                          batch.d_accept.ptr, dev, iters)
    ok = batch.accept()
    if dist is not None:
        # untimed: gather every shard's accept bytes back into request order (RCCL all-gather)
        from indy_plenum_amd import shard
        import torch
        full = shard.gather_accept(dist, ok, n * world, device=None if one_dev else torch.device("cuda", local))
        all_ok = bool(full.all())
    else:
        all_ok = bool(ok.all())

    if rank != 0:
        if dist is not None:
            dist.destroy_process_group()
        return
    achieved = MAIN_OPS * n / (main_ms * 1e-3)
    traffic, traffic_src = measured_traffic("edv_main_kernel", n, args.msg_len)
    whole = w_total(args.msg_len) * n / ((prep_ms + main_ms) * 1e-3)
    out = {
        "metric": "Ed25519 verifies/sec (256B msgs) + % of INT32 VALU peak",
        "value": value,
        "unit": "verifies/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_step,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "int32",
        "data": "synthetic: NYM-shaped signing bytes, distinct signers, keys+signatures made by the GPU batch signer",
        "config": {"workload": "C2: %d Ed25519 verifies per GPU per step, fixed %d-byte serialized requests, distinct "
                               "signers%s" % (n, args.msg_len, "" if world == 1 else "; C3-style shard by request index"),
                   "batch_per_gpu": n, "msg_len": args.msg_len, "parallelism": "shard-by-request-index x%d" % world},
        "roofline": {"bound": "valu_int32", "kernel": "edv_main_kernel",
                     "achieved": achieved / 1e12, "peak": PEAK_INT32 / 1e12, "unit": "TOP/s",
                     "frac": achieved / PEAK_INT32, "traffic": traffic, "traffic_unit": "bytes/launch",
                     "traffic_source": traffic_src, "algorithmic_bytes": (64 + 32 + args.msg_len + 8 + 1) * n,
                     "ops_per_launch": MAIN_OPS * n, "kernel_ms": main_ms, "prep_kernel_ms": prep_ms,
                     "whole_path_frac": whole / PEAK_INT32},
        "all_accepted": bool(all_ok),
        "timing": {"mode": "pipelined (prep of step k+1 beside main of step k)" if args.pipeline else "sequential",
                   "sequential_ms_per_step": 1e3 * seq_elapsed / args.steps,
                   "sequential_value": n * world * args.steps / seq_elapsed},
    }
    if world == 1 and not args.no_cpu_baseline:
        cb = cpu_baseline(batch, args.cpu_seconds)
        out["cpu_baseline"] = cb
        if cb:
            out["gpu_over_cpu"] = value / cb["value"]
    print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
