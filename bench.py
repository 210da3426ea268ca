#!/usr/bin/env python3
"""Benchmark: Ed25519 verifies/s on MI355X for Plenum's client-request
authentication hot path (BASELINE.json metric), with the INT32-VALU roofline
fraction, rocprof-counter VALU figures, the real C-ABI boundary timed on host
buffers, and the libsodium CPU baseline timed on the same box.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--reps R] [--batch B]
                  [--msg-len 256] [--total T] [--pipeline] [--no-e2e] [--no-cpu-baseline]

A "step" = one pass of the verifier (prep + main kernels) over one batch of
synthetic signed requests resident in HBM.  Default (BASELINE configs[1], C2):
B = 65,536 NYM-shaped 256-byte messages per GPU, distinct signers, all valid;
with N > 1 every rank verifies its own B-request shard (weak scaling).
--total T (C3, configs[2]): T requests split by request index over the ranks
(2,097,152 per GPU at T = 16,777,216 on 8 GPUs: strong scaling), 5 % of them
damaged (R bit, S + L, message byte, key bit) at known positions; every rank's
accept bytes are all-gathered (RCCL) and checked against the expected verdicts.

Timing: W warm-up steps (at least --warmup-seconds of them, so a short --warmup
gives the clocks the same settling time as a long one), then R repetitions of
exactly K steps, each bracketed by barrier + device sync; the max over ranks of
each repetition is taken and the MEDIAN repetition is reported.  The K steps
of a repetition are enqueued back to back on the library stream, strictly in
sequence (prep, main, prep, main, ...), so the kernel durations rocprofv3
reports for the run are the ones the roofline uses.  --pipeline times the
library's two-stream pipeline instead (prep of step k+1 beside main of step k).

The verify inputs are produced by the product's own GPU batch signer (row f-4),
never by the oracle; only the cpu_baseline leg uses oracle/ (the libsodium
harness oracle/sodium_batch.c, i.e. the reference's own CPU path).
"""
import argparse
import json
import os
import platform
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

from indy_plenum_amd import edv, shard, workload  # noqa: E402

# Algorithmic INT32 work per verify:
#   W(m) = 217,600 + 5,500 * ceil((m + 81) / 128)   (3,400 GF(p) mul/sq x 64 u32 mul-adds + SHA-512 blocks)
# The verify path is two launches per chunk (edv_prep_kernel, edv_main_kernel);
# the roofline prices the whole path: W(m) per verify over the sum of both
# kernels' HIP-event times.  (Round 1 priced the main kernel alone at
# (2,737 + 267) x 64 ops; with half-size scalars part of that work moved into
# prep and the rest shrank, so a per-kernel split of W would no longer mean
# anything.)
C3_TOTAL = 16777216


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


PMC_SUMMARY = os.path.join(ROOT, "profiles", "pmc_latest.json")


def pmc_figures(kernels, batch, msg_len, kernel_ms):
    """Counter-derived figures for the verify path (`kernels`, summed) from the
    committed rocprofv3 PMC summary (tools/pmc_summary.py), only if it was
    measured on these exact kernel sources at the default C2 shape; else
    (None, reason).  kernel_ms: the summed HIP-event time of those kernels."""
    if batch != 65536 or msg_len != 256 or not os.path.exists(PMC_SUMMARY):
        return None, "no PMC summary for this shape"
    with open(PMC_SUMMARY) as f:
        s = json.load(f)
    if s.get("kernel_source_sha256") != kernel_source_hash():
        return None, "PMC summary is stale (kernel sources changed since it was measured)"
    ks = [s["kernels"].get(k) for k in kernels]
    if not all(ks):
        return None, "kernel not in PMC summary"
    out = {"traffic": sum(k.get("hbm_bytes_per_launch", 0.0) for k in ks),
           "traffic_source": "%s: 2 x FETCH_SIZE + WRITE_SIZE per launch, prep + main (gfx950 correction; "
                             "Infinity-Cache (MALL) hits included, so an upper bound on DRAM bytes)"
                             % os.path.relpath(PMC_SUMMARY, ROOT)}
    cs = [k["counters"] for k in ks]
    if all("SQ_INSTS_VALU" in c for c in cs):
        valu = sum(c["SQ_INSTS_VALU"] for c in cs)  # wave-instructions per launch pair
        lane_ops = valu * 64  # one lane-op per active lane per VALU wave-instruction
        out.update({
            # a verify is one lane in each kernel (and in each prep side): per-lane
            # instructions = wave-instructions x 64 lanes / verifies
            "valu_insts_per_verify": valu * 64 / batch,
            "valu_int64_insts_per_verify": sum(c.get("SQ_INSTS_VALU_INT64", 0.0) for c in cs) * 64 / batch,
            "valu_int32_insts_per_verify": sum(c.get("SQ_INSTS_VALU_INT32", 0.0) for c in cs) * 64 / batch,
            "measured_valu_lane_ops_per_s": lane_ops / (kernel_ms * 1e-3),
            "measured_valu_frac_of_issue_peak": lane_ops / (kernel_ms * 1e-3) / PEAK_INT32,
            "per_kernel": {name: {"valu_insts_per_wave": k.get("valu_insts_per_wave"), "waves": k["counters"].get("SQ_WAVES"),
                                  "valu_busy": k.get("valu_busy"), "wave_cycle_split": k.get("wave_cycle_split"),
                                  "hbm_bytes_per_launch": k.get("hbm_bytes_per_launch")}
                           for name, k in zip(kernels, ks)},
        })
    return out, None


def w_total(m):
    return 217600 + 5500 * -(-(m + 81) // 128)


# INT32 VALU peak: 256 CUs x 64 lanes/clk (4 SIMDs at the 4-cycle VOP3 rate that
# v_mad_i64_i32 / v_mad_u64_u32 issue at, tools/ubench_valu.hip) x 2.4 GHz.
# Plain VOP2 ops (v_add_u32, v_xor_b32, ...) issue at twice that rate with two or
# more waves per SIMD (MI355X_MICROARCH.md "vector-instruction ISSUE cost"):
# PEAK_VOP2 is reported beside it.
PEAK_INT32 = 256 * 64 * 2.4e9
PEAK_VOP2 = 2 * PEAK_INT32


def cpu_info():
    model = platform.processor() or ""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else None
    return {"nproc": os.cpu_count(), "affinity_cpus": aff, "model": model,
            "omp_num_threads": os.environ.get("OMP_NUM_THREADS")}


def cpu_baseline(batch, budget_s):
    """libsodium 1.0.18 verify_detached over the same batch on the host cores,
    plus the reference's single-threaded Python chain (C1)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib as orc  # the baseline leg is the only oracle/ user here
    sb = orc.sodium_batch()
    if sb is None:
        return None
    sigs, pks, msgs, off = batch.host_copy()
    info = cpu_info()
    ncpu = info["affinity_cpus"] or info["nproc"] or 1
    # the GPU box's CPU share for one GPU is 16 threads (OMP_NUM_THREADS there);
    # the machine's nproc counts every CPU of the host, shared with other jobs
    threads = max(1, min(16, ncpu))
    acc = orc.sodium_verify_batch(sigs, pks, msgs, off, threads)  # warm + sanity
    assert acc.all()
    n = batch.n
    done, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < budget_s:
        orc.sodium_verify_batch(sigs, pks, msgs, off, threads)
        done += n
    dt = time.perf_counter() - t0
    k = min(n, 16384)
    t1 = time.perf_counter()
    orc.sodium_verify_batch(sigs[:64 * k], pks[:32 * k], msgs, off[:k + 1], 1)
    one = k / (time.perf_counter() - t1)
    out = {"value": done / dt, "unit": "verifies/s", "cores": threads, "kind": "reference",
           "sample": "%d passes over the %d-request batch (%d B msgs): libsodium %s crypto_sign_ed25519_verify_detached "
                     "(oracle/sodium_batch.c), %d threads, %.1f s" % (done // n, n, int(off[1] - off[0]),
                                                                      sb.sb_version().decode(), threads, dt),
           "one_thread_verifies_per_s": one, "host": info}
    try:
        out["c1_python_chain"] = c1_chain()
    except Exception as ex:  # the chain needs libsodium via ctypes; report why it is missing
        out["c1_python_chain"] = {"error": repr(ex)}
    return out


def c1_requests(n, seed=0xC1):
    """C1: NYM-style requests, distinct signers, identifier = b58(pk[:16]) and
    verkey '~' + b58(pk[16:]) registered, signed (GPU batch signer) over their
    SigningSerializer bytes (~150 B)."""
    from indy_plenum_amd import base58
    from indy_plenum_amd.client_authn import CoreAuthNr
    from indy_plenum_amd.signing_serializer import serialize_msg_for_signing
    rng = np.random.default_rng(seed)
    seeds = rng.integers(0, 256, size=(n, 32), dtype=np.uint8)
    pks, _ = edv.sign_arrays(seeds.tobytes(), b"\0" * 64, np.zeros(n + 1, dtype=np.uint64))
    pks = np.frombuffer(pks, np.uint8).reshape(n, 32)
    auth = CoreAuthNr()
    reqs = []
    for i in range(n):
        pk = pks[i].tobytes()
        idr = base58.b58encode(pk[:16]).decode()
        auth.addIdr(idr, "~" + base58.b58encode(pk[16:]).decode())
        reqs.append({"identifier": idr, "reqId": 1539648000000000 + i, "protocolVersion": 2,
                     "operation": {"type": "1", "dest": base58.b58encode(rng.bytes(16)).decode(),
                                   "verkey": "~" + base58.b58encode(rng.bytes(16)).decode()}})
    sers = [serialize_msg_for_signing(r) for r in reqs]
    off = np.zeros(n + 1, dtype=np.uint64)
    off[1:] = np.cumsum([len(s) for s in sers])
    _, sigs = edv.sign_arrays(seeds.tobytes(), b"".join(sers) + b"\0" * 64, off)
    sigs = sigs.tobytes()
    for i, r in enumerate(reqs):
        r["signature"] = base58.b58encode(sigs[64 * i:64 * i + 64]).decode()
    return auth, reqs


def c1_chain(n=3000):
    """The reference's CPU chain on C1: sequential CoreAuthNr.authenticate per
    request, Python restatement of P1-P7 + libsodium crypto_sign_open via ctypes
    (what libnacl does), one thread like the Node's Looper; native base58 and
    serializer off (the reference has none)."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import sodium_ref
    from indy_plenum_amd import base58, signing_serializer
    from indy_plenum_amd.client_authn import CoreAuthNr
    if sodium_ref.sodium() is None:
        return {"error": "libsodium not found"}
    auth, reqs = c1_requests(n)
    cpu = CoreAuthNr()
    cpu.clients = auth.clients
    saved = base58._native, signing_serializer._native
    base58._native = signing_serializer._native = None
    try:
        t0 = time.perf_counter()
        for r in reqs:
            assert cpu.authenticate(r, verifier=sodium_ref.SodiumVerifier) == [r["identifier"]]
        dt = time.perf_counter() - t0
    finally:
        base58._native, signing_serializer._native = saved
    return {"value": n / dt, "unit": "requests/s", "cores": 1, "requests": n,
            "what": "C1: sequential CoreAuthNr.authenticate (P1-P7 Python restatement) + libsodium crypto_sign_open "
                    "via ctypes, 1 thread"}


def median_time(f, reps):
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        f()
        ts.append(time.perf_counter() - t0)
    return statistics.median(ts)


def e2e_leg(batch, device_value, reps=5):
    """The drop-in boundary itself: edv_verify_batch on HOST buffers (H2D, kernels,
    D2H, synchronous), pageable numpy arrays and pinned (edv_host_alloc) arrays,
    median of `reps` calls each."""
    sigs, pks, msgs, off = batch.host_copy()
    n = batch.n
    want = batch.expected()
    acc = np.zeros(n, np.uint8)

    def call(s, p, m, o, a):
        edv._check(edv.lib().edv_verify_batch(s.ctypes.data, p.ctypes.data, m.ctypes.data, o.ctypes.data, n,
                                              a.ctypes.data, 1 << batch.device))

    call(sigs, pks, msgs, off, acc)  # warm: buffers sized, pinned staging allocated
    assert np.array_equal(acc, want)
    t_page = median_time(lambda: call(sigs, pks, msgs, off, acc), reps)
    # pinned: pack the same arrays into one page-locked arena
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
    call(ps, pp, pm, po, pa)
    assert np.array_equal(pa, want)
    t_pin = median_time(lambda: call(ps, pp, pm, po, pa), reps)
    # back to back through edv_verify_batch_async: batch k+1's copies run while
    # batch k computes (two verdict arrays in turn, waits one batch behind)
    pa2 = np.zeros(n, np.uint8)
    k_async = 10

    def stream_of_batches(s, p, m, o, accs):
        prev = None
        for k in range(k_async):
            t = edv.verify_async(s, p, m, o, accs[k % 2], device=batch.device)
            if prev is not None:
                edv.wait_async(prev, device=batch.device)
            prev = t
        edv.wait_async(prev, device=batch.device)

    acc2 = np.zeros(n, np.uint8)
    stream_of_batches(sigs, pks, msgs, off, (acc, acc2))
    assert np.array_equal(acc, want) and np.array_equal(acc2, want)
    t_apage = median_time(lambda: stream_of_batches(sigs, pks, msgs, off, (acc, acc2)), reps) / k_async
    stream_of_batches(ps, pp, pm, po, (pa, pa2))
    assert np.array_equal(pa, want) and np.array_equal(pa2, want)
    t_apin = median_time(lambda: stream_of_batches(ps, pp, pm, po, (pa, pa2)), reps) / k_async
    pb.free()
    return {"what": "edv_verify_batch on host buffers: H2D + kernels + D2H, synchronous, median of %d calls; "
                    "async_*: %d batches back to back through edv_verify_batch_async (waits one batch behind), "
                    "median of %d such runs" % (reps, k_async, reps),
            "async_pinned_verifies_per_s": n / t_apin, "async_pinned_ms_per_batch": 1e3 * t_apin,
            "async_pageable_verifies_per_s": n / t_apage, "async_pageable_ms_per_batch": 1e3 * t_apage,
            "async_pinned_vs_device_resident": (n / t_apin) / device_value,
            "requests": n, "pageable_verifies_per_s": n / t_page, "pageable_ms": 1e3 * t_page,
            "pinned_verifies_per_s": n / t_pin, "pinned_ms": 1e3 * t_pin,
            "pinned_vs_device_resident": (n / t_pin) / device_value,
            "pageable_vs_device_resident": (n / t_page) / device_value,
            "pcie_bytes_per_call": int(sigs.nbytes + pks.nbytes + off.nbytes + int(off[-1] - off[0]) + n)}


def node_path_leg(n=65536, reps=3):
    """f-1: CoreAuthNr.authenticate_batch over n C1-shaped requests on this GPU
    (native host prep, one verify call, replay)."""
    from indy_plenum_amd import _edvhost
    from indy_plenum_amd.req_authenticator import ReqAuthenticator
    auth, reqs = c1_requests(n, seed=0xF1)
    res = auth.authenticate_batch(reqs)
    assert all(x == [r["identifier"]] for x, r in zip(res, reqs))
    t = median_time(lambda: auth.authenticate_batch(reqs), reps)
    phases = _edvhost.last_phases()
    ra = ReqAuthenticator()
    ra.register_authenticator(auth)
    assert all(x == {r["identifier"]} for x, r in zip(ra.authenticate_batch(reqs), reqs))
    t_ra = median_time(lambda: ra.authenticate_batch(reqs), reps)
    return {"what": "CoreAuthNr.authenticate_batch, %d NYM requests (~150 B signing bytes), 1 GPU, median of %d; "
                    "native host prep on %d threads" % (n, reps, edv.PREP_THREADS),
            "requests_per_s": n / t, "ms": 1e3 * t, "phases_last_call_s": phases,
            "req_authenticator_requests_per_s": n / t_ra}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5, help="untimed steps first (at least --warmup-seconds of them)")
    ap.add_argument("--warmup-seconds", type=float, default=1.0)
    ap.add_argument("--reps", type=int, default=5, help="timed repetitions of --steps steps; the median is reported")
    ap.add_argument("--batch", type=int, default=65536, help="requests per GPU per step (C2)")
    ap.add_argument("--total", type=int, default=0,
                    help="C3: total requests per step, split by request index over the ranks (e.g. %d)" % C3_TOTAL)
    ap.add_argument("--msg-len", type=int, default=256)
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-e2e", action="store_true", help="skip the host-buffer boundary and node-path legs")
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
    # EDV_BENCH_FORCE_DIST=1 (check on a 1-GPU box): take the multi-rank path,
    # torch.cuda + RCCL beside libedv in one process, even for one rank
    json_out = sys.stdout
    if world > 1 or os.environ.get("EDV_BENCH_FORCE_DIST") == "1":
        # RCCL prints its version banner on stdout at communicator setup: keep
        # the original stdout for the one JSON line, send all else to stderr
        json_out = os.fdopen(os.dup(1), "w")
        sys.stdout.flush()
        os.dup2(2, 1)
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
    c3 = args.total > 0
    if c3:
        lo, hi = shard.shard_range(args.total, world, rank)   # one message length: equal counts
        n, start, damage = hi - lo, lo, 20
    else:
        n, start, damage = args.batch, rank * args.batch, 0
    batch = workload.DeviceBatch(n, device=dev, start=start, msg_len=args.msg_len, damage_every=damage)

    def step():
        if args.pipeline:
            batch.submit()
        else:
            batch.verify(stream=s)

    def drain():
        if args.pipeline:
            edv.pipeline_sync(dev)
        else:
            edv.sync(dev)

    s = edv.stream(dev)
    t0, done = time.perf_counter(), 0
    while done < args.warmup or time.perf_counter() - t0 < args.warmup_seconds:
        step()
        done += 1
        if done % 8 == 0:
            drain()
    drain()
    warm_steps = done
    ok = batch.accept()
    assert np.array_equal(ok, batch.expected()), "warm-up verdicts differ from the expected ones"

    def timed():
        drain()
        barrier()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            step()
        drain()
        t1 = time.perf_counter()
        barrier()
        return max_over_ranks(t1 - t0)

    reps = [timed() for _ in range(max(1, args.reps))]
    elapsed = statistics.median(reps)
    ms_step = 1e3 * elapsed / args.steps
    total = n * world * args.steps
    value = total / elapsed

    # per-kernel durations (HIP events on the kernels' own stream) on the first
    # chunk-sized slice of this rank's batch
    pn = min(n, 1 << 18)
    iters = max(3, min(args.steps, 10))
    prep_ms, main_ms = edv.profile_device(batch.d_sigs.ptr, batch.d_pks.ptr, batch.d_msgs.ptr, batch.d_off.ptr, pn,
                                          batch.d_accept.ptr, dev, iters)
    batch.verify()
    ok = batch.accept()
    if dist is not None:
        # untimed: gather every shard's accept bytes back into request order (RCCL all-gather)
        sys.path.insert(0, os.path.join(ROOT, "tools"))
        import torch
        from dist_gather import gather_accept
        bounds = ([shard.shard_range(args.total, world, r)[0] for r in range(world)] + [args.total] if c3
                  else [r * n for r in range(world + 1)])
        exp = np.ones(bounds[-1], np.uint8)
        exp[workload.damage_positions(0, bounds[-1], damage)] = 0
        full = gather_accept(dist, ok, bounds, device=None if one_dev else torch.device("cuda", local))
        verdicts_ok = bool(np.array_equal(full, exp))
    else:
        verdicts_ok = bool(np.array_equal(ok, batch.expected()))

    if rank != 0:
        if dist is not None:
            dist.destroy_process_group()
        return
    path_ms = prep_ms + main_ms
    ops = w_total(args.msg_len) * pn
    achieved = ops / (path_ms * 1e-3)
    pmc, why = pmc_figures(["edv_prep_kernel", "edv_main_kernel"], n, args.msg_len, path_ms)
    roofline = {"bound": "valu_int32", "kernel": "edv_prep_kernel + edv_main_kernel (the verify path, one launch each)",
                "achieved": achieved / 1e12, "peak": PEAK_INT32 / 1e12, "unit": "TOP/s",
                "frac": achieved / PEAK_INT32, "traffic": None, "traffic_unit": "bytes/launch pair",
                "traffic_source": why, "algorithmic_bytes": (64 + 32 + args.msg_len + 8 + 1) * pn,
                "ops_per_launch": ops, "kernel_ms": path_ms, "prep_kernel_ms": prep_ms, "main_kernel_ms": main_ms,
                "vop2_issue_peak": PEAK_VOP2 / 1e12,
                "convention": "achieved = SURVEY 8d W(m) INT32 ops per verify x verifies / (prep + main HIP-event "
                              "kernel time); peak = 256 CU x 64 lanes x 2.4 GHz (4-cycle VOP3 issue)"}
    if pmc:
        roofline.update(pmc)
    out = {
        "metric": "Ed25519 verifies/sec (256B msgs) + % of INT32 VALU peak",
        "value": value,
        "unit": "verifies/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_step,
        "higher_is_better": True,
        "scaling": "strong" if c3 else "weak",
        "vs_baseline": None,
        "dtype": "int32",
        "data": "synthetic: NYM-shaped signing bytes, distinct signers, keys+signatures made by the GPU batch signer"
                + ("; 5%% damaged at known positions" if c3 else ""),
        "config": ({"workload": "C3: %d Ed25519 verifies per step split by request index over %d GPU(s) (%d per GPU), "
                                "fixed %d-byte serialized requests, accept bytes all-gathered and checked"
                                % (args.total, world, n, args.msg_len),
                    "total_per_step": args.total, "per_gpu": n, "msg_len": args.msg_len,
                    "parallelism": "shard-by-request-index x%d" % world} if c3 else
                   {"workload": "C2: %d Ed25519 verifies per GPU per step, fixed %d-byte serialized requests, distinct "
                                "signers%s" % (n, args.msg_len, "" if world == 1 else "; shard by request index"),
                    "batch_per_gpu": n, "msg_len": args.msg_len, "parallelism": "shard-by-request-index x%d" % world}),
        "roofline": roofline,
        "verdicts_as_expected": verdicts_ok,
        "timing": {"mode": "pipelined (prep of step k+1 beside main of step k)" if args.pipeline else "sequential",
                   "reps_s": reps, "median_of": len(reps), "warmup_steps_run": warm_steps,
                   "kernel_sum_ms": prep_ms + main_ms,
                   "gap_ms_per_step": ms_step - (prep_ms + main_ms) * n / pn},
    }
    if world == 1 and not c3 and not args.no_e2e:
        out["e2e"] = e2e_leg(batch, value)
        try:
            out["node_path"] = node_path_leg()
        except Exception as ex:
            out["node_path"] = {"error": repr(ex)}
    if world == 1 and not args.no_cpu_baseline:
        cb = cpu_baseline(batch, args.cpu_seconds)
        out["cpu_baseline"] = cb
        if cb:
            out["gpu_over_cpu"] = value / cb["value"]
    print(json.dumps(out), file=json_out, flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
