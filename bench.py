#!/usr/bin/env python3
"""Benchmark: Ed25519 verifies/s on MI355X for Plenum's client-request
authentication hot path (BASELINE.json metric), with the INT32-VALU roofline
fraction, rocprof-counter VALU figures, the real C-ABI boundary timed on host
buffers, the C4/C5 configurations, and the libsodium CPU baseline timed on the
same box.  No PyTorch anywhere: the GPUs are driven through libedv.so only.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--reps R] [--batch B]
                  [--total T] [--weak] [--msg-len 256] [--pipeline] [--spawn]
                  [--no-e2e] [--no-extra] [--no-cpu-baseline]

A "step" = one pass of the verifier (prep + main kernels) over one batch of
synthetic signed requests resident in HBM.

  N = 1 (default):  BASELINE configs[1] (C2): B = 65,536 NYM-shaped 256-byte
                    messages, distinct signers, all valid.  --total T runs C3's
                    T requests on the one GPU instead.
  N > 1:            BASELINE configs[2] (C3): T = 16,777,216 requests per step
                    (--total overrides), split by request index into N
                    contiguous shards, one per GPU (strong scaling; 5 % of the
                    requests damaged at known positions, four kinds); after the
                    timed region every shard's accept bytes are copied (D2H) and
                    gathered into their slices of one host array on rank 0 and
                    checked.  --weak keeps C2's B requests per GPU instead.

Processes: one per GPU.  Under torch.distributed.run (RANK / WORLD_SIZE /
LOCAL_RANK in the environment) each rank drives device LOCAL_RANK.  Started
directly with --gpus N > 1 (or --spawn), this script launches the N ranks
itself, before anything touches a GPU, and only relays their exit status.  The
ranks meet over a loopback TCP rendezvous (class Rendezvous: barrier, max of
the per-rank times, gather of the accept bytes); there is no collective inside
verification.

Timing: W warm-up steps (at least --warmup-seconds of them), then R
repetitions of exactly K steps, each bracketed by barrier + device sync; the
max over ranks of each repetition is taken and the MEDIAN repetition is
reported.  value = requests of all ranks / that time.  The K steps are enqueued
back to back on the library stream (prep, main, prep, main, ...), so the kernel
durations rocprofv3 reports for the run are the ones the roofline uses.

The verify inputs are produced by the product's own GPU batch signer (row f-4),
never by the oracle; only the cpu_baseline leg uses oracle/ (the libsodium
harness oracle/sodium_batch.c, i.e. the reference's own CPU path).
"""
import argparse
import json
import math
import os
import platform
import socket
import statistics
import struct
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

METRIC = "Ed25519 verifies/sec at 1/8 MI355X (256B msgs) + % of INT32 VALU peak vs host CPU"
C3_TOTAL = 16777216
C3_DAMAGE_EVERY = 20      # 5 % invalid

# Algorithmic INT32 work per verify:
#   W(m) = 217,600 + 5,500 * ceil((m + 81) / 128)   (3,400 GF(p) mul/sq x 64 u32 mul-adds + SHA-512 blocks)
# The verify path is two launches per chunk (edv_prep_kernel, edv_main_kernel);
# the roofline prices the whole path: W(m) per verify over the sum of both
# kernels' HIP-event times.
# INT32 VALU peak: 256 CUs x 64 lanes/clk (4 SIMDs at the 4-cycle VOP3 rate that
# v_mad_i64_i32 / v_mad_u64_u32 issue at, tools/ubench_valu.hip) x 2.4 GHz.
# Plain VOP2 ops issue at twice that rate with two or more waves per SIMD
# (MI355X_MICROARCH.md "vector-instruction ISSUE cost"): PEAK_VOP2 beside it.
PEAK_INT32 = 256 * 64 * 2.4e9
PEAK_VOP2 = 2 * PEAK_INT32
PMC_SUMMARY = os.path.join(ROOT, "profiles", "pmc_latest.json")
PEAK_HBM = 8e12  # B/s, MI355X_MICROARCH.md "HBM"
# the R side's [S]B gathers per verify: kBTables (12) entries of 128 B (edv_verify_core.h)
SB_GATHER_BYTES = 12 * 128
# the controlled Infinity-Cache run (tools/flush_probe.py):
# main kernel time with every table line forced to DRAM between prep and main
FLUSH_PROBE = os.path.join(ROOT, "profiles", "r05", "flush_probe_s15.jsonl")


def w_blocks(m):
    return -(-(m + 81) // 128)


def w_total(m):
    return 217600 + 5500 * w_blocks(m)


def device_code_hash(lib=None):
    """SHA-256 of the gfx950 device code inside libedv.so (its .hip_fatbin ELF
    section): ties a committed PMC summary to the kernels it measured; host-only
    changes to the library leave it unchanged."""
    import hashlib
    import struct
    path = lib or os.path.join(ROOT, "indy-plenum_amd", "libedv.so")
    b = open(path, "rb").read()
    shoff = struct.unpack_from("<Q", b, 0x28)[0]
    shentsize, shnum, shstrndx = struct.unpack_from("<HHH", b, 0x3A)

    def sh(i):
        return struct.unpack_from("<IIQQQQ", b, shoff + i * shentsize)
    names = sh(shstrndx)[4]
    for i in range(shnum):
        nm, _typ, _fl, _addr, off, size = sh(i)
        if b[names + nm:b.index(b"\0", names + nm)] == b".hip_fatbin":
            return hashlib.sha256(b[off:off + size]).hexdigest()
    raise ValueError("no .hip_fatbin section in %s" % path)


# What the traffic figure is ("HBM traffic, calibrated"):
# profiles/r05/gather_calibration_s1.json, flush_probe_s1.jsonl.
TRAFFIC_NOTE = ("L2-to-fabric bytes, calibrated on known byte counts for this gather pattern "
                "(tools/ubench_gather.hip: 128 B x the L2's 128-B fabric read requests = the bytes, 2 x FETCH_SIZE "
                "agrees): the main kernel gathers one 160-B entry per window from each of two per-lane 1,440-B point "
                "tables the prep kernel wrote, ~4.9x re-read within the launch and served on die (L2 misses, "
                "Infinity-Cache hits; no gfx950 counter separates those from DRAM); the prep kernel's R side gathers "
                "12 x 128 B per verify from the 3 GiB shared [S]B tables (random lines: DRAM). What can reach DRAM "
                "is bounded by the distinct bytes: prep's reads + prep's writes + main's first reads of the tables")
def pmc_figures(kernels, batch, msg_len, kernel_ms):
    """Counter-derived figures for the verify path (`kernels`, summed) from the
    committed rocprofv3 PMC summary (tools/pmc_summary.py), only if it was
    measured on these exact kernel sources at the default C2 shape; else
    (None, reason).  kernel_ms: the summed HIP-event time of those kernels."""
    if batch != 65536 or msg_len != 256 or not os.path.exists(PMC_SUMMARY):
        return None, "no PMC summary for this shape"
    with open(PMC_SUMMARY) as f:
        s = json.load(f)
    if s.get("device_code_sha256") != device_code_hash():
        return None, "PMC summary is stale (the library's device code changed since it was measured)"
    ks = [s["kernels"].get(k) for k in kernels]
    if not all(ks):
        return None, "kernel not in PMC summary"
    out = {"traffic": sum(k.get("hbm_bytes_per_launch", 0.0) for k in ks),
           "traffic_source": "%s: fabric read bytes from the L2's request-size counters (128 x TCC_EA0_RDREQ_128B "
                             "+ 64 x _64B + 32 x _32B; 2 x FETCH_SIZE agrees) + WRITE_SIZE, per launch, prep + main; "
                             "Infinity-Cache (MALL) hits included, so an upper bound on DRAM bytes"
                             % os.path.relpath(PMC_SUMMARY, ROOT)}
    for key in ("dram_bytes_per_launch_bound", "dram_note"):
        if key in s:
            out[key] = s[key]
    out["traffic_per_verify_bytes"] = out["traffic"] / batch
    prep, main = s["kernels"].get("edv_prep_kernel", {}), s["kernels"].get("edv_main_kernel", {})
    if "read_bytes" in prep and "read_bytes" in main:
        split = {"inputs_and_sb_tables_read_by_prep": prep["read_bytes"] / batch,
                 "sb_table_gathers_algorithmic": SB_GATHER_BYTES,
                 "tables_and_digits_written_by_prep": prep["write_bytes"] / batch,
                 "tables_gathered_by_main": main["read_bytes"] / batch}
        out["traffic_split_per_verify_bytes"] = split
        # distinct bytes: what prep read (inputs, [S]B entries), what it wrote,
        # main's first read of the two per-lane tables
        dram = split["inputs_and_sb_tables_read_by_prep"] + split["tables_and_digits_written_by_prep"] + 2 * 1440
        out["dram_bytes_per_verify_upper_bound"] = dram
        out["dram_upper_bound_note"] = ("every distinct byte crossing DRAM once each way (nothing kept in the 256 MiB "
                                        "Infinity Cache from prep to main); the re-reads stay on die")
    out["traffic_note"] = TRAFFIC_NOTE
    if os.path.exists(FLUSH_PROBE):
        summ = [json.loads(ln) for ln in open(FLUSH_PROBE) if '"summary"' in ln]
        if summ:
            out["main_kernel_time_with_tables_forced_to_dram"] = {
                "ratio": summ[-1]["main_flushed_over_plain"],
                "source": os.path.relpath(FLUSH_PROBE, ROOT) + ": a 512 MiB read+rewrite between prep and main"}
    cs = [k["counters"] for k in ks]
    if all("SQ_INSTS_VALU" in c for c in cs):
        valu = sum(c["SQ_INSTS_VALU"] for c in cs)  # wave-instructions per launch pair
        lane_ops = valu * 64  # one lane-op per active lane per VALU wave-instruction
        out.update({
            "valu_insts_per_verify": valu * 64 / batch,

            "measured_valu_lane_ops_per_s": lane_ops / (kernel_ms * 1e-3),
            "measured_valu_frac_of_issue_peak": lane_ops / (kernel_ms * 1e-3) / PEAK_INT32,
            **({"valu_int64_insts_per_verify": sum(c["SQ_INSTS_VALU_INT64"] for c in cs) * 64 / batch,
                "valu_int32_insts_per_verify": sum(c["SQ_INSTS_VALU_INT32"] for c in cs) * 64 / batch}
               if all("SQ_INSTS_VALU_INT64" in c and "SQ_INSTS_VALU_INT32" in c for c in cs) else {}),
            "per_kernel": {name: {"valu_insts_per_wave": k.get("valu_insts_per_wave"), "waves": k["counters"].get("SQ_WAVES"),
                                  "valu_busy": k.get("valu_busy"), "wave_cycle_split": k.get("wave_cycle_split"),
                                  "hbm_bytes_per_launch": k.get("hbm_bytes_per_launch"),
                                  "l2_hit_rate": k.get("l2_hit_rate")}
                           for name, k in zip(kernels, ks)},
        })
    return out, None


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
    quota = None
    try:  # cgroup v2
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()
            quota = None if q == "max" else float(q) / float(per)
    except (OSError, ValueError):
        try:  # cgroup v1
            with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as f:
                q = float(f.read())
            with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
                per = float(f.read())
            quota = q / per if q > 0 else None
        except (OSError, ValueError):
            pass
    ncpu = aff or os.cpu_count() or 1
    # the CPUs this process can actually keep busy: its affinity, capped by the
    # cgroup's CPU-time quota (on the GPU box: 256 CPUs visible, 16 CPUs of time)
    effective = max(1, min(ncpu, int(math.ceil(quota)))) if quota else ncpu
    return {"nproc": os.cpu_count(), "affinity_cpus": aff, "cgroup_cpu_quota": quota, "effective_cpus": effective,
            "model": model, "omp_num_threads": os.environ.get("OMP_NUM_THREADS")}


# ------------------------------------------------------------------ ranks
class Rendezvous:
    """The ranks of one bench run on one node, over loopback TCP: rank 0
    listens on an ephemeral port it publishes in a file named by a token all
    ranks share (the launcher's, or torch.distributed.run's agent pid and
    MASTER_PORT); the others connect.  Collectives are synchronous: every rank
    sends, rank 0 answers.  Used only outside the timed region and for the
    barriers around it."""

    def __init__(self, rank, world, token, timeout=900.0):
        self.rank, self.world, self.peers, self.sock = rank, world, [], None
        if world == 1:
            return
        path = os.path.join(tempfile.gettempdir(), "edv_bench_%s.port" % token)
        deadline = time.time() + timeout
        if rank == 0:
            srv = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
            srv.bind(("127.0.0.1", 0))
            srv.listen(world)
            tmp = path + ".tmp%d" % os.getpid()
            with open(tmp, "w") as f:
                f.write(str(srv.getsockname()[1]))
            os.replace(tmp, path)
            srv.settimeout(timeout)
            peers = {}
            try:
                while len(peers) < world - 1:
                    c, _ = srv.accept()
                    c.settimeout(timeout)
                    peers[struct.unpack("<I", self._recvn(c, 4))[0]] = c
            finally:
                srv.close()
                try:
                    os.unlink(path)
                except OSError:
                    pass
            self.peers = [peers[r] for r in range(1, world)]
        else:
            while True:
                try:
                    with open(path) as f:
                        port = int(f.read())
                    self.sock = socket.create_connection(("127.0.0.1", port), timeout=10)
                    break
                except (OSError, ValueError):
                    if time.time() > deadline:
                        raise RuntimeError("rank %d: no rendezvous with rank 0 (%s)" % (rank, path))
                    time.sleep(0.05)
            self.sock.settimeout(timeout)
            self.sock.sendall(struct.pack("<I", rank))

    @staticmethod
    def _recvn(s, n):
        buf = bytearray()
        while len(buf) < n:
            b = s.recv(min(n - len(buf), 1 << 20))
            if not b:
                raise RuntimeError("bench rendezvous: a rank went away")
            buf += b
        return bytes(buf)

    def _send(self, s, payload):
        s.sendall(struct.pack("<Q", len(payload)) + payload)

    def _recv(self, s):
        return self._recvn(s, struct.unpack("<Q", self._recvn(s, 8))[0])

    def gather(self, payload, broadcast=True):
        """Every rank's payload (bytes), in rank order, on rank 0 (and on every
        rank when broadcast)."""
        if self.world == 1:
            return [payload]
        if self.rank == 0:
            got = [payload] + [self._recv(c) for c in self.peers]
            if broadcast:
                blob = b"".join(struct.pack("<Q", len(g)) + g for g in got)
                for c in self.peers:
                    self._send(c, blob)
            return got
        self._send(self.sock, payload)
        if not broadcast:
            return None
        blob, out, p = self._recv(self.sock), [], 0
        while p < len(blob):
            k = struct.unpack_from("<Q", blob, p)[0]
            out.append(blob[p + 8:p + 8 + k])
            p += 8 + k
        return out

    def barrier(self):
        self.gather(b"")

    def max(self, x):
        return max(struct.unpack("<d", g)[0] for g in self.gather(struct.pack("<d", x)))

    def close(self):
        for c in self.peers + ([self.sock] if self.sock else []):
            try:
                c.close()
            except OSError:
                pass


def launch_ranks(n):
    """Start N ranks of this script (RANK / LOCAL_RANK / WORLD_SIZE set, device
    = LOCAL_RANK) before anything here touches a GPU; relay their exit status.
    If one rank fails, the others are stopped (by their PIDs) instead of
    waiting at the next barrier."""
    token = "l%d_%d" % (os.getpid(), time.time_ns())
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   EDV_BENCH_TOKEN=token)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0 and rc == 0:
                rc = code
                for q in live:
                    q.kill()
        time.sleep(0.05)
    return rc if rc >= 0 else 1


def rank_env():
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    token = os.environ.get("EDV_BENCH_TOKEN") or "t%d_%s" % (os.getppid(), os.environ.get("MASTER_PORT", "0"))
    return world, rank, local, token


def narrow_to_own_gpu(local, world):
    """Before anything loads the HIP runtime: make this rank's GPU the only one
    it sees (HIP_VISIBLE_DEVICES = the LOCAL_RANK-th visible device), so each
    rank initialises one GPU, not all of them.  Returns the device index the
    rank then drives (0), or `local` unchanged when the ranks share logical
    devices of one GPU (EDV_VIRTUAL_DEVICES rehearsal) or there is one rank."""
    if world == 1 or os.environ.get("EDV_VIRTUAL_DEVICES"):
        return local, None
    vis = os.environ.get("HIP_VISIBLE_DEVICES")
    ids = [x.strip() for x in vis.split(",") if x.strip()] if vis is not None else None
    if ids == []:
        return local, None   # nothing visible: the device check below says so
    if ids is not None and local >= len(ids):
        sys.exit("bench.py: rank %d needs visible device %d, but HIP_VISIBLE_DEVICES=%s" % (local, local, vis))
    own = ids[local] if ids is not None else str(local)
    os.environ["HIP_VISIBLE_DEVICES"] = own
    return 0, own


# --------------------------------------------------------------- CPU baseline
CPU_SAMPLE = 65536   # requests of the CPU baseline's sample (the whole C2 batch; a prefix of a C3 shard)


def cpu_baseline(arrays, budget_s, what, chain=True):
    """libsodium 1.0.18 verify_detached over the same requests the GPU verified
    (`arrays` = (sigs, pks, msgs, off, expected), `what` says which) on the host
    cores this process can actually use: effective_cpus = its CPU affinity
    capped by the cgroup CPU quota (more threads than that only time-slice the
    same CPU share).  Also the one-thread rate, and from it a labelled
    projection to every core of the socket, which cannot be measured under the
    quota; plus (chain) the reference's single-threaded Python chain on C1."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib as orc  # the baseline leg is the only oracle/ user here
    sb = orc.sodium_batch()
    if sb is None:
        return None
    sigs, pks, msgs, off, expected = arrays
    info = cpu_info()
    eff = info["effective_cpus"]
    n = len(off) - 1
    acc = orc.sodium_verify_batch(sigs, pks, msgs, off, eff)  # warm + sanity
    assert np.array_equal(acc, expected), "libsodium and the construction disagree on the CPU sample"

    def rate(threads, seconds, k=n):
        done, t0 = 0, time.perf_counter()
        while True:
            orc.sodium_verify_batch(sigs[:64 * k], pks[:32 * k], msgs, off[:k + 1], threads)
            done += k
            dt = time.perf_counter() - t0
            if dt >= seconds:
                return done / dt, done // k, dt

    v_eff, p_eff, t_eff = rate(eff, budget_s)
    k1 = min(n, 8192)
    v_one, p_one, t_one = rate(1, max(2.0, budget_s / 4), k1)
    nproc = info["nproc"] or eff
    out = {"value": v_eff, "unit": "verifies/s", "cores": eff, "kind": "reference",
           "sample": "%d passes over %d requests (%s, %d B msgs): libsodium %s crypto_sign_ed25519_verify_detached "
                     "(oracle/sodium_batch.c) on %d threads = the CPUs this process can use (affinity %s, cgroup "
                     "quota %s CPUs), %.1f s; verdicts equal the GPU's construction"
                     % (p_eff, n, what, int(off[1] - off[0]), sb.sb_version().decode(), eff, info["affinity_cpus"],
                        info["cgroup_cpu_quota"], t_eff),
           "per_core_verifies_per_s": v_one,
           "per_core_sample": "1 thread, %d passes over the first %d requests, %.1f s" % (p_one, k1, t_one),
           "full_socket_projection_verifies_per_s": v_one * nproc,
           "full_socket_projection_note": "projection, not measurable under the quota: per-core rate x nproc (%d)"
                                          % nproc,
           "host": info}
    if chain:
        try:
            out["c1_python_chain"] = c1_chain()
        except Exception as ex:  # the chain needs libsodium via ctypes; report why it is missing
            out["c1_python_chain"] = {"error": repr(ex)}
    return out


def c1_requests(n, seed=0xC1):
    """C1: NYM-style requests, distinct signers, identifier = b58(pk[:16]) and
    verkey '~' + b58(pk[16:]), signed (GPU batch signer) over their
    SigningSerializer bytes (~150 B).  -> (verkeys {idr: '~...'}, reqs)."""
    from indy_plenum_amd import base58, edv
    from indy_plenum_amd.signing_serializer import serialize_msg_for_signing
    rng = np.random.default_rng(seed)
    seeds = rng.integers(0, 256, size=(n, 32), dtype=np.uint8)
    pks, _ = edv.sign_arrays(seeds.tobytes(), b"\0" * 64, np.zeros(n + 1, dtype=np.uint64))
    pks = np.frombuffer(pks, np.uint8).reshape(n, 32)
    verkeys, reqs = {}, []
    for i in range(n):
        pk = pks[i].tobytes()
        idr = base58.b58encode(pk[:16]).decode()
        verkeys[idr] = "~" + base58.b58encode(pk[16:]).decode()
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
    return verkeys, reqs


def c1_chain(n=10000):
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
    verkeys, reqs = c1_requests(n)
    cpu = CoreAuthNr()
    for idr, vk in verkeys.items():
        cpu.addIdr(idr, vk)
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


# ------------------------------------------------------------- other legs
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
    median of `reps` calls each; and back to back through edv_verify_batch_async."""
    from indy_plenum_amd import edv
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
    pa2 = np.zeros(n, np.uint8)
    k_async = 32   # a stream long enough that its first copy and last wait are ~3 % of it

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


def single_call_leg(calls=200):
    """Batch-of-one through the GPU (INTEGRATION.md ways 1 and 2): one request per
    call through nacl_wrappers.Verifier.verify (nacl_wrappers.py:232-242) and
    through ReqAuthenticator.authenticate (req_authenticator.py:22-44), median of
    `calls` calls each, next to the reference's per-call path on libsodium in the
    same run (crypto_sign_open via ctypes, as libnacl; DidVerifier key derivation)."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import sodium_ref
    from indy_plenum_amd import base58
    from indy_plenum_amd.client_authn import CoreAuthNr
    from indy_plenum_amd.nacl_wrappers import Verifier
    from indy_plenum_amd.req_authenticator import ReqAuthenticator
    from indy_plenum_amd.signing_serializer import serialize_msg_for_signing
    from indy_plenum_amd.verifier import DidVerifier
    verkeys, reqs = c1_requests(1, seed=0x51)
    req = reqs[0]
    idr, vk = req["identifier"], verkeys[req["identifier"]]
    sig = base58.b58decode(req["signature"])
    msg = serialize_msg_for_signing({k: v for k, v in req.items() if k != "signature"})
    pk = DidVerifier(vk, idr).batch_key()
    v = Verifier(pk)
    assert v.verify(sig, msg) and not v.verify(sig, msg + b"x")
    auth = CoreAuthNr()
    auth.addIdr(idr, vk)
    ra = ReqAuthenticator()
    ra.register_authenticator(auth)
    assert ra.authenticate(req) == {idr}

    def med_us(f):
        for _ in range(5):
            f()
        return 1e6 * median_time(f, calls)
    out = {"what": "one request per call, median of %d calls (after 5 warm calls); the GPU does every verify" % calls,
           "verifier_verify_gpu_us": med_us(lambda: v.verify(sig, msg)),
           "req_authenticator_gpu_us": med_us(lambda: ra.authenticate(req))}
    if sodium_ref.sodium() is not None:
        sv = sodium_ref.SodiumVerifier(vk, idr)
        assert sv.verify(sig, msg)
        out["verifier_verify_libsodium_us"] = med_us(lambda: sv.verify(sig, msg))
        cpu = sodium_ref.SodiumCoreAuthNr()
        cpu.addIdr(idr, vk)
        rc = ReqAuthenticator()
        rc.register_authenticator(cpu)
        out["req_authenticator_libsodium_us"] = med_us(lambda: rc.authenticate(req))
        out["verifier_gpu_over_libsodium_time"] = out["verifier_verify_gpu_us"] / out["verifier_verify_libsodium_us"]
        out["note"] = ("a batch of one takes the latency path (csrc/edv_quad.hip edv_rtl_kernel: one launch, "
                       "sixteen lanes per signature, ~0.18 ms of kernel bound by its serial chains at one wave per "
                       "SIMD, profiles/r06/rtl_kernel.txt); callers verify per prod (INTEGRATION.md way 3), where "
                       "one call carries hundreds of requests in the same time")
    return out


NODE_PROD = 400   # requests in a Node-sized batch (a prod at C5's load)


def footprint_child(path):
    """Child process of footprint_leg: a fresh process (no HIP runtime loaded
    yet) verifies the Node-sized batch in `path` through edv_verify_batch and
    reports the first call's latency (runtime init + context creation + table
    build + the verify), the warm latency and the library's device memory."""
    d = np.load(path)
    t0 = time.perf_counter()
    from indy_plenum_amd import edv
    edv.lib()
    t1 = time.perf_counter()
    acc = edv.verify_arrays(d["sigs"], d["pks"], d["msgs"], d["off"])
    t2 = time.perf_counter()
    assert np.array_equal(acc, d["expected"]), "cold-start call verdicts differ"
    mem = edv.context_memory(0)
    warm = median_time(lambda: edv.verify_arrays(d["sigs"], d["pks"], d["msgs"], d["off"]), 20)
    print(json.dumps({"load_library_ms": 1e3 * (t1 - t0), "first_call_ms": 1e3 * (t2 - t1),
                      "warm_call_ms": 1e3 * warm, "context_memory": mem}), flush=True)


def footprint_leg(batch, dev):
    """what a Node process costs a GPU.  A fresh process
    verifies one Node-sized batch (NODE_PROD requests, host buffers, the
    synchronous C-ABI): first-call latency with the HIP runtime and device
    context created inside it, warm latency, and the library's device memory
    afterwards (edv_context_memory, by kind); beside it, this bench process's
    own footprint after the C2 legs (large [S]B tables, 2^16-request scratch)."""
    arrays = batch.host_prefix(NODE_PROD)
    with tempfile.TemporaryDirectory() as td:
        path = os.path.join(td, "prod.npz")
        np.savez(path, sigs=arrays[0], pks=arrays[1], msgs=arrays[2], off=arrays[3], expected=arrays[4])
        env = dict(os.environ)
        if "HIP_VISIBLE_DEVICES" not in env and dev:
            env["HIP_VISIBLE_DEVICES"] = str(dev)
        r = subprocess.run([sys.executable, os.path.abspath(__file__), "--footprint-child", path], env=env,
                           capture_output=True, text=True, timeout=300)
    if r.returncode != 0:
        return {"error": "child rc %d: %s" % (r.returncode, r.stderr[-400:])}
    child = json.loads(r.stdout.strip().splitlines()[-1])
    from indy_plenum_amd import edv
    return {"what": "a fresh process verifying one %d-request batch (256 B msgs) through edv_verify_batch: "
                    "first call = HIP runtime + device context + [S]B table build + the verify" % NODE_PROD,
            "node_process": child,
            "node_process_total_mib": child["context_memory"]["total"] / 2**20,
            "this_process_after_c2_legs": edv.context_memory(dev),
            "table_policy": os.environ.get("EDV_SB_TABLES", "auto")}


class DictState:
    """A state with the reference's get(key, isCommitted) contract
    (PruningState.get, state/pruning_state.py), held in a dict: the NYM values
    of the state-backed node_path population.  A dict read is cheaper than the
    reference's trie + KV read, so this times everything but the storage."""

    def __init__(self):
        self.kv = {}

    def get(self, key, isCommitted=True):
        return self.kv.get(key)


def node_path_leg(n=65536, reps=3):
    """f-1: CoreAuthNr.authenticate_batch over n C1-shaped requests on this GPU
    (native host prep, one verify call, replay), with the verkeys (a) in the
    in-memory clients map and (b) only in the uncommitted state
    (client_authn.py:148-160, the NYMs not yet committed)."""
    from indy_plenum_amd import _edvhost, edv
    from indy_plenum_amd.client_authn import CoreAuthNr, nym_to_state_key
    from indy_plenum_amd.req_authenticator import ReqAuthenticator
    verkeys, reqs = c1_requests(n, seed=0xF1)
    auth = CoreAuthNr()
    for idr, vk in verkeys.items():
        auth.addIdr(idr, vk)
    res = auth.authenticate_batch(reqs)
    assert all(x == [r["identifier"]] for x, r in zip(res, reqs))
    t = median_time(lambda: auth.authenticate_batch(reqs), reps)
    phases = _edvhost.last_phases()
    ra = ReqAuthenticator()
    ra.register_authenticator(auth)
    assert all(x == {r["identifier"]} for x, r in zip(ra.authenticate_batch(reqs), reqs))
    t_ra = median_time(lambda: ra.authenticate_batch(reqs), reps)
    st = DictState()
    for idr, vk in verkeys.items():
        st.kv[nym_to_state_key(idr)] = json.dumps({"verkey": vk, "role": None}).encode()
    sauth = CoreAuthNr(state=st)
    calls = []
    real = edv.open_batch

    def counting(items, device_mask=0):   # requests the native path handed back to the Python plan
        items = list(items)
        calls.append(len(items))
        return real(items, device_mask)
    edv.open_batch = edv._OPEN_BATCH = counting   # both: the native path stays enabled
    try:
        res = sauth.authenticate_batch(reqs)
    finally:
        edv.open_batch = edv._OPEN_BATCH = real
    assert all(x == [r["identifier"]] for x, r in zip(res, reqs))
    t_st = median_time(lambda: sauth.authenticate_batch(reqs), reps)
    return {"what": "CoreAuthNr.authenticate_batch, %d NYM requests (~150 B signing bytes), 1 GPU, median of %d; "
                    "native host prep on %d threads" % (n, reps, edv.PREP_THREADS),
            "requests_per_s": n / t, "ms": 1e3 * t, "phases_last_call_s": phases,
            "req_authenticator_requests_per_s": n / t_ra,
            "state_backed": {"requests_per_s": n / t_st, "ms": 1e3 * t_st,
                             "native_path_hit_rate": 1.0 - sum(calls) / n,
                             "what": "the same requests with no clients entries: every verkey read from the "
                                     "uncommitted state (dict-backed get(key, isCommitted=False)); state keys by "
                                     "one GPU SHA-256 batch"}}


class StreamEvents:
    """HIP events on a HIP stream, through the runtime libedv.so itself links
    (libamdhip64.so.7: one runtime in the process): bracket the timed steps on
    the stream the kernels are launched on, so the kernels' own GPU time of the
    timed region is measured live, not re-measured in a separate profile."""

    def __init__(self):
        import ctypes
        self.ct = ctypes
        self.hip = ctypes.CDLL("libamdhip64.so.7")
        self.hip.hipEventRecord.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        self.hip.hipEventSynchronize.argtypes = [ctypes.c_void_p]
        self.hip.hipEventElapsedTime.argtypes = [ctypes.POINTER(ctypes.c_float), ctypes.c_void_p, ctypes.c_void_p]
        self.hip.hipEventDestroy.argtypes = [ctypes.c_void_p]
        self.ev = []
        for _ in range(2):
            e = ctypes.c_void_p()
            assert self.hip.hipEventCreate(ctypes.byref(e)) == 0
            self.ev.append(e)

    def start(self, stream):
        assert self.hip.hipEventRecord(self.ev[0], self.ct.c_void_p(stream)) == 0

    def stop(self, stream):
        assert self.hip.hipEventRecord(self.ev[1], self.ct.c_void_p(stream)) == 0

    def elapsed_ms(self):
        assert self.hip.hipEventSynchronize(self.ev[1]) == 0
        ms = self.ct.c_float(0)
        assert self.hip.hipEventElapsedTime(self.ct.byref(ms), self.ev[0], self.ev[1]) == 0
        return float(ms.value)


def timed_steps(step, drain, steps, reps, rdv, only_rank=None, own=None, events=None):
    """R repetitions of `steps` steps, each between barrier + sync; max over
    ranks per repetition -> list of seconds.  only_rank: that rank alone runs
    the steps (the others wait at the barriers).  own: gets this rank's time of
    each repetition.  events: (StreamEvents, stream, list) -- the GPU time of
    each repetition's steps on that stream is appended to the list (ms)."""
    out = []
    for _ in range(max(1, reps)):
        drain()
        rdv.barrier()
        t0 = time.perf_counter()
        if only_rank is None or rdv.rank == only_rank:
            if events:
                events[0].start(events[1])
            for _ in range(steps):
                step()
            if events:
                events[0].stop(events[1])
            drain()
            if events:
                events[2].append(events[0].elapsed_ms())
        t1 = time.perf_counter()
        rdv.barrier()
        if own is not None:
            own.append(t1 - t0)
        out.append(rdv.max(t1 - t0))
    return out


def c4_leg(dev, steps, reps, n=65536):
    """C4 (BASELINE configs[3]): n requests of 200..4,096 B (length-bucketed
    SHA-512), 5 % invalid over seven kinds (R bit, S + L, message byte, key bit,
    small-order R, non-canonical A, small-order A), device resident; verdicts
    checked against the construction."""
    from indy_plenum_amd import edv, workload
    b = workload.DeviceBatch(n, device=dev, seed=0xC4C4, var_range=(200, 4096), damage_every=20, damage_kinds=7,
                             keep_host=False)
    b.verify()
    got = b.accept()
    exp = b.expected()
    ok = bool(np.array_equal(got, exp))
    for _ in range(3):
        b.verify(stream=edv.stream(dev))
    edv.sync(dev)
    rdv = Rendezvous(0, 1, "")
    s = edv.stream(dev)
    ts = timed_steps(lambda: b.verify(stream=s), lambda: edv.sync(dev), steps, reps, rdv)
    el = statistics.median(ts)
    lens = np.diff(b.host_off).astype(np.int64)
    ops = float(np.sum(217600 + 5500 * ((lens + 81 + 127) // 128)))
    prep_ms, main_ms = edv.profile_device(b.d_sigs.ptr, b.d_pks.ptr, b.d_msgs.ptr, b.d_off.ptr, n, b.d_accept.ptr,
                                          dev, max(3, min(steps, 10)))
    # the same batches through the two-stream pipeline (prep of step k+1 beside main of step k): at C4
    # the prep kernel's SHA-512 tail runs one latency-bound wave per SIMD, so the overlap may pay here
    for _ in range(3):
        b.submit()
    edv.pipeline_sync(dev)
    tp = timed_steps(b.submit, lambda: edv.pipeline_sync(dev), steps, reps, rdv)
    okp = bool(np.array_equal(b.accept(), exp))
    # the split pipeline: only the hash side (one latency-bound SHA-512 chain per lane, ~17 blocks here)
    # of step k+1 beside main of step k, the issue-bound point sides in front of step k+1's main
    for _ in range(3):
        b.submit(edv.FLAG_SPLIT_PREP)
    edv.pipeline_sync(dev)
    b.d_accept.upload(np.full(n, 7, np.uint8))
    ts_split = timed_steps(lambda: b.submit(edv.FLAG_SPLIT_PREP), lambda: edv.pipeline_sync(dev), steps, reps, rdv)
    oks = bool(np.array_equal(b.accept(), exp))
    return {"workload": "C4: %d Ed25519 verifies per step, messages uniform in 200..4,096 B (mean %.0f B), "
                        "length-bucketed SHA-512, 5 %% invalid over %s" % (n, lens.mean(), ", ".join(workload.DAMAGE_KINDS)),
            "verifies_per_s": n * steps / el, "ms_per_step": 1e3 * el / steps, "reps_s": ts,
            "verdicts_as_expected": ok, "invalid": int(n - exp.sum()),
            "prep_kernel_ms": prep_ms, "main_kernel_ms": main_ms,
            "roofline_frac": ops / ((prep_ms + main_ms) * 1e-3) / PEAK_INT32,
            "w_ops_per_verify_mean": ops / n,
            "pipelined": {"verifies_per_s": n * steps / statistics.median(tp), "reps_s": tp,
                          "verdicts_as_expected": okp,
                          "what": "edv_verify_batch_dev_pipelined back to back (prep of step k+1 on a second stream "
                                  "beside main of step k)"},
            "pipelined_split": {"verifies_per_s": n * steps / statistics.median(ts_split), "reps_s": ts_split,
                                "verdicts_as_expected": oks,
                                "what": "edv_verify_batch_dev_pipelined with EDV_FLAG_SPLIT_PREP: the hash side of "
                                        "step k+1 beside main of step k, the point sides in front of step k+1's "
                                        "main"}}


def c3_shard_leg(dev, steps, reps, world_max=8):
    """The same-workload one-GPU reference for the driver's 1 -> 8 GPU curve: one
    rank's C3 shard at N = 8 (16,777,216 / 8 = 2,097,152 requests of 256 B, 5 %
    damaged, walked in 2^18-request launches), timed on this one GPU.  The N = 1
    line is C2 (65,536 per step), so value(N) / (N x this) is the curve's
    same-workload efficiency."""
    from indy_plenum_amd import edv, shard, workload
    lo, hi = shard.shard_range(C3_TOTAL, world_max, 0)
    b = workload.DeviceBatch(hi - lo, device=dev, start=lo, damage_every=C3_DAMAGE_EVERY, keep_host=False)
    b.verify()
    ok = bool(np.array_equal(b.accept(), b.expected()))
    s = edv.stream(dev)
    ts = timed_steps(lambda: b.verify(stream=s), lambda: edv.sync(dev), max(1, steps // 4), reps, Rendezvous(0, 1, ""))
    el = statistics.median(ts)
    return {"workload": "C3's shard at N = %d: %d requests of 256 B per step on one GPU, 5 %% damaged"
                        % (world_max, b.n),
            "verifies_per_s": b.n * max(1, steps // 4) / el, "reps_s": ts, "verdicts_as_expected": ok,
            "use": "same-workload reference for value(N) / (N x verifies_per_s) over --gpus 1, 2, 4, 8"}


def c5_leg(n=20000, n_cpu=2000):
    """C5 (BASELINE configs[4]): the 4-node pool (Alpha..Delta) under a client
    flood with the GPU verify_batch behind ReqAuthenticator, against the
    reference's one-message-at-a-time flow on libsodium (tools/bench_pool.py)."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import bench_pool
    out = bench_pool.c5(n, n_cpu)
    g = out["gpu_batched_overlap"]
    out["summary"] = {"gpu_ordered_req_per_s": g["ordered_req_per_s_one_process"],
                      "gpu_auth_share_of_node_time": g["auth_share_of_node_time"],
                      "gpu_auth_share_excluding_gc": g.get("auth_share_excluding_gc"),
                      "gpu_gc_share_of_node_time": g.get("gc_share_of_node_time"),
                      "gpu_vs_no_verify_ceiling": out["overlap_vs_ceiling"],
                      "gpu_vs_same_path_verify_skipped": out.get("overlap_vs_verify_skipped"),
                      "verify_skipped_ordered_req_per_s": out.get("gpu_overlap_verify_skipped", {}).get(
                          "ordered_req_per_s_one_process"),
                      "gpu_mode": ("overlap: authenticate_batch_submit per prod, handed over at the end of the same prod when "
                                   "the GPU is done by then (PendingProd.ready), else at the next prod"),
                      "early_handovers": out.get("gpu_batched_overlap", {}).get("early_handovers"),
                      "cpu_ordered_req_per_s": out.get("cpu_reference", {}).get("ordered_req_per_s_one_process"),
                      "cpu_auth_share_of_node_time": out.get("cpu_reference", {}).get("auth_share_of_node_time")}
    return out


# --------------------------------------------------------------------- main
def parse_args():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5, help="untimed steps first (at least --warmup-seconds of them)")
    ap.add_argument("--warmup-seconds", type=float, default=1.0)
    ap.add_argument("--reps", type=int, default=5, help="timed repetitions of --steps steps; the median is reported")
    ap.add_argument("--batch", type=int, default=65536, help="C2: requests per GPU per step")
    ap.add_argument("--total", type=int, default=0,
                    help="C3: total requests per step split by request index over the GPUs "
                         "(default %d when --gpus > 1)" % C3_TOTAL)
    ap.add_argument("--weak", action="store_true", help="with --gpus > 1: C2's --batch per GPU instead of C3")
    ap.add_argument("--msg-len", type=int, default=256)
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-e2e", action="store_true", help="skip the host-buffer boundary and node-path legs")
    ap.add_argument("--no-extra", action="store_true", help="skip the C4 and C5 legs")
    ap.add_argument("--spawn", action="store_true", help="launch the ranks from this process even for one GPU")
    ap.add_argument("--pipeline", action="store_true",
                    help="time the two-stream pipelined submission (prep of step k+1 beside main of step k)")
    ap.add_argument("--footprint-child", default=None, help=argparse.SUPPRESS)
    ap.add_argument("--split-prep", action="store_true",
                    help="with --pipeline: only the hash side of step k+1 beside main of step k, the point sides "
                         "after it (EDV_FLAG_SPLIT_PREP)")
    return ap.parse_args()


def main():
    args = parse_args()
    if args.footprint_child:
        return footprint_child(args.footprint_child)
    if "WORLD_SIZE" not in os.environ and (args.gpus > 1 or args.spawn):
        sys.exit(launch_ranks(args.gpus))
    world, rank, local, token = rank_env()
    if world != args.gpus:
        sys.exit("bench.py: --gpus %d but WORLD_SIZE=%d" % (args.gpus, world))
    dev, own_gpu = narrow_to_own_gpu(local, world)

    from indy_plenum_amd import edv, shard, workload
    ndev = edv.device_count()
    if dev >= ndev:
        sys.exit("bench.py: rank %d needs device %d, but %d gfx950 device(s) are visible (--gpus %d)"
                 % (rank, dev, ndev, args.gpus))
    rdv = Rendezvous(rank, world, token)

    c3 = args.total > 0 or (world > 1 and not args.weak)
    total = (args.total or C3_TOTAL) if c3 else args.batch * world
    if c3:
        lo, hi = shard.shard_range(total, world, rank)   # one message length: equal counts
        n, start, damage = hi - lo, lo, C3_DAMAGE_EVERY
    else:
        n, start, damage = args.batch, rank * args.batch, 0
    t_gen = time.perf_counter()
    batch = workload.DeviceBatch(n, device=dev, start=start, msg_len=args.msg_len, damage_every=damage)
    t_gen = time.perf_counter() - t_gen

    s = edv.stream(dev)

    split = edv.FLAG_SPLIT_PREP if args.split_prep else 0

    def step():
        if args.pipeline:
            batch.submit(split)
        else:
            batch.verify(stream=s)

    def drain():
        if args.pipeline:
            edv.pipeline_sync(dev)
        else:
            edv.sync(dev)

    t0, done = time.perf_counter(), 0
    while done < args.warmup or time.perf_counter() - t0 < args.warmup_seconds:
        step()
        done += 1
        if done % 8 == 0:
            drain()
    drain()
    warm_steps = done
    assert np.array_equal(batch.accept(), batch.expected()), "warm-up verdicts differ from the expected ones"

    alone = None
    if world > 1:
        # the same workload on one GPU: rank 0 times its own shard while the other
        # ranks wait at the barrier (one repetition of K steps), before the joint reps
        alone = timed_steps(step, drain, args.steps, 1, rdv, only_rank=0)[0]
    mine_s, gpu_ms = [], []
    # the kernels' GPU time inside the timed region: HIP events on the library
    # stream bracketing each repetition's steps (sequential mode: every kernel
    # of a step is on that stream)
    evs = None if args.pipeline else (StreamEvents(), s, gpu_ms)
    reps = timed_steps(step, drain, args.steps, args.reps, rdv, own=mine_s, events=evs)
    elapsed = statistics.median(reps)
    ms_step = 1e3 * elapsed / args.steps
    value = total * args.steps / elapsed
    per_rank_s = [struct.unpack("<d", g)[0] for g in rdv.gather(struct.pack("<d", statistics.median(mine_s)))]

    # the prep / main split of a launch pair (libedv_measure.so: each kernel
    # between HIP events, on the first chunk-sized slice of this rank's batch)
    pn = min(n, 1 << 18)
    iters = max(3, min(args.steps, 10))
    prep_ms, main_ms = edv.profile_device(batch.d_sigs.ptr, batch.d_pks.ptr, batch.d_msgs.ptr, batch.d_off.ptr, pn,
                                          batch.d_accept.ptr, dev, iters)
    # untimed: every rank verifies once more, packs its verdicts into a bitmask
    # on the device (N/8 bytes), copies it D2H and sends it to rank 0, which
    # places each shard's bits in its slice of one host array
    batch.verify()
    mine = batch.accept_bits()
    parts = rdv.gather(mine.tobytes(), broadcast=False)
    verdicts_ok = None
    if rank == 0:
        full = np.empty(total, np.uint8)
        bounds = ([shard.shard_range(total, world, r)[0] for r in range(world)] + [total] if c3
                  else [r * args.batch for r in range(world + 1)])
        for r, p in enumerate(parts):
            k = bounds[r + 1] - bounds[r]
            full[bounds[r]:bounds[r + 1]] = np.unpackbits(np.frombuffer(p, np.uint8), bitorder="little")[:k]
        gathered_bytes = sum(len(p) for p in parts)
        exp = np.ones(total, np.uint8)
        exp[workload.damage_positions(0, total, damage)] = 0
        verdicts_ok = bool(np.array_equal(full, exp))
    rdv.barrier()
    if rank != 0:
        rdv.close()
        return

    # per launch pair (pn requests): the timed region's own GPU time when the
    # events bracketed it, else the profile's sum
    pairs_per_step = n / pn
    pair_ms_timed = statistics.median(gpu_ms) / (args.steps * pairs_per_step) if gpu_ms else None
    path_ms = pair_ms_timed if pair_ms_timed is not None else prep_ms + main_ms
    ops = w_total(args.msg_len) * pn
    achieved = ops / (path_ms * 1e-3)
    # SURVEY 8d's whole-job fraction: the job's verifies/s x W(m) over N GPUs' peak
    # (includes step gaps, rank imbalance; the kernel fraction above does not)
    job_frac = value * w_total(args.msg_len) / (world * PEAK_INT32)
    pmc, why = pmc_figures(["edv_prep_kernel", "edv_main_kernel"], n, args.msg_len, path_ms)
    roofline = {"bound": "valu_int32", "kernel": "edv_prep_kernel + edv_main_kernel (the verify path, one launch each)",
                "achieved": achieved / 1e12, "peak": PEAK_INT32 / 1e12, "unit": "TOP/s",
                "frac": achieved / PEAK_INT32, "rank0_kernel_frac": achieved / PEAK_INT32,
                "job_frac": job_frac,
                "job_frac_what": "value x W(m) / (n_gpus x peak): the whole job's verifies/s, step gaps and the slowest "
                                 "rank included (SURVEY.md 8d)",
                "traffic": None, "traffic_unit": "bytes/launch pair",
                "traffic_source": why, "algorithmic_bytes": (64 + 32 + args.msg_len + 8 + 1) * pn,
                "ops_per_launch": ops, "kernel_ms": path_ms, "prep_kernel_ms": prep_ms, "main_kernel_ms": main_ms,
                "kernel_ms_source": ("HIP events on the library stream around each timed repetition's %d steps "
                                     "(median repetition), per prep + main launch pair" % args.steps
                                     if pair_ms_timed is not None else "prep + main profile (libedv_measure.so)"),
                "profile_pair_ms": prep_ms + main_ms,
                "profile_what": "prep_kernel_ms / main_kernel_ms: each kernel alone between HIP events "
                                "(libedv_measure.so, %d launch pairs, a sync after each)" % iters,
                "vop2_issue_peak": PEAK_VOP2 / 1e12,
                "convention": "achieved = SURVEY 8d W(m) INT32 ops per verify x verifies per launch pair / the pair's "
                              "GPU time; peak = 256 CU x 64 lanes x 2.4 GHz (4-cycle VOP3 issue)"}
    if pmc:
        roofline.update(pmc)
        if "dram_bytes_per_verify_upper_bound" in pmc:
            roofline["dram_frac_of_hbm_peak_upper_bound"] = pmc["dram_bytes_per_verify_upper_bound"] * value / PEAK_HBM
    if world > 1:
        one_gpu = n * args.steps / alone   # rank 0's shard, timed alone
        out_multi = {"per_gpu_verifies_per_s": value / world,
                     "per_rank_s": per_rank_s, "slowest_rank": int(np.argmax(per_rank_s)),
                     "slowest_rank_s": max(per_rank_s), "per_rank_what": "each rank's median repetition "
                     "(%d steps), its own clock between the barriers" % args.steps,
                     "one_gpu_same_workload_verifies_per_s": one_gpu,
                     "one_gpu_same_workload_what": "rank 0's shard (%d requests per step) timed alone, %d steps, the "
                                                   "other ranks idle at a barrier, before the joint repetitions"
                                                   % (n, args.steps),
                     "gathered_bytes": gathered_bytes,
                     "gathered": "accept bitmask, %d bytes from %d ranks (packed on each GPU, D2H, loopback TCP to "
                                 "rank 0, after the timed region)" % (gathered_bytes, world),
                     "gpu_isolation": ("HIP_VISIBLE_DEVICES=<the LOCAL_RANK-th device> per rank" if own_gpu is not None
                                       else "EDV_VIRTUAL_DEVICES=%s: logical devices sharing the visible GPU(s) "
                                            "(rehearsal)" % os.environ.get("EDV_VIRTUAL_DEVICES"))}
    if c3:
        config = {"workload": "C3: %d Ed25519 verifies per step split by request index over %d GPU(s) (%d per GPU), "
                              "fixed %d-byte serialized requests, 5 %% invalid, accept bitmask gathered to host and "
                              "checked" % (total, world, n, args.msg_len),
                  "total_per_step": total, "per_gpu": n, "msg_len": args.msg_len,
                  "parallelism": "shard-by-request-index x%d (one process per GPU)" % world}
    else:
        config = {"workload": "C2: %d Ed25519 verifies per GPU per step, fixed %d-byte serialized requests, distinct "
                              "signers%s" % (n, args.msg_len, "" if world == 1 else "; shard by request index"),
                  "batch_per_gpu": n, "msg_len": args.msg_len,
                  "parallelism": "shard-by-request-index x%d (one process per GPU)" % world}
    out = {
        "metric": METRIC,
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
                + ("; 5% damaged at known positions (R bit, S + L, message byte, key bit)" if c3 else ""),
        "config": config,
        "roofline": roofline,
        "verdicts_as_expected": verdicts_ok,
        "inputs": "device-resident: the batch is in HBM before the timed region (the host-buffer boundary "
                  "edv_verify_batch is timed in the e2e leg)",
        **({"multi_gpu": out_multi} if world > 1 else {}),
        "timing": {"mode": ("pipelined, split prep (hash side of step k+1 beside main of step k, point sides after "
                            "it)" if args.split_prep else "pipelined (prep of step k+1 beside main of step k)")
                           if args.pipeline else "sequential",
                   "reps_s": reps, "median_of": len(reps), "warmup_steps_run": warm_steps,
                   "kernel_sum_ms": path_ms, "gap_ms_per_step": ms_step - path_ms * n / pn,
                   "launch": "ranks started by bench.py" if os.environ.get("EDV_BENCH_TOKEN") else
                             ("torch.distributed.run ranks" if world > 1 else "single process"),
                   "input_generation_s": t_gen},
    }
    if world == 1 and not c3 and not args.no_e2e:
        out["e2e"] = e2e_leg(batch, value)
        out["boundary_async_pinned_vs_headline"] = out["e2e"]["async_pinned_vs_device_resident"]
        try:
            out["single_call"] = single_call_leg()
        except Exception as ex:
            out["single_call"] = {"error": repr(ex)}
        try:
            out["node_path"] = node_path_leg()
        except Exception as ex:
            out["node_path"] = {"error": repr(ex)}
    if world == 1 and not c3 and not args.no_extra:
        for name, leg in (("c3_shard", lambda: c3_shard_leg(dev, args.steps, args.reps)),
                          ("c4", lambda: c4_leg(dev, args.steps, args.reps)), ("c5", c5_leg)):
            try:
                out[name] = leg()
            except Exception as ex:
                out[name] = {"error": repr(ex)}
    if world == 1 and not c3 and not args.no_e2e:
        try:
            out["footprint"] = footprint_leg(batch, dev)
        except Exception as ex:
            out["footprint"] = {"error": repr(ex)}
    if not args.no_cpu_baseline:
        # rank 0, after the timed region and the gather (the other ranks have
        # left), on a bounded sample of the requests the GPUs verified: the
        # whole C2 batch, or the first CPU_SAMPLE requests of rank 0's C3 shard
        k = min(n, CPU_SAMPLE)
        what = ("the C2 batch" if not c3 else
                "the first %d requests of rank 0's C3 shard (5 %% damaged)" % k)
        cb = cpu_baseline(batch.host_prefix(k), args.cpu_seconds, what, chain=(world == 1 and not c3))
        out["cpu_baseline"] = cb
        if cb:
            out["gpu_over_cpu"] = value / cb["value"]
            out["gpu_over_cpu_full_socket_projection"] = value / cb["full_socket_projection_verifies_per_s"]
    print(json.dumps(out), flush=True)
    rdv.close()


if __name__ == "__main__":
    main()
