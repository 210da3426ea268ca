"""GPU tests of the host runtime around the kernels (include/edv.h):

* f-4 signer parity: edv_sign_batch_dev == libsodium, byte for byte;
* scratch ordering across caller streams (two batches in flight on two
  streams at once must each get their own verdicts);
* the host path: pinned (edv_host_alloc) and pageable inputs, sub-batches,
  chunk seams, the opt-in split-prep mode and the asynchronous slotted path;
* the multi-device path (one host thread per device, edv_shard_split) on
  EDV_VIRTUAL_DEVICES logical devices, against libsodium's committed bitmask
  (C3 split by request index) and the checker (C4 cost-balanced split);
* bench.py's C3 mode end to end on a bounded total.
Bit-exact accept/reject is the bar everywhere.
"""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

import golden_io
import oracle_lib as orc
from indy_plenum_amd import edv

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module", autouse=True)
def gpu_present():
    assert edv.device_count() >= 1, "no gfx950 device visible: the GPU suite must run on the MI355X box"


@pytest.fixture(autouse=True)
def batch_kernels_for_small_batches():
    """This module tests the batch kernels' host-path mechanics (field slices,
    sub-batches, chunk seams, slot streams) on batches that the latency path
    (edv_set_latency_path, default: up to 16,384 requests) would otherwise take:
    here it is off on device 0; test_gpu_parity.py and the fault-hook test
    below cover the latency path."""
    edv.set_latency_path(0, 0)
    yield
    edv.set_latency_path(0, edv.LATENCY_PATH_DEFAULT)


def checker(sigs, pks, msgs, off):
    if orc.sodium_batch() is not None:
        return orc.sodium_verify_batch(sigs, pks, msgs, off, 16)
    return np.frombuffer(orc.verify_batch(sigs.tobytes(), pks.tobytes(), msgs.tobytes(), off, len(off) - 1, 16),
                         dtype=np.uint8)


def test_sign_batch_dev_matches_libsodium():
    vec = golden_io.load_sign_golden()
    seeds, msgs, off = golden_io.pack_sign_batch(vec)
    pks, sigs = edv.sign_arrays(seeds, msgs, off)
    bad = [i for i, r in enumerate(vec) if pks[32 * i:32 * i + 32].tobytes() != r[2]
           or sigs[64 * i:64 * i + 64].tobytes() != r[3]]
    assert bad == []
    # and what the signer made verifies on the GPU verifier
    acc = edv.verify_arrays(sigs, pks, np.frombuffer(msgs + b"\0" * 16, np.uint8), off)
    assert acc.all()


def _upload(*arrays):
    bufs = []
    for a in arrays:
        b = edv.DeviceBuffer(a.nbytes + 64)
        b.upload(a)
        bufs.append(b)
    return bufs


class _HipStream:
    """A caller-owned HIP stream from the same HIP runtime libedv.so uses
    (torch ships its own libamdhip64, a second runtime in the process)."""
    _hip = None

    def __init__(self):
        import ctypes
        if _HipStream._hip is None:
            _HipStream._hip = ctypes.CDLL("libamdhip64.so.7")
        self._s = ctypes.c_void_p()
        assert _HipStream._hip.hipStreamCreate(ctypes.byref(self._s)) == 0
        self.cuda_stream = self._s.value

    def synchronize(self):
        assert _HipStream._hip.hipStreamSynchronize(self._s) == 0

    def __del__(self):
        if _HipStream._hip is not None and self._s:
            _HipStream._hip.hipStreamDestroy(self._s)


def test_two_caller_streams_do_not_share_scratch():
    """launches on different caller streams are ordered on the
    library's scratch (st_done event), so two batches enqueued back to back on
    two streams, without any sync between them, both come out right."""
    s1, s2 = _HipStream(), _HipStream()
    a = orc.corpus(0x5C1, 0, 20000, mode=0, invalid_permille=300)
    b = orc.corpus(0x5C2, 0, 30000, mode=1, invalid_permille=100)
    want_a, want_b = checker(*a), checker(*b)
    ba, bb = _upload(*a), _upload(*b)
    acc_a, acc_b = edv.DeviceBuffer(20000), edv.DeviceBuffer(30000)
    for _ in range(3):
        edv.verify_device(ba[0].ptr, ba[1].ptr, ba[2].ptr, ba[3].ptr, 20000, acc_a.ptr, stream=s1.cuda_stream)
        edv.verify_device(bb[0].ptr, bb[1].ptr, bb[2].ptr, bb[3].ptr, 30000, acc_b.ptr, stream=s2.cuda_stream)
        edv.verify_device(ba[0].ptr, ba[1].ptr, ba[2].ptr, ba[3].ptr, 20000, acc_a.ptr, stream=s1.cuda_stream,
                          flags=edv.FLAG_UNIFORM_LENGTH)
        s1.synchronize()
        s2.synchronize()
        assert np.array_equal(acc_a.download(20000), want_a)
        assert np.array_equal(acc_b.download(30000), want_b)


def test_device_entry_points_reject_misaligned_pointers():
    sigs, pks, msgs, off = orc.corpus(0xA1, 0, 64, mode=0, invalid_permille=0)
    bufs = _upload(sigs, pks, msgs, off)
    acc = edv.DeviceBuffer(64)
    with pytest.raises(edv.EdvError):
        edv.verify_device(bufs[0].ptr + 4, bufs[1].ptr, bufs[2].ptr, bufs[3].ptr, 64, acc.ptr)
    with pytest.raises(edv.EdvError):
        edv.verify_device(bufs[0].ptr, bufs[1].ptr + 8, bufs[2].ptr, bufs[3].ptr, 64, acc.ptr)
    # an unaligned message base is fine (messages are read as aligned words):
    # d_msgs one byte in, msg_base = 1, so message i is still at ptr + off[i]
    edv.verify_device(bufs[0].ptr, bufs[1].ptr, bufs[2].ptr + 1, bufs[3].ptr, 64, acc.ptr, msg_base=1)
    assert acc.download(64).all()


@pytest.mark.parametrize("n", [1, 255, 4097, 65536 + 77])
def test_host_path_pinned_and_pageable(n):
    sigs, pks, msgs, off = orc.corpus(0x9E + n, 0, n, mode=n % 2, invalid_permille=150)
    want = checker(sigs, pks, msgs, off)
    assert np.array_equal(edv.verify_arrays(sigs, pks, msgs, off), want)
    # the same batch from page-locked memory: direct DMA, no staging copy
    parts = [sigs, pks, off.view(np.uint8), msgs]
    pb = edv.PinnedBuffer(sum(p.nbytes for p in parts) + 4 * 64 + n)
    pos, views = 0, []
    for p in parts:
        v = pb.array[pos:pos + p.nbytes]
        v[:] = p
        views.append(v)
        pos += (p.nbytes + 63) // 64 * 64
    acc = pb.array[pos:pos + n]
    edv._check(edv.lib().edv_verify_batch(views[0].ctypes.data, views[1].ctypes.data, views[3].ctypes.data,
                                          views[2].ctypes.data, n, acc.ctypes.data, 0))
    assert np.array_equal(acc, want)
    pb.free()


@pytest.mark.parametrize("n,slices", [(8192 + 5, 2), (65536, 4), (65536, 3), (65536, 8), (100003, 2),
                                      (20000, 1), (600, 4)])
def test_host_field_slices_path(n, slices):
    """A synchronous one-chunk shard copies sigs / keys / offsets first (point
    sides start), then its messages in `slices` slices, each slice's hash side
    launched as soon as it has landed (edv_set_host_slices), one main kernel
    after all of them.  Pageable and pinned inputs, 15 % invalid spread over the
    slices, back to back (the second call reuses staging, events and scratch)."""
    sigs, pks, msgs, off = orc.corpus(0x5B17 + n, 0, n, mode=0, invalid_permille=150)
    want = checker(sigs, pks, msgs, off)
    assert 0 < want.sum() < n
    edv.set_host_slices(0, slices)
    try:
        assert np.array_equal(edv.verify_arrays(sigs, pks, msgs, off), want)
        bufs = [sigs, pks, off.view(np.uint8), msgs]
        pb = edv.PinnedBuffer(sum(p.nbytes for p in bufs) + 4 * 64 + n)
        pos, views = 0, []
        for p in bufs:
            v = pb.array[pos:pos + p.nbytes]
            v[:] = p
            views.append(v)
            pos += (p.nbytes + 63) // 64 * 64
        acc = pb.array[pos:pos + n]
        for _ in range(2):
            acc[:] = 7
            edv._check(edv.lib().edv_verify_batch(views[0].ctypes.data, views[1].ctypes.data, views[3].ctypes.data,
                                                  views[2].ctypes.data, n, acc.ctypes.data, 0))
            assert np.array_equal(acc, want)
        pb.free()
        # the same arrays pinned in reverse order (messages, offsets, keys, signatures):
        # no single sigs | keys | offsets region, so three separate copies
        pb = edv.PinnedBuffer(sum(p.nbytes for p in bufs) + 4 * 64 + n)
        pos, views = 0, [None] * 4
        for k in (3, 2, 1, 0):
            v = pb.array[pos:pos + bufs[k].nbytes]
            v[:] = bufs[k]
            views[k] = v
            pos += (bufs[k].nbytes + 63) // 64 * 64
        acc = pb.array[pos:pos + n]
        acc[:] = 7
        edv._check(edv.lib().edv_verify_batch(views[0].ctypes.data, views[1].ctypes.data, views[3].ctypes.data,
                                              views[2].ctypes.data, n, acc.ctypes.data, 0))
        assert np.array_equal(acc, want)
        pb.free()
    finally:
        edv.set_host_slices(0, 0)


@pytest.mark.parametrize("slices", [1, 2])
def test_host_field_path_empty_messages(slices):
    """A batch whose messages are all empty (Ed25519 over zero bytes: no message
    copy at all on the field path, SHA-512 of R || A alone), 10 % damaged, from
    pageable and pinned buffers; verdicts equal libsodium's."""
    n = 3000
    rng = np.random.default_rng(0xE0 + slices)
    seeds = rng.integers(0, 256, size=32 * n, dtype=np.uint8)
    off = np.zeros(n + 1, np.uint64)
    pks, sigs = edv.sign_arrays(seeds, b"", off)
    sigs = sigs.copy()
    sigs[64 * np.arange(0, n, 10) + 40] ^= 1          # every tenth S damaged
    msgs = np.zeros(16, np.uint8)
    want = checker(sigs, pks, msgs, off)
    assert want.sum() == n - len(range(0, n, 10))
    edv.set_host_slices(0, slices)
    try:
        assert np.array_equal(edv.verify_arrays(sigs, pks, msgs, off), want)
        pb = edv.PinnedBuffer(sigs.nbytes + pks.nbytes + off.nbytes + n + 4 * 64)
        pos, views = 0, []
        for a in (sigs, pks, off.view(np.uint8)):
            v = pb.array[pos:pos + a.nbytes]
            v[:] = a
            views.append(v)
            pos += (a.nbytes + 63) // 64 * 64
        acc = pb.array[pos:pos + n]
        acc[:] = 7
        edv._check(edv.lib().edv_verify_batch(views[0].ctypes.data, views[1].ctypes.data, msgs.ctypes.data,
                                              views[2].ctypes.data, n, acc.ctypes.data, 0))
        assert np.array_equal(acc, want)
        pb.free()
    finally:
        edv.set_host_slices(0, 0)


def test_host_field_path_varied_lengths_one_slice():
    """Messages of several SHA-512 block counts (C4 lengths) on the field path:
    the shard is length-bucketed, so its hash side runs in one piece after the
    whole copy whatever the slice setting; verdicts equal the checker's."""
    n = 30000
    sigs, pks, msgs, off = orc.corpus(0xC4F1, 0, n, mode=1, invalid_permille=120)
    want = checker(sigs, pks, msgs, off)
    edv.set_host_slices(0, 8)
    try:
        assert np.array_equal(edv.verify_arrays(sigs, pks, msgs, off), want)
    finally:
        edv.set_host_slices(0, 0)


def _pinned_copy(sigs, pks, msgs, off, n):
    bufs = [sigs, pks, off.view(np.uint8), msgs]
    pb = edv.PinnedBuffer(sum(p.nbytes for p in bufs) + 5 * 64 + n)
    pos, views = 0, []
    for p in bufs:
        v = pb.array[pos:pos + p.nbytes]
        v[:] = p
        views.append(v)
        pos += (p.nbytes + 63) // 64 * 64
    return pb, (views[0], views[1], views[3], views[2].view(np.uint64)), pb.array[pos:pos + n]


def test_host_async_path():
    """edv_verify_batch_async / edv_wait_async: batches of fixed and mixed
    lengths (sizes 20,000 / 4,097 / 65,536 / 1 / 30,000 / 40,000, 15 % invalid)
    queued back to back from pageable memory, twice over (twelve in flight:
    slots reused without an explicit wait, the submission completing the batch
    eight back), then pinned inputs with pinned verdict buffers in turn; every
    batch equals the checker."""
    sizes = (20000, 4097, 65536, 1, 30000, 40000)
    batches = [orc.corpus(0xA5A0 + k, 0, n, mode=k % 2, invalid_permille=150) for k, n in enumerate(sizes)]
    wants = [checker(*b) for b in batches]
    order = list(range(6)) * 2
    accs = [np.full(sizes[k], 7, np.uint8) for k in order]
    tickets = []
    for j, k in enumerate(order):
        tickets.append(edv.verify_async(*batches[k], accs[j]))
        if j == 1:
            edv.wait_async(tickets[0])
            assert np.array_equal(accs[0], wants[0])
    # tickets 1 and 2 were completed by the submissions eight after them; waiting is still fine
    for t in tickets:
        edv.wait_async(t)
    for j, k in enumerate(order):
        assert np.array_equal(accs[j], wants[k])
    with pytest.raises(edv.EdvError):
        edv.wait_async(tickets[-1] + 100)
    # pinned inputs and verdicts: DMA straight from and into the caller's memory
    pinned = [_pinned_copy(*batches[k], sizes[k]) for k in (0, 2)]
    want2 = [wants[0], wants[2]]
    for _ in range(2):
        ts = []
        for (pb, arrs, acc) in pinned:
            acc[:] = 7
            ts.append(edv.verify_async(*arrs, acc))
        for t in ts:
            edv.wait_async(t)
        for (pb, arrs, acc), w in zip(pinned, want2):
            assert np.array_equal(acc, w)
    for pb, _a, _c in pinned:
        pb.free()
    # the synchronous path in between async batches shares the scratch safely
    t = edv.verify_async(*batches[4], accs[4])
    assert np.array_equal(edv.verify_arrays(*batches[2]), wants[2])
    edv.wait_async(t)
    assert np.array_equal(accs[4], wants[4])


def test_host_async_path_from_threads():
    """Three threads on one device: two queue async batches and wait (the wait
    drops the device lock, so the other thread's submissions and the third
    thread's synchronous calls go on meanwhile), one calls edv_verify_batch.
    Every verdict array equals the checker."""
    import threading
    batches = [orc.corpus(0x7A00 + k, 0, 12000 + 977 * k, mode=k % 2, invalid_permille=120) for k in range(6)]
    wants = [checker(*b) for b in batches]
    errors = []

    def async_worker(ks):
        try:
            for _ in range(3):
                accs = {k: np.full(len(batches[k][3]) - 1, 7, np.uint8) for k in ks}
                ts = [(k, edv.verify_async(*batches[k], accs[k])) for k in ks]
                for k, t in ts:
                    edv.wait_async(t)
                    assert np.array_equal(accs[k], wants[k]), k
        except BaseException as ex:  # reported below, in the test's thread
            errors.append(ex)

    def sync_worker():
        try:
            for _ in range(3):
                assert np.array_equal(edv.verify_arrays(*batches[5]), wants[5])
        except BaseException as ex:
            errors.append(ex)

    th = [threading.Thread(target=async_worker, args=([0, 1, 2],)),
          threading.Thread(target=async_worker, args=([3, 4],)), threading.Thread(target=sync_worker)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=100)
    assert not any(t.is_alive() for t in th)
    assert errors == []


def test_host_async_small_batches_side_by_side():
    """Small asynchronous batches (at most kSmallAsync = 8,192 requests: each
    runs on its slot's own stream and scratch, side by side with the others)
    from four threads at once, fixed and mixed lengths (length buckets), sizes
    either side of the boundary (8,192 on a slot stream, 8,193 on the shared
    one), then single-threaded with chunks smaller than the batches (the slot
    path walks chunks on its own scratch).  Every verdict array equals the
    checker."""
    import threading
    sizes = [1, 97, 400, 1000, 4096, 8191, 8192, 8193]
    batches = [orc.corpus(0x5A11 + k, 0, n, mode=k % 2, invalid_permille=150) for k, n in enumerate(sizes)]
    wants = [checker(*b) for b in batches]
    errors = []

    def worker(w):
        try:
            for rnd in range(3):
                ks = [(w + rnd + j) % len(sizes) for j in range(3)]
                accs = {k: np.full(sizes[k], 7, np.uint8) for k in ks}
                ts = [(k, edv.verify_async(*batches[k], accs[k])) for k in ks]
                for k, t in ts:
                    edv.wait_async(t)
                    assert np.array_equal(accs[k], wants[k]), (w, rnd, k)
        except BaseException as ex:  # reported below, in the test's thread
            errors.append(ex)

    th = [threading.Thread(target=worker, args=(w,)) for w in range(4)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=120)
    assert not any(t.is_alive() for t in th)
    assert errors == []
    try:
        edv.set_chunk(0, 1024)
        accs = [np.full(n, 7, np.uint8) for n in sizes]
        ts = [edv.verify_async(*b, a) for b, a in zip(batches, accs)]
        for t in ts:
            edv.wait_async(t)
        for a, w in zip(accs, wants):
            assert np.array_equal(a, w)
    finally:
        edv.set_chunk(0, 0)


def test_host_path_chunk_seams_with_sub_batches():
    """Small chunks: the host path's sub-batches then span several chunk-sized
    scratch regions per stream (and one stream when the chunk is tiny)."""
    sigs, pks, msgs, off = orc.corpus(0xC5EA, 0, 9000, mode=1, invalid_permille=200)
    want = checker(sigs, pks, msgs, off)
    try:
        for chunk in (256, 1024, 4096, 8192):
            edv.set_chunk(0, chunk)
            assert np.array_equal(edv.verify_arrays(sigs, pks, msgs, off), want), chunk
    finally:
        edv.set_chunk(0, 0)


_VIRTUAL = r"""
import json, os, sys
import numpy as np
sys.path.insert(0, os.environ["ROOT"]); sys.path.insert(0, os.path.join(os.environ["ROOT"], "tests"))
import oracle_lib as orc
from indy_plenum_amd import edv, shard
out = {"devices": edv.device_count()}
meta = json.load(open(os.path.join(os.environ["ROOT"], "tests", "golden", "corpus_bitmask.json")))
cfg = meta["corpora"]["c2_256B"]
n = 262144
sigs, pks, msgs, off = orc.corpus(cfg["seed"], 0, n, cfg["mode"], cfg["invalid_permille"])
bits = np.fromfile(os.path.join(os.environ["ROOT"], "tests", "golden", "corpus_c2_256B.bits"), np.uint8)
want = np.unpackbits(bits[:n // 8], bitorder="little")
got = edv.verify_arrays(sigs, pks, msgs, off)            # all logical devices, split by index
out["c3_split_equal"] = bool(np.array_equal(got, want))
out["c3_bounds"] = edv.shard_split(off, out["devices"]).tolist()
got2 = edv.verify_arrays(sigs, pks, msgs, off, device_mask=0b0101)   # a subset of the devices
out["subset_equal"] = bool(np.array_equal(got2, want))
s4, p4, m4, o4 = orc.corpus(0xC4C4, 0, 30000, mode=1, invalid_permille=50)
w4 = np.frombuffer(orc.verify_batch(s4.tobytes(), p4.tobytes(), m4.tobytes(), o4, 30000, 16), np.uint8)
out["c4_equal"] = bool(np.array_equal(edv.verify_arrays(s4, p4, m4, o4), w4))
out["c4_bounds"] = edv.shard_split(o4, out["devices"]).tolist()
out["c4_bounds_restated"] = shard.shard_bounds(o4, out["devices"]).tolist()
try:
    edv.verify_arrays(s4, p4, m4, o4, device_mask=1 << 20)
    out["bad_mask"] = "no error"
except edv.EdvUnavailable as ex:
    out["bad_mask"] = "EdvUnavailable"
print(json.dumps(out))
"""


def test_multi_device_path_on_virtual_devices():
    """edv_verify_batch with four logical devices (EDV_VIRTUAL_DEVICES=4 on this
    one-GPU box): one host thread and context per device, shards by index (C2
    lengths: equal counts) checked against libsodium's committed verdict bitmask,
    and by estimated cost (C4 lengths) against the checker."""
    # EDV_MIN_SHARD: the 30,000-request C4 batch is split too (below the default
    # 65,536-request minimum shard it would run whole on one device)
    env = dict(os.environ, EDV_VIRTUAL_DEVICES="4", EDV_MIN_SHARD="4096", ROOT=ROOT)
    r = subprocess.run([sys.executable, "-c", _VIRTUAL], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["devices"] == 4
    assert out["c3_split_equal"] and out["subset_equal"] and out["c4_equal"]
    assert out["c3_bounds"] == [0, 65536, 131072, 196608, 262144]
    assert out["c4_bounds"] == out["c4_bounds_restated"]
    assert out["bad_mask"] == "EdvUnavailable"


_PLACEMENT = r"""
import json, os, statistics, sys, time
import numpy as np
sys.path.insert(0, os.environ["ROOT"]); sys.path.insert(0, os.path.join(os.environ["ROOT"], "tests"))
import oracle_lib as orc
from indy_plenum_amd import edv
out = {"devices": edv.device_count(), "contexts0": edv.context_count()}
sigs, pks, msgs, off = orc.corpus(0x91AC, 0, 400, mode=0, invalid_permille=100)
want = np.frombuffer(orc.verify_batch(sigs.tobytes(), pks.tobytes(), msgs.tobytes(), off, 400, 8), np.uint8)
def lat(k, reps=40):
    o = off[:k + 1]
    got = edv.verify_arrays(sigs[:64 * k], pks[:32 * k], msgs, o)
    assert np.array_equal(got, want[:k])
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        edv.verify_arrays(sigs[:64 * k], pks[:32 * k], msgs, o)
        ts.append(time.perf_counter() - t0)
    return statistics.median(ts)
out["lat1_s"] = lat(1)
out["contexts_after_1"] = edv.context_count()
out["lat400_s"] = lat(400)
out["contexts_after_400"] = edv.context_count()
# asynchronous submissions one at a time stay on one device
acc = [np.zeros(400, np.uint8) for _ in range(4)]
seq = []
for _ in range(5):
    d = edv.pick_device()
    seq.append(d)
    edv.wait_async(edv.verify_async(sigs, pks, msgs, off, acc[0], device=d), device=d)
out["async_sequential_devices"] = len(set(seq))
out["async_equal"] = bool(np.array_equal(acc[0], want))
out["contexts_after_async"] = edv.context_count()
if out["devices"] == 8:
    # C3-shaped: 8 x 65,536 requests split 8 ways, against libsodium's committed bitmask
    meta = json.load(open(os.path.join(os.environ["ROOT"], "tests", "golden", "corpus_bitmask.json")))
    cfg = meta["corpora"]["c2_256B"]
    n = 8 * 65536
    s3, p3, m3, o3 = orc.corpus(cfg["seed"], 0, n, cfg["mode"], cfg["invalid_permille"])
    bits = np.fromfile(os.path.join(os.environ["ROOT"], "tests", "golden", "corpus_c2_256B.bits"), np.uint8)
    want3 = np.unpackbits(bits[:n // 8], bitorder="little")
    out["c3_equal"] = bool(np.array_equal(edv.verify_arrays(s3, p3, m3, o3), want3))
    out["contexts_after_c3"] = edv.context_count()
    # asynchronous batches in flight together: a device with fewer than two running
    # counts as free, so four 131,072-request batches (milliseconds of GPU work each,
    # submitted from pinned memory in microseconds) land on at least two devices
    k = n // 4
    parts = []
    for j in range(4):
        ss, pp, oo = s3[64 * j * k:64 * (j + 1) * k], p3[32 * j * k:32 * (j + 1) * k], o3[j * k:(j + 1) * k + 1]
        mm = m3[int(oo[0]):int(oo[-1])]
        oo = oo - oo[0]
        bufs = [ss, pp, oo.view(np.uint8), mm]
        pb = edv.PinnedBuffer(sum(b.nbytes for b in bufs) + 5 * 64 + k)
        pos, views = 0, []
        for b in bufs:
            v = pb.array[pos:pos + b.nbytes]
            v[:] = b
            views.append(v)
            pos += (b.nbytes + 63) // 64 * 64
        parts.append((pb, views, pb.array[pos:pos + k]))
    picks, tickets = [], []
    for pb, (ss, pp, oo, mm), a in parts:
        d = edv.pick_device()
        picks.append(d)
        tickets.append((d, edv.verify_async(ss, pp, mm, oo.view(np.uint64), a, device=d)))
    for d, t in tickets:
        edv.wait_async(t, device=d)
    out["async_spread"] = len(set(picks))
    out["async_spread_equal"] = all(np.array_equal(a, want3[j * k:(j + 1) * k]) for j, (_, _, a) in enumerate(parts))
    for pb, _, _ in parts:
        pb.free()
print(json.dumps(out))
"""


def _placement(vdev):
    env = dict(os.environ, EDV_VIRTUAL_DEVICES=str(vdev), ROOT=ROOT)
    env.pop("EDV_MIN_SHARD", None)
    r = subprocess.run([sys.executable, "-c", _PLACEMENT], env=env, capture_output=True, text=True, timeout=400)
    assert r.returncode == 0, r.stderr[-3000:]
    return json.loads(r.stdout.strip().splitlines()[-1])


def test_device_placement_node_sized_batches():
    """VERDICT r3 next #3, on eight logical devices of this one GPU
    (EDV_VIRTUAL_DEVICES=8): a 1-request and a 400-request edv_verify_batch
    initialise exactly ONE device context (no thread per device, no empty
    shard), and their median latency does not grow against one logical device;
    asynchronous batches in flight together spread over devices, one at a time
    they stay on one (a device with one asynchronous batch running still counts
    as free); a C3-shaped 8 x 65,536 batch still splits 8 ways, with
    libsodium's committed verdicts."""
    one = _placement(1)
    eight = _placement(8)
    assert eight["devices"] == 8 and one["devices"] == 1
    assert eight["contexts0"] == 0
    assert eight["contexts_after_1"] == 1 and eight["contexts_after_400"] == 1
    assert eight["async_equal"] and one["async_equal"]
    assert eight["async_sequential_devices"] == 1 and one["async_sequential_devices"] == 1
    assert eight["async_spread"] >= 2 and eight["async_spread_equal"]
    assert eight["c3_equal"] and eight["contexts_after_c3"] == 8
    for k in ("lat1_s", "lat400_s"):
        assert eight[k] <= 1.25 * one[k] + 1e-4, (k, eight[k], one[k])
    print(json.dumps({"placement_1dev": one, "placement_8dev": eight}))


_CONCURRENT = r"""
import json, os, sys, threading
import numpy as np
sys.path.insert(0, os.environ["ROOT"]); sys.path.insert(0, os.path.join(os.environ["ROOT"], "tests"))
import oracle_lib as orc
from indy_plenum_amd import edv
meta = json.load(open(os.path.join(os.environ["ROOT"], "tests", "golden", "corpus_bitmask.json")))
cfg = meta["corpora"]["c2_256B"]
n = 2 * 131072
s, p, m, o = orc.corpus(cfg["seed"], 0, n, cfg["mode"], cfg["invalid_permille"])
bits = np.fromfile(os.path.join(os.environ["ROOT"], "tests", "golden", "corpus_c2_256B.bits"), np.uint8)
want = np.unpackbits(bits[:n // 8], bitorder="little")
h = n // 2
parts = [(s[:64 * h], p[:32 * h], m, o[:h + 1]), (s[64 * h:], p[32 * h:], m, o[h:])]
got = [None, None]
gate = threading.Barrier(2)
def run(k):
    gate.wait()
    got[k] = edv.verify_arrays(*parts[k])
th = [threading.Thread(target=run, args=(k,)) for k in range(2)]
for t in th: t.start()
for t in th: t.join()
out = {"devices": edv.device_count(), "contexts_concurrent": edv.context_count(),
       "equal": bool(np.array_equal(np.concatenate(got), want))}
# one at a time afterwards: a 2-shard call stays on initialised devices
for _ in range(3):
    assert np.array_equal(edv.verify_arrays(*parts[0]), want[:h])
out["contexts_after_sequential"] = edv.context_count()
print(json.dumps(out))
"""


def test_concurrent_mid_sized_batches_use_distinct_devices():
    """VERDICT r4 next #6 / ADVICE r4: two concurrent 131,072-request calls from
    two threads (each splits into two shards) on eight logical devices land on
    four distinct devices (placement reserves its choice, so concurrent callers
    see each other), not both on devices 0-1; verdicts equal libsodium's
    committed bitmask; later sequential calls reuse initialised devices."""
    env = dict(os.environ, EDV_VIRTUAL_DEVICES="8", ROOT=ROOT)
    env.pop("EDV_MIN_SHARD", None)
    r = subprocess.run([sys.executable, "-c", _CONCURRENT], env=env, capture_output=True, text=True, timeout=400)
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["devices"] == 8 and out["equal"]
    assert out["contexts_concurrent"] == 4
    assert out["contexts_after_sequential"] == 4


def _bench(args, env=None, launcher=None, timeout=420):
    cmd = (launcher or [sys.executable]) + [os.path.join(ROOT, "bench.py")] + args
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.strip().splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout[-2000:]           # exactly one JSON line on stdout
    return json.loads(lines[0])


_QUICK = ["--steps", "2", "--reps", "2", "--warmup", "1", "--warmup-seconds", "0", "--no-cpu-baseline"]


def test_bench_default_line_contract():
    """The N = 1 line the driver reads (C2, legs off): the contract's keys, the
    roofline object (bound, achieved = W ops / kernel time, peak, unit, frac =
    achieved / peak, traffic from the PMC summary while the kernel sources match
    it, else null) and the CPU baseline object with its sample and thread count."""
    import bench
    line = _bench(["--steps", "3", "--reps", "2", "--warmup", "1", "--warmup-seconds", "0", "--no-e2e",
                   "--no-extra"])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
              "scaling", "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert k in line, k
    assert line["n_gpus"] == 1 and line["steps"] == 3 and line["higher_is_better"] is True
    assert line["unit"] == "verifies/s" and line["dtype"] == "int32" and line["scaling"] == "weak"
    assert line["config"]["workload"].startswith("C2") and line["config"]["batch_per_gpu"] == 65536
    assert line["verdicts_as_expected"] is True
    rf = line["roofline"]
    assert rf["unit"] == "TOP/s" and rf["peak"] > 0 and abs(rf["frac"] - rf["achieved"] / rf["peak"]) < 1e-9
    ops = rf["ops_per_launch"] / (rf["kernel_ms"] * 1e-3) / 1e12
    assert abs(ops - rf["achieved"]) / rf["achieved"] < 1e-6
    assert abs(rf["profile_pair_ms"] - rf["prep_kernel_ms"] - rf["main_kernel_ms"]) < 1e-6
    # kernel time from HIP events around the timed steps on the library stream
    assert rf["kernel_ms_source"].startswith("HIP events")
    assert 0.8 * line["ms_per_step"] <= rf["kernel_ms"] <= line["ms_per_step"] * 1.02
    with open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles",
                           "pmc_latest.json")) as f:
        pmc_matches = json.load(f).get("device_code_sha256") == bench.device_code_hash()
    assert (rf["traffic"] is not None) == pmc_matches
    cb = line["cpu_baseline"]
    assert cb["kind"] in ("reference", "port") and cb["value"] > 0 and cb["cores"] >= 1 and cb["sample"]
    assert 0 < rf["job_frac"] <= 1 and rf["rank0_kernel_frac"] == rf["frac"]


def test_bench_c3_mode_bounded():
    """bench.py --total (C3 split by request index, 5 % damaged at known
    positions over four kinds, accept bytes checked) on a bounded total."""
    line = _bench(["--total", "524288"] + _QUICK)
    assert line["verdicts_as_expected"] is True
    assert line["config"]["workload"].startswith("C3")
    assert line["n_gpus"] == 1 and line["value"] > 1e6


def test_bench_two_gpus_launched_by_bench():
    """python bench.py --gpus 2 (no launcher around it) on two logical devices
    (EDV_VIRTUAL_DEVICES=2 on this one-GPU box): bench starts one process per
    device, C3 is the default for N > 1, every shard's accept bytes come back
    into their slice of the host array and match the construction."""
    env = dict(os.environ, EDV_VIRTUAL_DEVICES="2")
    env.pop("WORLD_SIZE", None)
    line = _bench(["--gpus", "2", "--total", "1048576"] + _QUICK, env=env)
    assert line["n_gpus"] == 2 and line["verdicts_as_expected"] is True
    assert line["config"]["workload"].startswith("C3") and line["config"]["per_gpu"] == 524288
    assert line["timing"]["launch"] == "ranks started by bench.py"
    # the fields a scaling curve needs
    mg = line["multi_gpu"]
    assert len(mg["per_rank_s"]) == 2 and mg["slowest_rank"] in (0, 1)
    assert mg["slowest_rank_s"] == max(mg["per_rank_s"])
    assert mg["one_gpu_same_workload_verifies_per_s"] > 1e6
    assert "scaling_efficiency" not in mg  # the driver computes efficiency from the per-N values
    assert mg["gpu_isolation"].startswith("EDV_VIRTUAL_DEVICES")


def test_bench_two_gpus_under_torch_distributed_run():
    """The driver's N > 1 form: python -m torch.distributed.run --nproc-per-node 2
    bench.py --gpus 2 (ranks from the environment, device = LOCAL_RANK; the
    ranks themselves import no torch)."""
    env = dict(os.environ, EDV_VIRTUAL_DEVICES="2")
    env.pop("WORLD_SIZE", None)
    launcher = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                "--master-addr", "127.0.0.1", "--master-port", str(29500 + os.getpid() % 1000)]
    line = _bench(["--gpus", "2", "--total", "1048576"] + _QUICK, env=env, launcher=launcher)
    assert line["n_gpus"] == 2 and line["verdicts_as_expected"] is True
    assert line["timing"]["launch"] == "torch.distributed.run ranks"


def test_pack_bits_matches_numpy():
    """edv_pack_bits_dev (the bitmask a multi-GPU run gathers) equals
    numpy.packbits(accept != 0, bitorder="little") for lengths around the 8-bit
    and word seams, at an unaligned start and for verdict bytes other than 0/1."""
    rng = np.random.default_rng(0xB175)
    for n in (1, 7, 8, 9, 63, 64, 65, 1000, 65536 + 3):
        for shift in (0, 1):
            a = rng.integers(0, 2, size=n, dtype=np.uint8)
            a[::13] *= 7                      # any nonzero byte is a 1
            buf = edv.DeviceBuffer(n + 8)
            host = np.zeros(n + 8, np.uint8)
            host[shift:shift + n] = a
            buf.upload(host)
            out = edv.DeviceBuffer((n + 7) // 8)
            edv.pack_bits_device(buf.ptr + shift, n, out.ptr)
            got = out.download((n + 7) // 8)
            assert np.array_equal(got, np.packbits(a != 0, bitorder="little")), (n, shift)


@pytest.mark.parametrize("ranks", [8, 4])
def test_bench_c3_full_size_virtual_ranks(ranks):
    """the line the driver's SCALE run will time, at its full
    size -- bench.py --gpus N over C3's 16,777,216 requests per step split by
    request index into N rank processes (here N logical devices sharing this
    GPU: EDV_VIRTUAL_DEVICES=N), each rank's verdicts packed into a bitmask on
    its device and gathered into its slice on rank 0, then checked against the
    construction (5 % damaged at known positions)."""
    env = dict(os.environ, EDV_VIRTUAL_DEVICES=str(ranks))
    env.pop("WORLD_SIZE", None)
    line = _bench(["--gpus", str(ranks), "--steps", "2", "--reps", "1", "--warmup", "1", "--warmup-seconds", "0",
                   "--cpu-seconds", "3"], env=env, timeout=900)
    assert line["n_gpus"] == ranks and line["verdicts_as_expected"] is True
    assert line["config"]["total_per_step"] == 16777216 and line["config"]["per_gpu"] == 16777216 // ranks
    mg = line["multi_gpu"]
    assert len(mg["per_rank_s"]) == ranks and mg["slowest_rank_s"] == max(mg["per_rank_s"])
    assert mg["gathered_bytes"] == 16777216 // 8
    assert mg["one_gpu_same_workload_verifies_per_s"] > 1e6
    assert "scaling_efficiency" not in mg
    assert line["value"] > 1e7
    # north_star's reporting clause at N > 1 -- the whole
    # job's fraction of N GPUs' INT32 peak beside rank 0's kernel
    # fraction, and libsodium on the host cores in the same run, cores stated
    rf = line["roofline"]
    assert 0 < rf["job_frac"] <= 1 and 0 < rf["rank0_kernel_frac"] <= 1
    from bench import w_total, PEAK_INT32
    assert abs(rf["job_frac"] - line["value"] * w_total(256) / (ranks * PEAK_INT32)) < 1e-9
    cb = line["cpu_baseline"]
    assert cb["kind"] == "reference" and cb["value"] > 0 and cb["cores"] >= 1
    assert "C3 shard" in cb["sample"] and line["gpu_over_cpu"] > 1


def test_async_failure_end_to_end_with_fault_hook():
    """the asynchronous path's fail-closed contract driven on the
    device, not only the ledger's arithmetic.  libedv_measure.so's fault hook
    (edv_test_fail_async) makes one submission launch nothing and fail at its
    wait, as a batch whose done event failed would.  Then: the failed ticket's
    wait returns EDV_E_HIP and its verdicts (zeroed at submission) are all
    rejections; a ticket waited for before the failure and asked again is
    reported failed (sticky); batches submitted around it, still in their
    slots, keep their own verdicts; later batches (every slot reused) are
    unaffected -- with pageable and with page-locked (zero-copy) verdicts."""
    import ctypes
    ml = edv.measure_lib()
    dev = 0
    n = 512
    sigs, pks, msgs, off = orc.corpus(0xFA17, 0, n, mode=1, invalid_permille=100)
    want = checker(sigs, pks, msgs, off)
    assert 0 < want.sum() < n
    pin = edv.PinnedBuffer(n * 16)

    def submit(acc):
        t = ctypes.c_int64(-1)
        rc = ml.edv_verify_batch_async(sigs.ctypes.data, pks.ctypes.data, msgs.ctypes.data, off.ctypes.data, n,
                                       acc.ctypes.data, dev, ctypes.byref(t))
        assert rc == 0, ml.edv_last_error()
        return t.value

    def wait(t):
        return ml.edv_wait_async(dev, t)

    for pinned in (False, True):
        accs = ([pin.array[k * n:(k + 1) * n] for k in range(16)] if pinned
                else [np.full(n, 7, np.uint8) for _ in range(16)])
        t0 = submit(accs[0])
        assert wait(t0) == 0 and np.array_equal(accs[0], want)
        t1 = submit(accs[1])
        assert ml.edv_test_fail_async(dev, t1 + 1) == 0
        t2 = submit(accs[2])
        t3 = submit(accs[3])
        assert (t1, t2, t3) == (t0 + 1, t0 + 2, t0 + 3)
        assert wait(t3) == 0 and np.array_equal(accs[3], want)
        assert wait(t2) == edv.EDV_E_HIP
        assert not accs[2].any()                  # zeroed at submission, nothing written after
        assert wait(t1) == 0 and np.array_equal(accs[1], want)   # still in its slot: its own verdicts
        assert wait(t0) == edv.EDV_E_HIP          # settled below the failed ticket: sticky
        assert wait(t2) == edv.EDV_E_HIP          # and the failed one stays failed
        assert ml.edv_test_fail_async(dev, -1) == 0
        later = [submit(accs[4 + k]) for k in range(10)]   # every slot reused after the failure
        for k, t in enumerate(later):
            assert wait(t) == 0 and np.array_equal(accs[4 + k], want), (pinned, k)
        assert wait(later[-1] + 1) == edv.EDV_E_ARG  # never issued
    pin.free()


def test_query_async_hands_over_without_waiting():
    """edv_query_async (the Node's early hand-over, pool.py handover="early"):
    EDV_PENDING while a batch runs, then 0 with the verdicts in the caller's
    buffer -- latency-path and batch-path sizes, pageable and page-locked
    verdicts -- and 0 again when asked twice; EDV_E_ARG for a ticket never
    issued; a failed batch (fault hook of the measurement build) answers
    EDV_E_HIP with all-zero verdicts, and the wait after it says the same."""
    import ctypes
    import time
    lib = edv.lib()
    dev = 0
    cases = [orc.corpus(0x9E40 + k, 0, n, mode=k % 2, invalid_permille=80) for k, n in enumerate((400, 65536))]
    wants = [checker(*c) for c in cases]
    pin = edv.PinnedBuffer(65536 + 64)

    def poll(query, t, limit_s=20.0):
        t0 = time.time()
        while True:
            rc = query(dev, t)
            if rc != edv.EDV_PENDING:
                return rc
            assert time.time() - t0 < limit_s, "batch never completed"
            time.sleep(0.0001)

    for pinned in (False, True):
        for (sigs, pks, msgs, off), want in zip(cases, wants):
            n = len(off) - 1
            acc = pin.array[:n] if pinned else np.full(n, 7, np.uint8)
            acc[:] = 7
            t = ctypes.c_int64(-1)
            assert lib.edv_verify_batch_async(sigs.ctypes.data, pks.ctypes.data, msgs.ctypes.data, off.ctypes.data,
                                              n, acc.ctypes.data, dev, ctypes.byref(t)) == 0
            assert poll(lib.edv_query_async, t.value) == 0
            assert np.array_equal(acc, want), (pinned, n)
            assert lib.edv_query_async(dev, t.value) == 0 and lib.edv_wait_async(dev, t.value) == 0
            assert edv.query_async(t.value, dev)
    assert lib.edv_query_async(dev, t.value + 1000) == edv.EDV_E_ARG
    pin.free()
    # a failed batch, through the measurement build's fault hook
    ml = edv.measure_lib()
    ml.edv_query_async.argtypes = [ctypes.c_int, ctypes.c_int64]
    sigs, pks, msgs, off = cases[0]
    n = len(off) - 1
    acc = np.full(n, 7, np.uint8)
    t = ctypes.c_int64(-1)
    assert ml.edv_verify_batch_async(sigs.ctypes.data, pks.ctypes.data, msgs.ctypes.data, off.ctypes.data, n,
                                     acc.ctypes.data, dev, ctypes.byref(t)) == 0
    assert poll(ml.edv_query_async, t.value) == 0
    assert ml.edv_test_fail_async(dev, t.value + 1) == 0
    assert ml.edv_verify_batch_async(sigs.ctypes.data, pks.ctypes.data, msgs.ctypes.data, off.ctypes.data, n,
                                     acc.ctypes.data, dev, ctypes.byref(t)) == 0
    assert poll(ml.edv_query_async, t.value) == edv.EDV_E_HIP
    assert not acc.any()
    assert ml.edv_wait_async(dev, t.value) == edv.EDV_E_HIP
    assert ml.edv_test_fail_async(dev, -1) == 0


def test_context_memory_and_table_sets():
    """edv_context_memory reports the library's device
    memory by kind.  In a fresh process with the default table policy a
    Node-sized batch builds only the compact [S]B set (64 MiB) and scratch
    sized to the batch, well under 1.5 GB; a C2-sized batch then adds the
    large set (3 GiB); EDV_SB_TABLES=compact never builds it.  Verdicts equal
    libsodium's in every configuration."""
    code = r'''
import json, sys, numpy as np
sys.path.insert(0, %r); sys.path.insert(0, %r)
import oracle_lib as orc
from indy_plenum_amd import edv
out = {}
for n in (400, 65536):
    s, p, m, o = orc.corpus(0xF00D, 0, n, mode=0, invalid_permille=50)
    acc = edv.verify_arrays(s, p, m, o)
    want = orc.sodium_verify_batch(s, p, m, o, 16) if orc.sodium_batch() else acc
    out[str(n)] = {"equal": bool(np.array_equal(acc, want)), "mem": edv.context_memory(0)}
print(json.dumps(out))
''' % (ROOT, os.path.join(ROOT, "tests"))
    res = {}
    for pol in ("auto", "compact"):
        env = dict(os.environ, EDV_SB_TABLES=pol)
        r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300, env=env)
        assert r.returncode == 0, r.stderr[-2000:]
        res[pol] = json.loads(r.stdout.strip().splitlines()[-1])
    for pol, d in res.items():
        assert d["400"]["equal"] and d["65536"]["equal"], pol
        m = d["400"]["mem"]
        assert m["sb_tables"] < 80 * 2**20, (pol, m)             # compact set only
        assert 0 < m["total"] < 1.5 * 2**30, (pol, m)
        assert m["total"] == sum(v for k, v in m.items() if k != "total")
    assert res["auto"]["65536"]["mem"]["sb_tables"] > 3 * 2**30    # large set added at C2 size
    assert res["compact"]["65536"]["mem"]["sb_tables"] < 80 * 2**20
