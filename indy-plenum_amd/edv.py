"""ctypes binding of the gfx950 batch verifier C-ABI (include/edv.h, libedv.so).

This is the thin shim between Plenum's authenticator layer (client_authn.py,
req_authenticator.py, verifier.py, nacl_wrappers.py in this package) and the
HIP kernels.  There is no CPU fallback here: if libedv.so is missing or no
gfx950 device is visible, every call raises EdvUnavailable, loudly.

Reference behaviour reproduced at this layer:
  stp_core/crypto/nacl_wrappers.py:232-242  Verifier.verify(signature, msg)
      -> crypto_sign_open(signature + msg, pk): the first 64 bytes of the
         CONCATENATION are the signature and the rest is the message, so a
         non-64-byte "signature" re-splits positionally (open_batch below);
         fewer than 64 bytes in total rejects (libsodium: smlen < 64).
"""
import ctypes
import os
import threading

import numpy as np

from . import _edvhost  # native host-side packing (csrc/edv_host.cpp, row f-1)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("EDV_LIB", os.path.join(_HERE, "libedv.so"))
# the benchmark/profiling build (include/edv_measure.h): loaded only by the
# measurement helpers below (bench.py, tools/, the GPU tests' fault hook),
# never by the authenticators
MEASURE_LIB_PATH = os.path.join(_HERE, "libedv_measure.so")
MEASUREMENT_TAG = "MEASUREMENT-ONLY"  # in edv_version() of builds whose verdicts are not libsodium's

EDV_OK = 0
EDV_E_ARG = -1
EDV_E_NODEV = -2
EDV_E_HIP = -3
EDV_E_OOM = -4
FLAG_UNIFORM_LENGTH = 1  # every message has the same SHA-512 block count: no length buckets
FLAG_BUCKETS = 2         # always bucket by SHA-512 block count
FLAG_SPLIT_PREP = 4      # pipelined path: batch k+1's hash side beside batch k's main kernel


class EdvUnavailable(RuntimeError):
    """libedv.so cannot be loaded or no gfx950 device is visible."""


class EdvError(RuntimeError):
    """The C-ABI returned an error code."""

    def __init__(self, code, what):
        super().__init__("edv error {}: {}".format(code, what))
        self.code = code


_lock = threading.Lock()
_lib = None


def lib():
    """The loaded libedv.so (raises EdvUnavailable if it is not built)."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise EdvUnavailable("libedv.so not built at {} (run __graft_entry__.build())".format(LIB_PATH))
        h = ctypes.CDLL(LIB_PATH)
        h.edv_version.restype = ctypes.c_char_p
        ver = h.edv_version().decode(errors="replace")
        if MEASUREMENT_TAG in ver and os.environ.get("EDV_ALLOW_MEASUREMENT_LIB") != "1":
            # a measurement build (e.g. variants/libedv_noverify.so reports every
            # signature valid) must never authenticate requests: fail closed,
            # as the reference's Verifier never returns True without libsodium's
            # check (nacl_wrappers.py:232-242)
            raise EdvUnavailable("{} is a measurement-only build ({}); refusing to load it "
                                 "(EDV_ALLOW_MEASUREMENT_LIB=1 is for benchmarks only)".format(LIB_PATH, ver))
        vp, u64 = ctypes.c_void_p, ctypes.c_uint64
        h.edv_verify_batch.argtypes = [vp, vp, vp, vp, u64, vp, ctypes.c_uint32]
        h.edv_verify_batch.restype = ctypes.c_int
        h.edv_verify_batch_dev.argtypes = [vp, vp, vp, vp, u64, u64, vp, ctypes.c_int, vp]
        h.edv_verify_batch_dev.restype = ctypes.c_int
        h.edv_sha256_batch.argtypes = [vp, vp, u64, vp, ctypes.c_uint32]
        h.edv_sha256_batch.restype = ctypes.c_int
        h.edv_sha256_batch_dev.argtypes = [vp, vp, u64, u64, vp, ctypes.c_int, vp]
        h.edv_sha256_batch_dev.restype = ctypes.c_int
        h.edv_verify_batch_dev_flags.argtypes = [vp, vp, vp, vp, u64, u64, vp, ctypes.c_int, vp, ctypes.c_uint32]
        h.edv_verify_batch_dev_flags.restype = ctypes.c_int
        h.edv_verify_batch_dev_pipelined.argtypes = [vp, vp, vp, vp, u64, u64, vp, ctypes.c_int, ctypes.c_uint32]
        h.edv_verify_batch_dev_pipelined.restype = ctypes.c_int
        h.edv_verify_batch_async.argtypes = [vp, vp, vp, vp, u64, vp, ctypes.c_int, ctypes.POINTER(ctypes.c_int64)]
        h.edv_verify_batch_async.restype = ctypes.c_int
        h.edv_verify_digest_batch_async.argtypes = [vp, vp, vp, vp, u64, vp, vp, ctypes.c_int,
                                                    ctypes.POINTER(ctypes.c_int64)]
        h.edv_verify_digest_batch_async.restype = ctypes.c_int
        h.edv_wait_async.argtypes = [ctypes.c_int, ctypes.c_int64]
        h.edv_wait_async.restype = ctypes.c_int
        h.edv_query_async.argtypes = [ctypes.c_int, ctypes.c_int64]
        h.edv_query_async.restype = ctypes.c_int
        h.edv_pipeline_sync.argtypes = [ctypes.c_int]
        h.edv_pipeline_sync.restype = ctypes.c_int
        h.edv_sign_batch_dev.argtypes = [vp, vp, vp, u64, u64, vp, vp, ctypes.c_int, vp]
        h.edv_sign_batch_dev.restype = ctypes.c_int
        h.edv_stream.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)]
        h.edv_stream.restype = ctypes.c_int
        h.edv_sync.argtypes = [ctypes.c_int]
        h.edv_sync.restype = ctypes.c_int
        h.edv_set_latency_path.argtypes = [ctypes.c_int, u64]
        h.edv_set_latency_path.restype = ctypes.c_int
        h.edv_set_length_buckets.argtypes = [ctypes.c_int, ctypes.c_int]
        h.edv_set_length_buckets.restype = ctypes.c_int
        h.edv_set_chunk.argtypes = [ctypes.c_int, u64]
        h.edv_set_chunk.restype = ctypes.c_int
        h.edv_set_host_slices.argtypes = [ctypes.c_int, ctypes.c_int]
        h.edv_set_host_slices.restype = ctypes.c_int
        h.edv_shard_split.argtypes = [vp, u64, ctypes.c_uint32, vp]
        h.edv_shard_split.restype = ctypes.c_int
        h.edv_host_alloc.argtypes = [u64, ctypes.POINTER(ctypes.c_void_p)]
        h.edv_host_alloc.restype = ctypes.c_int
        h.edv_host_free.argtypes = [vp]
        h.edv_host_free.restype = ctypes.c_int
        h.edv_device_count.argtypes = []
        h.edv_device_count.restype = ctypes.c_int
        h.edv_context_count.argtypes = []
        h.edv_context_count.restype = ctypes.c_int
        h.edv_pick_device.argtypes = [ctypes.c_uint32]
        h.edv_pick_device.restype = ctypes.c_int
        h.edv_pack_bits_dev.argtypes = [vp, u64, vp, ctypes.c_int, vp]
        h.edv_pack_bits_dev.restype = ctypes.c_int
        h.edv_context_memory.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_uint64)]
        h.edv_context_memory.restype = ctypes.c_int
        h.edv_dev_alloc.argtypes = [ctypes.c_int, u64, ctypes.POINTER(ctypes.c_void_p)]
        h.edv_dev_free.argtypes = [ctypes.c_int, vp]
        h.edv_h2d.argtypes = [ctypes.c_int, vp, vp, u64]
        h.edv_d2h.argtypes = [ctypes.c_int, vp, vp, u64]
        h.edv_version.restype = ctypes.c_char_p
        h.edv_last_error.restype = ctypes.c_char_p
        _lib = h
        return h


_mlib = None


def measure_lib():
    """libedv_measure.so: the same verifier plus kernel timing and the fault hook
    (include/edv_measure.h).  Its device contexts are its own (a second [S]B
    table set and scratch per GPU in this process); device pointers from either
    library may be passed to the other."""
    global _mlib
    if _mlib is not None:
        return _mlib
    with _lock:
        if _mlib is not None:
            return _mlib
        if not os.path.exists(MEASURE_LIB_PATH):
            raise EdvUnavailable("libedv_measure.so not built at {} (run __graft_entry__.build())"
                                 .format(MEASURE_LIB_PATH))
        h = ctypes.CDLL(MEASURE_LIB_PATH)
        vp, u64, f32p = ctypes.c_void_p, ctypes.c_uint64, ctypes.POINTER(ctypes.c_float)
        h.edv_time_batch_dev.argtypes = [vp, vp, vp, vp, u64, u64, vp, ctypes.c_int, ctypes.c_int, f32p]
        h.edv_profile_batch_dev.argtypes = [vp, vp, vp, vp, u64, u64, vp, ctypes.c_int, ctypes.c_int, f32p, f32p]
        h.edv_profile_batch_dev_flush.argtypes = [vp, vp, vp, vp, u64, u64, vp, ctypes.c_int, ctypes.c_int, u64,
                                                  f32p, f32p, f32p]
        h.edv_profile_prep_sides.argtypes = [vp, vp, vp, vp, u64, u64, vp, ctypes.c_int, ctypes.c_int, f32p]
        h.edv_test_fail_async.argtypes = [ctypes.c_int, ctypes.c_int64]
        h.edv_verify_batch_async.argtypes = [vp, vp, vp, vp, u64, vp, ctypes.c_int, ctypes.POINTER(ctypes.c_int64)]
        h.edv_wait_async.argtypes = [ctypes.c_int, ctypes.c_int64]
        h.edv_last_error.restype = ctypes.c_char_p
        h.edv_version.restype = ctypes.c_char_p
        _mlib = h
        return h


def _mcheck(rc):
    if rc != EDV_OK:
        what = measure_lib().edv_last_error().decode(errors="replace")
        if rc == EDV_E_NODEV:
            raise EdvUnavailable(what)
        raise EdvError(rc, what)


def version() -> str:
    return lib().edv_version().decode()


CONTEXT_MEMORY_FIELDS = ("total", "sb_tables", "chunk_scratch", "async_slots", "pipelined_sets", "sync_inputs",
                         "signer_comb")


def context_memory(device: int = 0) -> dict:
    """Device bytes the library holds for `device` in this process
    (edv_context_memory), by kind; all zero before the context exists."""
    out = (ctypes.c_uint64 * 7)()
    _check(lib().edv_context_memory(device, out))
    return dict(zip(CONTEXT_MEMORY_FIELDS, (int(x) for x in out)))


def device_count() -> int:
    return lib().edv_device_count()


def context_count() -> int:
    """Devices whose context the library has initialised (placement tests)."""
    return lib().edv_context_count()


def pick_device(device_mask: int = 0) -> int:
    """The device edv_pick_device chooses for a one-device batch (include/edv.h)."""
    d = lib().edv_pick_device(device_mask)
    if d < 0:
        _check(d)
    return d


def batch_device() -> int:
    """Device of the next native asynchronous whole-batch submission: BATCH_DEVICE
    if set, else the library's choice among BATCH_DEVICE_MASK (an idle
    initialised device, else a fresh one), so the Nodes of one process spread
    over the GPUs while a lone caller stays on one context."""
    return BATCH_DEVICE if BATCH_DEVICE is not None else pick_device(BATCH_DEVICE_MASK)


def stream(device: int = 0) -> int:
    """The library's HIP stream of `device` (for asynchronous edv_*_dev calls)."""
    p = ctypes.c_void_p()
    _check(lib().edv_stream(device, ctypes.byref(p)))
    return p.value


def sync(device: int = 0):
    """Wait for everything enqueued on the library stream of `device`."""
    _check(lib().edv_sync(device))


def set_length_buckets(device: int, mode: int):
    """SHA-512 length buckets on the device paths: 0 never, 1 always, 2 auto (default)."""
    _check(lib().edv_set_length_buckets(device, mode))


LATENCY_PATH_DEFAULT = 16384


def set_latency_path(device: int, max_requests: int):
    """Batches of at most max_requests (0 = never) run on the four-lanes-per-
    signature latency kernel (edv_set_latency_path).  Never changes verdicts."""
    _check(lib().edv_set_latency_path(device, max_requests))


def set_chunk(device: int, chunk: int):
    """Signatures per prep/main kernel pair (0 = default).  Never changes verdicts."""
    _check(lib().edv_set_chunk(device, chunk))


def set_host_slices(device: int, slices: int):
    """Message slices of a synchronous one-chunk shard (edv_set_host_slices; 0 = default)."""
    _check(lib().edv_set_host_slices(device, slices))


def _check(rc):
    if rc != EDV_OK:
        what = lib().edv_last_error().decode(errors="replace")
        if rc == EDV_E_NODEV:
            raise EdvUnavailable(what)
        raise EdvError(rc, what)


def verify_arrays(sigs, pks, msgs, offsets, device_mask: int = 0) -> np.ndarray:
    """Verify n detached 64-byte signatures laid out as the C-ABI expects.

    sigs: n*64 bytes, pks: n*32 bytes, msgs: concatenated messages, offsets:
    n+1 uint64 byte offsets.  Returns a uint8 array of n verdicts (1 = accept),
    bit-exact with libsodium crypto_sign_ed25519_verify_detached.
    """
    off = np.ascontiguousarray(offsets, dtype=np.uint64)
    n = len(off) - 1
    if n <= 0:
        return np.zeros(0, dtype=np.uint8)
    sigs = np.frombuffer(bytes(sigs), dtype=np.uint8) if not isinstance(sigs, np.ndarray) else sigs
    pks = np.frombuffer(bytes(pks), dtype=np.uint8) if not isinstance(pks, np.ndarray) else pks
    if not isinstance(msgs, np.ndarray):
        msgs = np.frombuffer(bytes(msgs) or b"\0", dtype=np.uint8)
    if sigs.nbytes != 64 * n or pks.nbytes != 32 * n:
        raise ValueError("sigs/pks size does not match offsets")
    if int(off[-1]) > msgs.nbytes:
        raise ValueError("offsets exceed the message buffer")
    accept = np.zeros(n, dtype=np.uint8)
    _check(lib().edv_verify_batch(sigs.ctypes.data, pks.ctypes.data, msgs.ctypes.data, off.ctypes.data, n,
                                  accept.ctypes.data, device_mask))
    return accept


def verify_async(sigs: np.ndarray, pks: np.ndarray, msgs: np.ndarray, offsets: np.ndarray, accept: np.ndarray,
                 device: int = 0) -> int:
    """Queue one host batch (edv_verify_batch_async) and return its ticket.

    The arrays (uint8 sigs/pks/msgs/accept, uint64 offsets, C-ABI layout) must
    stay alive and unchanged, and `accept` unread, until wait_async(ticket)."""
    off = offsets
    n = len(off) - 1
    if off.dtype != np.uint64 or not off.flags.c_contiguous:
        raise ValueError("offsets must be a contiguous uint64 array")
    if sigs.nbytes != 64 * n or pks.nbytes != 32 * n or accept.nbytes < n:
        raise ValueError("sigs/pks/accept size does not match offsets")
    if n > 0 and int(off[-1]) > msgs.nbytes:
        raise ValueError("offsets exceed the message buffer")
    t = ctypes.c_int64(-1)
    _check(lib().edv_verify_batch_async(sigs.ctypes.data, pks.ctypes.data, msgs.ctypes.data, off.ctypes.data, n,
                                        accept.ctypes.data, device, ctypes.byref(t)))
    return t.value


def wait_async(ticket: int, device: int = 0) -> None:
    """Wait until batch `ticket` has its verdicts in its accept array."""
    _check(lib().edv_wait_async(device, ticket))


EDV_PENDING = 1


def query_async(ticket: int, device: int = 0) -> bool:
    """wait_async without the wait: False while batch `ticket` is still on the
    GPU, True once it is done (its verdicts then handed over, as wait_async
    would); raises as wait_async would for a failed batch."""
    rc = lib().edv_query_async(device, ticket)
    if rc == EDV_PENDING:
        return False
    _check(rc)
    return True


def sha256_arrays(msgs, offsets, device_mask: int = 0) -> np.ndarray:
    """SHA-256 of n messages in the C-ABI layout -> (n, 32) uint8 digests (row f-3)."""
    off = np.ascontiguousarray(offsets, dtype=np.uint64)
    n = len(off) - 1
    if n <= 0:
        return np.zeros((0, 32), dtype=np.uint8)
    if not isinstance(msgs, np.ndarray):
        msgs = np.frombuffer(bytes(msgs) or b"\0", dtype=np.uint8)
    if int(off[-1]) > msgs.nbytes:
        raise ValueError("offsets exceed the message buffer")
    out = np.zeros((n, 32), dtype=np.uint8)
    _check(lib().edv_sha256_batch(msgs.ctypes.data, off.ctypes.data, n, out.ctypes.data, device_mask))
    return out


def sha256_batch(messages, device_mask: int = 0):
    """list[bytes] -> list[32-byte digest] (hashlib.sha256(m).digest() for each m)."""
    messages = list(messages)
    if not messages:
        return []
    off = np.zeros(len(messages) + 1, dtype=np.uint64)
    off[1:] = np.cumsum([len(m) for m in messages])
    d = sha256_arrays(b"".join(messages), off, device_mask)
    return [bytes(r) for r in d]


def pack_bits_device(d_accept, n, d_bits, device=0, stream=None):
    """Device accept bytes -> bitmask (ceil(n/8) bytes, little-endian bit order)."""
    _check(lib().edv_pack_bits_dev(d_accept, n, d_bits, device, stream))


def sha256_device(d_msgs, d_off, n, d_out, device=0, msg_base=0, stream=None):
    """Device-resident batch SHA-256: d_out gets n x 32 bytes."""
    _check(lib().edv_sha256_batch_dev(d_msgs, d_off, msg_base, n, d_out, device, stream))


def verify_detached_batch(items, device_mask: int = 0):
    """items: iterable of (sig64: bytes, msg: bytes, pk32: bytes) -> list[bool]."""
    items = list(items)
    if not items:
        return []
    for s, _m, p in items:
        if len(s) != 64 or len(p) != 32:
            raise ValueError("verify_detached_batch needs 64-byte sigs and 32-byte keys")
    off = np.zeros(len(items) + 1, dtype=np.uint64)
    off[1:] = np.cumsum([len(m) for _s, m, _p in items])
    acc = verify_arrays(b"".join(s for s, _m, _p in items), b"".join(p for _s, _m, p in items),
                        b"".join(m for _s, m, _p in items), off, device_mask)
    return [bool(a) for a in acc]


def open_batch(items, device_mask: int = 0):
    """crypto_sign_open semantics on (signature, msg, pk) triples, batched.

    Mirrors nacl_wrappers.Verifier.verify (nacl_wrappers.py:232-242): the signed
    message is signature + msg and libsodium splits it positionally, so a
    signature of any length is accepted iff (sm[:64], sm[64:]) verifies; sm
    shorter than 64 bytes rejects without reaching the GPU.  pk must be 32 bytes.
    """
    items = list(items)
    if not items:
        return []
    addr = verify_address()
    try:
        out = _edvhost.open_verify(items, addr, device_mask)
    except TypeError:  # bytearray / memoryview / list items: normalise, then pack
        items = [(bytes(s), bytes(m), bytes(p)) for s, m, p in items]
        out = _edvhost.open_verify(items, addr, device_mask)
    if isinstance(out, int):  # the C-ABI's error code
        _check(out)
    return out


_OPEN_BATCH = open_batch        # the genuine entry point (tests may monkeypatch open_batch)
_verify_addr = None
_sha_addr = None
BATCH_DEVICE_MASK = 0          # devices used by the native whole-batch authenticator path
PREP_THREADS = int(os.environ.get("EDV_PREP_THREADS", "0")) or max(1, min(8, (os.cpu_count() or 2) // 2))


def verify_address() -> int:
    """Address of edv_verify_batch (the native whole-batch authenticator calls it
    with the GIL released); also hands edv_host_alloc/free to _edvhost so its
    batch arenas are page-locked."""
    global _verify_addr
    if _verify_addr is None:
        h = lib()
        _edvhost.set_host_allocator(ctypes.cast(h.edv_host_alloc, ctypes.c_void_p).value,
                                    ctypes.cast(h.edv_host_free, ctypes.c_void_p).value)
        _verify_addr = ctypes.cast(h.edv_verify_batch, ctypes.c_void_p).value
    return _verify_addr


_async_addrs = None


def async_addresses():
    """(edv_verify_digest_batch_async, edv_wait_async) addresses for the native
    asynchronous whole-batch path (_edvhost.auth_core_submit / _finish)."""
    global _async_addrs
    if _async_addrs is None:
        verify_address()  # page-locked arenas
        h = lib()
        _async_addrs = (ctypes.cast(h.edv_verify_digest_batch_async, ctypes.c_void_p).value,
                        ctypes.cast(h.edv_wait_async, ctypes.c_void_p).value)
    return _async_addrs


_query_addr = None


def query_address() -> int:
    """Address of edv_query_async (the native batch handles' ready() calls it)."""
    global _query_addr
    if _query_addr is None:
        _query_addr = ctypes.cast(lib().edv_query_async, ctypes.c_void_p).value
    return _query_addr


BATCH_DEVICE = None            # device of the native asynchronous whole-batch path (None: batch_device())


def sha256_address() -> int:
    """Address of edv_sha256_batch (the native request-digest batch calls it with
    the GIL released)."""
    global _sha_addr
    if _sha_addr is None:
        _sha_addr = ctypes.cast(lib().edv_sha256_batch, ctypes.c_void_p).value
    return _sha_addr


def native_batch_enabled() -> bool:
    """The native whole-batch path calls edv_verify_batch itself, so it is used
    only while open_batch is the genuine entry point."""
    return open_batch is _OPEN_BATCH and os.environ.get("EDV_NATIVE_BATCH", "1") != "0"


class DeviceBuffer:
    """A raw device allocation through the C-ABI (no PyTorch needed)."""

    def __init__(self, nbytes: int, device: int = 0):
        self.device = device
        self.nbytes = nbytes
        p = ctypes.c_void_p()
        _check(lib().edv_dev_alloc(device, nbytes, ctypes.byref(p)))
        self.ptr = p.value

    def upload(self, host):
        a = np.ascontiguousarray(host)
        assert a.nbytes <= self.nbytes
        _check(lib().edv_h2d(self.device, self.ptr, a.ctypes.data, a.nbytes))

    def download(self, nbytes=None, dtype=np.uint8):
        nbytes = self.nbytes if nbytes is None else nbytes
        out = np.empty(nbytes, dtype=np.uint8)
        _check(lib().edv_d2h(self.device, out.ctypes.data, self.ptr, nbytes))
        return out.view(dtype)

    def download_at(self, offset, nbytes, dtype=np.uint8):
        """Bytes [offset, offset + nbytes) of the buffer."""
        assert 0 <= offset and offset + nbytes <= self.nbytes
        out = np.empty(nbytes, dtype=np.uint8)
        if nbytes:
            _check(lib().edv_d2h(self.device, out.ctypes.data, self.ptr + offset, nbytes))
        return out.view(dtype)

    def free(self):
        if self.ptr:
            lib().edv_dev_free(self.device, self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


def verify_device(d_sigs, d_pks, d_msgs, d_off, n, d_accept, device=0, msg_base=0, stream=None, flags=0):
    """Device-resident verify (pointers are ints); async on `stream` if given.
    flags: FLAG_UNIFORM_LENGTH / FLAG_BUCKETS (per-call length-bucket hint)."""
    _check(lib().edv_verify_batch_dev_flags(d_sigs, d_pks, d_msgs, d_off, msg_base, n, d_accept, device, stream,
                                            flags))


def verify_device_pipelined(d_sigs, d_pks, d_msgs, d_off, n, d_accept, device=0, msg_base=0, flags=0):
    """Enqueue a device-resident batch on the library's two-stream pipeline (the
    prep kernel of the next batch overlaps the main kernel of this one); the
    verdicts are in d_accept after pipeline_sync(device)."""
    _check(lib().edv_verify_batch_dev_pipelined(d_sigs, d_pks, d_msgs, d_off, msg_base, n, d_accept, device,
                                                flags))


def shard_split(offsets, g: int) -> np.ndarray:
    """The C-ABI's shard split (edv_shard_split; host only, no GPU): g+1 bounds,
    shard k = requests [b[k], b[k+1]).  Equal counts for one SHA-512 block count,
    else equal estimated cost sum(40 + blocks)."""
    off = np.ascontiguousarray(offsets, dtype=np.uint64)
    n = len(off) - 1
    b = np.zeros(g + 1, dtype=np.uint64)
    _check(lib().edv_shard_split(off.ctypes.data if n > 0 else None, max(n, 0), g, b.ctypes.data))
    return b


class PinnedBuffer:
    """Page-locked host memory (edv_host_alloc): batches packed here reach the
    device by DMA without the library's staging copy.  `.array` is a uint8 view."""

    def __init__(self, nbytes: int):
        p = ctypes.c_void_p()
        _check(lib().edv_host_alloc(nbytes, ctypes.byref(p)))
        self.ptr, self.nbytes = p.value, nbytes
        self.array = np.ctypeslib.as_array((ctypes.c_uint8 * max(nbytes, 1)).from_address(p.value))[:nbytes]

    def view(self, dtype, offset: int = 0, count: int = -1):
        return np.frombuffer(self.array, dtype=dtype, count=count, offset=offset)

    def free(self):
        if self.ptr:
            self.array = None
            lib().edv_host_free(self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


def pipeline_sync(device: int = 0):
    """Wait for every pipelined batch submitted on `device`."""
    _check(lib().edv_pipeline_sync(device))


def sign_device(d_seeds, d_msgs, d_off, n, d_pks, d_sigs, device=0, msg_base=0, stream=None):
    """Device-resident batch signing (row f-4): seeds -> pks, detached sigs."""
    _check(lib().edv_sign_batch_dev(d_seeds, d_msgs, d_off, msg_base, n, d_pks, d_sigs, device, stream))


def sign_arrays(seeds, msgs, offsets, device=0):
    """Host-array convenience over sign_device -> (pks n*32, sigs n*64) uint8 arrays."""
    off = np.ascontiguousarray(offsets, dtype=np.uint64)
    n = len(off) - 1
    seeds = np.ascontiguousarray(np.frombuffer(bytes(seeds), np.uint8) if not isinstance(seeds, np.ndarray) else seeds)
    msgs = np.frombuffer(bytes(msgs) + b"\0" * 16, np.uint8) if not isinstance(msgs, np.ndarray) else msgs
    if n <= 0:
        return np.zeros(0, np.uint8), np.zeros(0, np.uint8)
    bufs = [DeviceBuffer(max(a.nbytes, 1) + 64, device) for a in (seeds, msgs, off)]
    for b, a in zip(bufs, (seeds, msgs, off)):
        b.upload(a)
    dp, ds = DeviceBuffer(32 * n, device), DeviceBuffer(64 * n, device)
    sign_device(bufs[0].ptr, bufs[1].ptr, bufs[2].ptr, n, dp.ptr, ds.ptr, device)
    return dp.download(32 * n), ds.download(64 * n)


# ---- measurement helpers: libedv_measure.so (include/edv_measure.h)
def time_device(d_sigs, d_pks, d_msgs, d_off, n, d_accept, device=0, iters=1, msg_base=0) -> float:
    """Milliseconds for `iters` back-to-back kernel launches (HIP events on the kernel's stream)."""
    ms = ctypes.c_float(0)
    _mcheck(measure_lib().edv_time_batch_dev(d_sigs, d_pks, d_msgs, d_off, msg_base, n, d_accept, device, iters,
                                             ctypes.byref(ms)))
    return float(ms.value)


def profile_device(d_sigs, d_pks, d_msgs, d_off, n, d_accept, device=0, iters=1, msg_base=0):
    """(prep_ms, main_ms): average per-launch kernel times from HIP events on the kernels' stream."""
    a, b = ctypes.c_float(0), ctypes.c_float(0)
    _mcheck(measure_lib().edv_profile_batch_dev(d_sigs, d_pks, d_msgs, d_off, msg_base, n, d_accept, device, iters,
                                                ctypes.byref(a), ctypes.byref(b)))
    return float(a.value), float(b.value)


def profile_device_flush(d_sigs, d_pks, d_msgs, d_off, n, d_accept, device=0, iters=1, flush_bytes=0, msg_base=0):
    """(prep_ms, flush_ms, main_ms) with a cache-evicting kernel of flush_bytes between
    prep and main (edv_profile_batch_dev_flush)."""
    a, f, b = ctypes.c_float(0), ctypes.c_float(0), ctypes.c_float(0)
    _mcheck(measure_lib().edv_profile_batch_dev_flush(d_sigs, d_pks, d_msgs, d_off, msg_base, n, d_accept, device,
                                                      iters, flush_bytes, ctypes.byref(a), ctypes.byref(f),
                                                      ctypes.byref(b)))
    return float(a.value), float(f.value), float(b.value)


PREP_SIDE_KEYS = ("hash_side", "a_side", "r_side", "all_three", "point_sides")


def profile_prep_sides(d_sigs, d_pks, d_msgs, d_off, n, d_accept, device=0, iters=1, msg_base=0) -> dict:
    """The prep kernel's sides timed apart (edv_profile_prep_sides), ms per launch."""
    ms = (ctypes.c_float * 5)()
    _mcheck(measure_lib().edv_profile_prep_sides(d_sigs, d_pks, d_msgs, d_off, msg_base, n, d_accept, device, iters,
                                                 ms))
    return dict(zip(PREP_SIDE_KEYS, (float(x) for x in ms)))
