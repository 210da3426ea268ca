"""ctypes access to the CPU oracle (oracle/liboref.so) -- TEST INFRASTRUCTURE.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use this,
and only as the checker / the timed CPU baseline.  See oracle/ed25519_oracle.c.
"""
import ctypes
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
ORACLE_SO = os.path.join(ORACLE_DIR, "liboref.so")

_lib = None


def load():
    """Load (building if needed) the oracle shared library."""
    global _lib
    if _lib is not None:
        return _lib
    src = os.path.join(ORACLE_DIR, "ed25519_oracle.c")
    if not os.path.exists(ORACLE_SO) or os.path.getmtime(ORACLE_SO) < os.path.getmtime(src):
        subprocess.check_call(["make", "-s", "-C", ORACLE_DIR])
    lib = ctypes.CDLL(ORACLE_SO)
    u8p = ctypes.c_char_p
    lib.oref_verify_detached.argtypes = [u8p, u8p, ctypes.c_uint64, u8p]
    lib.oref_sign_open.argtypes = [u8p, ctypes.c_uint64, u8p]
    lib.oref_sign_detached.argtypes = [ctypes.c_void_p, u8p, ctypes.c_uint64, u8p]
    lib.oref_seed_keypair.argtypes = [ctypes.c_void_p, ctypes.c_void_p, u8p]
    lib.oref_sha512.argtypes = [ctypes.c_void_p, u8p, ctypes.c_uint64]
    lib.oref_sc_reduce64.argtypes = [ctypes.c_void_p, u8p]
    lib.oref_point_add.argtypes = [ctypes.c_void_p, u8p, u8p]
    lib.oref_scalarmult.argtypes = [ctypes.c_void_p, u8p, u8p]
    lib.oref_scalarmult_base.argtypes = [ctypes.c_void_p, u8p]
    lib.oref_verify_batch.argtypes = [ctypes.c_void_p] * 4 + [ctypes.c_uint64, ctypes.c_void_p, ctypes.c_int]
    _lib = lib
    return lib


def verify(sig: bytes, msg: bytes, pk: bytes) -> bool:
    assert len(sig) == 64 and len(pk) == 32
    return load().oref_verify_detached(sig, msg, len(msg), pk) == 0


def sign_open(sm: bytes, pk: bytes) -> bool:
    return load().oref_sign_open(sm, len(sm), pk) == 0


def keypair(seed: bytes):
    pk, sk = ctypes.create_string_buffer(32), ctypes.create_string_buffer(64)
    load().oref_seed_keypair(pk, sk, seed)
    return pk.raw, sk.raw


def sign(msg: bytes, sk: bytes) -> bytes:
    sig = ctypes.create_string_buffer(64)
    load().oref_sign_detached(sig, msg, len(msg), sk)
    return sig.raw


def point_add(p: bytes, q: bytes):
    out = ctypes.create_string_buffer(32)
    return out.raw if load().oref_point_add(out, p, q) == 0 else None


def scalarmult(k: bytes, p: bytes):
    out = ctypes.create_string_buffer(32)
    return out.raw if load().oref_scalarmult(out, k, p) == 0 else None


def scalarmult_base(k: bytes) -> bytes:
    out = ctypes.create_string_buffer(32)
    load().oref_scalarmult_base(out, k)
    return out.raw


def sc_reduce64(s: bytes) -> bytes:
    out = ctypes.create_string_buffer(32)
    load().oref_sc_reduce64(out, s)
    return out.raw


def verify_batch(sigs: bytes, pks: bytes, msgs: bytes, offs, n: int, threads: int = 1) -> bytes:
    import numpy as np
    off = np.ascontiguousarray(offs, dtype=np.uint64)
    acc = ctypes.create_string_buffer(max(n, 1))
    rc = load().oref_verify_batch(sigs, pks, msgs if msgs else b"\0", off.ctypes.data, n, acc, threads)
    assert rc == 0
    return acc.raw[:n]


def corpus_lengths(seed: int, start: int, count: int, mode: int):
    import numpy as np
    lib = load()
    lib.oref_corpus_len.restype = ctypes.c_uint64
    lib.oref_corpus_len.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_int]
    if mode == 0:
        return np.full(count, 256, dtype=np.uint64)
    # same splitmix64 as the C generator, vectorised
    x = (np.uint64(seed) * np.uint64(0x100000001B3)) ^ (np.arange(start, start + count, dtype=np.uint64)) ^ np.uint64(0xC4C4C4C4)
    with np.errstate(over="ignore"):
        x = x + np.uint64(0x9E3779B97F4A7C15)
        x = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        x = (x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        x = x ^ (x >> np.uint64(31))
    return np.uint64(200) + x % np.uint64(3897)


def corpus(seed: int, start: int, count: int, mode: int = 0, invalid_permille: int = 50, threads: int = None):
    """Deterministic signed-request corpus (items [start, start+count)):
    -> (sigs, pks, msgs, off) numpy uint8/uint64 arrays in the C-ABI layout."""
    import numpy as np
    lib = load()
    threads = threads or min(16, os.cpu_count() or 1)
    lens = corpus_lengths(seed, start, count, mode)
    off = np.zeros(count + 1, dtype=np.uint64)
    off[1:] = np.cumsum(lens)
    sigs = np.zeros(64 * count, dtype=np.uint8)
    pks = np.zeros(32 * count, dtype=np.uint8)
    msgs = np.zeros(int(off[-1]) + 64, dtype=np.uint8)
    lib.oref_corpus_gen.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_int, ctypes.c_int,
                                    ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
    rc = lib.oref_corpus_gen(seed, start, count, mode, invalid_permille, sigs.ctypes.data, pks.ctypes.data,
                             msgs.ctypes.data, off.ctypes.data, threads)
    assert rc == 0
    return sigs, pks, msgs, off


SODIUM_SO = os.path.join(ORACLE_DIR, "libsodium_batch.so")
_sb = None


def sodium_batch():
    """libsodium 1.0.18 batch harness (oracle/sodium_batch.c) or None if the
    image's libsodium is absent."""
    global _sb
    if _sb is None:
        if not os.path.exists(SODIUM_SO):
            subprocess.call(["make", "-s", "-C", ORACLE_DIR, "libsodium_batch.so"])
        if not os.path.exists(SODIUM_SO):
            return None
        try:
            lib = ctypes.CDLL(SODIUM_SO)
        except OSError:
            return None
        lib.sb_version.restype = ctypes.c_char_p
        lib.sb_verify_batch.argtypes = [ctypes.c_void_p] * 4 + [ctypes.c_uint64, ctypes.c_void_p, ctypes.c_int]
        _sb = lib
    return _sb


def sodium_verify_batch(sigs, pks, msgs, off, threads: int = 1):
    import numpy as np
    lib = sodium_batch()
    n = len(off) - 1
    acc = np.zeros(n, dtype=np.uint8)
    off = np.ascontiguousarray(off, dtype=np.uint64)
    assert lib.sb_verify_batch(sigs.ctypes.data, pks.ctypes.data, msgs.ctypes.data, off.ctypes.data, n,
                               acc.ctypes.data, threads) == 0
    return acc
