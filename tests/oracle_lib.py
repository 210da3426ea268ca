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
