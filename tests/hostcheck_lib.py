"""ctypes access to libedv_hostcheck.so: the KERNEL's own math and per-signature
algorithm (indy-plenum_amd/csrc/edv_math.h, edv_verify_core.h, edv_sha256.h) compiled for the
CPU.  Test harness only."""
import ctypes
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "indy-plenum_amd", "csrc")
SO = os.path.join(ROOT, "indy-plenum_amd", "libedv_hostcheck.so")
_lib = None


def load():
    global _lib
    if _lib is None and os.environ.get("EDV_HOSTCHECK_OVERRIDE"):
        _lib = _bind(ctypes.CDLL(os.environ["EDV_HOSTCHECK_OVERRIDE"]))  # an instrumented build (tools/asan_host.sh)
    if _lib is None:
        srcs = [os.path.join(CSRC, f) for f in ("edv_hostcheck.cpp", "edv_math.h", "edv_verify_core.h", "edv_sha256.h", "edv_ledger.h")]
        if not os.path.exists(SO) or os.path.getmtime(SO) < max(os.path.getmtime(s) for s in srcs):
            subprocess.check_call(["make", "-s", "-C", CSRC, "../libedv_hostcheck.so"])
        _lib = _bind(ctypes.CDLL(SO))
    return _lib


def _bind(lib):
    lib.hc_hram.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_uint64, ctypes.c_void_p]
    lib.hc_sha256.argtypes = [ctypes.c_char_p, ctypes.c_uint64, ctypes.c_int, ctypes.c_void_p]
    lib.hc_recode.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_void_p]
    lib.hc_btab_entries_of.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
    lib.hc_rside_point.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_void_p]
    lib.hc_btab_entries_of_bits.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_int,
                                            ctypes.c_void_p]
    lib.hc_rside_point_bits.argtypes = [ctypes.c_int, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_void_p]
    lib.hc_half_scalars.argtypes = [ctypes.c_char_p, ctypes.c_void_p, ctypes.c_void_p]
    lib.hc_verify_batch.argtypes = [ctypes.c_char_p] * 3 + [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p]
    lib.hc_layout.argtypes = [ctypes.c_void_p]
    lib.hc_ledger.argtypes = [ctypes.c_int64, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int,
                              ctypes.c_void_p]
    return lib


def layout():
    """The walk's layout constants as built (edv_verify_core.h)."""
    out = (ctypes.c_int32 * 4)()
    load().hc_layout(out)
    return dict(zip(("awin", "aentries", "bbits", "btables"), list(out)))


def ledger(n, failed, queries):
    """edv_ledger.h AsyncLedger: issue n tickets, fail `failed`, settled() per query."""
    import numpy as np
    f = np.asarray(failed, np.int64)
    q = np.asarray(queries, np.int64)
    out = np.zeros(len(q), np.int32)
    load().hc_ledger(n, f.ctypes.data, len(f), q.ctypes.data, len(q), out.ctypes.data)
    return out.tolist()
