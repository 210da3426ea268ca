"""The reference's CPU verify path for benchmarks: libsodium
crypto_sign_open(signature + msg, pk) through ctypes, which is what libnacl
does under stp_core/crypto/nacl_wrappers.py:232-242.  Key derivation is the
DidVerifier one (plenum/common/verifier.py:26-52).  Bench infrastructure only."""
import ctypes

from indy_plenum_amd.client_authn import CoreAuthNr
from indy_plenum_amd.verifier import DidVerifier, Verifier

_sodium = None


def sodium():
    global _sodium
    if _sodium is None:
        for path in ("/opt/conda/lib/libsodium.so.23", "libsodium.so.23", "libsodium.so"):
            try:
                _sodium = ctypes.CDLL(path)
                break
            except OSError:
                continue
        if _sodium is not None:
            _sodium.sodium_init()
    return _sodium


class SodiumVerifier(Verifier):
    """DidVerifier key derivation + crypto_sign_open, as libnacl does it."""

    def __init__(self, verkey, identifier=None):
        self.pk = DidVerifier(verkey, identifier).batch_key()

    def verify(self, sig, msg):
        sm = bytes(sig) + bytes(msg)
        m = ctypes.create_string_buffer(len(sm))
        mlen = ctypes.c_ulonglong(0)
        return sodium().crypto_sign_open(m, ctypes.byref(mlen), sm, ctypes.c_ulonglong(len(sm)), self.pk) == 0


class SodiumCoreAuthNr(CoreAuthNr):
    """CoreAuthNr whose verifier is libsodium on the CPU (the reference's Node)."""

    def authenticate(self, req_data, identifier=None, signature=None, verifier=None):
        return super().authenticate(req_data, identifier, signature, verifier=SodiumVerifier)
