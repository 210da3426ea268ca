"""GPU-backed counterparts of the reference's libnacl wrappers on the verify
path (stp_core/crypto/nacl_wrappers.py:62-108 VerifyKey, :212-242 Verifier).

Same constructor rules and results; the arithmetic runs in the gfx950 kernels
through edv.open_batch instead of libnacl.crypto_sign_open.  Signing, Box and
Curve25519 classes of that module are not on the verification hot path and
are out of scope.
"""
import binascii

from . import edv


class RawEncoder(object):
    @staticmethod
    def encode(data):
        return data

    @staticmethod
    def decode(data):
        return data


class HexEncoder(object):
    @staticmethod
    def encode(data):
        return binascii.hexlify(data)

    @staticmethod
    def decode(data):
        return binascii.unhexlify(data)


class Encodable(object):
    def encode(self, encoder=RawEncoder):
        return encoder.encode(bytes(self))


PUBLICKEYBYTES = 32


class VerifyKey(Encodable):
    """Ed25519 public key (nacl_wrappers.py:62-108)."""

    def __init__(self, key, encoder=RawEncoder):
        key = encoder.decode(key)
        if len(key) != PUBLICKEYBYTES:
            raise ValueError("The key must be exactly %s bytes long" % PUBLICKEYBYTES)
        self._key = key

    def __bytes__(self):
        return self._key

    def verify(self, smessage, signature=None, encoder=RawEncoder):
        """Return the message of a valid signed message, else raise ValueError
        (libnacl.crypto_sign_open semantics: sm[:64] is the signature)."""
        if signature is not None:
            smessage = signature + smessage
        smessage = encoder.decode(smessage)
        if not edv.open_batch([(smessage, b"", self._key)])[0]:
            raise ValueError("Failed to validate message")
        return smessage[64:]


class Verifier:
    """Used to verify messages with an Ed25519 signature (nacl_wrappers.py:212-242)."""

    def __init__(self, key=None):
        if key:
            if not isinstance(key, VerifyKey):
                if len(key) == 32:
                    key = VerifyKey(key, RawEncoder)
                else:
                    key = VerifyKey(key, HexEncoder)
        self.key = key
        if isinstance(self.key, VerifyKey):
            self.keyhex = self.key.encode(HexEncoder)
            self.keyraw = self.key.encode(RawEncoder)
        else:
            self.keyhex = ''
            self.keyraw = ''

    def verify(self, signature, msg):
        if not self.key:
            return False
        return edv.open_batch([(signature, msg, bytes(self.key))])[0]

    # batch hook used by client_authn.authenticate_batch: the 32-byte key the
    # crypto_sign_open(signature + msg, key) call would use, or None (-> False)
    def batch_key(self):
        return bytes(self.key) if self.key else None
