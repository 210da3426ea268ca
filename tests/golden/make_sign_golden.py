#!/usr/bin/env python3
"""Generate tests/golden/sign_golden.bin: Ed25519 SIGNING vectors whose outputs
come from libsodium 1.0.18 itself -- crypto_sign_seed_keypair + crypto_sign_detached,
the pair behind the reference's client-side signing
(stp_core/crypto/nacl_wrappers.py:162-176 SigningKey.sign ->
libnacl.crypto_sign; plenum/common/signer_did.py:122-129 DidSigner.sign).

Run here (the container has /opt/conda/lib/libsodium.so.23); the GPU box only
reads the committed .bin.  Row f-4 (edv_sign_batch_dev, the GPU batch signer)
and its CPU build (hc_sign_batch) must reproduce every pk and sig byte for byte.

Cases: the RFC 8032 section 7.1 Ed25519 test vectors 1-3 (checked against
libsodium here), seeds with every byte 0x00 / 0xff, and random seeds with
message lengths 0..4096 spanning every SHA-512 block boundary of the nonce and
challenge hashes (lengths 63..65 + 128k, 111..113 + 128k, ...).

File format (little-endian): magic b"EDVSIGN1", u32 count, then per record:
  u32 mlen, seed[32], pk[32], sig[64], msg[mlen]
"""
import ctypes
import os
import random
import struct

HERE = os.path.dirname(os.path.abspath(__file__))

na = ctypes.CDLL("/opt/conda/lib/libsodium.so.23")
assert na.sodium_init() >= 0
na.sodium_version_string.restype = ctypes.c_char_p
assert na.sodium_version_string() == b"1.0.18", na.sodium_version_string()

# RFC 8032 section 7.1, TEST 1..3: (secret seed, public key, message, signature)
RFC8032 = [
    ("9d61b19deffd5a60ba844af492ec2cc44449c5697b326919703bac031cae7f60",
     "d75a980182b10ab7d54bfed3c964073a0ee172f3daa62325af021a68f707511a", "",
     "e5564300c360ac729086e2cc806e828a84877f1eb8e5d974d873e065224901555fb8821590a33bacc61e39701cf9b46bd25bf5f0595bbe24655141438e7a100b"),
    ("4ccd089b28ff96da9db6c346ec114e0f5b8a319f35aba624da8cf6ed4fb8a6fb",
     "3d4017c3e843895a92b70aa74d1b7ebc9c982ccf2ec4968cc0cd55f12af4660c", "72",
     "92a009a9f0d4cab8720e820b5f642540a2b27b5416503f8fb3762223ebdb69da085ac1e43e15996e458f3613d0f11d8c387b2eaeb4302aeeb00d291612bb0c00"),
    ("c5aa8df43f9f837bedb7442f31dcb7b166d38535076f094b85ce3a2e0b4458f7",
     "fc51cd8e6218a1a38da47ed00230f0580816ed13ba3303ac5deb911548908025", "af82",
     "6291d657deec24024827e69c3abe01a30ce548a284743a445e3680d7db5ac3ac18ff9b538d16f290ae67f760984dc6594a7c15e9716ed28dc027beceea1ec40a"),
]


def sodium_keypair_sign(seed: bytes, msg: bytes):
    pk, sk = ctypes.create_string_buffer(32), ctypes.create_string_buffer(64)
    assert na.crypto_sign_seed_keypair(pk, sk, seed) == 0
    sig = ctypes.create_string_buffer(64)
    assert na.crypto_sign_detached(sig, None, msg, ctypes.c_ulonglong(len(msg)), sk) == 0
    return pk.raw, sig.raw


def cases():
    for seed, pk, msg, sig in RFC8032:
        seed, pk, msg, sig = (bytes.fromhex(x) for x in (seed, pk, msg, sig))
        got_pk, got_sig = sodium_keypair_sign(seed, msg)
        assert (got_pk, got_sig) == (pk, sig), "libsodium disagrees with RFC 8032"
        yield seed, msg
    yield b"\0" * 32, b""
    yield b"\xff" * 32, b"\xff" * 300
    r = random.Random(0x516E)
    lens = list(range(0, 140)) + [k * 128 + d for k in range(1, 33) for d in (-17, -16, -15, 47, 48, 49)]
    lens += [r.randrange(0, 4097) for _ in range(300)] + [4096]
    for n in lens:
        if 0 <= n <= 4096:
            yield bytes(r.getrandbits(8) for _ in range(32)), bytes(r.getrandbits(8) for _ in range(n))


def main():
    recs = []
    for seed, msg in cases():
        pk, sig = sodium_keypair_sign(seed, msg)
        recs.append(struct.pack("<I", len(msg)) + seed + pk + sig + msg)
    with open(os.path.join(HERE, "sign_golden.bin"), "wb") as f:
        f.write(b"EDVSIGN1" + struct.pack("<I", len(recs)) + b"".join(recs))
    print("wrote %d signing vectors" % len(recs))


if __name__ == "__main__":
    main()
