#!/usr/bin/env python3
"""Generate tests/golden/ed25519_golden.bin: Ed25519 verify cases whose verdicts
come from libsodium 1.0.18 itself (the library the reference reaches through
libnacl.crypto_sign_open, stp_core/crypto/nacl_wrappers.py:86-108).

Run here (the container has /opt/conda/lib/libsodium.so.23); the GPU box only
reads the committed .bin.  Inputs are built with the oracle's point arithmetic
(oracle/liboref.so) and Python integers; every VERDICT is libsodium's
crypto_sign_ed25519_verify_detached (or crypto_sign_open for the positional-split
cases in ed25519_open_golden.json).

Categories follow SURVEY.md section 8c.  File format (little-endian):
  magic b"EDVGOLD1", u32 count, then per record:
  u8 verdict (1 accept), u8 category, u16 0, u32 mlen, sig[64], pk[32], msg[mlen]
"""
import ctypes
import hashlib
import json
import os
import random
import struct
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import oracle_lib as orc  # noqa: E402

P = 2**255 - 19
L = 2**252 + 27742317777372353535851937790883648493

CATEGORIES = [
    "valid", "valid_long", "flip_msg", "flip_r", "flip_s", "s_plus_kl", "s_high_garbage",
    "small_order_a", "noncanon_a", "offcurve_a", "small_order_r", "small_order_r_eq_holds",
    "mixed_order_a", "mixed_order_r", "wrong_key", "noncanon_r", "empty_msg", "s_ge_2_252_lt_l",
    "zero_sig", "random_bytes",
]
CAT = {c: i for i, c in enumerate(CATEGORIES)}

na = ctypes.CDLL("/opt/conda/lib/libsodium.so.23")
assert na.sodium_init() >= 0
na.sodium_version_string.restype = ctypes.c_char_p
assert na.sodium_version_string() == b"1.0.18", na.sodium_version_string()


def sodium_verify(sig: bytes, msg: bytes, pk: bytes) -> int:
    return 1 if na.crypto_sign_ed25519_verify_detached(sig, msg, ctypes.c_ulonglong(len(msg)), pk) == 0 else 0


def sodium_open(sm: bytes, pk: bytes) -> int:
    m = ctypes.create_string_buffer(max(len(sm), 1))
    mlen = ctypes.c_ulonglong(0)
    return 1 if na.crypto_sign_open(m, ctypes.byref(mlen), sm, ctypes.c_ulonglong(len(sm)), pk) == 0 else 0


def sodium_sign(msg: bytes, sk: bytes) -> bytes:
    sig = ctypes.create_string_buffer(64)
    na.crypto_sign_ed25519_detached(sig, None, msg, ctypes.c_ulonglong(len(msg)), sk)
    return sig.raw


def sodium_keypair(seed: bytes):
    pk, sk = ctypes.create_string_buffer(32), ctypes.create_string_buffer(64)
    na.crypto_sign_ed25519_seed_keypair(pk, sk, seed)
    return pk.raw, sk.raw


def le(x: int) -> bytes:
    return x.to_bytes(32, "little")


def H(*parts) -> int:
    return int.from_bytes(hashlib.sha512(b"".join(parts)).digest(), "little")


def secret_scalar(seed: bytes) -> int:
    h = bytearray(hashlib.sha512(seed).digest()[:32])
    h[0] &= 248
    h[31] &= 127
    h[31] |= 64
    return int.from_bytes(h, "little")


def torsion_points():
    """All 8 points of the torsion subgroup, canonical encodings; T8 of order 8."""
    rng = random.Random(7)
    while True:
        y = rng.randrange(P)
        enc = le(y)
        t = orc.scalarmult(le(L), enc)
        if t is None:
            continue
        pts = [le(1)]  # identity
        cur = t
        for _ in range(7):
            pts.append(cur)
            cur = orc.point_add(cur, t)
        if len(set(pts)) == 8:
            return pts  # pts[k] = [k]T8


def main():
    rng = random.Random(0x5EED2025)
    recs = []

    def add(cat, sig, pk, msg):
        recs.append((sodium_verify(sig, msg, pk), CAT[cat], sig, pk, msg))

    def rbytes(n):
        return bytes(rng.getrandbits(8) for _ in range(n))

    def keyed():
        pk, sk = sodium_keypair(rbytes(32))
        return pk, sk

    T = torsion_points()
    tor_encs = set(T)
    # non-canonical / sign-bit variants of the torsion encodings
    tor_variants = set()
    for e in T:
        tor_variants.add(e)
        b = bytearray(e)
        b[31] ^= 0x80
        tor_variants.add(bytes(b))
    for y in (0, 1):  # y + p (non-canonical) for y = 0, 1, both sign bits
        v = (y + P).to_bytes(32, "little")
        tor_variants.add(v)
        b = bytearray(v)
        b[31] |= 0x80
        tor_variants.add(bytes(b))
    tor_variants = sorted(tor_variants)

    # valid, short/medium messages
    for i in range(1200):
        pk, sk = keyed()
        m = rbytes(rng.choice([0, 1, 31, 32, 47, 48, 63, 64, 111, 112, 113, 127, 128, 150, 256, rng.randrange(300)]))
        add("valid", sodium_sign(m, sk), pk, m)
    # valid, C4 lengths 200 B .. 4 KB
    for i in range(80):
        pk, sk = keyed()
        m = rbytes(rng.randrange(200, 4097))
        add("valid_long", sodium_sign(m, sk), pk, m)
    # flipped bits
    for cat, lo, hi in (("flip_msg", None, None), ("flip_r", 0, 32), ("flip_s", 32, 64)):
        for i in range(250):
            pk, sk = keyed()
            m = rbytes(rng.randrange(1, 300))
            sig = bytearray(sodium_sign(m, sk))
            if cat == "flip_msg":
                mm = bytearray(m)
                mm[rng.randrange(len(mm))] ^= 1 << rng.randrange(8)
                add(cat, bytes(sig), pk, bytes(mm))
            else:
                sig[rng.randrange(lo, hi)] ^= 1 << rng.randrange(8)
                add(cat, bytes(sig), pk, m)
    # malleated S + k L (k = 1..15 keeps S < 2^256)
    for i in range(150):
        pk, sk = keyed()
        m = rbytes(rng.randrange(0, 300))
        sig = sodium_sign(m, sk)
        s = int.from_bytes(sig[32:], "little") + L * (1 + i % 15)
        if s < 2**256:
            add("s_plus_kl", sig[:32] + le(s), pk, m)
    # S = L, S = L + 1, random S >= 2^253 and top nibble garbage
    pk, sk = keyed()
    m = b"edv"
    sig = sodium_sign(m, sk)
    for s in (L, L + 1, L - 1, 2**253, 2**256 - 1, 2**255, 2**252, 2**252 - 1):
        add("s_high_garbage", sig[:32] + le(s), pk, m)
    for i in range(60):
        pk, sk = keyed()
        m = rbytes(64)
        sig = sodium_sign(m, sk)
        add("s_high_garbage", sig[:32] + le(rng.randrange(2**252, 2**256)), pk, m)
    # S in [2^252, L): passes V2, wrong equation (random R)
    for i in range(30):
        pk, sk = keyed()
        add("s_ge_2_252_lt_l", rbytes(32) + le(rng.randrange(2**252, L)), pk, rbytes(40))
    # small-order A (every torsion encoding and variant), random and "honest-looking" sigs
    for enc in tor_variants:
        for k in range(3):
            m = rbytes(rng.randrange(0, 100))
            add("small_order_a", rbytes(32) + le(rng.randrange(L)), enc, m)
        # R = [r]B, S = r: equation [S]B - [h]A = R holds for A of small order only if [h]A = 0
        r = rng.randrange(1, L)
        add("small_order_a", orc.scalarmult_base(le(r)) + le(r), enc, b"abc")
    # non-canonical A: y + p for y < 19 (on-curve or not), both sign bits, and y >= p
    for y in range(0, 19):
        for sb in (0, 0x80):
            b = bytearray((y + P).to_bytes(32, "little"))
            b[31] |= sb
            pk, sk = keyed()
            m = rbytes(20)
            sig = sodium_sign(m, sk)
            add("noncanon_a", sig, bytes(b), m)
    for i in range(20):
        b = bytearray(b"\xff" * 32)
        b[0] = rng.randrange(0xED, 0x100)
        b[31] = 0x7F | (0x80 if i & 1 else 0)
        add("noncanon_a", rbytes(64), bytes(b), rbytes(10))
    # off-curve A: small y values and random y until not decodable
    for y in range(2, 12):
        add("offcurve_a", rbytes(64), le(y), b"x")
    cnt = 0
    while cnt < 60:
        y = rbytes(32)
        if orc.point_add(y, le(1)) is None:
            add("offcurve_a", rbytes(64), y, rbytes(rng.randrange(0, 64)))
            cnt += 1
    # small-order R with random S
    for enc in tor_variants:
        pk, sk = keyed()
        add("small_order_r", enc + le(rng.randrange(L)), pk, rbytes(30))
        add("small_order_r", enc + le(0), pk, rbytes(30))
    # small-order R where the cofactorless equation HOLDS (libsodium still rejects):
    # A = A0 + T8, S = h*a0  =>  [S]B - [h]A = -[h]T8; search M so that -[h]T8 == R.
    found = 0
    tries = 0
    while found < 24 and tries < 5000:
        tries += 1
        seed = rbytes(32)
        a0 = secret_scalar(seed)
        A0 = orc.scalarmult_base(le(a0 % L))
        k = rng.randrange(1, 8)
        A = orc.point_add(A0, T[k])
        target = T[rng.randrange(8)]
        m = rbytes(16)
        h = H(target, A, m) % L
        # -[h]T_k = [(-h*k) mod 8] T8
        if T[(-h * k) % 8] == target:
            s = (h * a0) % L
            add("small_order_r_eq_holds", target + le(s), A, m)
            found += 1
    # mixed-order A = A0 + T, honest signer (knows a0): accept iff [h]T == 0
    for i in range(400):
        seed = rbytes(32)
        a0 = secret_scalar(seed)
        A0 = orc.scalarmult_base(le(a0 % L))
        k = rng.randrange(1, 8)
        A = orc.point_add(A0, T[k])
        m = rbytes(rng.randrange(0, 200))
        r = rng.randrange(1, L)
        R = orc.scalarmult_base(le(r))
        h = H(R, A, m) % L
        s = (r + h * a0) % L
        add("mixed_order_a", R + le(s), A, m)
    # mixed-order R = [r]B + T
    for i in range(60):
        pk, sk = keyed()
        a = secret_scalar(sk[:32])
        m = rbytes(rng.randrange(0, 100))
        r = rng.randrange(1, L)
        R = orc.point_add(orc.scalarmult_base(le(r)), T[rng.randrange(1, 8)])
        h = H(R, pk, m) % L
        add("mixed_order_r", R + le((r + h * a) % L), pk, m)
    # wrong key
    for i in range(150):
        pk, sk = keyed()
        pk2, _ = keyed()
        m = rbytes(rng.randrange(0, 200))
        add("wrong_key", sodium_sign(m, sk), pk2, m)
    # non-canonical R: y_R + p when y_R < 19 cannot come from a signer; random S
    for y in range(0, 19):
        b = (y + P).to_bytes(32, "little")
        pk, sk = keyed()
        add("noncanon_r", b + le(rng.randrange(L)), pk, rbytes(8))
    # empty messages
    for i in range(40):
        pk, sk = keyed()
        add("empty_msg", sodium_sign(b"", sk), pk, b"")
    add("zero_sig", b"\0" * 64, keyed()[0], b"hello")
    for i in range(100):
        add("random_bytes", rbytes(64), rbytes(32), rbytes(rng.randrange(0, 130)))

    out = bytearray(b"EDVGOLD1")
    out += struct.pack("<I", len(recs))
    for v, c, sig, pk, m in recs:
        out += struct.pack("<BBHI", v, c, 0, len(m)) + sig + pk + m
    path = os.path.join(HERE, "ed25519_golden.bin")
    with open(path, "wb") as f:
        f.write(out)
    acc = sum(r[0] for r in recs)
    per = {}
    for v, c, *_ in recs:
        per.setdefault(CATEGORIES[c], [0, 0])
        per[CATEGORIES[c]][v] += 1
    meta = {
        "generator": "tests/golden/make_golden.py",
        "verdicts_from": "libsodium 1.0.18 crypto_sign_ed25519_verify_detached (/opt/conda/lib/libsodium.so.23)",
        "count": len(recs),
        "accepted": acc,
        "sha256": hashlib.sha256(out).hexdigest(),
        "categories": CATEGORIES,
        "per_category_reject_accept": per,
    }
    with open(os.path.join(HERE, "ed25519_golden.json"), "w") as f:
        json.dump(meta, f, indent=1, sort_keys=True)

    # crypto_sign_open-level cases: the reference's positional split of sig + msg
    # (nacl_wrappers.py:239), including non-64-byte "signatures"
    opens = []
    pk, sk = keyed()
    for n in (0, 1, 5, 64, 200):
        m = rbytes(n)
        sig = sodium_sign(m, sk)
        opens.append((sig, m, pk))                       # normal
        opens.append((sig[:63], m, pk))                  # 63-byte signature
        opens.append((sig + b"\x00", m, pk))             # 65 bytes, different message
        if n:
            x = m[:1]
            sig2 = sodium_sign(x + m, sk)
            opens.append((sig2 + x, m, pk))              # 65-byte sig(x||M)||x : ACCEPTED
            opens.append((sig2[:60], sig2[60:] + x + m, pk))  # split inside the signature
    opens.append((b"", b"", pk))
    opens.append((b"\x01" * 10, b"", pk))
    opens.append((b"", b"\x02" * 63, pk))
    rows = [{"sig": s.hex(), "msg": m.hex(), "pk": p.hex(), "accept": sodium_open(s + m, p)} for s, m, p in opens]
    with open(os.path.join(HERE, "ed25519_open_golden.json"), "w") as f:
        json.dump({"verdicts_from": "libsodium 1.0.18 crypto_sign_open(sig + msg, pk)", "cases": rows}, f, indent=1)
    print(json.dumps({k: meta[k] for k in ("count", "accepted", "sha256")}))
    print(json.dumps(per))


if __name__ == "__main__":
    main()
