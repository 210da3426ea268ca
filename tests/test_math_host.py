"""The kernel's field/scalar/SHA-512 code and its whole per-signature algorithm,
compiled for the CPU (libedv_hostcheck.so), against Python integers, hashlib
and libsodium's golden verdicts.  Catches arithmetic bugs before the GPU."""
import ctypes
import hashlib
import random

import pytest

import golden_io
import hostcheck_lib

P = 2**255 - 19
L = 2**252 + 27742317777372353535851937790883648493
POS = [0, 26, 51, 77, 102, 128, 153, 179, 204, 230]
# input bound the multiply is specified for: |f_i| <= 1.65 * 2^26 (even i), 1.65 * 2^25 (odd i)
BOUND = [int(1.65 * 2**26) if i % 2 == 0 else int(1.65 * 2**25) for i in range(10)]


def val(l):
    return sum(int(x) << POS[i] for i, x in enumerate(l))


def arr(l):
    return (ctypes.c_int32 * 10)(*l)


def limbs(x):
    return [(x >> POS[i]) & ((1 << (26 if i % 2 == 0 else 25)) - 1) for i in range(10)]


def rand_limbs(r, extreme=False):
    if extreme:
        return [r.choice([-BOUND[i], BOUND[i], BOUND[i] - 1, -BOUND[i] + 1]) for i in range(10)]
    return [r.randrange(-BOUND[i], BOUND[i] + 1) for i in range(10)]


def out_ok(h):
    # outputs must be reduced enough to feed another multiply after one add/sub
    return all(abs(h[i]) <= (2**25 + 2**20 if i % 2 == 0 else 2**24 + 2**20) for i in range(10))


def test_fe_mul_sq_against_python():
    hc = hostcheck_lib.load()
    r = random.Random(5)
    h = (ctypes.c_int32 * 10)()
    for it in range(3000):
        f = rand_limbs(r, extreme=(it % 3 == 0))
        g = rand_limbs(r, extreme=(it % 5 == 0))
        hc.hc_fe_mul(arr(f), arr(g), h)
        assert val(h) % P == val(f) * val(g) % P and out_ok(h)
        hc.hc_fe_sq(arr(f), h)
        assert val(h) % P == val(f) ** 2 % P and out_ok(h)
        hc.hc_fe_sq2(arr(f), h)
        assert val(h) % P == 2 * val(f) ** 2 % P and out_ok(h)


def test_fe_sq_floor_chain():
    """fe_sq_floor (the exponentiations' squaring runs): a signed reduced input
    (what fe_mul returns) and then its own unsigned outputs, 40 squarings deep,
    at the limb extremes of both forms: exact mod p, limbs in [0, 2^26) /
    [0, 2^25) (h1 within 2^17), so the next squaring's premultiplied operands
    stay inside int32."""
    hc = hostcheck_lib.load()
    r = random.Random(9)
    h = (ctypes.c_int32 * 10)()
    top = [(1 << 26) - 1 if i % 2 == 0 else (1 << 25) - 1 for i in range(10)]
    starts = [[r.randrange(-2**25, 2**25) if i % 2 == 0 else r.randrange(-2**24, 2**24) for i in range(10)]
              for _ in range(300)]
    starts += [[(2**25 if i % 2 == 0 else 2**24) * s for i in range(10)] for s in (1, -1)]
    starts += [top, [t if i != 1 else (1 << 25) + (1 << 17) for i, t in enumerate(top)]]
    for f in starts:
        x = val(f) % P
        cur = f
        for _ in range(40):
            hc.hc_fe_sq_floor(arr(cur), h)
            x = x * x % P
            cur = list(h)
            assert val(cur) % P == x
            assert all(0 <= cur[i] < (1 << (26 if i % 2 == 0 else 25)) for i in range(10) if i != 1)
            assert -(1 << 17) <= cur[1] < (1 << 25) + (1 << 17)


def test_digits_windows():
    """The window count from the packed 4-bit digits (count-leading-zeros form)
    is 1 + the index of the top nonzero digit, 0 for no digits."""
    hc = hostcheck_lib.load()
    r = random.Random(11)
    cases = [[0] * 8, [1] + [0] * 7, [0] * 7 + [0xF0000000], [0] * 7 + [1], [0x80000000] + [0] * 7]
    for _ in range(3000):
        w = [0] * 8
        top = r.randrange(64)
        for k in range(top + 1):
            w[k // 8] |= r.randrange(16) << (4 * (k % 8))
        w[top // 8] |= r.randrange(1, 16) << (4 * (top % 8))
        cases.append(w)
    for w in cases:
        digits = [(w[k // 8] >> (4 * (k % 8))) & 15 for k in range(64)]
        want = max([k + 1 for k in range(64) if digits[k]], default=0)
        assert hc.hc_digits_windows((ctypes.c_uint32 * 8)(*w)) == want


def test_fe_tobytes_canonical_and_frombytes():
    hc = hostcheck_lib.load()
    r = random.Random(6)
    out = ctypes.create_string_buffer(32)
    h = (ctypes.c_int32 * 10)()
    specials = [0, 1, P - 1, P, P + 1, 2 * P - 1, 2**255 - 1, 2**255 - 20, 19, 2**255 - 19 - 1]
    for x in specials + [r.randrange(2**255) for _ in range(2000)]:
        hc.hc_fe_frombytes(x.to_bytes(32, "little"), h)
        y = x & (2**255 - 1)  # bit 255 (the sign bit) is ignored by the decoder
        assert val(h) % P == y % P and out_ok(h)
        hc.hc_fe_tobytes(h, out)
        assert int.from_bytes(out.raw, "little") == y % P
    for _ in range(2000):  # tobytes of non-canonical reduced limb vectors
        f = [r.randrange(-2**25, 2**25) if i % 2 == 0 else r.randrange(-2**24, 2**24) for i in range(10)]
        hc.hc_fe_tobytes(arr(f), out)
        assert int.from_bytes(out.raw, "little") == val(f) % P


def test_fe_invert_and_pow22523():
    hc = hostcheck_lib.load()
    r = random.Random(7)
    h = (ctypes.c_int32 * 10)()
    for x in [1, 2, P - 1] + [r.randrange(1, P) for _ in range(30)]:
        hc.hc_fe_invert(arr(limbs(x)), h)
        assert val(h) % P == pow(x, P - 2, P)
        hc.hc_fe_pow22523(arr(limbs(x)), h)
        assert val(h) % P == pow(x, (P - 5) // 8, P)


def test_fe_invert_safegcd():
    """The divsteps inversion the encode uses (V9) against pow(x, p - 2, p), on
    canonical, non-canonical and bound-extreme limb vectors."""
    hc = hostcheck_lib.load()
    r = random.Random(17)
    h = (ctypes.c_int32 * 10)()
    xs = [1, 2, 3, 19, P - 1, P - 2, (P - 1) // 2, 2**254, 2**255 - 20] + [r.randrange(1, P) for _ in range(3000)]
    for x in xs:
        hc.hc_fe_invert_safegcd(arr(limbs(x)), h)
        assert val(h) % P == pow(x, P - 2, P) and out_ok(h), x
    for it in range(3000):  # arbitrary (non-canonical, signed) limb vectors within the mul input bounds
        f = rand_limbs(r, extreme=(it % 2 == 0))
        if val(f) % P == 0:
            continue
        hc.hc_fe_invert_safegcd(arr(f), h)
        assert val(h) % P == pow(val(f) % P, P - 2, P) and out_ok(h)
    hc.hc_fe_invert_safegcd(arr([0] * 10), h)
    assert val(h) % P == 0


def test_sc_reduce_canonical():
    hc = hostcheck_lib.load()
    r = random.Random(8)
    out = ctypes.create_string_buffer(32)
    vals = [0, 1, L - 1, L, L + 1, 2 * L - 1, 2 * L, 2**512 - 1, 2**511, 2**253 - 1, 8 * L + 7]
    vals += [k * L + d for k in (1, 2**100, 2**258 - 1) for d in (-1, 0, 1)]
    vals += [r.randrange(2**512) for _ in range(3000)]
    for v in vals:
        if not 0 <= v < 2**512:
            continue
        hc.hc_sc_reduce(v.to_bytes(64, "little"), out)
        assert int.from_bytes(out.raw, "little") == v % L, hex(v)


def test_hram_sha512_all_lengths():
    hc = hostcheck_lib.load()
    r = random.Random(9)
    d = ctypes.create_string_buffer(64)
    for n in list(range(0, 300)) + [4096, 4095, 1000, 111 - 64 + 64]:
        R = bytes(r.getrandbits(8) for _ in range(32))
        A = bytes(r.getrandbits(8) for _ in range(32))
        m = bytes(r.getrandbits(8) for _ in range(n))
        hc.hc_hram(R, A, m, len(m), d)
        assert d.raw == hashlib.sha512(R + A + m).digest(), n


def test_sha256_all_lengths_and_alignments():
    """The kernel's SHA-256 (row f-3) vs hashlib: every length across the 1-, 2-
    and 3-block padding boundaries, long messages, and all 4 misalignments."""
    hc = hostcheck_lib.load()
    r = random.Random(10)
    d = ctypes.create_string_buffer(32)
    for n in list(range(0, 200)) + [247, 255, 256, 1000, 4095, 4096, 4097]:
        m = bytes(r.getrandbits(8) for _ in range(n))
        for mis in range(4):
            hc.hc_sha256(m, len(m), mis, d)
            assert d.raw == hashlib.sha256(m).digest(), (n, mis)


def test_kernel_algorithm_on_cpu_matches_libsodium_golden(golden, golden_meta):
    hc = hostcheck_lib.load()
    sigs, pks, msgs, off = golden_io.pack_batch(golden)
    acc = ctypes.create_string_buffer(len(golden))
    hc.hc_verify_batch(sigs, pks, msgs or b"\0", off.ctypes.data, len(golden), acc)
    cats = golden_meta["categories"]
    bad = [(i, cats[g[1]]) for i, g in enumerate(golden) if acc.raw[i] != g[0]]
    assert bad == []


def _digits(packed, bits):
    """Digit k at bits [bits k, bits k + bits) of the packed 256-bit value."""
    v = sum(w << (32 * i) for i, w in enumerate(packed))
    out = []
    for k in range(256 // bits):
        raw = (v >> (bits * k)) & ((1 << bits) - 1)
        out.append(raw - (1 << bits) if raw >> (bits - 1) else raw)
    return out


def test_scalar_recoding_radix_4_5_8():
    """Signed digits: radix 16 (the main loop's windows, digit in [-8, 7], so |d|
    indexes the 0..8 per-lane table) and radix 32, signer scalars (radix 256);
    sum d_k * 2^(bits*k) must give back the scalar."""
    hc = hostcheck_lib.load()
    r = random.Random(12)
    out = (ctypes.c_uint32 * 8)()
    # V2 admits every S < 2^252 and canonical S < L; h and signer scalars are < L
    edge = [0, 1, L - 1, 2**252 - 1, 2**252, 2**253 - 1 - (2**253 - L)]
    edge += [int("8000" * 16, 16) % L, int("7fff" * 16, 16) % L, int("ffff" * 15, 16), int("80" * 31, 16)]
    edge += [int("88" * 31, 16), int("77" * 31, 16)]
    vals = [v for v in edge if 0 <= v < L] + [r.randrange(L) for _ in range(2000)]
    for bits, lo, hi in ((4, -8, 7), (5, -16, 15), (8, -128, 127)):
        for v in vals:
            assert hc.hc_recode(v.to_bytes(32, "little"), bits, out) == 0
            d = _digits(list(out), bits)
            assert sum(x << (bits * k) for k, x in enumerate(d)) == v, (bits, hex(v))
            assert all(lo <= x <= hi for x in d[:-1]), (bits, hex(v))
            assert 0 <= d[-1] <= hi, (bits, hex(v))


def test_walk_layout_constants():
    """The default build walks 4-bit windows (9-entry per-lane tables); the R
    side computes [S]B from 12 signed radix-2^22 digits against 12 tables."""
    lay = hostcheck_lib.layout()
    assert lay == {"awin": 4, "aentries": 9, "bbits": 22, "btables": 12}
    # every S < 2^253 fits the digits, the top one (carry included) its table
    assert lay["bbits"] * lay["btables"] >= 253 and 253 - lay["bbits"] * (lay["btables"] - 1) <= lay["bbits"] - 1


def _btab_entries(hc, t, js, bits=22):
    import numpy as np
    js = np.asarray(js, np.int32)
    out = np.zeros(32 * len(js), np.int32)
    assert hc.hc_btab_entries_of_bits(bits, t, js.ctypes.data, len(js), out.ctypes.data) == 0
    return out.reshape(len(js), 32)


# the two [S]B table sets (edv_verify_core.h SbShape): large (the default
# layout above) and compact (16 digits of 16 bits, 64 MiB)
SB_SHAPES = {22: 12, 16: 16}


@pytest.mark.parametrize("bb", sorted(SB_SHAPES))
def test_btab_entries_are_multiples_of_2_16t_B(bb):
    """Table t of the R side's [S]B: entry j = j x 2^(bbits t) B (affine y+x, y-x,
    2dxy limbs) against the oracle's fixed-base multiplication, for the first,
    a middle and the last table, in both table sets."""
    import oracle_lib as orc
    hc = hostcheck_lib.load()
    if bb == 22:
        assert hc.hc_btab_entries() == 2**(hostcheck_lib.layout()["bbits"] - 1) + 1
    n = 2**(bb - 1) + 1
    d = (-121665 * pow(121666, P - 2, P)) % P
    inv2 = pow(2, P - 2, P)
    r = random.Random(13)
    nt = SB_SHAPES[bb]
    assert bb * nt >= 253 and 253 - bb * (nt - 1) <= bb - 1
    for t in (0, 1, nt // 2, nt - 1):
        js = [0, 1, 2, 3, 127, 128, 255, 256, 4097, 16384, n - 2, n - 1] + [r.randrange(n) for _ in range(12)]
        for j, e in zip(js, _btab_entries(hc, t, js, bb)):
            e = list(e)
            ypx, ymx, xy2d = val(e[0:10]) % P, val(e[10:20]) % P, val(e[20:30]) % P
            y, x = (ypx + ymx) * inv2 % P, (ypx - ymx) * inv2 % P
            assert xy2d == 2 * d * x * y % P, (t, j)
            enc = int.to_bytes(y | ((x & 1) << 255), 32, "little")
            assert enc == orc.scalarmult_base(((j << (bb * t)) % L).to_bytes(32, "little")), (t, j)


def _ed_add(p1, p2):
    d = (-121665 * pow(121666, P - 2, P)) % P
    (x1, y1), (x2, y2) = p1, p2
    t = d * x1 * x2 * y1 * y2 % P
    return ((x1 * y2 + y1 * x2) * pow(1 + t, P - 2, P) % P, (y1 * y2 + x1 * x2) * pow(1 - t, P - 2, P) % P)


def _ed_decode(b):
    d = (-121665 * pow(121666, P - 2, P)) % P
    v = int.from_bytes(b, "little")
    y, sign = v & ((1 << 255) - 1), v >> 255
    if y >= P:
        return None
    u, w = (y * y - 1) % P, (d * y * y + 1) % P
    x = pow(u * pow(w, P - 2, P), (P + 3) // 8, P)
    if (w * x * x - u) % P:
        x = x * pow(2, (P - 1) // 4, P) % P
    if (w * x * x - u) % P:
        return None
    if x == 0 and sign:
        return None
    if (x & 1) != sign:
        x = P - x
    return x, y


def _ed_encode(pt):
    x, y = pt
    return int.to_bytes(y | ((x & 1) << 255), 32, "little")


@pytest.mark.parametrize("bb", sorted(SB_SHAPES))
def test_r_side_point_is_SB_minus_R(bb):
    """The prep kernel's R side: Q = [S]B - R from the signed radix-2^bbits digits of S,
    against Python affine arithmetic on the oracle's [S]B, for S over the range
    V2 admits (edges and random, below L and below 2^252) and R of every
    order: a valid signature's R, torsion-shifted R, the identity-adjacent
    cases; rejected R (small order, non-canonical, not on the curve) gives -1."""
    import oracle_lib as orc
    hc = hostcheck_lib.load()
    r = random.Random(31)
    out = ctypes.create_string_buffer(32)
    rside = lambda R, S, o: hc.hc_rside_point_bits(bb, R, S, o)  # noqa: E731
    # digit edges: |d| = 2^(bb-1) (the last entry) with and without carries, all-ones runs
    Ss = [0, 1, 2, 2**bb - 1, 2**bb, 2**(bb - 1), 2**(bb - 1) - 1, 2**(bb - 1) + 1, L - 1, L - 2, 2**252 - 1]
    nt = SB_SHAPES[bb]
    Ss += [2**(bb * k) - 1 for k in range(2, nt) if 2**(bb * k) < L] + [2**(bb - 1) * (2**(bb * k) - 1) // (2**bb - 1) % L for k in (3, nt - 1)]
    Ss += [2**240, 2**252 - 2**240, sum(2**(bb * k + bb - 1) for k in range(nt - 1)) % L]
    Ss += [int("8000" * 16, 16) % L, int("7fff" * 16, 16) % L] + [r.randrange(L) for _ in range(60)]
    pts = []
    for _ in range(8):
        k = r.randrange(1, L)
        pts.append(orc.scalarmult_base(k.to_bytes(32, "little")))
    # a mixed-order R: a valid point plus the order-2 point (0, -1)
    q = _ed_decode(pts[0])
    pts.append(_ed_encode(_ed_add(q, (0, P - 1))))
    for S in Ss:
        sb = _ed_decode(orc.scalarmult_base(S.to_bytes(32, "little")))
        for Rb in pts + ([orc.scalarmult_base(S.to_bytes(32, "little"))] if S else []):  # R = [S]B: Q = identity
            Rp = _ed_decode(Rb)
            want = _ed_encode(_ed_add(sb, ((P - Rp[0]) % P, Rp[1])))
            assert rside(Rb, S.to_bytes(32, "little"), out) == 0, (hex(S), Rb.hex())
            assert out.raw == want, (hex(S), Rb.hex())
    # S with bits above 2^253 (rejected by the hash side): no fault, some point
    for S in (2**256 - 1, 2**255 + 12345, 2**253):
        assert rside(pts[1], S.to_bytes(32, "little"), out) == 0
    # rejected R: identity (small order), y >= p (non-canonical), not on the curve
    bad = [_ed_encode((0, 1)), (P + 1).to_bytes(32, "little")]
    y = 2
    while _ed_decode(y.to_bytes(32, "little")) is not None:
        y += 1
    bad.append(y.to_bytes(32, "little"))
    for Rb in bad:
        assert rside(Rb, (5).to_bytes(32, "little"), out) == -1, Rb.hex()


N8L = 8 * L


def _half(hc, h):
    a, u = ctypes.create_string_buffer(32), ctypes.create_string_buffer(32)
    neg = hc.hc_half_scalars(h.to_bytes(32, "little"), a, u)
    a, u = int.from_bytes(a.raw, "little"), int.from_bytes(u.raw, "little")
    return a, (-u if neg else u)


def test_half_scalars_lattice_reduction():
    """The prep kernel's lattice reduction: a = b h (mod 8L), b odd (so [b]Q = 0
    iff Q = 0 for Q in a group of order 8L), a >= 0, a < 2^253, |b| < 2^192 for
    every h < L, and both about 2^128 for hash-like h."""
    hc = hostcheck_lib.load()
    r = random.Random(21)
    edge = [0, 1, 2, 3, L - 1, L - 2, 2**128 - 1, 2**128, 2**128 + 1, 2**252, 2**252 - 1, 8, 2**64, 2**64 + 1]
    # large partial quotients (the binary long-division path): h near N8L / 2^k and N8L * j / k
    edge += [N8L >> k for k in (4, 40, 64, 100, 124, 130, 200) if (N8L >> k) < L]
    edge += [(N8L >> k) + 1 for k in (40, 100, 126)]
    edge += [(N8L * j // k) % L for j, k in ((1, 3), (2, 7), (5, 11), (1, 2**33 + 1), (7, 2**61 - 1))]
    edge += [(2**140 * x) % L for x in (1, 3, 5)]
    # a huge quotient after a few ordinary ones (negative cofactor at that point)
    for k in (33, 40, 70, 110):
        for q1 in (1, 2, 3):
            x = N8L * 2**k // (q1 * 2**k + 1)          # N8L / h = q1 + 1/2^k
            edge += [x % L, (x + 12345) % L]
            x = N8L * (2**k + 1) // (2 * 2**k + 3)     # quotients 1, 1, ~2^(k-1), ...
            edge += [x % L]
    vals = edge + [r.randrange(L) for _ in range(20000)]
    lens = []
    for h in vals:
        a, b = _half(hc, h)
        assert 0 <= a < 2**253 and abs(b) < 2**192, hex(h)
        assert b % 2 == 1, hex(h)
        assert (a - b * h) % N8L == 0, hex(h)
        lens.append(max(a.bit_length(), abs(b).bit_length()))
    rand = sorted(lens[len(edge):])
    assert rand[len(rand) // 2] <= 128 and rand[-1] <= 142, (rand[len(rand) // 2], rand[-1])


def test_kernel_algorithm_on_cpu_matches_libsodium_corpus_slice():
    """The kernel algorithm (half-size scalars) on the CPU against libsodium's
    committed verdict bits for the first 12,000 requests of the C2 and C4
    corpora (5 % damaged: flipped R/S/A/message bits, S >= L, small-order and
    non-canonical points)."""
    import json
    import os
    import numpy as np
    import oracle_lib as orc
    hc = hostcheck_lib.load()
    gdir = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
    meta = json.load(open(os.path.join(gdir, "corpus_bitmask.json")))
    for name, n in (("c2_256B", 12000), ("c4_var", 4000)):
        cfg = meta["corpora"][name]
        sigs, pks, msgs, off = orc.corpus(cfg["seed"], 0, n, cfg["mode"], cfg["invalid_permille"])
        bits = np.fromfile(os.path.join(gdir, "corpus_%s.bits" % name), dtype=np.uint8)
        want = np.unpackbits(bits[:n // 8], bitorder="little")
        acc = ctypes.create_string_buffer(n)
        hc.hc_verify_batch(sigs.tobytes(), pks.tobytes(), msgs.tobytes(), off.ctypes.data, n, acc)
        got = np.frombuffer(acc.raw, dtype=np.uint8)
        assert np.array_equal(got, want), (name, np.nonzero(got != want)[0][:10])
