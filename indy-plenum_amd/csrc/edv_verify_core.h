// edv_verify_core.h -- the per-signature verification algorithm (one lane),
// __host__ __device__ so the exact kernel logic is unit-tested on the CPU
// (libedv_hostcheck.so, tests only) before it runs on gfx950.
//
// Follows libsodium 1.0.18 crypto_sign_ed25519_verify_detached, the function
// behind the reference's only verify call site
// (stp_core/crypto/nacl_wrappers.py:86-108 -> libnacl.crypto_sign_open);
// SURVEY.md section 8a rows V2-V9.
#pragma once
#include "edv_math.h"

namespace edv {

// [h](-A): 51 fixed signed windows of 5 bits (digits in [-16, 15], the top one in
// [0, 8]) against a per-lane table 0..16 x (-A); [S]B: 17 signed radix-2^15
// digits against a shared table 0..2^14 x B, one every third window (15 = 3 x 5
// bits, so the B additions land on window boundaries).  Against 4-bit windows
// (64 additions) and radix 2^16 (16 mixed additions): 13 fewer additions, one
// more mixed addition, two fewer doublings per verify, and a 2 MiB B table that
// fits one XCD's 4 MiB L2.
constexpr int kAWin = 5;                        // bits per [h](-A) window
constexpr int kAWindows = 51;                   // 51 x 5 = 255 bits >= 253
constexpr int kAEntries = 17;                   // per-lane table 0..16 x (-A), cached form (entry 0 = identity)
constexpr int kBBits = 15;                      // radix 2^15 digits of S
constexpr int kBDigits = 17;                    // 17 x 15 = 255 bits >= 253
constexpr int kBEvery = kBBits / kAWin;         // a B digit every third window
constexpr int kBEntries = (1 << (kBBits - 1)) + 1; // shared table 0..2^14 x B, affine precomp form (2 MiB)
static_assert(kBBits % kAWin == 0, "B digits must land on window boundaries");
constexpr int kCombEntries = 129;               // signer comb rows: 0..128 x 256^i B
constexpr int kBStride = 32;                    // words per B / comb entry (30 used; 128-byte aligned)

// ------------------------------------------------------------- message words
EDV_HD uint32_t alignbyte(uint32_t hi, uint32_t lo, uint32_t sh) {
  return uint32_t(((uint64_t(hi) << 32) | lo) >> (8 * sh));
}
// N big-endian SHA words of message bytes [q, q + 8N) that lie wholly inside the
// message: funnel-shifted aligned loads, none of msg_words_tail's clamp/pad work.
template <int N>
EDV_HD void msg_words_full(uint64_t* W, const uint8_t* m, uint64_t q) {
  const uintptr_t a = reinterpret_cast<uintptr_t>(m + q);
  const uint32_t sh = uint32_t(a & 3);
  const uint32_t* p = reinterpret_cast<const uint32_t*>(a - sh);
  uint32_t d[2 * N + 1];
#pragma unroll
  for (int t = 0; t < 2 * N + 1; t++) d[t] = p[t];
#pragma unroll
  for (int t = 0; t < N; t++)
    W[t] = be64_from_le_words(alignbyte(d[2 * t + 1], d[2 * t], sh), alignbyte(d[2 * t + 2], d[2 * t + 1], sh));
}

// N big-endian SHA words of message bytes [q0, q0 + 8N) of which some (or all)
// lie past the message end: 0x80 pad byte at mlen, zeros after it.  Branch-free:
// every dword address is clamped to the dword holding byte mlen (readable: the
// buffer extends 16 bytes past the message), so all 2N+1 loads issue together
// and the block waits for memory once.  (A per-word `if (bytes remain) load`
// compiled to a load + wait per word: ~16 serialized memory latencies in the
// last block of every message.)
template <int N>
EDV_HD void msg_words_tail(uint64_t* W, const uint8_t* m, uint64_t mlen, uint64_t q0) {
  const uintptr_t a = reinterpret_cast<uintptr_t>(m) + q0;
  const uint32_t sh = uint32_t(a & 3);
  const uintptr_t base = a - sh;
  const uintptr_t last = (reinterpret_cast<uintptr_t>(m) + mlen) & ~uintptr_t(3);
  uint32_t d[2 * N + 1];
#pragma unroll
  for (int t = 0; t < 2 * N + 1; t++) {
    const uintptr_t ad = base + 4 * uintptr_t(t);
    d[t] = *reinterpret_cast<const uint32_t*>(ad < last ? ad : last);
  }
  // byte masks without selects (a VCC-mask v_cndmask_b32 costs ~23 cycles on
  // gfx950): keep(k) = low k bytes set, as two shifts of at most 32 so k = 8 works
  const int32_t rem0 = int32_t(int64_t(mlen) - int64_t(q0));  // messages are far below 2 GiB
#pragma unroll
  for (int t = 0; t < N; t++) {
    const int32_t r = rem0 - 8 * t;
    const int32_t nv = r < 0 ? 0 : (r > 8 ? 8 : r);            // v_med3_i32
    const int32_t nv1 = r + 1 < 0 ? 0 : (r + 1 > 8 ? 8 : r + 1);
    const uint64_t keep = ((uint64_t(1) << (4 * nv)) << (4 * nv)) - 1;
    const uint64_t keep1 = ((uint64_t(1) << (4 * nv1)) << (4 * nv1)) - 1;
    uint64_t v = (uint64_t(alignbyte(d[2 * t + 2], d[2 * t + 1], sh)) << 32) | alignbyte(d[2 * t + 1], d[2 * t], sh);
    // the 0x80 pad byte sits at byte r when 0 <= r < 8: the one byte keep1 adds to keep
    v = (v & keep) | ((keep ^ keep1) & 0x8080808080808080ULL);
    W[t] = be64_from_le_words(uint32_t(v), uint32_t(v >> 32));
  }
}

// SHA-512(P || M) for a 32- or 64-byte prefix P given as little-endian words,
// -> 16 little-endian words of the 64-byte digest.
template <int PB>
EDV_HD void sha512_pm(uint32_t out[16], const uint32_t* P, const uint8_t* m, uint64_t mlen) {
  static_assert(PB == 32 || PB == 64, "prefix is 32 or 64 bytes");
  uint64_t H[8] = {0x6a09e667f3bcc908ULL, 0xbb67ae8584caa73bULL, 0x3c6ef372fe94f82bULL, 0xa54ff53a5f1d36f1ULL,
                   0x510e527fade682d1ULL, 0x9b05688c2b3e6c1fULL, 0x1f83d9abfb41bd6bULL, 0x5be0cd19137e2179ULL};
  constexpr int PW = PB / 8;  // prefix 64-bit SHA words
  const uint64_t total = PB + mlen;
  const uint64_t nb = (total + 17 + 127) / 128;
  uint64_t W[16];
#pragma unroll
  for (int t = 0; t < PW; t++) W[t] = be64_from_le_words(P[2 * t], P[2 * t + 1]);
  if (mlen >= uint64_t(128 - PB)) {
    msg_words_full<16 - PW>(W + PW, m, 0);
  } else {
    msg_words_tail<16 - PW>(W + PW, m, mlen, 0);
  }
  if (nb == 1) { W[14] = total >> 61; W[15] = total << 3; }
  sha512_compress(H, W);
#pragma unroll 1
  for (uint64_t b = 1; b < nb; b++) {
    const uint64_t q0 = 128 * b - PB;
    if (q0 + 128 <= mlen) {
      msg_words_full<16>(W, m, q0);
    } else {
      msg_words_tail<16>(W, m, mlen, q0);
    }
    if (b == nb - 1) { W[14] = total >> 61; W[15] = total << 3; }
    sha512_compress(H, W);
  }
#pragma unroll
  for (int i = 0; i < 8; i++) {
    out[2 * i] = bswap32(uint32_t(H[i] >> 32));
    out[2 * i + 1] = bswap32(uint32_t(H[i]));
  }
}

// SHA-512(R || A || M) (V6)
EDV_HD void hram(uint32_t out[16], const uint32_t R[8], const uint32_t A[8], const uint8_t* m, uint64_t mlen) {
  uint32_t P[16];
#pragma unroll
  for (int k = 0; k < 8; k++) { P[k] = R[k]; P[8 + k] = A[k]; }
  sha512_pm<64>(out, P, m, mlen);
}

// ------------------------------------------------------------ scalar recoding
// NDIG signed radix-2^BITS digits of a 256-bit scalar s (8 little-endian words),
// digit k in [-2^(BITS-1), 2^(BITS-1)) packed as BITS-bit two's complement at
// bits [BITS k, BITS k + BITS) of out; the top digit takes the final carry and
// stays non-negative (callers keep s < 2^253, so it stays in range).
template <int BITS, int NDIG>
EDV_HD void recode_signed(uint32_t out[8], const uint32_t s[8]) {
  static_assert(BITS * NDIG <= 256 && BITS <= 31, "digits must fit 256 bits");
  constexpr uint32_t kMask = (1u << BITS) - 1;
#pragma unroll
  for (int w = 0; w < 8; w++) out[w] = 0;
  int carry = 0;
#pragma unroll
  for (int k = 0; k < NDIG; k++) {
    const int pos = BITS * k, wi = pos >> 5, sh = pos & 31;
    const uint64_t win = uint64_t(s[wi]) | (wi + 1 < 8 ? uint64_t(s[wi + 1]) << 32 : 0);
    int e = int(uint32_t(win >> sh) & kMask) + carry;
    carry = (k == NDIG - 1) ? 0 : ((e + (1 << (BITS - 1))) >> BITS);
    e -= carry * (1 << BITS);
    const uint64_t pe = uint64_t(uint32_t(e) & kMask) << sh;
    out[wi] |= uint32_t(pe);
    if (wi + 1 < 8) out[wi + 1] |= uint32_t(pe >> 32);
  }
}
// h < L: the 51 radix-32 digits of the [h](-A) windows
EDV_HD void recode5(uint32_t out[8], const uint32_t h[8]) { recode_signed<kAWin, kAWindows>(out, h); }
// h < L: 64 signed radix-16 digits in [-8, 7] (kept for the recoding tests)
EDV_HD void recode4(uint32_t out[8], const uint32_t h[8]) { recode_signed<4, 64>(out, h); }
// S (signer scalars): 32 signed radix-256 digits in [-128, 127] (k < 2^253 keeps
// the top digit <= 32).
EDV_HD void recode8(uint32_t out[8], const uint32_t s[8]) {
  int carry = 0;
#pragma unroll
  for (int w = 0; w < 8; w++) {
    uint32_t packed = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) {
      int e = int((s[w] >> (8 * k)) & 255) + carry;
      carry = (w == 7 && k == 3) ? 0 : ((e + 128) >> 8);
      e -= carry * 256;
      packed |= uint32_t(e & 255) << (8 * k);
    }
    out[w] = packed;
  }
}
// S (verify, V8): 17 signed radix-2^15 digits in [-2^14, 2^14).  V2 leaves
// S < 2^253, so the top digit is <= 2^13 and stays inside the 0..2^14 table.
EDV_HD void recode15(uint32_t out[8], const uint32_t s[8]) { recode_signed<kBBits, kBDigits>(out, s); }
EDV_HD void recode16(uint32_t out[8], const uint32_t s[8]) { recode_signed<16, 16>(out, s); }
// shift a 256-bit little-endian word vector left by N bits (0 < N < 32)
template <int N>
EDV_HD void shl256(uint32_t v[8]) {
#pragma unroll
  for (int i = 7; i > 0; i--) v[i] = (v[i] << N) | (v[i - 1] >> (32 - N));
  v[0] <<= N;
}

EDV_HD ge_precomp precomp_from_words(const int32_t* w) {
  ge_precomp q;
#pragma unroll
  for (int l = 0; l < 10; l++) { q.ypx.v[l] = w[l]; q.ymx.v[l] = w[10 + l]; q.xy2d.v[l] = w[20 + l]; }
  return q;
}

// j * B for j in [0, 2^15], affine precomp form, written as kBStride words.
EDV_HD void btab_entry(int32_t* o, int j) {
  const uint32_t Bw[8] = {0x66666658u, 0x66666666u, 0x66666666u, 0x66666666u,
                          0x66666666u, 0x66666666u, 0x66666666u, 0x66666666u};
  ge_p3 nB;
  ge_frombytes_negate(nB, Bw);
  const ge_p3 B{fe_neg(nB.X), nB.Y, nB.Z, fe_neg(nB.T)};
  const ge_cached Bc = ge_p3_to_cached(B);
  ge_p3 acc = ge_p3_identity();
  for (int bit = kBBits - 1; bit >= 0; bit--) {
    acc = ge_p1p1_to_p3(ge_p2_dbl(ge_p3_to_p2(acc)));
    if ((j >> bit) & 1) acc = ge_p1p1_to_p3(ge_add(acc, Bc));
  }
  const fe zi = fe_invert(acc.Z);
  const fe x = fe_mul(acc.X, zi), y = fe_mul(acc.Y, zi);
  const fe ypx = fe_carry32(fe_add(y, x)), ymx = fe_carry32(fe_sub(y, x));
  const fe xy2d = fe_mul(fe_mul(x, y), fe_d2());
  for (int l = 0; l < 10; l++) { o[l] = ypx.v[l]; o[10 + l] = ymx.v[l]; o[20 + l] = xy2d.v[l]; }
  o[30] = 0;
  o[31] = 0;
}

// Phase 1 of one signature (kernel edv_prep_kernel): strictness checks V2-V4,
// decompression V5, h = SHA-512(R || A || M) mod L (V6, V7), digit recoding and
// the 0..16 x (-A) table (entry 0 the identity, so a zero digit needs no select).  Returns false if the signature is already rejected
// (then hd/sd/table are unspecified).  ATab provides store(e, cached).
template <class ATab>
EDV_HD bool prep_one(const uint32_t R[8], const uint32_t S[8], const uint32_t A[8], const uint8_t* m, uint64_t mlen,
                     ATab& at, uint32_t hd[8], uint32_t sd[8]) {
  bool ok = !((S[7] & 0xF0000000u) && !sc_is_canonical(S));
  ok = ok && !has_small_order(R);
  ok = ok && ge_is_canonical(A) && !has_small_order(A);
  if (!ok) return false;
  ge_p3 nA;
  if (!ge_frombytes_negate(nA, A)) return false;
  uint32_t dig[16], h[8];
  hram(dig, R, A, m, mlen);
  sc_reduce(h, dig);
  recode5(hd, h);
  recode15(sd, S);
  const ge_cached c1 = ge_p3_to_cached(nA);
  // -A comes out of the decompression affine (Z = 1, T = XY), so its cached form
  // doubles as precomp form and each further entry is a mixed addition (3 field
  // products instead of 4: 14 products saved per signature)
  const ge_precomp p1{c1.YpX, c1.YmX, c1.T2d};
  at.store(0, ge_cached_identity());
  at.store(1, c1);
  ge_p3 cur = ge_p1p1_to_p3(ge_p2_dbl(ge_p3_to_p2(nA)));
  at.store(2, ge_p3_to_cached(cur));
#pragma unroll 1
  for (int e = 3; e < kAEntries; e++) {
    cur = ge_p1p1_to_p3(ge_madd(cur, p1));
    at.store(e, ge_p3_to_cached(cur));
  }
  return true;
}

// Phase 2 (kernel edv_main_kernel): V8 R' = [h](-A) + [S]B by a joint
// fixed-window walk, top digit first -- every lane adds at the same positions,
// so a wave never diverges -- then V9 encode(R') == R.  51 windows of 5 bits for
// [h](-A) (one table addition each); [S]B adds one radix-2^15 digit every third
// window.  ATab provides load(e); BTab provides entry(j) -> precomp.
template <class ATab, class BTab>
EDV_HD bool main_one(const uint32_t R[8], uint32_t hd[8], uint32_t sd[8], const ATab& at, const BTab& bt) {
  ge_p2 acc = ge_p2_identity();
  int bphase = (kAWindows - 1) % kBEvery;  // windows until the next B digit
#pragma unroll 1
  for (int w = kAWindows - 1; w >= 0; --w) {
    // table reads first, so their latency hides under this window's doublings
    const int dA = int32_t(hd[7] << 1) >> (32 - kAWin);  // digit at bits [250, 255)
    shl256<kAWin>(hd);
    ge_cached c = at.load(dA < 0 ? -dA : dA);
    const bool addB = bphase == 0;
    bphase = addB ? kBEvery - 1 : bphase - 1;
    int dB = 0;
    ge_precomp q;
    if (addB) {
      dB = int32_t(sd[7] << 1) >> (32 - kBBits);  // digit at bits [240, 255)
      shl256<kBBits>(sd);
      // shift before the loads are issued: scheduled after them, the shift's
      // temporaries landed in the loads' destination VGPRs and forced a vmcnt
      // wait right behind the loads
      sched_fence();
      q = bt.entry(dB < 0 ? -dB : dB);
    }
    ge_p3 p3;
    if (w == kAWindows - 1) {
      p3 = ge_p3_identity();
    } else {
#pragma unroll
      for (int d = 0; d < kAWin - 1; d++) acc = ge_p1p1_to_p2(ge_p2_dbl(acc));
      p3 = ge_p1p1_to_p3(ge_p2_dbl(acc));
    }
    c = ge_cached_cneg(c, dA < 0);
    ge_p1p1 t = ge_add(p3, c);
    if (addB) {
      p3 = ge_p1p1_to_p3(t);
      t = ge_madd(p3, ge_precomp_cneg(q, dB < 0));
    }
    acc = ge_p1p1_to_p2(t);
  }
  uint32_t enc[8];
  ge_p2_tobytes(enc, acc);
  bool match = true;
#pragma unroll
  for (int k = 0; k < 8; k++) match = match && (enc[k] == R[k]);
  return match;
}

// The whole verdict for one signature: true iff libsodium's verify_detached
// would return 0.
template <class ATab, class BTab>
EDV_HD bool verify_one(const uint32_t R[8], const uint32_t S[8], const uint32_t A[8], const uint8_t* m, uint64_t mlen,
                       ATab& at, const BTab& bt) {
  uint32_t hd[8], sd[8];
  if (!prep_one(R, S, A, m, mlen, at, hd, sd)) return false;
  return main_one(R, hd, sd, at, bt);
}

// ------------------------------------------------ batch signing (row f-4)
// Fixed-base comb for [k]B without doublings: entry (i, j) = j * 256^i * B,
// i < 32, j <= 128, affine precomp form; [k]B = sum_i T[i][d_i] over the signed
// radix-256 digits of k < L.
constexpr int kCombRows = 32;
EDV_HD void comb_entry(int32_t* o, int i, int j) {
  const uint32_t Bw[8] = {0x66666658u, 0x66666666u, 0x66666666u, 0x66666666u,
                          0x66666666u, 0x66666666u, 0x66666666u, 0x66666666u};
  ge_p3 nB;
  ge_frombytes_negate(nB, Bw);
  ge_p3 base{fe_neg(nB.X), nB.Y, nB.Z, fe_neg(nB.T)};
  for (int k = 0; k < 8 * i; k++) base = ge_p1p1_to_p3(ge_p2_dbl(ge_p3_to_p2(base)));
  const ge_cached bc = ge_p3_to_cached(base);
  ge_p3 acc = ge_p3_identity();
  for (int bit = 7; bit >= 0; bit--) {
    acc = ge_p1p1_to_p3(ge_p2_dbl(ge_p3_to_p2(acc)));
    if ((j >> bit) & 1) acc = ge_p1p1_to_p3(ge_add(acc, bc));
  }
  const fe zi = fe_invert(acc.Z);
  const fe x = fe_mul(acc.X, zi), y = fe_mul(acc.Y, zi);
  const fe ypx = fe_carry32(fe_add(y, x)), ymx = fe_carry32(fe_sub(y, x));
  const fe xy2d = fe_mul(fe_mul(x, y), fe_d2());
  for (int l = 0; l < 10; l++) { o[l] = ypx.v[l]; o[10 + l] = ymx.v[l]; o[20 + l] = xy2d.v[l]; }
  o[30] = 0;
  o[31] = 0;
}
// [k]B for k < L (8 words); CombTab provides entry(i, j) -> precomp
template <class CombTab>
EDV_HD ge_p3 scalarmult_base(const uint32_t k[8], const CombTab& ct) {
  uint32_t d[8];
  recode8(d, k);
  ge_p3 acc = ge_p3_identity();
#pragma unroll 1
  for (int i = 0; i < kCombRows; i++) {
    const int di = int(int8_t(uint8_t(d[i >> 2] >> (8 * (i & 3)))));
    const int ui = di < 0 ? -di : di;
    acc = ge_p1p1_to_p3(ge_madd(acc, ge_precomp_cneg(ct.entry(i, ui), di < 0)));
  }
  return acc;
}
EDV_HD void ge_p3_tobytes(uint32_t w[8], const ge_p3& p) { ge_p2_tobytes(w, ge_p3_to_p2(p)); }

// (a * b + c) mod L for 8-word little-endian scalars
EDV_HD void sc_muladd(uint32_t out[8], const uint32_t a[8], const uint32_t b[8], const uint32_t c[8]) {
  uint32_t t[16];
  uint64_t carry = 0;
#pragma unroll
  for (int k = 0; k < 16; k++) {
    // column k of a*b (+ c_k): accumulate 32x32 products into a 96-bit column sum
    uint64_t lo = carry + (k < 8 ? c[k] : 0), hi = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
      const int j = k - i;
      if (j < 0 || j > 7) continue;
      const uint64_t p = uint64_t(a[i]) * b[j];
      const uint64_t s = lo + p;
      hi += (s < lo);
      lo = s;
    }
    t[k] = uint32_t(lo);
    carry = (lo >> 32) | (hi << 32);
  }
  sc_reduce(out, t);
}

// RFC 8032 / libsodium crypto_sign_seed_keypair + crypto_sign_detached for one
// (seed, M): deterministic, so results are comparable byte for byte.
template <class CombTab>
EDV_HD void sign_one(uint32_t pk[8], uint32_t sig[16], const uint32_t seed[8], const uint8_t* m, uint64_t mlen,
                     const CombTab& ct) {
  uint32_t az[16];
  sha512_pm<32>(az, seed, m, 0);
  az[0] &= ~7u;
  az[7] = (az[7] & 0x7fffffffu) | 0x40000000u;
  uint32_t a64[16], a[8];
#pragma unroll
  for (int k = 0; k < 16; k++) a64[k] = k < 8 ? az[k] : 0;
  sc_reduce(a, a64);  // [a]B = [a mod L]B; keeps the radix-256 digits in range
  ge_p3_tobytes(pk, scalarmult_base(a, ct));
  uint32_t nonce[16], r[8];
  sha512_pm<32>(nonce, az + 8, m, mlen);
  sc_reduce(r, nonce);
  ge_p3_tobytes(sig, scalarmult_base(r, ct));
  uint32_t hr[16], h[8];
  hram(hr, sig, pk, m, mlen);
  sc_reduce(h, hr);
  uint32_t aclamped[8];
#pragma unroll
  for (int k = 0; k < 8; k++) aclamped[k] = az[k];
  sc_muladd(sig + 8, h, aclamped, r);
}

}  // namespace edv
