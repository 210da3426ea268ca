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

// Half-size scalars (V8).  libsodium's R' = [S]B + [h](-A)
// with a 253-bit h costs 252 doublings.  Instead the prep kernel finds, by a
// 2-dimensional lattice reduction, a ~128-bit pair (a, b) with a = b h (mod 8L)
// and b odd, and the main kernel checks
//     [a](-A) + [b]([S]B - R) == identity
// which is [b](R' - R) == 0 ([b]([S]B) = [b S mod L]B: B has order L): since b is odd and 0 < |b| < L, that holds iff
// R' == R (the group has order 8L; a = b h mod 8L, not just mod L, keeps the
// torsion part of a mixed-order A exact).  R' == R is libsodium's
// encode(R') == R bytes for canonical, decodable R; any other R is rejected
// up front, as libsodium's compare would.  ~130 doublings instead of 252, and
// no inversion at the end; the price is a second decompression (R) and a
// second per-lane table in the prep kernel.  [S]B needs only the signature,
// not h: the prep kernel's R side computes it (12 mixed additions against
// shared tables) and builds the second table on [S]B - R, so the main kernel's
// walk has no fixed-base part and the h-dependent critical path of a
// synchronous call (copy -> hash side -> main) carries none of that work.
//
// [a](-A), [b](S B - R): fixed signed windows of kAWin bits against per-lane
// tables 0..2^(kAWin-1) x (-A) and x (S B - R); the window count is the wave's
// maximum over its lanes.  Default kAWin = 4: digits in [-8, 7] (the top one >= 0),
// 9-entry tables, 33 windows in practice (34 for a few waves), at most 64.
// (5-bit windows -- 17-entry tables, ~27 windows -- made the prep kernel 17 %
// slower for a main kernel 3 % faster, net -5 %: profiles/r02/ab_w4_s43.jsonl.)
constexpr int kAWin = 4;                        // bits per [a](-A) / [b](SB - R) window
constexpr int kAWindows = (255 + kAWin - 1) / kAWin;  // at most: 64 x 4 = 256 bits >= 253
constexpr int kAEntries = (1 << (kAWin - 1)) + 1;     // per-lane table 0..8 x P, cached form (entry 0 = identity)
// [S]B (prep kernel, R side): signed radix-2^bits digits of S against shared
// tables t of 0..2^(bits-1) x 2^(bits t) B (affine precomp form).  Two shapes,
// chosen per launch (SbShape below): the LARGE one, 12
// digits of 22 bits against 3 GiB of tables (256 MiB each), built in a device
// context once a batch of at least one wave per SIMD arrives (memory the 288 GB
// of HBM has to spare buys mixed additions: radix 2^16 made the C2 step 1.1 %
// slower, 2^19 0.8 %, profiles/r05/ab_bbits_s13.jsonl; the gathers are staged
// ahead, so the tables' size costs no latency), and the COMPACT one, 16 digits
// of 16 bits against 64 MiB, which every context builds first and which is all
// a Node verifying prods of a few hundred requests ever allocates.
constexpr int kBBits = 22;                             // the large shape
constexpr int kBTables = (253 + kBBits - 1) / kBBits;  // 12: digit t of S against table t
constexpr int kBEntries = (1 << (kBBits - 1)) + 1;     // per table 0..2^(kBBits-1) x base
constexpr int kBBitsCompact = 16;
constexpr int kBTablesCompact = (253 + kBBitsCompact - 1) / kBBitsCompact;  // 16
constexpr int kBEntriesCompact = (1 << (kBBitsCompact - 1)) + 1;
// the top digit, (S >> bits (tables - 1)) + carry, must index its table too
static_assert(253 - kBBits * (kBTables - 1) <= kBBits - 1, "top [S]B digit out of table range");
static_assert(253 - kBBitsCompact * (kBTablesCompact - 1) <= kBBitsCompact - 1, "top [S]B digit out of table range");
struct SbShape {
  int bits, tables, entries;
};
EDV_HD constexpr SbShape sb_large() { return SbShape{kBBits, kBTables, kBEntries}; }
EDV_HD constexpr SbShape sb_compact() { return SbShape{kBBitsCompact, kBTablesCompact, kBEntriesCompact}; }
constexpr int kCombEntries = 129;               // signer comb rows: 0..128 x 256^i B
constexpr int kBStride = 32;                    // words per B / comb entry (30 used; 128-byte aligned)

EDV_HD int mx(int a, int b) { return a > b ? a : b; }
// all ones iff x != 0, in plain VOP2 arithmetic: the or-value and the mask are
// opaque, so LLVM can fold neither the shift nor a later AND with the mask
// back into a compare and a VCC-mask v_cndmask_b32 (~23 cycles on gfx950)
EDV_HD uint32_t nz_mask(uint32_t x) { return uint32_t(opaque_i32(opaque_i32(int32_t(x | (0u - x))) >> 31)); }

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
  const int32_t lim = int32_t(int64_t(last) - int64_t(base));  // < 0 for a block wholly past the end
  uint32_t d[2 * N + 1];
#pragma unroll
  for (int t = 0; t < 2 * N + 1; t++) {
    // min(base + 4t, last) as last - max(lim - 4t, 0): one v_max_i32 instead of
    // a 64-bit compare and two VCC-mask selects
    const int32_t back = lim - 4 * t;
    d[t] = *reinterpret_cast<const uint32_t*>(last - uintptr_t(uint32_t(back > 0 ? back : 0)));
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
// scalar < 2^253: the kAWindows signed radix-2^kAWin digits of the main loop's windows
EDV_HD void recode5(uint32_t out[8], const uint32_t h[8]) { recode_signed<kAWin, kAWindows>(out, h); }
EDV_HD void recode5_fixed(uint32_t out[8], const uint32_t h[8]) { recode_signed<5, 51>(out, h); }
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

// Number of windows the packed radix-2^kAWin digits need: 1 + index of the
// top nonzero digit (0 for a zero scalar).
// bit length: one count-leading-zeros per word and an integer max, no selects
// (a VCC-mask v_cndmask_b32 costs ~23 cycles on gfx950)
EDV_HD int w8_bitlen(const uint32_t a[8]) {
  int n = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const uint32_t x = a[i];
    // zero-defined form (32 for x == 0: v_ffbh_u32 + v_min_u32), so no poison
    // value can reach the window count that bounds the main loop
#if defined(__clang__)
    const int lz = __builtin_clzg(x, 32);
#else
    const int lz = x ? __builtin_clz(x) : 32;
#endif
    n = mx(n, (32 * (i + 1) - lz) & int32_t(nz_mask(x)));
  }
  return n;
}
EDV_HD int digits5_windows(const uint32_t d[8]) {
  if (kAWin == 4) {
    // 4-bit fields never straddle a word: windows = ceil(bit length / 4) (the
    // per-field scan below compiled to 64 v_cndmask_b32 per scalar)
    return (w8_bitlen(d) + 3) >> 2;
  }
  int n = 0;
#pragma unroll
  for (int k = 0; k < kAWindows; k++) {
    const int pos = kAWin * k, wi = pos >> 5, sh = pos & 31;
    const uint64_t win = uint64_t(d[wi]) | (wi + 1 < 8 ? uint64_t(d[wi + 1]) << 32 : 0);
    n = ((win >> sh) & ((1u << kAWin) - 1)) ? k + 1 : n;
  }
  return n;
}

// ------------------------------------------- 256-bit words (lattice reduction)
EDV_HD bool w8_lt(const uint32_t a[8], const uint32_t b[8]) {
  bool lt = false, eq = true;
#pragma unroll
  for (int i = 7; i >= 0; i--) {
    lt = lt || (eq && a[i] < b[i]);
    eq = eq && a[i] == b[i];
  }
  return lt;
}
EDV_HD void w8_add(uint32_t a[8], const uint32_t b[8]) {
  uint64_t c = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    c += uint64_t(a[i]) + b[i];
    a[i] = uint32_t(c);
    c >>= 32;
  }
}
EDV_HD void w8_sub(uint32_t a[8], const uint32_t b[8]) {
  int64_t br = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const int64_t s = int64_t(a[i]) - int64_t(b[i]) + br;
    a[i] = uint32_t(s);
    br = s >> 32;
  }
}
EDV_HD double w8_to_f64(const uint32_t a[8]) {
  double d = 0.0;
#pragma unroll
  for (int i = 7; i >= 0; i--) d = d * 4294967296.0 + double(a[i]);  // x 2^32 is exact; one rounding per word
  return d;
}
EDV_HD void w8_shl1(uint32_t a[8]) {
#pragma unroll
  for (int i = 7; i > 0; i--) a[i] = (a[i] << 1) | (a[i - 1] >> 31);
  a[0] <<= 1;
}
EDV_HD void w8_sar1(uint32_t a[8]) {
#pragma unroll
  for (int i = 0; i < 7; i++) a[i] = (a[i] >> 1) | (a[i + 1] << 31);
  a[7] = uint32_t(int32_t(a[7]) >> 1);
}
EDV_HD void w8_shr1(uint32_t a[8]) {
#pragma unroll
  for (int i = 0; i < 7; i++) a[i] = (a[i] >> 1) | (a[i + 1] << 31);
  a[7] >>= 1;
}

// a / b to about 2^-50 relative.  On the GPU: v_rcp_f64 and one Newton step
// (4 instructions) in place of the IEEE-exact division sequence (div_scale x 2,
// rcp, five fma, div_fmas, div_fixup); every caller corrects its quotient
// afterwards, so exactness is not needed (see fdiv_floor and euclid_div).
#ifndef EDV_RCP_DIV
#define EDV_RCP_DIV 1
#endif
EDV_HD double approx_div(double a, double b) {
#if defined(__HIP_DEVICE_COMPILE__)
  if (EDV_RCP_DIV) {
    double r = __builtin_amdgcn_rcp(b);
    r = __builtin_fma(r, __builtin_fma(-b, r, 1.0), r);
    return a * r;
  }
#endif
  return a / b;
}
// One Euclidean division step of the lattice reduction: q = floor(r0 / r1)
// (r0 >= r1 > 0), r0 <- r0 - q r1, t0 <- t0 - q t1 (cofactors signed, two's
// complement mod 2^256).  q comes from a double-precision quotient of the two
// values scaled down by 2^-44 (relative error of the doubles < 2^-49), so for
// q < 2^31 the estimate is q or q - 1 and one masked subtraction finishes it
// (no branch); a larger quotient takes exact binary long division.
EDV_HD void euclid_div(uint32_t r0[8], uint32_t t0[8], const uint32_t r1[8], const uint32_t t1[8]) {
  const double qd = __builtin_floor(approx_div(w8_to_f64(r0), w8_to_f64(r1)) * (1.0 - 0x1p-44));
  uint32_t q = 0;
  if (qd < 2147483648.0) {
    q = uint32_t(qd);
    uint64_t c = 0;
    int64_t br = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
      const uint64_t p = uint64_t(q) * r1[i] + c;
      c = p >> 32;
      const int64_t s = int64_t(r0[i]) - int64_t(uint32_t(p)) + br;
      r0[i] = uint32_t(s);
      br = s >> 32;
    }
  } else {
    // binary long division over quotient bits e..0, 2^e <= qd <= q: r1 << e
    // stays below r0, so nothing overflows
    uint32_t d[8], v[8];
#pragma unroll
    for (int i = 0; i < 8; i++) { d[i] = r1[i]; v[i] = t1[i]; }
    const int e = int((__builtin_bit_cast(uint64_t, qd) >> 52) & 0x7ff) - 1023;  // floor(log2 qd), qd >= 2^31
#pragma unroll 1
    for (int k = 0; k < e; k++) { w8_shl1(d); w8_shl1(v); }
#pragma unroll 1
    for (int k = e; k >= 0; k--) {
      if (!w8_lt(r0, d)) { w8_sub(r0, d); w8_sub(t0, v); }
      w8_shr1(d);
      w8_sar1(v);  // t1 2^k, sign-extended (|t1 2^e| < 2^255: exact)
    }
  }
  // quotient one too small: subtract r1 once more (masked, no branch)
  const uint32_t m = w8_lt(r0, r1) ? 0u : ~0u;
  int64_t br = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const int64_t s = int64_t(r0[i]) - int64_t(r1[i] & m) + br;
    r0[i] = uint32_t(s);
    br = s >> 32;
  }
  q -= m;  // + 1 when m = ~0
  uint64_t c = 0;
  int64_t bt = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const uint64_t p = uint64_t(q) * t1[i] + c;
    c = p >> 32;
    const int64_t s = int64_t(t0[i]) - int64_t(uint32_t(p)) + bt;
    t0[i] = uint32_t(s);
    bt = s >> 32;
  }
}

EDV_HD bool w8_ge128(const uint32_t r[8]) { return (r[4] | r[5] | r[6] | r[7]) != 0; }

// floor(r / 2^s) for r < 2^(s + 53), as an exact double
EDV_HD double w8_window53(const uint32_t r[8], int s) {
  const int wi = s >> 5, b = s & 31;
  // words wi, wi + 1, wi + 2 picked by arithmetic masks (per-lane index; the
  // select form compiled to 24 VCC-mask v_cndmask_b32 at ~23 cycles each)
  uint32_t w0 = 0, w1 = 0, w2 = 0;
#pragma unroll
  for (int k = 0; k < 8; k++) {
    const uint32_t d = uint32_t(k - wi);  // 0, 1, 2 for the three slots
    const uint32_t m0 = ~nz_mask(d), m1 = ~nz_mask(d - 1u), m2 = ~nz_mask(d - 2u);
    w0 |= r[k] & m0;
    w1 |= r[k] & m1;
    w2 |= r[k] & m2;
  }
  const uint64_t lo = (uint64_t(w1) << 32) | w0;
  const uint64_t v = b == 0 ? lo : ((lo >> b) | (uint64_t(w2) << (64 - b)));
  return double(v);
}
// floor(a / b) for exact non-negative integers a < 2^54, 0 < b < 2^54 in doubles:
// exact whenever the quotient is below 2^50 (the estimate is then within one
// of it and the remainder test fixes that); larger quotients may be off, and
// every caller rejects a quotient that large (Lehmer: cofactor above 2^30).
EDV_HD double fdiv_floor(double a, double b) {
  double q = __builtin_floor(approx_div(a, b));
  const double r = __builtin_fma(-q, b, a);
  q = r < 0 ? q - 1 : (r >= b ? q + 1 : q);
  return q;
}
// (a x + b y) mod 2^256 for cofactor rows with a, b of opposite signs (or zero)
EDV_HD void w8_lin(uint32_t out[8], const uint32_t x[8], const uint32_t y[8], int32_t a, int32_t b) {
  int64_t c = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const int64_t v = int64_t(a) * int64_t(uint64_t(x[i])) + int64_t(b) * int64_t(uint64_t(y[i])) + c;
    out[i] = uint32_t(v);
    c = v >> 32;
  }
}

// One Lehmer round: Euclid simulated on the leading 53 bits of (r0, r1) in
// doubles, quotients taken only while both ends of the truncation interval give
// the same one (Knuth 4.5.2, Algorithm L), and only while the true remainder
// provably stays >= 2^128, so the first remainder below 2^128 is still reached
// by exact steps; then the cofactor matrix is applied to (r0, r1) and (t0, t1)
// once.  About 25 bits of reduction per round for one multiword pass instead of
// ~15 exact divisions.  Returns false if no quotient could be taken.
EDV_HD bool lehmer_round(uint32_t r0[8], uint32_t r1[8], uint32_t t0[8], uint32_t t1[8]) {
  const int n = w8_bitlen(r0);
  const int s = n > 53 ? n - 53 : 0;
  double x = w8_window53(r0, s), y = w8_window53(r1, s);
  const double thr = __builtin_ldexp(1.0, 128 - s);
  double A = 1, B = 0, C = 0, D = 1;
#pragma unroll 1
  for (int k = 0; k < 60; k++) {
    const double yc = y + C, yd = y + D;
    if (!(yc > 0 && yd > 0)) break;
    const double q = fdiv_floor(x + A, yc);
    // the other end of the interval gives the same quotient iff
    // 0 <= (x + B) - q (y + D) < y + D: one fma (exact: an integer below 2^53
    // whenever it is in range) instead of a second division
    const double r2 = __builtin_fma(-q, yd, x + B);
    if (!(r2 >= 0 && r2 < yd)) break;
    const double yn = x - q * y, Cn = A - q * C, Dn = B - q * D;
    // true next remainder > (yn - |Cn| - |Dn|) 2^s; keep the cofactors < 2^30
    if (yn - __builtin_fabs(Cn) - __builtin_fabs(Dn) < thr || __builtin_fabs(Cn) + __builtin_fabs(Dn) > 0x1p30) break;
    A = C; B = D; C = Cn; D = Dn;
    x = y; y = yn;
  }
  if (B == 0) return false;
  const int32_t a = int32_t(A), b = int32_t(B), c = int32_t(C), d = int32_t(D);
  uint32_t n0[8], n1[8];
  w8_lin(n0, r0, r1, a, b);
  w8_lin(n1, r0, r1, c, d);
#pragma unroll
  for (int i = 0; i < 8; i++) { r0[i] = n0[i]; r1[i] = n1[i]; }
  w8_lin(n0, t0, t1, a, b);
  w8_lin(n1, t0, t1, c, d);
#pragma unroll
  for (int i = 0; i < 8; i++) { t0[i] = n0[i]; t1[i] = n1[i]; }
  return true;
}

EDV_HD bool w8_neg_(const uint32_t t[8]) { return t[7] >> 31; }
EDV_HD void w8_abs(uint32_t out[8], const uint32_t t[8]) {
  const uint32_t m = w8_neg_(t) ? ~0u : 0u;
  uint64_t c = m & 1;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    c += uint64_t(t[i] ^ m);
    out[i] = uint32_t(c);
    c >>= 32;
  }
}

// The lattice reduction: (a, u, neg) with a = b h (mod 8L), b = (neg ? -u : u)
// odd, a >= 0, both about 2^128 (Euclid on (8L, h) stopped at the first
// remainder below 2^128: r_i = t_i h (mod 8L) throughout, and |t_i| <= 8L /
// r_(i-1) <= 2^127 at the stop).  Consecutive cofactors are coprime, so if
// that t_i is even its neighbours are odd; the shorter of them is taken.
// Always a < 2^253 and u < 2^192.  Lehmer rounds take the bulk of the
// reduction; exact divisions (two per trip, so the pairs trade places instead
// of being copied) take the last few steps down to the threshold.
EDV_HD void half_scalars(const uint32_t h[8], uint32_t a[8], uint32_t u[8], bool& neg) {
  uint32_t r0[8] = {0xe7ae9f68u, 0xc09318d2u, 0x17bce6b2u, 0xa6f7cef5u, 0u, 0u, 0u, 0x80000000u};  // 8L
  uint32_t r1[8], t0[8], t1[8];
#pragma unroll
  for (int i = 0; i < 8; i++) { r1[i] = h[i]; t0[i] = 0; t1[i] = i == 0; }
#pragma unroll 1
  for (int it = 0; it < 40 && w8_bitlen(r1) > 140; it++) {
    if (!lehmer_round(r0, r1, t0, t1)) break;
  }
  bool flip = false;  // the current pair is (r0, t0) rather than (r1, t1)
  if (w8_ge128(r1)) {
#pragma unroll 1
    for (int it = 0; it < 200; it++) {
      euclid_div(r0, t0, r1, t1);
      if (!w8_ge128(r0)) { flip = true; break; }
      euclid_div(r1, t1, r0, t0);
      if (!w8_ge128(r1)) break;
    }
  }
  if (flip) {
#pragma unroll
    for (int i = 0; i < 8; i++) {
      const uint32_t tr = r0[i], tt = t0[i];
      r0[i] = r1[i]; t0[i] = t1[i];
      r1[i] = tr; t1[i] = tt;
    }
  }
  // candidates: cur = (r1, t1), prev = (r0, t0); if cur's cofactor is even,
  // next = prev - q cur (only when r1 >= 2^64, which keeps its cofactor below
  // 2^192)
  uint32_t u0[8], u1[8];
  w8_abs(u0, t0);
  w8_abs(u1, t1);
  const bool cur_ok = u1[0] & 1, prev_ok = u0[0] & 1;
  const int cur_len = mx(w8_bitlen(r1), w8_bitlen(u1)), prev_len = mx(w8_bitlen(r0), w8_bitlen(u0));
  if (cur_ok && (!prev_ok || cur_len <= prev_len)) {
#pragma unroll
    for (int i = 0; i < 8; i++) { a[i] = r1[i]; u[i] = u1[i]; }
    neg = w8_neg_(t1);
    return;
  }
  // prev is odd here (cur is even, or cur is longer)
#pragma unroll
  for (int i = 0; i < 8; i++) { a[i] = r0[i]; u[i] = u0[i]; }
  neg = w8_neg_(t0);
  if (!cur_ok && (r1[2] | r1[3])) {
    euclid_div(r0, t0, r1, t1);  // (r0, t0) = next
    w8_abs(u0, t0);
    if (mx(w8_bitlen(r0), w8_bitlen(u0)) < prev_len) {
#pragma unroll
      for (int i = 0; i < 8; i++) { a[i] = r0[i]; u[i] = u0[i]; }
      neg = w8_neg_(t0);
    }
  }
}

// shift a 256-bit little-endian word vector left by N bits (0 < N < 32)
template <int N>
EDV_HD void shl256(uint32_t v[8]) {
#pragma unroll
  for (int i = 7; i > 0; i--) v[i] = (v[i] << N) | (v[i - 1] >> (32 - N));
  v[0] <<= N;
}
// ... and right by N bits (0 < N < 32)
template <int N>
EDV_HD void shr256(uint32_t v[8]) {
#pragma unroll
  for (int i = 0; i < 7; i++) v[i] = (v[i] >> N) | (v[i + 1] << (32 - N));
  v[7] >>= N;
}

EDV_HD ge_precomp precomp_from_words(const int32_t* w) {
  ge_precomp q;
#pragma unroll
  for (int l = 0; l < 10; l++) { q.ypx.v[l] = w[l]; q.ymx.v[l] = w[10 + l]; q.xy2d.v[l] = w[20 + l]; }
  return q;
}

// [2^shift] B
EDV_HD ge_p3 base_point(int shift) {
  const uint32_t Bw[8] = {0x66666658u, 0x66666666u, 0x66666666u, 0x66666666u,
                          0x66666666u, 0x66666666u, 0x66666666u, 0x66666666u};
  ge_p3 nB;
  ge_frombytes_negate(nB, Bw);
  ge_p3 B{fe_neg(nB.X), nB.Y, nB.Z, fe_neg(nB.T)};
  for (int k = 0; k < shift; k++) B = ge_p1p1_to_p3(ge_p2_dbl(ge_p3_to_p2(B)));
  return B;
}
// j * base for j in [0, 2^(kBBits-1)] (j < 2^kBBits), affine precomp form, written as kBStride words.
EDV_HD void btab_entry(int32_t* o, int j, const ge_p3& base) {
  const ge_cached Bc = ge_p3_to_cached(base);
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

// Device words of a table set: tables x entries x kBStride, then the tables'
// base points 2^(bits t) B as scratch for the build (launch_btab_kernel).
EDV_HD constexpr size_t sb_words(SbShape sh) { return size_t(sh.tables) * size_t(sh.entries) * kBStride; }
EDV_HD constexpr size_t sb_alloc_bytes(SbShape sh) { return 4 * sb_words(sh) + size_t(sh.tables) * sizeof(ge_p3); }

// Per-lane outputs of phase 1 that phase 2 consumes.
struct PrepDigits {
  uint32_t da[8];        // packed signed radix-2^kAWin digits of a ([a](-A))
  uint32_t db[8];        // packed signed radix-2^kAWin digits of |b| ([b](SB - R), sign folded into the walk)
  int nwin;              // windows this lane needs (max over a and |b|)
  bool negR;             // b < 0: the second table's digits are negated ([b]Q = [|b|](-Q))
};

// 0..kAEntries-1 x P into a per-lane table (entry 0 the identity, so a zero digit needs
// no select).  P comes out of a decompression affine (Z = 1, T = XY), so its
// cached form doubles as precomp form and each further entry is a mixed
// addition (3 field products instead of 4).
template <class Tab>
EDV_HD void build_table(Tab& tab, const ge_p3& P) {
  const ge_cached c1 = ge_p3_to_cached(P);
  const ge_precomp p1{c1.YpX, c1.YmX, c1.T2d};
  tab.store(0, ge_cached_identity());
  tab.store(1, c1);
  ge_p3 cur = ge_p1p1_to_p3(ge_p2_dbl(ge_p3_to_p2(P)));
  tab.store(2, ge_p3_to_cached(cur));
#pragma unroll 1
  for (int e = 3; e < kAEntries; e++) {
    cur = ge_p1p1_to_p3(ge_madd(cur, p1));
    tab.store(e, ge_p3_to_cached(cur));
  }
}
// The same for a projective P (Z != 1): full additions of P's cached form,
// which Stash keeps outside the registers between them (put(c), get(); on the
// GPU the lane's LDS slice) -- held live across the loop, its 40 registers
// made the prep kernel spill inside it (prep +9 % at C2).
template <class Tab, class Stash>
EDV_HD void build_table_projective(Tab& tab, const ge_p3& P, Stash& st) {
  {
    const ge_cached c1 = ge_p3_to_cached(P);
    tab.store(0, ge_cached_identity());
    tab.store(1, c1);
    st.put(c1);
  }
  ge_p3 cur = ge_p1p1_to_p3(ge_p2_dbl(ge_p3_to_p2(P)));
  tab.store(2, ge_p3_to_cached(cur));
#pragma unroll 1
  for (int e = 3; e < kAEntries; e++) {
    cur = ge_p1p1_to_p3(ge_add(cur, st.get()));
    tab.store(e, ge_p3_to_cached(cur));
  }
}

// Phase 1, hash side (kernel edv_prep_kernel): strictness checks V2-V4,
// h = SHA-512(R || A || M) mod L (V6, V7), the half-size scalars (a, b) and
// their digit recoding.  Returns false if the signature is already rejected
// (then the digits are unspecified).
EDV_HD bool prep_one(const uint32_t R[8], const uint32_t S[8], const uint32_t A[8], const uint8_t* m, uint64_t mlen,
                     PrepDigits& pd) {
  bool ok = !((S[7] & 0xF0000000u) && !sc_is_canonical(S));
  ok = ok && !has_small_order(R);
  ok = ok && ge_is_canonical(A) && !has_small_order(A);
  if (!ok) return false;
  uint32_t dig[16], h[8];
  hram(dig, R, A, m, mlen);
  sc_reduce(h, dig);
  uint32_t a[8], u[8];
  bool neg;
  half_scalars(h, a, u, neg);
  recode5(pd.da, a);
  recode5(pd.db, u);
  pd.nwin = mx(digits5_windows(pd.da), digits5_windows(pd.db));
  pd.negR = neg;
  return true;
}

// Phase 1, A side (kernel edv_prep_kernel, concurrent with the hash side):
// decompress -A and build its 0..kAEntries-1 x (-A) table (V4, V5: libsodium's
// checks on the key).  Returns false on rejection.
template <class ATab>
EDV_HD bool prep_point(const uint32_t P[8], ATab& tab) {
  if (!ge_is_canonical(P) || has_small_order(P)) return false;
  ge_p3 nP;
  if (!ge_frombytes_negate(nP, P)) return false;
  build_table(tab, nP);
  return true;
}

// Phase 1, R side: Q = [S]B - R and its 0..kAEntries-1 x Q table.  encode(R')
// is canonical and a curve point's encoding, so R bytes that are
// non-canonical, of small order (libsodium's blocklist) or decode to no point
// can never pass: the same three checks as for A reject them.  [S]B is the
// sum of entry |d_t| of table t (negated for d_t < 0) over the sh.tables signed
// radix-2^sh.bits digits d_t of S (sh = bt.shape(): the large or the compact
// tables), added to -R by mixed additions; BTab provides stage(t, j) then
// fetch() -> j x 2^(bits t) B (precomp).  S < L for every signature that can
// pass (the hash side's V2 check rejects the rest); S is cut to 253 bits so
// that any 256-bit S keeps its digits inside the tables.  BTab also stashes
// Q's cached form for the table (build_table_projective).
EDV_HD void shr256_var(uint32_t v[8], int n) {  // 0 < n < 32
#pragma unroll
  for (int i = 0; i < 7; i++) v[i] = (v[i] >> n) | (v[i + 1] << (32 - n));
  v[7] >>= n;
}
// q += [S]B: the sh.tables mixed additions of the signed radix-2^sh.bits
// digits of S (cut to 253 bits) against BTab's tables
template <class BTab>
EDV_HD void add_sb(ge_p3& q, const uint32_t S[8], BTab& bt) {
  const SbShape sh = bt.shape();
  uint32_t s[8];
#pragma unroll
  for (int i = 0; i < 8; i++) s[i] = S[i];
  s[7] &= 0x1fffffffu;
  // signed digits, least significant first, taken off the bottom of s as the
  // walk goes: d = (s mod 2^bits) + carry in [-2^(bits-1), 2^(bits-1)); the
  // top digit keeps its carry (static_asserts above: it stays in range)
  int carry = 0;
  const int bits = sh.bits;
  auto next_digit = [&](bool top) {
    int e = int(s[0] & ((1u << bits) - 1)) + carry;
    shr256_var(s, bits);
    carry = top ? 0 : (e + (1 << (bits - 1))) >> bits;
    return e - carry * (1 << bits);
  };
  // entry t + 1 is staged (on the GPU: straight into LDS) while entry t is added
  int dt = next_digit(sh.tables == 1);
  bt.stage(0, dt < 0 ? -dt : dt);
#pragma unroll 1
  for (int t = 0; t < sh.tables; t++) {
    const ge_precomp e = ge_precomp_cneg(bt.fetch(), dt < 0);
    if (t + 1 < sh.tables) {
      dt = next_digit(t + 2 == sh.tables);
      bt.stage(t + 1, dt < 0 ? -dt : dt);
    }
    q = ge_p1p1_to_p3(ge_madd(q, e));
  }
}
// Q = [S]B - R (projective) for a decodable R; false if R is rejected
template <class BTab>
EDV_HD bool rpoint_q(const uint32_t R[8], const uint32_t S[8], BTab& bt, ge_p3& q) {
  if (!ge_is_canonical(R) || has_small_order(R)) return false;
  if (!ge_frombytes_negate(q, R)) return false;
  add_sb(q, S, bt);
  return true;
}
template <class ATab, class BTab>
EDV_HD bool prep_rpoint(const uint32_t R[8], const uint32_t S[8], ATab& tab, BTab& bt) {
  ge_p3 q;
  if (!rpoint_q(R, S, bt, q)) return false;
  build_table_projective(tab, q, bt);
  return true;
}

// Phase 2 (kernel edv_main_kernel): Q = [a](-A) + [|b|](+-([S]B - R)) by a
// joint fixed-window walk, top window first -- every lane adds at the same
// positions, so a wave never diverges -- then Q == identity.  nwin: windows to
// walk (the wave's maximum; >= every lane's own count); da/db are consumed
// from the top (shifted left kAWin bits per window).  ATab provides stage(e)
// then fetch() -> cached entry e.
template <class ATab>
EDV_HD bool main_one(uint32_t da[8], uint32_t db[8], int nwin, bool negR, ATab& at, ATab& rt) {
  // align window nwin-1 with the top window, bits [kTop, kTop + kAWin)
  constexpr int kTop = kAWin * (kAWindows - 1);       // 250 (252)
  constexpr int kTopShl = 32 - kAWin - (kTop - 224);  // 1 (0)
#pragma unroll 1
  for (int k = nwin; k < kAWindows; k++) {
    shl256<kAWin>(da);
    shl256<kAWin>(db);
  }
  ge_p2 acc = ge_p2_identity();
#pragma unroll 1
  for (int w = nwin - 1; w >= 0; --w) {
    // stage(...) starts this window's table reads (on the GPU: straight into
    // LDS, no registers held), fetch() picks them up after the doublings
    const int dA = int32_t(da[7] << kTopShl) >> (32 - kAWin);  // digit at bits [kTop, kTop + kAWin)
    const int dR = int32_t(db[7] << kTopShl) >> (32 - kAWin);
    shl256<kAWin>(da);
    shl256<kAWin>(db);
    at.stage(dA < 0 ? -dA : dA);
    rt.stage(dR < 0 ? -dR : dR);
    ge_p3 p3;
    if (w == nwin - 1) {
      p3 = ge_p3_identity();
    } else {
#pragma unroll 1  // a doubling is ~1k instructions: unrolling buys nothing but code size
      for (int d = 0; d < kAWin - 1; d++) acc = ge_p1p1_to_p2(ge_p2_dbl(acc));
      p3 = ge_p1p1_to_p3(ge_p2_dbl(acc));
    }
    const ge_cached ea = at.fetch();
    p3 = ge_p1p1_to_p3(ge_add(p3, ge_cached_cneg(ea, dA < 0)));
    const ge_cached er = rt.fetch();
    acc = ge_p1p1_to_p2(ge_add(p3, ge_cached_cneg(er, (dR < 0) != negR)));
  }
  // identity: X = 0 and Y = Z (mod p)
  return fe_iszero(acc.X) && fe_iszero(fe_carry32(fe_sub(acc.Y, acc.Z)));
}

// The whole verdict for one signature: true iff libsodium's verify_detached
// would return 0.
template <class ATab, class BTab>
EDV_HD bool verify_one(const uint32_t R[8], const uint32_t S[8], const uint32_t A[8], const uint8_t* m, uint64_t mlen,
                       ATab& at, ATab& rt, BTab& bt) {
  PrepDigits pd;
  if (!prep_one(R, S, A, m, mlen, pd)) return false;
  if (!prep_point(A, at) || !prep_rpoint(R, S, rt, bt)) return false;
  return main_one(pd.da, pd.db, pd.nwin, pd.negR, at, rt);
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
