// edv_math.h -- GF(2^255-19), edwards25519 group, scalar mod L and SHA-512
// for the MI355X batch Ed25519 verifier.  One signature per lane.
//
// What this replaces: the arithmetic behind the reference's single verify call
// site, stp_core/crypto/nacl_wrappers.py:86-108 (VerifyKey.verify ->
// libnacl.crypto_sign_open), i.e. libsodium 1.0.18
// crypto_sign_ed25519_verify_detached.
//
// Representation (DESIGN.md "Field arithmetic"): signed 32-bit limbs in radix
// 2^25.5 (26/25/26/... bits).  A product is 100 32x32->64 multiply-adds
// (v_mad_i64_i32, ~4.6 cycles/wave-instr on gfx950, measured in
// tools/ubench_valu.hip) into ten 64-bit column accumulators with the 2^255 = 19
// fold applied to pre-multiplied operands, so no column ever needs a carry
// word; additions and subtractions are plain 32-bit limb ops (v_add_u32 class,
// ~2.3 cycles) with no carry at all.  Limb bounds follow the classic radix-2^25.5
// analysis: mul/sq accept |f_i| <= 1.65*2^26 (even i) / 1.65*2^25 (odd i) and
// return |h_i| <= 2^25 / 2^24 (+ tiny), so sums/differences of up to three
// reduced values can feed a multiply directly.
//
// Everything is __host__ __device__ so the identical code is unit-tested on the
// CPU (tests/test_math_host.py via libedv_hostcheck.so) before it runs on gfx950.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define EDV_HD __host__ __device__ __forceinline__
#else  // plain C++ build of the same math for the CPU unit tests (tests only)
#define EDV_HD inline
#endif

namespace edv {

struct fe { int32_t v[10]; };

// ---------------------------------------------------------------- constants
// d = -121665/121666, 2d, sqrt(-1): limbs computed from the integers
// (tools/derive_constants.py), unsigned within limb widths.
EDV_HD fe fe_d() { return fe{{56195235, 13857412, 51736253, 6949390, 114729, 24766616, 60832955, 30306712, 48412415, 21499315}}; }
EDV_HD fe fe_d2() { return fe{{45281625, 27714825, 36363642, 13898781, 229458, 15978800, 54557047, 27058993, 29715967, 9444199}}; }
EDV_HD fe fe_sqrtm1() { return fe{{34513072, 25610706, 9377949, 3500415, 12389472, 33281959, 41962654, 31548777, 326685, 11406482}}; }

EDV_HD fe fe_zero() { return fe{{0, 0, 0, 0, 0, 0, 0, 0, 0, 0}}; }
EDV_HD fe fe_one() { return fe{{1, 0, 0, 0, 0, 0, 0, 0, 0, 0}}; }

EDV_HD fe fe_add(const fe& f, const fe& g) {
  fe h;
#pragma unroll
  for (int i = 0; i < 10; i++) h.v[i] = f.v[i] + g.v[i];
  return h;
}
EDV_HD fe fe_sub(const fe& f, const fe& g) {
  fe h;
#pragma unroll
  for (int i = 0; i < 10; i++) h.v[i] = f.v[i] - g.v[i];
  return h;
}
EDV_HD fe fe_neg(const fe& f) {
  fe h;
#pragma unroll
  for (int i = 0; i < 10; i++) h.v[i] = -f.v[i];
  return h;
}
EDV_HD fe fe_select(const fe& a, const fe& b, bool take_b) {
  fe h;
#pragma unroll
  for (int i = 0; i < 10; i++) h.v[i] = take_b ? b.v[i] : a.v[i];
  return h;
}

// One signed rounding carry step on a 64-bit column: returns the new 32-bit limb
// (in [-2^(w-1), 2^(w-1))) and adds the carry into `next`.
template <int W>
EDV_HD int32_t carry_step(int64_t h, int64_t& next) {
  const int64_t t = h + (int64_t(1) << (W - 1));
  next += t >> W;  // arithmetic shift
  return int32_t(uint32_t(t) & ((1u << W) - 1)) - (1 << (W - 1));
}

// Reduce ten 64-bit columns to limbs (radix-2^25.5 carry order that keeps every
// intermediate inside int64 and leaves |h_i| <= 2^25 / 2^24 (+2^(small))).
EDV_HD fe fe_carry64(int64_t h0, int64_t h1, int64_t h2, int64_t h3, int64_t h4, int64_t h5, int64_t h6,
                     int64_t h7, int64_t h8, int64_t h9) {
  h0 = carry_step<26>(h0, h1);
  h4 = carry_step<26>(h4, h5);
  h1 = carry_step<25>(h1, h2);
  h5 = carry_step<25>(h5, h6);
  h2 = carry_step<26>(h2, h3);
  h6 = carry_step<26>(h6, h7);
  h3 = carry_step<25>(h3, h4);
  h7 = carry_step<25>(h7, h8);
  h4 = carry_step<26>(h4, h5);
  h8 = carry_step<26>(h8, h9);
  int64_t c9 = 0;
  h9 = carry_step<25>(h9, c9);
  h0 += c9 * 19;
  h0 = carry_step<26>(h0, h1);
  return fe{{int32_t(h0), int32_t(h1), int32_t(h2), int32_t(h3), int32_t(h4), int32_t(h5), int32_t(h6),
             int32_t(h7), int32_t(h8), int32_t(h9)}};
}

// Rounding bias of column k (2^(W_k - 1)).  The product kernels START their
// column accumulators at this value (it rides in as the addend of the first
// v_mad_i64_i32), so each first-pass carry step below is one 64-bit shift, one
// 64-bit add and a mask: the separate 64-bit bias add of carry_step is gone
// (10 of the 12 steps).  On the device the bias is read from constant memory:
// as a literal, LLVM's reassociation moves it to the END of the column sum and
// emits exactly the 64-bit add this saves (main kernel: 1,383 -> 704
// v_lshl_add_u64, 11.3k -> 10.7k instructions, 204 -> 193 VGPRs).
EDV_HD constexpr int64_t col_bias(int k) { return (k & 1) ? (int64_t(1) << 24) : (int64_t(1) << 25); }
#if defined(__HIP_DEVICE_COMPILE__)
__constant__ int64_t c_col_bias[3] = {int64_t(1) << 25, int64_t(1) << 24, 0};
EDV_HD int64_t bias_reg(int k) { return c_col_bias[k & 1]; }
// an opaque zero addend: keeps an unbiased column's first product one
// v_mad_i64_i32 (a literal 0 would make it a mul_lo/mul_hi pair)
EDV_HD int64_t zero_reg() { return c_col_bias[2]; }
#else
EDV_HD int64_t bias_reg(int k) { return col_bias(k); }
EDV_HD int64_t zero_reg() { return 0; }
#endif
template <int W>
EDV_HD int32_t carry_biased(int64_t t, int64_t& next) {
  next += t >> W;  // arithmetic shift of the biased column = rounded carry
  return int32_t(uint32_t(t) & ((1u << W) - 1)) - (1 << (W - 1));
}
// fe_carry64 for columns that carry their col_bias (same carry order, same
// rounding, hence the same output bounds).  A column that has already been
// reduced to a limb and then receives a carry (h4, and h0 after the 19-fold)
// is unbiased, so its second step is an ordinary carry_step.
EDV_HD fe fe_carry64_biased(int64_t h0, int64_t h1, int64_t h2, int64_t h3, int64_t h4, int64_t h5, int64_t h6,
                            int64_t h7, int64_t h8, int64_t h9) {
  // One sequential pass 0 -> 9, the 2^255 = 19 fold, then 0 -> 1: eleven steps
  // (ten of them on biased columns) against twelve for ref10's two interleaved
  // chains, which need h4 carried twice.  Every column is carried once before it
  // is read as a limb, so the output bounds are those of fe_carry64: a column
  // is < 2^62, its carry < 2^37 adds into the next 64-bit column, 19 * c9 < 2^42
  // lands on the reduced h0 and h0's last carry (< 2^17) on the reduced h1.
  h0 = carry_biased<26>(h0, h1);
  h1 = carry_biased<25>(h1, h2);
  h2 = carry_biased<26>(h2, h3);
  h3 = carry_biased<25>(h3, h4);
  h4 = carry_biased<26>(h4, h5);
  h5 = carry_biased<25>(h5, h6);
  h6 = carry_biased<26>(h6, h7);
  h7 = carry_biased<25>(h7, h8);
  h8 = carry_biased<26>(h8, h9);
  int64_t c9 = 0;
  h9 = carry_biased<25>(h9, c9);
  h0 += c9 * 19;
  h0 = carry_step<26>(h0, h1);
  return fe{{int32_t(h0), int32_t(h1), int32_t(h2), int32_t(h3), int32_t(h4), int32_t(h5), int32_t(h6),
             int32_t(h7), int32_t(h8), int32_t(h9)}};
}

// h = f * g.  Column k collects f_i g_j with i + j = k (weight 1) or k + 10
// (weight 19 via the pre-multiplied g_j*19); odd*odd products carry an extra 2
// because of the 26/25 limb alternation (applied to the odd f_i when k is even).
// Keeps the machine scheduler from interleaving independent field products:
// interleaving buys little ILP but multiplies live registers (measured: a point
// addition went from 421 to 135 VGPRs), and occupancy is what hides latency here.
EDV_HD void sched_fence() {
#if defined(__HIP_DEVICE_COMPILE__) && !defined(EDV_NO_SCHED_FENCE)
  __builtin_amdgcn_sched_barrier(0);
#endif
}

EDV_HD fe fe_mul(const fe& f, const fe& g) {
  sched_fence();
  int32_t g19[10], f2[10];
#pragma unroll
  for (int i = 0; i < 10; i++) {
    g19[i] = 19 * g.v[i];
    f2[i] = (i & 1) ? 2 * f.v[i] : f.v[i];
  }
  const int32_t f38_9 = 38 * f.v[9];
  int64_t h[10];
#pragma unroll
  for (int k = 0; k < 10; k++) {
    int64_t acc = 0;
#pragma unroll
    for (int i = 0; i < 10; i++) {
      const int j = k - i;
      // f_9 g_j with j odd wraps with weight 2 * 19: as (38 f_9) g_j, so
      // neither 2 f_9 nor 19 g_1 is needed (13 premultiplied operands, not 14)
      const bool f9w = (i == 9) && (j < 0) && ((j + 10) & 1);
      const int32_t a = f9w ? f38_9 : ((k & 1) == 0) ? f2[i] : f.v[i];
      const int32_t b = f9w ? g.v[j + 10] : (j >= 0) ? g.v[j] : g19[j + 10];
      acc = (i == 0) ? int64_t(a) * int64_t(b) + bias_reg(k) : acc + int64_t(a) * int64_t(b);
    }
    h[k] = acc;
  }
  const fe r = fe_carry64_biased(h[0], h[1], h[2], h[3], h[4], h[5], h[6], h[7], h[8], h[9]);
  sched_fence();
  return r;
}

// Squaring columns (55 products): term f_i f_j (i <= j) carries the constant
// (i<j ? 2 : 1) * (i,j both odd ? 2 : 1) * (i+j >= 10 ? 19 : 1) (* 2 for
// DOUBLE, i.e. 2 f^2), applied as (x f_i) * (y f_j) with x y = that constant.
// The split {x, y} below keeps each premultiplied operand inside int32 under
// the mul input bounds (x <= 19 on even limbs, <= 38 on odd limbs) and uses the
// fewest distinct premultiplied operands, one instruction each: 13 for f^2 and
// 21 for 2 f^2 (tools/derive_sq_split.py, a small 0/1 ILP; the earlier hand
// rule needed 17 and 27).  Columns start at col_bias.
struct sq_split { int8_t x, y; };
constexpr sq_split kSqSplit[2][10][10] = {
    {
        {{1, 1}, {1, 2}, {1, 2}, {2, 1}, {2, 1}, {2, 1}, {2, 1}, {2, 1}, {2, 1}, {2, 1}},
        {{0, 0}, {1, 2}, {2, 1}, {2, 2}, {2, 1}, {2, 2}, {1, 2}, {2, 2}, {2, 1}, {2, 38}},
        {{0, 0}, {0, 0}, {1, 1}, {1, 2}, {2, 1}, {1, 2}, {1, 2}, {1, 2}, {2, 19}, {1, 38}},
        {{0, 0}, {0, 0}, {0, 0}, {1, 2}, {2, 1}, {2, 2}, {2, 1}, {2, 38}, {2, 19}, {2, 38}},
        {{0, 0}, {0, 0}, {0, 0}, {0, 0}, {1, 1}, {1, 2}, {2, 19}, {1, 38}, {2, 19}, {1, 38}},
        {{0, 0}, {0, 0}, {0, 0}, {0, 0}, {0, 0}, {19, 2}, {2, 19}, {2, 38}, {2, 19}, {2, 38}},
        {{0, 0}, {0, 0}, {0, 0}, {0, 0}, {0, 0}, {0, 0}, {19, 1}, {1, 38}, {2, 19}, {1, 38}},
        {{0, 0}, {0, 0}, {0, 0}, {0, 0}, {0, 0}, {0, 0}, {0, 0}, {1, 38}, {2, 19}, {2, 38}},
        {{0, 0}, {0, 0}, {0, 0}, {0, 0}, {0, 0}, {0, 0}, {0, 0}, {0, 0}, {1, 19}, {1, 38}},
        {{0, 0}, {0, 0}, {0, 0}, {0, 0}, {0, 0}, {0, 0}, {0, 0}, {0, 0}, {0, 0}, {1, 38}},
    },
    {
        {{1, 2}, {1, 4}, {2, 2}, {1, 4}, {2, 2}, {2, 2}, {2, 2}, {2, 2}, {2, 2}, {1, 4}},
        {{0, 0}, {4, 1}, {4, 1}, {8, 1}, {4, 1}, {8, 1}, {1, 4}, {4, 2}, {4, 1}, {8, 19}},
        {{0, 0}, {0, 0}, {2, 1}, {1, 4}, {2, 2}, {4, 1}, {2, 2}, {4, 1}, {4, 19}, {4, 19}},
        {{0, 0}, {0, 0}, {0, 0}, {1, 4}, {1, 4}, {4, 2}, {1, 4}, {4, 38}, {4, 19}, {4, 38}},
        {{0, 0}, {0, 0}, {0, 0}, {0, 0}, {1, 2}, {4, 1}, {4, 19}, {2, 38}, {4, 19}, {4, 19}},
        {{0, 0}, {0, 0}, {0, 0}, {0, 0}, {0, 0}, {38, 2}, {38, 2}, {4, 38}, {4, 19}, {38, 4}},
        {{0, 0}, {0, 0}, {0, 0}, {0, 0}, {0, 0}, {0, 0}, {2, 19}, {2, 38}, {4, 19}, {19, 4}},
        {{0, 0}, {0, 0}, {0, 0}, {0, 0}, {0, 0}, {0, 0}, {0, 0}, {38, 2}, {38, 2}, {38, 4}},
        {{0, 0}, {0, 0}, {0, 0}, {0, 0}, {0, 0}, {0, 0}, {0, 0}, {0, 0}, {2, 19}, {19, 4}},
        {{0, 0}, {0, 0}, {0, 0}, {0, 0}, {0, 0}, {0, 0}, {0, 0}, {0, 0}, {0, 0}, {19, 4}},
    }};
template <bool DOUBLE, bool BIAS = true>
EDV_HD void fe_sq_cols(const fe& f, int64_t h[10]) {
  bool first[10];
#pragma unroll
  for (int k = 0; k < 10; k++) first[k] = true;
#pragma unroll
  for (int i = 0; i < 10; i++) {
#pragma unroll
    for (int j = i; j < 10; j++) {
      const int k = (i + j) % 10;
      const sq_split m = kSqSplit[DOUBLE ? 1 : 0][i][j];
      const int32_t a = f.v[i] * int32_t(m.x), b = f.v[j] * int32_t(m.y);
      h[k] = first[k] ? int64_t(a) * int64_t(b) + (BIAS ? bias_reg(k) : zero_reg()) : h[k] + int64_t(a) * int64_t(b);
      first[k] = false;
    }
  }
}
EDV_HD fe fe_sq(const fe& f) {
  sched_fence();
  int64_t h[10];
  fe_sq_cols<false>(f, h);
  const fe r = fe_carry64_biased(h[0], h[1], h[2], h[3], h[4], h[5], h[6], h[7], h[8], h[9]);
  sched_fence();
  return r;
}
// f^2 with floor carries (no rounding bias): limbs come out in [0, 2^26) /
// [0, 2^25) (h1 within 2^16 of that range), one 32-bit subtraction per limb
// cheaper than fe_sq.  Twice fe_sq's limb magnitude, so an output may feed
// fe_sq / fe_sq_floor / fe_mul directly (inside their input bounds:
// 19 x 2^26 and 38 x (2^25 + 2^16) < 2^31 for the premultiplied operands,
// columns < 2^59), but not a sum or difference into a product.  Used for the
// runs of squarings in the exponentiations (fe_sqn).
template <int W>
EDV_HD int32_t carry_floor(int64_t t, int64_t& next) {
  next += t >> W;  // arithmetic shift: floor
  return int32_t(uint32_t(t) & ((1u << W) - 1));
}
EDV_HD fe fe_sq_floor(const fe& f) {
  sched_fence();
  int64_t h[10];
  fe_sq_cols<false, false>(f, h);
  int64_t c9 = 0;
  int32_t o[10];
  o[0] = carry_floor<26>(h[0], h[1]);
  o[1] = carry_floor<25>(h[1], h[2]);
  o[2] = carry_floor<26>(h[2], h[3]);
  o[3] = carry_floor<25>(h[3], h[4]);
  o[4] = carry_floor<26>(h[4], h[5]);
  o[5] = carry_floor<25>(h[5], h[6]);
  o[6] = carry_floor<26>(h[6], h[7]);
  o[7] = carry_floor<25>(h[7], h[8]);
  o[8] = carry_floor<26>(h[8], h[9]);
  o[9] = carry_floor<25>(h[9], c9);
  int64_t t0 = int64_t(o[0]) + 19 * c9, t1 = o[1];
  o[0] = carry_floor<26>(t0, t1);
  o[1] = int32_t(t1);
  const fe r{{o[0], o[1], o[2], o[3], o[4], o[5], o[6], o[7], o[8], o[9]}};
  sched_fence();
  return r;
}
// 2 f^2
EDV_HD fe fe_sq2(const fe& f) {
  sched_fence();
  int64_t h[10];
  fe_sq_cols<true>(f, h);
  const fe r = fe_carry64_biased(h[0], h[1], h[2], h[3], h[4], h[5], h[6], h[7], h[8], h[9]);
  sched_fence();
  return r;
}

// Weak 32-bit carry: brings limbs of a (sum of few reduced values) back to the
// reduced range without 64-bit work.
EDV_HD fe fe_carry32(const fe& f) {
  int64_t h[10];
#pragma unroll
  for (int i = 0; i < 10; i++) h[i] = f.v[i];
  return fe_carry64(h[0], h[1], h[2], h[3], h[4], h[5], h[6], h[7], h[8], h[9]);
}

// Canonical little-endian encoding as 8 words.  Input: reduced limbs.
EDV_HD void fe_tobytes(uint32_t w[8], const fe& f) {
  int32_t h[10];
#pragma unroll
  for (int i = 0; i < 10; i++) h[i] = f.v[i];
  // q = floor(value / p) in {0, 1} for reduced input (value in (-2^255, 2^256))
  int32_t q = (19 * h[9] + (1 << 24)) >> 25;
#pragma unroll
  for (int i = 0; i < 10; i++) q = (h[i] + q) >> ((i & 1) ? 25 : 26);
  h[0] += 19 * q;
  // value - q*p, then propagate with floor carries; drop the 2^255 carry
#pragma unroll
  for (int i = 0; i < 9; i++) {
    const int s = (i & 1) ? 25 : 26;
    const int32_t c = h[i] >> s;
    h[i + 1] += c;
    h[i] -= c * (1 << s);
  }
  h[9] &= (1 << 25) - 1;
  const uint32_t u0 = h[0], u1 = h[1], u2 = h[2], u3 = h[3], u4 = h[4], u5 = h[5], u6 = h[6], u7 = h[7],
                 u8 = h[8], u9 = h[9];
  w[0] = u0 | (u1 << 26);
  w[1] = (u1 >> 6) | (u2 << 19);
  w[2] = (u2 >> 13) | (u3 << 13);
  w[3] = (u3 >> 19) | (u4 << 6);
  w[4] = u5 | (u6 << 25);
  w[5] = (u6 >> 7) | (u7 << 19);
  w[6] = (u7 >> 13) | (u8 << 12);
  w[7] = (u8 >> 20) | (u9 << 6);
}

// 255 low bits of 8 little-endian words; bit 255 ignored; value may be >= p.
// Output is carried (centered) so it meets the reduced bounds.
EDV_HD fe fe_frombytes(const uint32_t w[8]) {
  fe h;
  h.v[0] = w[0] & 0x3ffffff;
  h.v[1] = ((w[0] >> 26) | (w[1] << 6)) & 0x1ffffff;
  h.v[2] = ((w[1] >> 19) | (w[2] << 13)) & 0x3ffffff;
  h.v[3] = ((w[2] >> 13) | (w[3] << 19)) & 0x1ffffff;
  h.v[4] = (w[3] >> 6) & 0x3ffffff;
  h.v[5] = w[4] & 0x1ffffff;
  h.v[6] = ((w[4] >> 25) | (w[5] << 7)) & 0x3ffffff;
  h.v[7] = ((w[5] >> 19) | (w[6] << 13)) & 0x1ffffff;
  h.v[8] = ((w[6] >> 12) | (w[7] << 20)) & 0x3ffffff;
  h.v[9] = (w[7] >> 6) & 0x1ffffff;
  return fe_carry32(h);
}

EDV_HD bool fe_iszero(const fe& f) {
  uint32_t w[8];
  fe_tobytes(w, f);
  return (w[0] | w[1] | w[2] | w[3] | w[4] | w[5] | w[6] | w[7]) == 0;
}
EDV_HD bool fe_isnegative(const fe& f) {
  uint32_t w[8];
  fe_tobytes(w, f);
  return w[0] & 1;
}

#ifndef EDV_SQN_FLOOR
#define EDV_SQN_FLOOR 1
#endif
EDV_HD fe fe_sqn(fe f, int n) {
#pragma unroll 1
  for (int i = 0; i < n; i++) f = EDV_SQN_FLOOR ? fe_sq_floor(f) : fe_sq(f);
  return f;
}
// z^(2^250 - 1) and z^11 (shared prefix of the inversion and sqrt chains)
EDV_HD fe fe_pow2_250_1(const fe& z, fe& z11) {
  fe z2 = fe_sq(z);
  fe z8 = fe_sq(fe_sq(z2));
  fe z9 = fe_mul(z, z8);
  z11 = fe_mul(z2, z9);
  fe z_5_0 = fe_mul(z9, fe_sq(z11));            // 2^5 - 1
  fe z_10_0 = fe_mul(fe_sqn(z_5_0, 5), z_5_0);  // 2^10 - 1
  fe z_20_0 = fe_mul(fe_sqn(z_10_0, 10), z_10_0);
  fe z_40_0 = fe_mul(fe_sqn(z_20_0, 20), z_20_0);
  fe z_50_0 = fe_mul(fe_sqn(z_40_0, 10), z_10_0);
  fe z_100_0 = fe_mul(fe_sqn(z_50_0, 50), z_50_0);
  fe z_200_0 = fe_mul(fe_sqn(z_100_0, 100), z_100_0);
  return fe_mul(fe_sqn(z_200_0, 50), z_50_0);  // 2^250 - 1
}
// z^(p-2) = z^(2^255 - 21)
EDV_HD fe fe_invert(const fe& z) {
  fe z11;
  fe t = fe_pow2_250_1(z, z11);
  return fe_mul(fe_sqn(t, 5), z11);
}
// z^((p-5)/8) = z^(2^252 - 3)
EDV_HD fe fe_pow22523(const fe& z) {
  fe z11;
  fe t = fe_pow2_250_1(z, z11);
  return fe_mul(fe_sqn(t, 2), z);
}

// ------------------------------------------------ inversion by safegcd (V9)
// z^-1 by Bernstein-Yang constant-time divsteps ("Fast constant-time gcd
// computation and modular inversion", 2019), in the eta ("hddivstep") form with
// 20 batches of 30 divsteps (600 >= the 590 proven sufficient for 256-bit
// moduli), on signed 30-bit limbs.  About 13.5k instructions per lane against
// ~30k for z^(p-2) (254 squarings + 11 products); every lane runs the same
// fixed schedule, so the wave never diverges.
//   f, g  the gcd pair (f = p, g = z), 9 signed limbs of 30 bits
//   d, e  d*z = f and e*z = g (mod p) throughout; at the end g = 0, f = +-1
struct s30 { int32_t v[9]; };
// A masked limb is known non-negative, so LLVM widens it with zext; a signed x
// zext 32x32 product then matches neither v_mad_i64_i32 nor v_mad_u64_u32 and
// becomes a 64-bit multiply (mul_lo + mad_u64 + add).  Hiding the value range
// keeps every limb product one v_mad_i64_i32.
EDV_HD int32_t opaque_i32(int32_t x) {
#if defined(__HIP_DEVICE_COMPILE__)
  asm("" : "+v"(x));
#endif
  return x;
}
constexpr int32_t kM30 = 0x3fffffff;
constexpr uint32_t kPInv30 = 0x179435e5u;  // p^-1 mod 2^30 (p = -19 mod 2^30)
// p = -19 + 2^15 * 2^240 in signed-30 limbs: limb 0 = -19, limb 8 = 2^15, the rest 0.

// 30 divsteps on the low 30 bits of f and g: returns the new eta and the
// transition matrix [u v; q r] scaled by 2^30 ((f', g') = T (f, g) / 2^30).
EDV_HD int32_t divsteps_30(int32_t eta, uint32_t f, uint32_t g, int32_t t[4]) {
  uint32_t u = 1, v = 0, q = 0, r = 1;
#pragma unroll
  for (int i = 0; i < 30; i++) {
    uint32_t c1 = uint32_t(eta >> 31);   // eta < 0
    const uint32_t c2 = 0u - (g & 1u);   // g odd
    const uint32_t x = (f ^ c1) - c1, y = (u ^ c1) - c1, z = (v ^ c1) - c1;
    g += x & c2;
    q += y & c2;
    r += z & c2;
    c1 &= c2;                            // swap step: eta < 0 and g odd
    eta = int32_t((uint32_t(eta) ^ c1) - 1u);
    f += g & c1;
    u += q & c1;
    v += r & c1;
    g >>= 1;
    u <<= 1;
    v <<= 1;
  }
  t[0] = int32_t(u); t[1] = int32_t(v); t[2] = int32_t(q); t[3] = int32_t(r);
  return eta;
}
// (f, g) <- T (f, g) / 2^30 (exact)
EDV_HD void update_fg(s30& f, s30& g, const int32_t t[4]) {
  int64_t cf = int64_t(t[0]) * f.v[0] + int64_t(t[1]) * g.v[0];
  int64_t cg = int64_t(t[2]) * f.v[0] + int64_t(t[3]) * g.v[0];
  cf >>= 30;
  cg >>= 30;
#pragma unroll
  for (int i = 1; i < 9; i++) {
    cf += int64_t(t[0]) * f.v[i] + int64_t(t[1]) * g.v[i];
    cg += int64_t(t[2]) * f.v[i] + int64_t(t[3]) * g.v[i];
    f.v[i - 1] = opaque_i32(int32_t(cf) & kM30);
    g.v[i - 1] = opaque_i32(int32_t(cg) & kM30);
    cf >>= 30;
    cg >>= 30;
  }
  f.v[8] = int32_t(cf);
  g.v[8] = int32_t(cg);
}
// (d, e) <- T (d, e) / 2^30 mod p, keeping both in (-2p, p): first add the
// multiples of p that make a negative input non-negative in effect (md, me start
// at the matrix entries of a negative d / e), then the ones that clear the low
// 30 bits of the numerator.
EDV_HD void update_de(s30& d, s30& e, const int32_t t[4]) {
  const int32_t u = t[0], v = t[1], q = t[2], r = t[3];
  const int32_t sd = d.v[8] >> 31, se = e.v[8] >> 31;
  int32_t md = (u & sd) + (v & se);
  int32_t me = (q & sd) + (r & se);
  int64_t cd = int64_t(u) * d.v[0] + int64_t(v) * e.v[0];
  int64_t ce = int64_t(q) * d.v[0] + int64_t(r) * e.v[0];
  md -= int32_t((kPInv30 * uint32_t(cd) + uint32_t(md)) & uint32_t(kM30));
  me -= int32_t((kPInv30 * uint32_t(ce) + uint32_t(me)) & uint32_t(kM30));
  cd += int64_t(-19) * md;
  ce += int64_t(-19) * me;
  cd >>= 30;
  ce >>= 30;
#pragma unroll
  for (int i = 1; i < 9; i++) {
    cd += int64_t(u) * d.v[i] + int64_t(v) * e.v[i];
    ce += int64_t(q) * d.v[i] + int64_t(r) * e.v[i];
    if (i == 8) {
      cd += int64_t(32768) * md;
      ce += int64_t(32768) * me;
    }
    d.v[i - 1] = opaque_i32(int32_t(cd) & kM30);
    e.v[i - 1] = opaque_i32(int32_t(ce) & kM30);
    cd >>= 30;
    ce >>= 30;
  }
  d.v[8] = int32_t(cd);
  e.v[8] = int32_t(ce);
}
EDV_HD fe fe_invert_safegcd(const fe& z) {
  uint32_t w[8];
  fe_tobytes(w, z);  // canonical 0 <= z < p
  s30 f, g, d, e;
  g.v[0] = int32_t(w[0] & kM30);
#pragma unroll
  for (int i = 1; i < 8; i++) {
    const int pos = 30 * i, wi = pos >> 5, sh = pos & 31;
    g.v[i] = int32_t(((w[wi] >> sh) | (sh ? (w[wi + 1] << (32 - sh)) : 0u)) & uint32_t(kM30));
  }
  g.v[8] = int32_t(w[7] >> 16);  // bits 240..255
#pragma unroll
  for (int i = 0; i < 9; i++) g.v[i] = opaque_i32(g.v[i]);
#pragma unroll
  for (int i = 0; i < 9; i++) { f.v[i] = 0; d.v[i] = 0; e.v[i] = 0; }
  f.v[0] = -19;
  f.v[8] = 32768;
  e.v[0] = 1;
  int32_t eta = -1;
#pragma unroll 1
  for (int it = 0; it < 20; it++) {
    int32_t t[4];
    eta = divsteps_30(eta, uint32_t(f.v[0]), uint32_t(g.v[0]), t);
    update_de(d, e, t);
    update_fg(f, g, t);
  }
  // f = +-1: z^-1 = sign(f) * d (mod p); d (|d| < 2p) regrouped into the
  // radix-2^25.5 columns, then carried (bits above 2^255 fold in with 19)
  const int64_t sgn = (f.v[8] >> 31) | 1;  // f.v[8] is 0 or -1 when f = +-1
  constexpr int kPos[10] = {0, 26, 51, 77, 102, 128, 153, 179, 204, 230};
  int64_t h[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
  for (int i = 0; i < 9; i++) {
    const int pos = 30 * i;
    int k = 0;  // the radix-2^25.5 limb whose range holds bit 30 i
#pragma unroll
    for (int j = 0; j < 10; j++)
      if (kPos[j] <= pos) k = j;
    h[k] += (sgn * int64_t(d.v[i])) * (int64_t(1) << (pos - kPos[k]));
  }
  return fe_carry64(h[0], h[1], h[2], h[3], h[4], h[5], h[6], h[7], h[8], h[9]);
}

// ---------------------------------------------------------------- the group
struct ge_p2 { fe X, Y, Z; };
struct ge_p3 { fe X, Y, Z, T; };
struct ge_p1p1 { fe X, Y, Z, T; };       // x = X/Z, y = Y/T
struct ge_cached { fe YpX, YmX, Z, T2d; };
struct ge_precomp { fe ypx, ymx, xy2d; };  // affine, Z = 1

EDV_HD ge_p2 ge_p2_identity() { return ge_p2{fe_zero(), fe_one(), fe_one()}; }
EDV_HD ge_p3 ge_p3_identity() { return ge_p3{fe_zero(), fe_one(), fe_one(), fe_zero()}; }
EDV_HD ge_cached ge_cached_identity() { return ge_cached{fe_one(), fe_one(), fe_one(), fe_zero()}; }
EDV_HD ge_precomp ge_precomp_identity() { return ge_precomp{fe_one(), fe_one(), fe_zero()}; }

// Operand order: fe_mul(f, g) premultiplies f's odd limbs (x 2, 38 f_9) and
// g's limbs (x 19), so X and Z go first and Y and T second in every product:
// each coordinate's premultiplied forms are made once and shared by its two
// products (the same column sums either way: the product is symmetric).
EDV_HD ge_p2 ge_p1p1_to_p2(const ge_p1p1& p) {
  return ge_p2{fe_mul(p.X, p.T), fe_mul(p.Z, p.Y), fe_mul(p.Z, p.T)};
}
EDV_HD ge_p3 ge_p1p1_to_p3(const ge_p1p1& p) {
  return ge_p3{fe_mul(p.X, p.T), fe_mul(p.Z, p.Y), fe_mul(p.Z, p.T), fe_mul(p.X, p.Y)};
}
EDV_HD ge_p2 ge_p3_to_p2(const ge_p3& p) { return ge_p2{p.X, p.Y, p.Z}; }
EDV_HD ge_cached ge_p3_to_cached(const ge_p3& p) {
  return ge_cached{fe_add(p.Y, p.X), fe_sub(p.Y, p.X), p.Z, fe_mul(p.T, fe_d2())};
}

// dbl-2008-hwcd for a = -1, output in p1p1
EDV_HD ge_p1p1 ge_p2_dbl(const ge_p2& p) {
  ge_p1p1 r;
  const fe XX = fe_sq(p.X);
  const fe YY = fe_sq(p.Y);
  const fe B = fe_sq2(p.Z);
  const fe A = fe_sq(fe_add(p.X, p.Y));
  r.Y = fe_add(YY, XX);
  r.Z = fe_sub(YY, XX);
  r.X = fe_sub(A, r.Y);
  r.T = fe_sub(B, r.Z);
  return r;
}
// p + q (unified, complete for edwards25519)
EDV_HD ge_p1p1 ge_add(const ge_p3& p, const ge_cached& q) {
  ge_p1p1 r;
  const fe A = fe_mul(fe_add(p.Y, p.X), q.YpX);
  const fe B = fe_mul(fe_sub(p.Y, p.X), q.YmX);
  const fe C = fe_mul(q.T2d, p.T);
  const fe ZZ = fe_mul(p.Z, q.Z);
  const fe D = fe_add(ZZ, ZZ);
  r.X = fe_sub(A, B);
  r.Y = fe_add(A, B);
  r.Z = fe_add(D, C);
  r.T = fe_sub(D, C);
  return r;
}
// p + q with q affine (mixed addition)
EDV_HD ge_p1p1 ge_madd(const ge_p3& p, const ge_precomp& q) {
  ge_p1p1 r;
  const fe A = fe_mul(fe_add(p.Y, p.X), q.ypx);
  const fe B = fe_mul(fe_sub(p.Y, p.X), q.ymx);
  const fe C = fe_mul(q.xy2d, p.T);
  const fe D = fe_add(p.Z, p.Z);
  r.X = fe_sub(A, B);
  r.Y = fe_add(A, B);
  r.Z = fe_add(D, C);
  r.T = fe_sub(D, C);
  return r;
}
// Conditional negation by an all-ones/zero lane mask in plain VOP2 logic (xor
// swap, (t ^ m) - m): the mask is opaque, so LLVM cannot turn it back into the
// 60 v_cndmask_b32 per window a select-based version compiles to.
EDV_HD void fe_cswap_mask(fe& a, fe& b, int32_t m) {
#pragma unroll
  for (int i = 0; i < 10; i++) {
    const int32_t t = (a.v[i] ^ b.v[i]) & m;
    a.v[i] ^= t;
    b.v[i] ^= t;
  }
}
EDV_HD fe fe_cneg_mask(const fe& a, int32_t m) {
  fe h;
#pragma unroll
  for (int i = 0; i < 10; i++) h.v[i] = (a.v[i] ^ m) - m;
  return h;
}
EDV_HD ge_cached ge_cached_cneg(ge_cached c, bool neg) {
  const int32_t m = opaque_i32(-int32_t(neg));
  fe_cswap_mask(c.YpX, c.YmX, m);
  c.T2d = fe_cneg_mask(c.T2d, m);
  return c;
}
EDV_HD ge_precomp ge_precomp_cneg(ge_precomp c, bool neg) {
  const int32_t m = opaque_i32(-int32_t(neg));
  fe_cswap_mask(c.ypx, c.ymx, m);
  c.xy2d = fe_cneg_mask(c.xy2d, m);
  return c;
}

// libsodium ge25519_frombytes_negate_vartime: decode, return -P.  false = not on curve.
EDV_HD bool ge_frombytes_negate(ge_p3& h, const uint32_t s[8]) {
  const fe one = fe_one();
  h.Y = fe_frombytes(s);
  h.Z = one;
  fe u = fe_sq(h.Y);
  fe v = fe_mul(u, fe_d());
  u = fe_sub(u, one);  // y^2 - 1
  v = fe_add(v, one);  // d y^2 + 1
  fe v3 = fe_mul(fe_sq(v), v);
  fe x = fe_mul(fe_mul(fe_sq(v3), v), u);  // u v^7
  x = fe_pow22523(x);
  x = fe_mul(fe_mul(x, v3), u);  // u v^3 (u v^7)^((p-5)/8)
  const fe vxx = fe_mul(fe_sq(x), v);
  const bool m_ok = fe_iszero(fe_sub(vxx, u));
  const bool p_ok = fe_iszero(fe_add(vxx, u));
  x = fe_select(x, fe_mul(x, fe_sqrtm1()), !m_ok);
  const bool neg = fe_isnegative(x) == bool(s[7] >> 31);
  x = fe_select(x, fe_neg(x), neg);
  h.X = fe_carry32(x);
  h.T = fe_mul(h.X, h.Y);
  return m_ok || p_ok;
}

EDV_HD void ge_p2_tobytes(uint32_t w[8], const ge_p2& p) {
  const fe zi = fe_invert_safegcd(p.Z);
  const fe x = fe_mul(p.X, zi);
  const fe y = fe_mul(p.Y, zi);
  fe_tobytes(w, y);
  w[7] ^= uint32_t(fe_isnegative(x)) << 31;
}

// ---------------------------------------------------------- strictness (V2-V4)
// S < L (libsodium sc25519_is_canonical), S as 8 LE words
EDV_HD bool sc_is_canonical(const uint32_t s[8]) {
  const uint32_t L[8] = {0x5cf5d3edu, 0x5812631au, 0xa2f79cd6u, 0x14def9deu, 0, 0, 0, 0x10000000u};
  bool lt = false, eq = true;
#pragma unroll
  for (int i = 7; i >= 0; i--) {
    lt = lt || (eq && s[i] < L[i]);
    eq = eq && s[i] == L[i];
  }
  return lt;
}
// ge25519_has_small_order: 7-entry blocklist, sign bit masked
EDV_HD bool has_small_order(const uint32_t s[8]) {
  const uint32_t top = s[7] & 0x7fffffffu;
  const bool low_zero = (s[1] | s[2] | s[3] | s[4] | s[5] | s[6]) == 0;
  const bool low_ones = (s[1] & s[2] & s[3] & s[4] & s[5] & s[6]) == 0xffffffffu;
  bool r = false;
  r = r || (low_zero && top == 0 && (s[0] == 0 || s[0] == 1));                         // 0, 1
  r = r || (low_ones && top == 0x7fffffffu && (s[0] == 0xffffffecu || s[0] == 0xffffffedu ||
                                                s[0] == 0xffffffeeu));                  // p-1, p, p+1
  // order-8 points (26e8958f... and c7176a70...)
  r = r || (s[0] == 0x8f95e826u && s[1] == 0xb027b2c2u && s[2] == 0x89f4c345u && s[3] == 0xf098eff2u &&
            s[4] == 0x05acdfd5u && s[5] == 0x3933c6d3u && s[6] == 0x880238b1u && top == 0x05fc536du);
  r = r || (s[0] == 0x706a17c7u && s[1] == 0x4fd84d3du && s[2] == 0x760b3cbau && s[3] == 0x0f67100du &&
            s[4] == 0xfa53202au && s[5] == 0xc6cc392cu && s[6] == 0x77fdc74eu && top == 0x7a03ac92u);
  return r;
}
// ge25519_is_canonical: low 255 bits < p
EDV_HD bool ge_is_canonical(const uint32_t s[8]) {
  const bool high_ones = (s[1] & s[2] & s[3] & s[4] & s[5] & s[6]) == 0xffffffffu && (s[7] & 0x7fffffffu) == 0x7fffffffu;
  return !(high_ones && s[0] >= 0xffffffedu);
}

// --------------------------------------------------------- scalars mod L (V7)
// 2^252 = -delta (mod L) with -delta = sum c_t 2^(21 t)
EDV_HD int64_t sc_bits(const uint32_t* in, int pos, int len) {
  const int wi = pos >> 5, sh = pos & 31;
  uint64_t w = in[wi];
  if (sh + len > 32) w |= uint64_t(in[wi + 1]) << 32;
  return int64_t((w >> sh) & ((uint64_t(1) << len) - 1));
}
template <int K>
EDV_HD void sc_fold(int64_t s[24]) {
  const int64_t c0 = 666643, c1 = 470296, c2 = 654183, c3 = -997805, c4 = 136657, c5 = -683901;
  const int64_t x = s[K];
  s[K - 12] += x * c0;
  s[K - 11] += x * c1;
  s[K - 10] += x * c2;
  s[K - 9] += x * c3;
  s[K - 8] += x * c4;
  s[K - 7] += x * c5;
  s[K] = 0;
}
EDV_HD void sc_carry_round(int64_t s[24], int k) {
  const int64_t c = (s[k] + (int64_t(1) << 20)) >> 21;
  s[k + 1] += c;
  s[k] -= c * (int64_t(1) << 21);
}
EDV_HD void sc_carry_floor(int64_t s[24], int k) {
  const int64_t c = s[k] >> 21;
  s[k + 1] += c;
  s[k] -= c * (int64_t(1) << 21);
}
// out = in mod L, canonical (0 <= out < L); in = 64 bytes as 16 LE words
EDV_HD void sc_reduce(uint32_t out[8], const uint32_t in[16]) {
  int64_t s[24];
#pragma unroll
  for (int k = 0; k < 23; k++) s[k] = sc_bits(in, 21 * k, 21);
  s[23] = sc_bits(in, 483, 29);
  sc_fold<23>(s); sc_fold<22>(s); sc_fold<21>(s); sc_fold<20>(s); sc_fold<19>(s); sc_fold<18>(s);
#pragma unroll
  for (int k = 6; k <= 16; k++) sc_carry_round(s, k);
  sc_fold<17>(s); sc_fold<16>(s); sc_fold<15>(s); sc_fold<14>(s); sc_fold<13>(s); sc_fold<12>(s);
#pragma unroll
  for (int k = 0; k <= 11; k++) sc_carry_round(s, k);
  sc_fold<12>(s);
#pragma unroll
  for (int k = 0; k <= 11; k++) sc_carry_floor(s, k);
  sc_fold<12>(s);
#pragma unroll
  for (int k = 0; k <= 10; k++) sc_carry_floor(s, k);
  // s[0..11] are 21-bit digits (s[11] may hold more); pack 256 bits
  uint32_t w[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
  for (int k = 0; k < 12; k++) {
    const uint64_t v = uint64_t(s[k]);
    const int pos = 21 * k, wi = pos >> 5, sh = pos & 31;
    w[wi] |= uint32_t(v << sh);
    if (wi + 1 < 8) w[wi + 1] |= uint32_t((v << sh) >> 32);
    if (sh + 21 > 64 && wi + 2 < 8) w[wi + 2] |= uint32_t(v >> (64 - sh));
  }
  // final conditional subtraction keeps the result canonical
  const uint32_t L[8] = {0x5cf5d3edu, 0x5812631au, 0xa2f79cd6u, 0x14def9deu, 0, 0, 0, 0x10000000u};
  uint32_t d[8];
  uint64_t br = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const uint64_t t = uint64_t(w[i]) - L[i] - br;
    d[i] = uint32_t(t);
    br = (t >> 63) & 1;
  }
#pragma unroll
  for (int i = 0; i < 8; i++) out[i] = br ? w[i] : d[i];
}

// ------------------------------------------------------------------ SHA-512 (V6)
// 64-bit rotate as two 32-bit funnel shifts (v_alignbit_b32 each): the plain
// (x >> n) | (x << 64-n) form compiles to two 64-bit shifts and two ORs.
EDV_HD uint32_t funnel32(uint32_t hi, uint32_t lo, int n) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_alignbit(hi, lo, n);  // opaque: keeps one v_alignbit_b32 per half
#else
  return uint32_t(((uint64_t(hi) << 32) | lo) >> n);
#endif
}
struct u32x2 { uint32_t lo, hi; };
EDV_HD uint64_t pack64(uint32_t lo, uint32_t hi) { return __builtin_bit_cast(uint64_t, u32x2{lo, hi}); }
EDV_HD uint64_t rotr64(uint64_t x, int n) {
  const u32x2 p = __builtin_bit_cast(u32x2, x);
  // rotr by n < 32: lo' = (hi:lo) >> n, hi' = (lo:hi) >> n; n >= 32 swaps the halves first
  if (n >= 32) return pack64(funnel32(p.lo, p.hi, n - 32), funnel32(p.hi, p.lo, n - 32));
  return pack64(funnel32(p.hi, p.lo, n), funnel32(p.lo, p.hi, n));
}

// A 64-bit value the optimizer cannot look into: a pair packed from two 32-bit
// halves is otherwise rewritten as zext(lo) + (hi << 32) and the two pieces are
// added separately into the round's 64-bit sums (two v_lshl_add_u64 and a
// v_mov_b32 more per use).
EDV_HD uint64_t opaque_u64(uint64_t x) {
#if defined(__HIP_DEVICE_COMPILE__)
  asm("" : "+v"(x));
#endif
  return x;
}
// Three-input bitwise functions as one v_bitop3_b32 per 32-bit half (gfx950):
// LLVM does not form bitop3 from the 64-bit expressions, which cost two
// v_xor_b32 per half for a three-way xor and four ops per half for Maj.  Both
// truth tables are symmetric in their inputs, so operand order cannot matter.
EDV_HD uint32_t xor3_32(uint32_t x, uint32_t y, uint32_t z) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_bitop3_b32(x, y, z, 0x96);
#else
  return x ^ y ^ z;
#endif
}
EDV_HD uint32_t maj32(uint32_t x, uint32_t y, uint32_t z) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_bitop3_b32(x, y, z, 0xE8);
#else
  return (x & y) ^ (x & z) ^ (y & z);
#endif
}
EDV_HD uint64_t xor3_64(uint64_t x, uint64_t y, uint64_t z) {
#if defined(__HIP_DEVICE_COMPILE__)
  const u32x2 a = __builtin_bit_cast(u32x2, x), b = __builtin_bit_cast(u32x2, y), c = __builtin_bit_cast(u32x2, z);
  return opaque_u64(pack64(__builtin_amdgcn_bitop3_b32(a.lo, b.lo, c.lo, 0x96),
                           __builtin_amdgcn_bitop3_b32(a.hi, b.hi, c.hi, 0x96)));
#else
  return x ^ y ^ z;
#endif
}
EDV_HD uint64_t maj64(uint64_t x, uint64_t y, uint64_t z) {
#if defined(__HIP_DEVICE_COMPILE__)
  const u32x2 a = __builtin_bit_cast(u32x2, x), b = __builtin_bit_cast(u32x2, y), c = __builtin_bit_cast(u32x2, z);
  return opaque_u64(pack64(__builtin_amdgcn_bitop3_b32(a.lo, b.lo, c.lo, 0xE8),
                           __builtin_amdgcn_bitop3_b32(a.hi, b.hi, c.hi, 0xE8)));
#else
  return (x & y) ^ (x & z) ^ (y & z);
#endif
}

EDV_HD void sha512_round(uint64_t& a, uint64_t& b, uint64_t& c, uint64_t& d, uint64_t& e, uint64_t& f, uint64_t& g,
                         uint64_t& h, uint64_t kw) {
  const uint64_t S1 = xor3_64(rotr64(e, 14), rotr64(e, 18), rotr64(e, 41));
  const uint64_t ch = (e & f) ^ (~e & g);
  const uint64_t t1 = h + S1 + ch + kw;
  const uint64_t S0 = xor3_64(rotr64(a, 28), rotr64(a, 34), rotr64(a, 39));
  const uint64_t mj = maj64(a, b, c);
  d += t1;
  h = t1 + S0 + mj;
}
// One compression.  Rounds run 16 at a time with the register rotation
// unrolled, so every W index is a compile-time constant (no dynamic register
// indexing) while the code stays one 16-round body.
EDV_HD void sha512_compress(uint64_t H[8], uint64_t W[16]) {
  const uint64_t K[80] = {
      0x428a2f98d728ae22ULL, 0x7137449123ef65cdULL, 0xb5c0fbcfec4d3b2fULL, 0xe9b5dba58189dbbcULL,
      0x3956c25bf348b538ULL, 0x59f111f1b605d019ULL, 0x923f82a4af194f9bULL, 0xab1c5ed5da6d8118ULL,
      0xd807aa98a3030242ULL, 0x12835b0145706fbeULL, 0x243185be4ee4b28cULL, 0x550c7dc3d5ffb4e2ULL,
      0x72be5d74f27b896fULL, 0x80deb1fe3b1696b1ULL, 0x9bdc06a725c71235ULL, 0xc19bf174cf692694ULL,
      0xe49b69c19ef14ad2ULL, 0xefbe4786384f25e3ULL, 0x0fc19dc68b8cd5b5ULL, 0x240ca1cc77ac9c65ULL,
      0x2de92c6f592b0275ULL, 0x4a7484aa6ea6e483ULL, 0x5cb0a9dcbd41fbd4ULL, 0x76f988da831153b5ULL,
      0x983e5152ee66dfabULL, 0xa831c66d2db43210ULL, 0xb00327c898fb213fULL, 0xbf597fc7beef0ee4ULL,
      0xc6e00bf33da88fc2ULL, 0xd5a79147930aa725ULL, 0x06ca6351e003826fULL, 0x142929670a0e6e70ULL,
      0x27b70a8546d22ffcULL, 0x2e1b21385c26c926ULL, 0x4d2c6dfc5ac42aedULL, 0x53380d139d95b3dfULL,
      0x650a73548baf63deULL, 0x766a0abb3c77b2a8ULL, 0x81c2c92e47edaee6ULL, 0x92722c851482353bULL,
      0xa2bfe8a14cf10364ULL, 0xa81a664bbc423001ULL, 0xc24b8b70d0f89791ULL, 0xc76c51a30654be30ULL,
      0xd192e819d6ef5218ULL, 0xd69906245565a910ULL, 0xf40e35855771202aULL, 0x106aa07032bbd1b8ULL,
      0x19a4c116b8d2d0c8ULL, 0x1e376c085141ab53ULL, 0x2748774cdf8eeb99ULL, 0x34b0bcb5e19b48a8ULL,
      0x391c0cb3c5c95a63ULL, 0x4ed8aa4ae3418acbULL, 0x5b9cca4f7763e373ULL, 0x682e6ff3d6b2b8a3ULL,
      0x748f82ee5defb2fcULL, 0x78a5636f43172f60ULL, 0x84c87814a1f0ab72ULL, 0x8cc702081a6439ecULL,
      0x90befffa23631e28ULL, 0xa4506cebde82bde9ULL, 0xbef9a3f7b2c67915ULL, 0xc67178f2e372532bULL,
      0xca273eceea26619cULL, 0xd186b8c721c0c207ULL, 0xeada7dd6cde0eb1eULL, 0xf57d4f7fee6ed178ULL,
      0x06f067aa72176fbaULL, 0x0a637dc5a2c898a6ULL, 0x113f9804bef90daeULL, 0x1b710b35131c471bULL,
      0x28db77f523047d84ULL, 0x32caab7b40c72493ULL, 0x3c9ebe0a15c9bebcULL, 0x431d67c49c100d4cULL,
      0x4cc5d4becb3e42b6ULL, 0x597f299cfc657e2aULL, 0x5fcb6fab3ad6faecULL, 0x6c44198c4a475817ULL};
  uint64_t a = H[0], b = H[1], c = H[2], d = H[3], e = H[4], f = H[5], g = H[6], h = H[7];
#pragma unroll 1
  for (int r = 0; r < 80; r += 16) {
    if (r > 0) {
#pragma unroll
      for (int t = 0; t < 16; t++) {
        const uint64_t w15 = W[(t + 1) & 15], w2 = W[(t + 14) & 15];
        const uint64_t s0 = xor3_64(rotr64(w15, 1), rotr64(w15, 8), opaque_u64(w15 >> 7));
        const uint64_t s1 = xor3_64(rotr64(w2, 19), rotr64(w2, 61), opaque_u64(w2 >> 6));
        W[t] += s0 + W[(t + 9) & 15] + s1;
      }
    }
    sha512_round(a, b, c, d, e, f, g, h, K[r + 0] + W[0]);
    sha512_round(h, a, b, c, d, e, f, g, K[r + 1] + W[1]);
    sha512_round(g, h, a, b, c, d, e, f, K[r + 2] + W[2]);
    sha512_round(f, g, h, a, b, c, d, e, K[r + 3] + W[3]);
    sha512_round(e, f, g, h, a, b, c, d, K[r + 4] + W[4]);
    sha512_round(d, e, f, g, h, a, b, c, K[r + 5] + W[5]);
    sha512_round(c, d, e, f, g, h, a, b, K[r + 6] + W[6]);
    sha512_round(b, c, d, e, f, g, h, a, K[r + 7] + W[7]);
    sha512_round(a, b, c, d, e, f, g, h, K[r + 8] + W[8]);
    sha512_round(h, a, b, c, d, e, f, g, K[r + 9] + W[9]);
    sha512_round(g, h, a, b, c, d, e, f, K[r + 10] + W[10]);
    sha512_round(f, g, h, a, b, c, d, e, K[r + 11] + W[11]);
    sha512_round(e, f, g, h, a, b, c, d, K[r + 12] + W[12]);
    sha512_round(d, e, f, g, h, a, b, c, K[r + 13] + W[13]);
    sha512_round(c, d, e, f, g, h, a, b, K[r + 14] + W[14]);
    sha512_round(b, c, d, e, f, g, h, a, K[r + 15] + W[15]);
  }
  H[0] += a; H[1] += b; H[2] += c; H[3] += d; H[4] += e; H[5] += f; H[6] += g; H[7] += h;
}

EDV_HD uint32_t bswap32(uint32_t x) {
  return (x >> 24) | ((x >> 8) & 0xff00u) | ((x << 8) & 0xff0000u) | (x << 24);
}
// two LE words (bytes b0..b7) -> big-endian 64-bit word
EDV_HD uint64_t be64_from_le_words(uint32_t lo, uint32_t hi) {
  return (uint64_t(bswap32(lo)) << 32) | bswap32(hi);
}

}  // namespace edv
