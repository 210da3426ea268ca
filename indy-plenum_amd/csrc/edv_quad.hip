// edv_quad.hip -- the latency path: one kernel launch verifies a small batch
// (a Node's prod, a single Verifier.verify) with several lanes per signature:
// edv_rtl_kernel (sixteen lanes, no tables, at most 4,096 requests: below) and
// edv_quad_kernel (eight lanes, per-signature tables, up to 16,384 requests),
// described first.
//
// The batch path (edv_prep.hip, edv_verify.hip) runs one signature per lane:
// best for throughput, but a lane's serial chain -- two exponentiations, ~130
// doublings, ~70 additions, every field product one after the other -- sets
// the latency of any batch that leaves most of the chip idle (~0.55 ms of
// kernels for n <= 16k: one wave per SIMD at most).  Here a 256-thread
// workgroup takes 32 signatures:
//
//   phase 1  wave-specialised (uniform within a wave, so no divergence):
//              wave 0: V2-V4 byte checks, V6/V7 h = SHA-512(R || A || M) mod L,
//                      the half-size scalars (a, b) and their digits
//              wave 1: canonical / small-order checks, decompress -A
//              wave 2: the same for R
//              wave 3: [S]B from the shared tables (from identity)
//            results through LDS, then one barrier;
//   phase 2  per signature two quads (4 consecutive lanes each): quad 0 builds
//            the 0..8 x (-A) table, quad 1 computes Q = [S]B - R and builds
//            0..8 x Q, in global scratch;
//   phase 3  quad 0 walks [a](-A), quad 1 walks [b](+-Q) -- the batch path's
//            fixed signed 4-bit windows, split into the
//            two scalars' walks -- then [a](-A) == -[b](+-Q) projectively.
//
// Quad arithmetic.  A point is DISTRIBUTED: lane q of a quad holds coordinate
// q of (X : Y : Z : T).  The extended-coordinate formulas have four
// independent field products per stage, so each lane computes one: a doubling
// is two product latencies (X^2 | Y^2 | 2Z^2 | (X+Y)^2, then X1 T1 | Y1 Z1 |
// Z1 T1 | X1 Y1) instead of seven, an addition two instead of eight.  The
// operands a lane needs are gathered from its quad with DPP quad_perm moves
// (v_mov_b32_dpp / DPP-modified VOP2 adds: the exchange costs a few VOP2 per
// limb, no LDS); per-lane signs and selects are mask arithmetic and v_bfi_b32
// (no VCC-mask v_cndmask_b32, ~23 cycles on gfx950).  A table entry is read
// one coordinate per lane (48-byte slots): the digit's sign picks which slot
// (YpX <-> YmX) and negates T2d, so no data is selected after the load.
//
// Same verdicts as the batch path (same strictness checks, same lattice
// scalars, same windows), checked against libsodium's golden and corpus
// verdicts by the GPU tests; the field arithmetic is edv_math.h's.
#define EDV_NO_SCHED_FENCE 1
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "edv_kernels.h"
#include "edv_launch.h"

namespace edv {
namespace {

constexpr int kQSigs = 32;                           // signatures per 256-thread workgroup (8 lanes each)
constexpr int kQCoordWords = 12;                     // one coordinate of a table entry, padded to 48 B
constexpr int kQEntryWords = 4 * kQCoordWords;       // YpX | YmX | T2d | Z
constexpr int kQTableWords = kAEntries * kQEntryWords;
static_assert(kQSigWords == 2 * kQTableWords, "edv_kernels.h kQSigWords: tables of -A and Q per signature");

// ------------------------------------------------------------ quad helpers
constexpr int qp(int a, int b, int c, int d) { return a | (b << 2) | (c << 4) | (d << 6); }
template <int C>
__device__ __forceinline__ int32_t dpp(int32_t x) {
  return __builtin_amdgcn_mov_dpp(x, C, 0xf, 0xf, true);
}
template <int C>
__device__ __forceinline__ fe fdpp(const fe& f) {
  fe r;
#pragma unroll
  for (int i = 0; i < 10; i++) r.v[i] = dpp<C>(f.v[i]);
  return r;
}
__device__ __forceinline__ fe fand(const fe& f, int32_t m) {
  fe r;
#pragma unroll
  for (int i = 0; i < 10; i++) r.v[i] = f.v[i] & m;
  return r;
}
// s = 0: f; s = -1: -f
__device__ __forceinline__ fe fcneg(const fe& f, int32_t s) {
  fe r;
#pragma unroll
  for (int i = 0; i < 10; i++) r.v[i] = (f.v[i] ^ s) - s;
  return r;
}
// m = -1: a; m = 0: b -- one v_bfi_b32 per limb (LLVM makes the AND / OR
// form two instructions: v_and_b32 + v_and_or_b32)
__device__ __forceinline__ int32_t bfi(int32_t m, int32_t a, int32_t b) {
  int32_t r;
  asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(r) : "v"(m), "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ fe fsel(int32_t m, const fe& a, const fe& b) {
  fe r;
#pragma unroll
  for (int i = 0; i < 10; i++) r.v[i] = bfi(m, a.v[i], b.v[i]);
  return r;
}
__device__ __forceinline__ fe fshl(const fe& f, int32_t sh) {
  fe r;
#pragma unroll
  for (int i = 0; i < 10; i++) r.v[i] = f.v[i] << sh;
  return r;
}

// Per-lane constants of a quad (opaque, so LLVM keeps them as mask arithmetic)
struct QLane {
  int32_t q;           // lane within the quad
  int32_t m1, m2, m3;  // all ones on lane 1 / 2 / 3
  int32_t m01;         // all ones on lanes 0 and 1
  int32_t m13;         // all ones on lanes 1 and 3
  int32_t s1;          // -1 on lane 1
  int32_t s03, s02;    // -1 on lanes 0, 3 / lanes 0, 2
  int32_t sh2, sh3;    // 1 on lane 2 / lane 3 (shift amounts)
  __device__ explicit QLane(int lane) {
    q = lane & 3;
    m1 = opaque_i32(-int32_t(q == 1));
    m2 = opaque_i32(-int32_t(q == 2));
    m3 = opaque_i32(-int32_t(q == 3));
    m01 = opaque_i32(-int32_t(q < 2));
    m13 = opaque_i32(-int32_t(q & 1));
    s1 = m1;
    s03 = opaque_i32(-int32_t(q == 0 || q == 3));
    s02 = opaque_i32(-int32_t(q == 0 || q == 2));
    sh2 = opaque_i32(int32_t(q == 2));
    sh3 = opaque_i32(int32_t(q == 3));
  }
};

// f^2, doubled on lanes where sh = 1 (2 Z^2 for the doubling's lane 2): the
// unbiased columns are shifted before the rounding bias goes in, so the one
// biased carry chain reduces either (output bounds of fe_sq)
__device__ __forceinline__ fe fe_sq_shift(const fe& f, int32_t sh) {
  int64_t h[10];
  fe_sq_cols<false, false>(f, h);
#pragma unroll
  for (int k = 0; k < 10; k++) {
    // (h << sh) + bias in one v_lshl_add_u64 (its shift may be a VGPR, low 3 bits)
    int64_t r;
    asm("v_lshl_add_u64 %0, %1, %2, %3" : "=v"(r) : "v"(h[k]), "v"(sh), "v"(bias_reg(k)));
    h[k] = r;
  }
  return fe_carry64_biased(h[0], h[1], h[2], h[3], h[4], h[5], h[6], h[7], h[8], h[9]);
}

// Doubling of a distributed point (dbl-2008-hwcd, a = -1), T ignored on
// input, all four of X3 Y3 Z3 T3 out.
__device__ __forceinline__ fe quad_dbl(const fe& p, const QLane& L) {
  // stage A: X^2 | Y^2 | 2 Z^2 | (X + Y)^2
  const fe y3 = fand(fdpp<qp(1, 1, 1, 1)>(p), L.m3);   // Y on lane 3
  const fe u = fe_add(fdpp<qp(0, 1, 2, 0)>(p), y3);     // X | Y | Z | X + Y
  const fe r = fe_sq_shift(u, L.sh2);
  // stage B: Y1 = YY + XX, Z1 = YY - XX, X1 = A - Y1, T1 = B - Z1
  const fe a0 = fdpp<qp(0, 0, 0, 0)>(r), a1 = fdpp<qp(1, 1, 1, 1)>(r);
  const fe S = fe_add(a1, a0), D = fe_sub(a1, a0);
  const fe X1 = fe_sub(fdpp<qp(3, 3, 3, 3)>(r), S);
  const fe T1 = fe_sub(fdpp<qp(2, 2, 2, 2)>(r), D);
  const fe uu = fsel(L.m1, S, fsel(L.m2, D, X1));  // X1 | Y1 | Z1 | X1
  const fe vv = fsel(L.m1, D, fsel(L.m3, S, T1));  // T1 | Z1 | T1 | Y1
  return fe_mul(uu, vv);                           // X3 | Y3 | Z3 | T3
}

// Addition of a distributed point and one cached-form coordinate per lane
// (e: YpX | YmX | T2d | Z of the addend, already negated if need be).
__device__ __forceinline__ fe quad_add(const fe& p, const fe& e, const QLane& L) {
  // stage A: A = (Y+X) YpX | B = (Y-X) YmX | C = T T2d | ZZ = Z Z'
  const fe x = fcneg(fand(fdpp<qp(0, 0, 0, 0)>(p), L.m01), L.s1);  // X | -X | 0 | 0
  const fe u = fe_add(fdpp<qp(1, 1, 3, 2)>(p), x);                   // Y+X | Y-X | T | Z
  const fe r = fshl(fe_mul(u, e), L.sh3);                            // A | B | C | D = 2 ZZ
  // stage B: X1 = A - B, Y1 = A + B, Z1 = D + C, T1 = D - C
  const fe uu = fe_add(fdpp<qp(0, 0, 3, 0)>(r), fcneg(fdpp<qp(1, 1, 2, 1)>(r), L.s03));  // X1 | Y1 | Z1 | X1
  const fe vv = fe_add(fdpp<qp(3, 3, 3, 0)>(r), fcneg(fdpp<qp(2, 2, 2, 1)>(r), L.s02));  // T1 | Z1 | T1 | Y1
  return fe_mul(uu, vv);                                                                  // X3 | Y3 | Z3 | T3
}

// Cached form of a distributed point, one coordinate per lane:
// YpX | YmX | T2d | Z (the table slot order, quad_add's e)
__device__ __forceinline__ fe quad_cached(const fe& p, const QLane& L) {
  const fe x = fcneg(fand(fdpp<qp(0, 0, 0, 0)>(p), L.m01), L.s1);
  const fe w = fe_add(fdpp<qp(1, 1, 3, 2)>(p), x);  // Y+X | Y-X | T | Z
  return fe_mul(w, fsel(L.m2, fe_d2(), fe_one()));  // x 1 | x 1 | x 2d | x 1
}

// the lane's coordinate of a table entry: 10 limbs at a 48-byte slot
__device__ __forceinline__ void slot_store(int32_t* s, const fe& f) {
  int4* p = reinterpret_cast<int4*>(s);
  p[0] = make_int4(f.v[0], f.v[1], f.v[2], f.v[3]);
  p[1] = make_int4(f.v[4], f.v[5], f.v[6], f.v[7]);
  p[2] = make_int4(f.v[8], f.v[9], 0, 0);
}
__device__ __forceinline__ fe slot_load(const int32_t* s) {
  const int4* p = reinterpret_cast<const int4*>(s);
  const int4 a = p[0], b = p[1], c = p[2];
  return fe{{a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w, c.x, c.y}};
}

// ------------------------------------------------------------ LDS layout
// per workgroup: phase-1 results for its 32 signatures (structure of arrays:
// word w of signature j at [w][j]), and wave 3's [S]B staging slice
constexpr int kQDigWords = 17;  // da[8] | db[8] | nwin | negR << 8
constexpr int kQPtWords = 40;   // X | Y | Z | T, 10 limbs each
struct QuadLds {
  uint32_t dig[kQDigWords][kQSigs];
  int32_t pt[3][kQPtWords][kQSigs];  // 0: -A, 1: -R, 2: [S]B
  uint8_t ok[3][kQSigs];              // hash side, A, R
  int32_t stage[kLdsBWaveWords];      // wave 3: LdsBStage slice
};

template <class Lds>
__device__ __forceinline__ void lds_put_point(Lds& L, int k, int j, const ge_p3& p) {
#pragma unroll
  for (int i = 0; i < 10; i++) {
    L.pt[k][i][j] = p.X.v[i];
    L.pt[k][10 + i][j] = p.Y.v[i];
    L.pt[k][20 + i][j] = p.Z.v[i];
    L.pt[k][30 + i][j] = p.T.v[i];
  }
}
// coordinate q of a point stored [word][signature] (X | Y | Z | T, 10 limbs
// each): the quad's distributed form of signature j
template <int S>
__device__ __forceinline__ fe coord_get(const int32_t (&pt)[kQPtWords][S], int j, int q) {
  fe f;
#pragma unroll
  for (int i = 0; i < 10; i++) f.v[i] = pt[10 * q + i][j];
  return f;
}
template <int S>
__device__ __forceinline__ void coord_put(int32_t (&pt)[kQPtWords][S], int j, int q, const fe& f) {
#pragma unroll
  for (int i = 0; i < 10; i++) pt[10 * q + i][j] = f.v[i];
}
template <class Lds>
__device__ __forceinline__ fe lds_coord(const Lds& L, int k, int j, int q) {
  return coord_get(L.pt[k], j, q);
}

// [S]B from identity (wave 3 of phase 1)
template <int BITS>
__device__ __forceinline__ ge_p3 sb_point(const uint32_t S[8], const int32_t* btab, int32_t* stage, int lane) {
  LdsBStage<BITS> bs{btab, stage, lane};
  ge_p3 q = ge_p3_identity();
  add_sb(q, S, bs);
  return q;
}

// A batch of fewer than kQMinLive requests is worked as if it had kQMinLive:
// the slots past its end repeat its last request (no verdict is written for
// them).  Measured on MI355X (profiles/r06/quad_sizes_s8.csv): with at most 8
// live signatures the kernel took 290-360 us on most launches (236 us on one
// or two of every eight consecutive dispatches), with 12 or more it took
// 232-240 us on every launch, for the same per-signature work -- an effect of
// how little of the chip such a launch keeps busy, not of the code path; the
// padding costs nothing measurable (the extra lanes are idle otherwise).
constexpr uint64_t kQMinLive = 16;

// ---- phase 1 of both latency kernels: one role per wave (uniform, so no
// divergence), one signature per lane (lanes 0 .. NS - 1); results into L.dig,
// L.pt and L.ok for the later phases (one barrier after it)
template <int BITS, int NS, class Lds>
__device__ __forceinline__ void phase1(const VerifyArgs& a, Lds& L, uint64_t g0, int wave, int lane) {
  if (lane < NS) {
    const uint64_t jl = g0 + uint64_t(lane);
    const bool in = jl < a.n || jl < kQMinLive;         // worked: a request, or padding of a tiny batch
    const uint64_t j = jl < a.n ? jl : a.n - 1;           // padding repeats the last request
    const uint64_t i = a.base + (in ? j : 0);
    if (wave == 0) {
      bool ok = false;
      PrepDigits pd;
      if (in) {
        uint32_t R[8], S[8], A[8];
        load_words(R, a.sigs + 16 * i, 2);
        load_words(S, a.sigs + 16 * i + 8, 2);
        load_words(A, a.pks + 8 * i, 2);
        const uint64_t o0 = a.off[i] - a.msg_base, o1 = a.off[i + 1] - a.msg_base;
        ok = prep_one(R, S, A, a.msgs + o0, o1 - o0, pd);
      }
#pragma unroll
      for (int k = 0; k < 8; k++) {
        L.dig[k][lane] = ok ? pd.da[k] : 0u;
        L.dig[8 + k][lane] = ok ? pd.db[k] : 0u;
      }
      L.dig[16][lane] = ok ? (uint32_t(pd.nwin) | (pd.negR ? 0x100u : 0u)) : 0u;
      L.ok[0][lane] = ok ? 1 : 0;
    } else if (wave == 1 || wave == 2) {
      uint32_t P[8];
      bool ok = false;
      ge_p3 p = ge_p3_identity();
      if (in) {
        load_words(P, wave == 1 ? a.pks + 8 * i : a.sigs + 16 * i, 2);
        ok = ge_is_canonical(P) && !has_small_order(P) && ge_frombytes_negate(p, P);
        if (!ok) p = ge_p3_identity();
      }
      lds_put_point(L, wave - 1, lane, p);
      L.ok[wave][lane] = ok ? 1 : 0;
    } else {
      uint32_t S[8];
      ge_p3 p = ge_p3_identity();
      if (in) {
        load_words(S, a.sigs + 16 * i + 8, 2);
        p = sb_point<BITS>(S, a.btab, L.stage, lane);
      }
      lds_put_point(L, 2, lane, p);
    }
  }
}

// The latency-path kernel: workgroup g verifies requests base + 32 g .. + 31,
// eight lanes per signature from phase 2 on: two quads, h = 0 walking
// [a](-A) and h = 1 walking [b](+-Q), so each window is four doublings and ONE
// addition per quad (the joint walk of the batch path adds both entries to one
// accumulator: two additions in a row), and each quad builds one table.  The
// verdict is [a](-A) == -[b](+-Q), compared projectively at the end.
template <int BITS>
__device__ __forceinline__ void quad_body(const VerifyArgs& a, int32_t* qtab, QuadLds& L) {
  const int tid = int(threadIdx.x), wave = tid >> 6, lane = tid & 63;
  const uint64_t g0 = uint64_t(blockIdx.x) * kQSigs;
  phase1<BITS, kQSigs>(a, L, g0, wave, lane);
  __syncthreads();
  // ---- phases 2 and 3: signature js, its quad h
  const QLane Q(lane);
  const int js = tid >> 3, h = (tid >> 2) & 1;
  const uint64_t j = g0 + uint64_t(js);
  const bool in = j < a.n;                              // a verdict to write
  const bool alive = (in || j < kQMinLive) && L.ok[0][js] && L.ok[1][js] && L.ok[2][js];
  int32_t* tab = qtab + uint64_t(blockIdx.x * kQSigs + js) * kQSigWords + h * kQTableWords;  // this quad's table
  {
    // identity entry: YpX = 1, YmX = 1, T2d = 0, Z = 1
    fe id = fe_zero();
    id.v[0] = Q.q == 2 ? 0 : 1;
    slot_store(tab + Q.q * kQCoordWords, id);
  }
  // the quad's point: h = 0: -A (plus the identity: the same code in both quads,
  // no divergence); h = 1: Q = [S]B + (-R); then its table 1..8 x point
  {
    fe idc = fe_zero();
    idc.v[0] = Q.q == 2 ? 0 : 1;
    const fe cr = quad_cached(lds_coord(L, 1, js, Q.q), Q);  // cached(-R)
    const int32_t mh = opaque_i32(-int32_t(h));
    const fe p = quad_add(lds_coord(L, h ? 2 : 0, js, Q.q), fsel(mh, cr, idc), Q);
    const fe e1 = quad_cached(p, Q);
    slot_store(tab + kQEntryWords + Q.q * kQCoordWords, e1);
    fe cur = quad_dbl(p, Q);
#pragma unroll 1
    for (int e = 2; e < kAEntries; e++) {
      if (e > 2) cur = quad_add(cur, e1, Q);
      slot_store(tab + e * kQEntryWords + Q.q * kQCoordWords, quad_cached(cur, Q));
    }
  }
  // the table was written by the quad's lanes: make it visible to their
  // neighbours (the walk reads the slot its digit's sign selects)
  __syncthreads();
  // ---- phase 3: this quad's walk, window count = the wave's maximum
  uint32_t d[8];
#pragma unroll
  for (int k = 0; k < 8; k++) d[k] = L.dig[8 * h + k][js];  // a (h = 0) or |b| (h = 1)
  const uint32_t wf = alive ? L.dig[16][js] : 0u;
  int nwin = int(wf & 0xff);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) nwin = max(nwin, __shfl_xor(nwin, o));
  nwin = __builtin_amdgcn_readfirstlane(nwin);
  const bool flip = h == 1 && ((wf >> 8) & 1);  // b < 0: the Q walk's digits are negated
  constexpr int kTop = kAWin * (kAWindows - 1);
  constexpr int kTopShl = 32 - kAWin - (kTop - 224);
#pragma unroll 1
  for (int k = nwin; k < kAWindows; k++) shl256<kAWin>(d);
  // identity, distributed: X = 0 | Y = 1 | Z = 1 | T = 0
  fe acc = fe_zero();
  acc.v[0] = (Q.q == 1 || Q.q == 2) ? 1 : 0;
#pragma unroll 1
  for (int w = nwin - 1; w >= 0; --w) {
    const int dg = int32_t(d[7] << kTopShl) >> (32 - kAWin);
    shl256<kAWin>(d);
    // this lane's slot of the entry: YpX and YmX trade places for a negative
    // digit, and T2d is negated (below)
    const bool ng = (dg < 0) != flip;
    const int c = Q.q < 2 ? (Q.q ^ int(ng)) : Q.q;
    fe e = slot_load(tab + (dg < 0 ? -dg : dg) * kQEntryWords + c * kQCoordWords);
    if (w != nwin - 1) {
#pragma unroll 1
      for (int k = 0; k < kAWin; k++) acc = quad_dbl(acc, Q);
    }
    acc = quad_add(acc, fcneg(e, opaque_i32(-int32_t(ng && Q.q == 2))), Q);
  }
  // Pa + Pb == identity  <=>  Xa Zb = -Xb Za  and  Ya Zb = Yb Za  (own = this
  // quad's point, other = the partner quad's, 4 lanes away; symmetric)
  fe other;
#pragma unroll
  for (int i = 0; i < 10; i++) other.v[i] = __shfl_xor(acc.v[i], 4);
  const fe u = fsel(Q.m13, fdpp<qp(0, 0, 1, 1)>(other), fdpp<qp(0, 0, 1, 1)>(acc));   // Xa | Xb | Ya | Yb
  const fe v = fsel(Q.m13, fdpp<qp(2, 2, 2, 2)>(acc), fdpp<qp(2, 2, 2, 2)>(other));   // Zb | Za | Zb | Za
  const fe r = fe_mul(u, v);
  const fe w2 = fe_add(r, fcneg(fdpp<qp(1, 1, 3, 3)>(r), Q.m2));                      // lane 0: XaZb + XbZa, lane 2: YaZb - YbZa
  const int32_t z = fe_iszero(w2) ? 1 : 0;
  const int32_t ok = dpp<qp(0, 0, 0, 0)>(z) & dpp<qp(2, 2, 2, 2)>(z);
  if (in && h == 0 && Q.q == 0) a.accept[a.base + j] = (alive && ok) ? 1 : 0;
}

// ------------------------------------------------ the right-to-left kernel
// For batches of at most kRtlMax requests: sixteen lanes per signature, four
// waves with one role each from phase 2 on, and no tables.  [a]P = sum_j d_j
// 16^j P (signed 4-bit digits from the least significant end): a DOUBLER wave
// runs the chain P, 16 P, 16^2 P, ... (four distributed doublings per window,
// the walk's whole serial part, started as soon as phase 1 has P) and
// publishes each 16^j P in LDS; an ADDER wave adds +-16^j P into bucket |d_j|
// (bucket 0 takes the zero digits), one cached addition per window, beside the
// doubler's next four doublings; at the end sum_d d B_d = sum_k T_k with the
// running sums T_k = B_8 + ... + B_k, the doubler forming T_k while the adder
// adds up the T's one step behind.  Waves 1 (doubler) and 0 (adder) walk
// [a](-A), waves 2 and 3 walk [b](+-Q) with Q = [S]B - R; the verdict is
// [a](-A) == -[b](+-Q), projectively.  The doubler and the adder of a walk
// meet through two LDS counters, not barriers: the doubler publishes 16^j P
// into slot j % kRing and then its count (release), the adder waits for the
// count (acquire), reads the slot and then advances its own count, which the
// doubler checks before reusing a slot kRing windows later; the adder, with
// ~half the doubler's work per window, is almost never waited for.  Measured
// on MI355X (profiles/r06/rtl_kernel.txt): 174-187 us a launch (box to box)
// against 198-214 us for edv_quad_kernel; the same code with one barrier per
// window instead of the counters: +10 us.
constexpr int kRSigs = 16;                 // signatures per 256-thread workgroup
constexpr int kRing = 4;                   // published points in flight per walk
struct RtlLds {
  uint32_t dig[kQDigWords][kRSigs];
  int32_t pt[3][kQPtWords][kRSigs];        // phase 1: -A, -R, [S]B
  uint8_t ok[3][kRSigs];
  int32_t pub[2][kRing][kQPtWords][kRSigs];  // [walk][slot]: the doubler's 16^j P in slot j % kRing (then running sums)
  int32_t published[2];                    // [walk]: points published so far (the doubler's count)
  int32_t consumed[2];                     // [walk]: points the adder has read
  int32_t buckets_done[2];                 // [walk]: the adder's last bucket write is visible
  int32_t bkt[2][kAEntries][kQPtWords][kRSigs];  // [walk][|digit|]: bucket sums, extended
  int32_t res[kQPtWords][kRSigs];          // the [b](+-Q) walk's result for the final check
  int32_t stage[kLdsBWaveWords];           // wave 3 of phase 1: [S]B staging
  // pads the allocation above half a CU's 160 KiB: one workgroup per CU, so
  // each role wave has a SIMD of its own (kRtlMax requests fill 256 CUs)
  int32_t pad[1024];
};
static_assert(sizeof(RtlLds) > 80 * 1024, "one workgroup per CU");

__device__ __forceinline__ int lds_acquire(const int32_t* c) {
  return __hip_atomic_load(c, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_release(int32_t* c, int v) {
  __hip_atomic_store(c, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
// spin (with a short sleep) until *c >= v; every lane of the wave reads the same count
__device__ __forceinline__ void lds_wait_ge(const int32_t* c, int v) {
  while (lds_acquire(c) < v) __builtin_amdgcn_s_sleep(1);
}

__device__ __forceinline__ fe quad_identity(const QLane& L) {
  fe f = fe_zero();
  f.v[0] = (L.q == 1 || L.q == 2) ? 1 : 0;  // X = 0 | Y = 1 | Z = 1 | T = 0
  return f;
}
// the cached form of +-P (YpX | YmX | T2d | Z): for -P, YpX and YmX trade
// places and T2d changes sign
__device__ __forceinline__ fe quad_cached_signed(const fe& p, int32_t neg, const QLane& L) {
  const fe c = quad_cached(p, L);
  const fe sw = fsel(neg & L.m01, fdpp<qp(1, 0, 2, 3)>(c), c);
  return fcneg(sw, neg & L.m2);
}

template <int BITS>
__device__ __forceinline__ void rtl_body(const VerifyArgs& a, RtlLds& L) {
  const int tid = int(threadIdx.x), wave = tid >> 6, lane = tid & 63;
  const uint64_t g0 = uint64_t(blockIdx.x) * kRSigs;
  phase1<BITS, kRSigs>(a, L, g0, wave, lane);
  __syncthreads();
  const QLane Q(lane);
  const int js = lane >> 2;                     // every wave: 16 signatures x 4 lanes
  const uint64_t j = g0 + uint64_t(js);
  const bool in = j < a.n;                      // a verdict to write
  const bool alive = (in || j < kQMinLive) && L.ok[0][js] && L.ok[1][js] && L.ok[2][js];
  const int walk = (wave == 2 || wave == 3) ? 1 : 0;
  const bool doubler = wave == 1 || wave == 2;
  const uint32_t wf = alive ? L.dig[16][js] : 0u;
  // windows: the workgroup's maximum (all four waves run the same barriers)
  int nwin = int(wf & 0xff);
#pragma unroll
  for (int o = 32; o >= 4; o >>= 1) nwin = max(nwin, __shfl_xor(nwin, o));
  nwin = __builtin_amdgcn_readfirstlane(nwin);
  uint32_t d[8];
#pragma unroll
  for (int k = 0; k < 8; k++) d[k] = alive ? L.dig[8 * walk + k][js] : 0u;  // a, or |b|; dead: all zero
  const int32_t flip = opaque_i32(-int32_t(walk == 1 && ((wf >> 8) & 1)));  // b < 0: the digits' signs flip
  fe P;  // the doubler's 16^j P; the adder's sum at the end
  if (doubler) {
    if (walk == 0) {
      P = lds_coord(L, 0, js, Q.q);                                   // -A
    } else {
      const fe cr = quad_cached(lds_coord(L, 1, js, Q.q), Q);         // cached(-R)
      P = quad_add(lds_coord(L, 2, js, Q.q), cr, Q);                  // Q = [S]B - R
    }
  } else {
    const fe id = quad_identity(Q);
#pragma unroll 1
    for (int k = 0; k < kAEntries; k++) coord_put(L.bkt[walk][k], js, Q.q, id);
  }
  if (tid < 2) {
    L.published[tid] = 0;
    L.consumed[tid] = 0;
    L.buckets_done[tid] = 0;
  }
  __syncthreads();
  if (doubler) {
#pragma unroll 1
    for (int w = 0; w < nwin; w++) {
      if (w > 0) {
#pragma unroll 1
        for (int k = 0; k < kAWin; k++) P = quad_dbl(P, Q);
      }
      if (w >= kRing) lds_wait_ge(&L.consumed[walk], w - kRing + 1);  // slot w % kRing is free
      coord_put(L.pub[walk][w % kRing], js, Q.q, P);
      lds_release(&L.published[walk], w + 1);
    }
  } else {
#pragma unroll 1
    for (int w = 0; w < nwin; w++) {
      const int dg = int32_t(d[0] << (32 - kAWin)) >> (32 - kAWin);  // digit w, signed
      shr256<kAWin>(d);
      const int32_t ng = opaque_i32(-int32_t(dg < 0)) ^ flip;
      const int ad = dg < 0 ? -dg : dg;
      lds_wait_ge(&L.published[walk], w + 1);
      const fe pw = coord_get(L.pub[walk][w % kRing], js, Q.q);
      lds_release(&L.consumed[walk], w + 1);  // after the slot's reads (release waits for them)
      const fe e = quad_cached_signed(pw, ng, Q);
      coord_put(L.bkt[walk][ad], js, Q.q, quad_add(coord_get(L.bkt[walk][ad], js, Q.q), e, Q));
    }
    lds_release(&L.buckets_done[walk], 1);
  }
  // sum_d d B_d = sum_k T_k, T_k = B_8 + ... + B_(8 - k): the doubler forms the
  // T's from the finished buckets and publishes them as points nwin + k; the
  // adder adds them up as they come (the same two counters)
  constexpr int kTop = kAEntries - 1;
  if (doubler) {
    lds_wait_ge(&L.buckets_done[walk], 1);
#pragma unroll 1
    for (int k = 0; k < kTop; k++) {
      const fe b = coord_get(L.bkt[walk][kTop - k], js, Q.q);
      P = k == 0 ? b : quad_add(P, quad_cached(b, Q), Q);
      const int w = nwin + k;
      lds_wait_ge(&L.consumed[walk], w - kRing + 1);
      coord_put(L.pub[walk][w % kRing], js, Q.q, P);
      lds_release(&L.published[walk], w + 1);
    }
  } else {
#pragma unroll 1
    for (int k = 0; k < kTop; k++) {
      const int w = nwin + k;
      lds_wait_ge(&L.published[walk], w + 1);
      const fe t = coord_get(L.pub[walk][w % kRing], js, Q.q);
      lds_release(&L.consumed[walk], w + 1);
      P = k == 0 ? t : quad_add(P, quad_cached(t, Q), Q);
    }
  }
  if (wave == 3) coord_put(L.res, js, Q.q, P);
  __syncthreads();
  if (wave != 0) return;
  // [a](-A) + [b](+-Q) == identity  <=>  Xa Zb = -Xb Za  and  Ya Zb = Yb Za
  const fe other = coord_get(L.res, js, Q.q);
  const fe u = fsel(Q.m13, fdpp<qp(0, 0, 1, 1)>(other), fdpp<qp(0, 0, 1, 1)>(P));   // Xa | Xb | Ya | Yb
  const fe v = fsel(Q.m13, fdpp<qp(2, 2, 2, 2)>(P), fdpp<qp(2, 2, 2, 2)>(other));   // Zb | Za | Zb | Za
  const fe r = fe_mul(u, v);
  const fe w2 = fe_add(r, fcneg(fdpp<qp(1, 1, 3, 3)>(r), Q.m2));                     // lane 0: XaZb + XbZa, lane 2: YaZb - YbZa
  const int32_t z = fe_iszero(w2) ? 1 : 0;
  const int32_t ok = dpp<qp(0, 0, 0, 0)>(z) & dpp<qp(2, 2, 2, 2)>(z);
  if (in && Q.q == 0) a.accept[a.base + j] = (alive && ok) ? 1 : 0;
}

__global__ __launch_bounds__(256) void edv_rtl_kernel(VerifyArgs a) {
  __shared__ RtlLds lds;
  rtl_body<kBBits>(a, lds);
}
__global__ __launch_bounds__(256) void edv_rtl_kernel_compact(VerifyArgs a) {
  __shared__ RtlLds lds;
  rtl_body<kBBitsCompact>(a, lds);
}

__global__ __launch_bounds__(256) void edv_quad_kernel(VerifyArgs a, int32_t* qtab) {
  __shared__ QuadLds lds;
  quad_body<kBBits>(a, qtab, lds);
}
__global__ __launch_bounds__(256) void edv_quad_kernel_compact(VerifyArgs a, int32_t* qtab) {
  __shared__ QuadLds lds;
  quad_body<kBBitsCompact>(a, qtab, lds);
}

}  // namespace

hipError_t launch_rtl_kernel(hipStream_t s, const VerifyArgs& va) {
  const unsigned blocks = unsigned((va.n + kRSigs - 1) / kRSigs);
  if (va.sb.bits == kBBits) edv_rtl_kernel<<<dim3(blocks), dim3(256), 0, s>>>(va);
  else edv_rtl_kernel_compact<<<dim3(blocks), dim3(256), 0, s>>>(va);
  return hipGetLastError();
}

hipError_t launch_quad_kernel(hipStream_t s, const VerifyArgs& va, int32_t* qtab) {
  const unsigned blocks = unsigned((va.n + kQSigs - 1) / kQSigs);
  if (va.sb.bits == kBBits) edv_quad_kernel<<<dim3(blocks), dim3(256), 0, s>>>(va, qtab);
  else edv_quad_kernel_compact<<<dim3(blocks), dim3(256), 0, s>>>(va, qtab);
  return hipGetLastError();
}

}  // namespace edv
