// edv_kernels.h -- what the prep kernel (edv_prep.hip) and the main kernel and
// host runtime (edv_verify.hip) share: the per-chunk state layout, the kernel
// arguments, the per-signature table view used by the prep kernel, and the
// prep launch entry point.  Two translation units so the prep kernel is built
// without the scheduling fences of the field arithmetic (edv_math.h
// sched_fence): they keep the main kernel's registers in check, while the
// prep kernel's serial exponentiations and table chain run faster when LLVM
// may interleave independent products (measured: prep -7 %, main +3 % with
// the fences removed everywhere, profiles/r02/ab_fence_s23.jsonl).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "edv_verify_core.h"

namespace edv {

constexpr int kBlock = 256;
constexpr int kEntryWords = 40;           // cached point = 4 x 10 limbs, 160 B
constexpr int kAWords = kAEntries * kEntryWords;  // per-signature table (9 entries: 360 words = 1,440 B)
// dig words per signature: da (8), db (8), window count and sign (1)
constexpr int kDigWords = 8 + 8 + 1;
constexpr int kDigNwin = 16;
constexpr uint64_t kChunkDefault = uint64_t(1) << 18;  // signatures per prep/main launch pair
constexpr int kBuckets = 64;  // SHA-512 length buckets (block counts 0..62, 63 = 63 or more)
// the latency path (edv_quad.hip): per signature, tables 0..8 x (-A) and 0..8 x Q
// in global scratch, 4 coordinates x 12 words (48-byte slots) per entry
constexpr int kQSigWords = 2 * kAEntries * 4 * 12;

// Per-chunk state handed from the prep kernel to the main kernel, SoA so every
// wave-wide load/store touches 64 consecutive words:
//   atab[kAWords * i + w]  word w of signature i's 0..kAEntries-1 x (-A) table
//   rtab[kAWords * i + w]  the same for its 0..kAEntries-1 x ([S]B - R) table
//   dig[w * cap + i]   w 0..7: packed radix-2^kAWin digits of a, 8..15: of |b|,
//                      16: windows needed | (b < 0) << 8
//   alive[k cap + i]   1 if prep side k (0 hash, 1 A, 2 R) passed for slot i (the
//                      main kernel skips lanes where any side failed)
struct ChunkState {
  int32_t* atab;
  int32_t* rtab;
  uint32_t* dig;
  uint8_t* alive;
  uint64_t cap;
  const uint32_t* perm;   // slot j -> request base + perm[j] (length buckets); null = identity
};

struct VerifyArgs {
  const uint32_t* sigs;   // n x 16 words
  const uint32_t* pks;    // n x 8 words
  const uint8_t* msgs;
  const uint64_t* off;    // n + 1
  uint64_t msg_base;
  uint64_t base;          // first signature of this chunk
  uint64_t n;             // signatures in this chunk
  uint8_t* accept;        // indexed by global signature index
  ChunkState st;
  const int32_t* btab;    // sb.tables x sb.entries x kBStride (the prep kernel's R side)
  SbShape sb;             // which [S]B table set btab is (large or compact, edv_verify_core.h)
  // prep sides this launch runs: workgroup b runs side side0 + b % nsides
  // (0 hash, 1 A, 2 R); 0 / 3 = all three, 0 / 1 = the hash side, 1 / 2 = the points
  int32_t side0;
  int32_t nsides;
};

// Per-signature A table in HBM, signature-major: signature i's 360 words are
// contiguous at slot = atab + 360*i, so a lane's digit-dependent gather reads
// 160 contiguous bytes (10 x 16-byte loads) instead of touching one line per
// word for every distinct digit in the wave (the word-major layout measured
// 39 KB of L2-miss traffic per verify, 8x the useful bytes).
struct GlobalATab {
  int32_t* slot;
  // one entry = 40 contiguous words (160 B, 16-byte aligned): ten 16-byte stores.
  // (Packing an entry into 128 B -- four canonical 255-bit encodings, one line
  // per gather -- halved main's fabric reads but made the C2 step 3.4 % slower:
  // profiles/r05/ab_packed_s2.jsonl.)
  __device__ __forceinline__ void store(int e, const ge_cached& c) const {
    int32_t t[40];
#pragma unroll
    for (int l = 0; l < 10; l++) {
      t[l] = c.YpX.v[l]; t[10 + l] = c.YmX.v[l]; t[20 + l] = c.Z.v[l]; t[30 + l] = c.T2d.v[l];
    }
    int4* p = reinterpret_cast<int4*>(slot + e * kEntryWords);
#pragma unroll
    for (int q = 0; q < 10; q++) p[q] = make_int4(t[4 * q], t[4 * q + 1], t[4 * q + 2], t[4 * q + 3]);
  }
};
__device__ __forceinline__ void load_words(uint32_t* out, const uint32_t* p, int n4) {
  const uint4* q = reinterpret_cast<const uint4*>(p);
#pragma unroll
  for (int k = 0; k < n4; k++) {
    const uint4 v = q[k];
    out[4 * k] = v.x; out[4 * k + 1] = v.y; out[4 * k + 2] = v.z; out[4 * k + 3] = v.w;
  }
}

namespace {  // per translation unit (the prep kernel's codegen depends on it: +368 B of scratch otherwise)
// The R side's view of the [S]B tables: stage() copies the lane's entry
// straight into the wave's 10 KiB LDS slice (global_load_lds_dwordx4, 64 lanes
// x 16 B per instruction), so the gather flies during the previous entry's
// addition without holding registers; fetch() waits and reads it back.  After
// the last entry the slice holds Q's cached form for the table (put / get).
constexpr int kBPieces = 8;         // 128-byte entry (30 words used)
constexpr int kStashPieces = 10;    // cached point, 160 B
__device__ __forceinline__ void wait_vmem() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
__device__ __forceinline__ void wait_lds() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }
// BITS: the table set (a compile-time shape: with the shape read at run time
// the R side's loop kept ~90 more dwords spilled, prep +7 %)
template <int BITS>
struct LdsBStage {
  const int32_t* w;  // the shared tables
  int32_t* lds;      // the wave's slice: kStashPieces x 64 lanes x 4 words
  int lane;
  static constexpr SbShape kShape = BITS == kBBits ? sb_large() : sb_compact();
  __device__ __forceinline__ SbShape shape() const { return kShape; }
  __device__ __forceinline__ void stage(int t, int j) {
    const int32_t* g = w + (size_t(t) * kShape.entries + j) * kBStride;
#pragma unroll
    for (int q = 0; q < kBPieces; q++)
      __builtin_amdgcn_global_load_lds(const_cast<int32_t*>(g + 4 * q), lds + q * 256, 16, 0, 0);
  }
  __device__ __forceinline__ ge_precomp fetch() {
    wait_vmem();
    int32_t v[32];
#pragma unroll
    for (int q = 0; q < kBPieces; q++) {
      const int4 x = reinterpret_cast<const int4*>(lds + q * 256)[lane];
      v[4 * q] = x.x; v[4 * q + 1] = x.y; v[4 * q + 2] = x.z; v[4 * q + 3] = x.w;
    }
    wait_lds();  // the slice is restaged right after this: the reads must have landed
    return precomp_from_words(v);
  }
  __device__ __forceinline__ void put(const ge_cached& c) {
    int32_t v[40];
#pragma unroll
    for (int l = 0; l < 10; l++) { v[l] = c.YpX.v[l]; v[10 + l] = c.YmX.v[l]; v[20 + l] = c.Z.v[l]; v[30 + l] = c.T2d.v[l]; }
#pragma unroll
    for (int q = 0; q < kStashPieces; q++)
      reinterpret_cast<int4*>(lds + q * 256)[lane] = make_int4(v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]);
  }
  __device__ __forceinline__ ge_cached get() const {
    asm volatile("" ::: "memory");  // read at each use, not once ahead of the loop
    int32_t v[40];
#pragma unroll
    for (int q = 0; q < kStashPieces; q++) {
      const int4 x = reinterpret_cast<const int4*>(lds + q * 256)[lane];
      v[4 * q] = x.x; v[4 * q + 1] = x.y; v[4 * q + 2] = x.z; v[4 * q + 3] = x.w;
    }
    ge_cached c;
#pragma unroll
    for (int l = 0; l < 10; l++) { c.YpX.v[l] = v[l]; c.YmX.v[l] = v[10 + l]; c.Z.v[l] = v[20 + l]; c.T2d.v[l] = v[30 + l]; }
    return c;
  }
};
constexpr int kLdsBWaveWords = kStashPieces * 256;
}  // namespace

// Launches edv_prep_kernel (edv_prep.hip) over `grid` workgroups on stream s;
// the R side's LDS staging is dynamic shared memory, reserved only by launches
// that run the R side (a hash-side or A-side launch is not capped at four
// workgroups per CU by 40 KiB it never touches).
hipError_t launch_prep_kernel(unsigned grid, hipStream_t s, const VerifyArgs& va);

}  // namespace edv
