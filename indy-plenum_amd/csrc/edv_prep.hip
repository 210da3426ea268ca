// edv_prep.hip -- the prep kernel (phase 1 of a chunk: SURVEY.md section 8a
// rows V2-V7 plus the half-size scalars and the per-signature point tables),
// in its own translation unit so it is compiled without the field
// arithmetic's scheduling fences (see edv_kernels.h).
#define EDV_NO_SCHED_FENCE 1
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "edv_kernels.h"

namespace edv {
namespace {

// Phase 1 in three independent sides, interleaved by workgroup (block b runs
// side side0 + b % nsides of slots [(b / nsides) 256, +256); all three by
// default, the split pipeline launches the hash side and the two point sides
// apart): 0 = V2-V4 checks, V6/V7 hash, half-size scalars and digits; 1 =
// decompress A, 0..8 x (-A) table; 2 = decompress R, Q = [S]B - R, 0..8 x Q
// table.  They share no data, so they run side by side (three waves per SIMD at
// 64k signatures where one kernel per side would leave one wave each to hide
// its own latencies), and the two exponentiations no longer sit behind the
// hash in one lane.

// The R side's view of the [S]B tables: stage() copies the lane's entry
// straight into the wave's 10 KiB LDS slice (global_load_lds_dwordx4, 64 lanes
// x 16 B per instruction), so the gather flies during the previous entry's
// addition without holding registers; fetch() waits and reads it back.  After
// the last entry the slice holds Q's cached form for the table (put / get).
constexpr int kBPieces = 8;         // 128-byte entry (30 words used)
constexpr int kStashPieces = 10;    // cached point, 160 B
__device__ __forceinline__ void wait_staged() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
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
    wait_staged();
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

template <int BITS>
__device__ __forceinline__ void prep_point_side(const VerifyArgs& a, uint64_t j, int side, int32_t* lds) {
  if (j >= a.n) return;
  const uint64_t i = a.base + (a.st.perm ? a.st.perm[j] : j);
  uint32_t P[8];
  bool ok;
  if (side == 1) {
    load_words(P, a.pks + 8 * i, 2);
    GlobalATab tab{a.st.atab + j * kAWords};
    ok = prep_point(P, tab);
  } else {
    uint32_t S[8];
    load_words(P, a.sigs + 16 * i, 2);
    load_words(S, a.sigs + 16 * i + 8, 2);
    GlobalATab tab{a.st.rtab + j * kAWords};
    LdsBStage<BITS> bs{a.btab, lds + (threadIdx.x >> 6) * kLdsBWaveWords, int(threadIdx.x & 63)};
    ok = prep_rpoint(P, S, tab, bs);
  }
  a.st.alive[side * a.st.cap + j] = ok ? 1 : 0;
  if (!ok) a.accept[i] = 0;
}
// The kernel body for table set BITS (one kernel per set, below).
template <int BITS>
__device__ __forceinline__ void prep_body(const VerifyArgs& a, int32_t* lds_b) {
  const uint32_t ns = uint32_t(a.nsides);
  const int side = a.side0 + int(blockIdx.x % ns);
  const uint64_t j = uint64_t(blockIdx.x / ns) * kBlock + threadIdx.x;  // slot within the chunk
  if (side != 0) {
    prep_point_side<BITS>(a, j, side, lds_b);
    return;
  }
  if (j >= a.n) return;
  const uint64_t i = a.base + (a.st.perm ? a.st.perm[j] : j);
  uint32_t R[8], S[8], A[8];
  load_words(R, a.sigs + 16 * i, 2);
  load_words(S, a.sigs + 16 * i + 8, 2);
  load_words(A, a.pks + 8 * i, 2);
  const uint64_t o0 = a.off[i] - a.msg_base, o1 = a.off[i + 1] - a.msg_base;
  PrepDigits pd;
  const bool ok = prep_one(R, S, A, a.msgs + o0, o1 - o0, pd);
  a.st.alive[j] = ok ? 1 : 0;
  if (ok) {
    uint32_t* d = a.st.dig + j;
    const uint64_t cap = a.st.cap;
#pragma unroll
    for (int k = 0; k < 8; k++) {
      d[uint64_t(k) * cap] = pd.da[k];
      d[uint64_t(8 + k) * cap] = pd.db[k];
    }
    d[uint64_t(kDigNwin) * cap] = uint32_t(pd.nwin) | (pd.negR ? 0x100u : 0u);
  } else {
    a.accept[i] = 0;
  }
}

// the register budget allows at least three waves per SIMD (the three sides);
// the R side's LDS staging, (kBlock / 64) * kLdsBWaveWords words, is dynamic
// shared memory that only launches running the R side reserve
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(3, 8))) void edv_prep_kernel(
    VerifyArgs a) {
  extern __shared__ int32_t lds_b[];
  prep_body<kBBits>(a, lds_b);
}
// the same against the compact [S]B tables (edv_verify_core.h SbShape)
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(3, 8))) void edv_prep_kernel_compact(
    VerifyArgs a) {
  extern __shared__ int32_t lds_b[];
  prep_body<kBBitsCompact>(a, lds_b);
}

}  // namespace

hipError_t launch_prep_kernel(unsigned grid, hipStream_t s, const VerifyArgs& va) {
  const bool rside = va.side0 + va.nsides > 2;  // sides side0 .. side0 + nsides - 1 include side 2
  const size_t lds = rside ? size_t(kBlock / 64) * kLdsBWaveWords * sizeof(int32_t) : 0;
  if (va.sb.bits == kBBits) edv_prep_kernel<<<dim3(grid), dim3(kBlock), lds, s>>>(va);
  else edv_prep_kernel_compact<<<dim3(grid), dim3(kBlock), lds, s>>>(va);
  return hipGetLastError();
}

}  // namespace edv
