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
