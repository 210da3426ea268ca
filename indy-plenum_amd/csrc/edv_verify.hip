// edv_verify.hip -- the gfx950 kernels of libedv.so other than the prep kernel
// (edv_prep.hip), and their launch wrappers (edv_launch.h) for the host
// runtime and C-ABI in edv_runtime.hip.
//
// One signature per lane, 256-thread workgroups; a chunk of signatures is two
// launches (libsodium 1.0.18 semantics):
//   edv_prep_kernel (edv_prep.hip), three sides side by side:
//     hash side  V2-V4 byte predicates, V6/V7 h = SHA-512(R || A || M) mod L
//                straight from the caller's message buffer, the half-size
//                scalars (a, b) with a = b h (mod 8L), b odd, recoded into
//                fixed signed windows
//     A side     decompress -A (one sqrt exponentiation), 0..8 x (-A) table
//     R side     decompress -R, Q = [S]B - R (12 mixed additions against
//                shared 0..2^21 x 2^(22 t) B tables), 0..8 x Q table
//                (per-signature tables in cached form, HBM scratch)
//   edv_main_kernel (below): [a](-A) + [b]([S]B - R) == identity by one
//     joint walk of ~33 four-bit windows (FIXED windows, so all 64 lanes of a
//     wave stay in lock-step), table entries staged through LDS; no inversion.
//   DESIGN.md section 2 has the argument that this is libsodium's verdict.
// No MFMA: this is scalar bignum integer work (v_mad_i64_i32 chains).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "edv_verify_core.h"
#include "edv_kernels.h"
#include "edv_launch.h"
#include "edv_sha256.h"

using namespace edv;

namespace {

// ---------------------------------------------------------------- kernels
// The main kernel's views of the tables: stage() copies the entry a lane needs
// this window from global memory straight into the wave's LDS slice
// (global_load_lds_dwordx4: 64 lanes x 16 B per instruction, lane-linear), so
// nothing of it sits in registers during the window's doublings; fetch()
// waits for the copies and reads the lane's 16-byte pieces back.  Per wave:
// A 10 KiB + R 10 KiB = 20 KiB (80 KiB per 256-thread workgroup), so two
// 256-thread workgroups fit a CU (2 waves/SIMD once a chunk has more than one
// wave per SIMD).
constexpr int kEntryPieces = 10;  // one cached entry: 10 pieces of 64 lanes x 4 words
constexpr int kLdsAWords = kEntryPieces * 256;
constexpr int kLdsWaveWords = 2 * kLdsAWords;
__device__ __forceinline__ void wait_staged() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
struct LdsATab {
  const int32_t* slot;  // this lane's table in global memory
  int32_t* lds;         // the wave's LDS region for this table
  int lane;
  __device__ __forceinline__ void stage(int e) {
    const int32_t* g = slot + e * kEntryWords;
#pragma unroll
    for (int q = 0; q < kEntryPieces; q++)
      __builtin_amdgcn_global_load_lds(const_cast<int32_t*>(g + 4 * q), lds + q * 256, 16, 0, 0);
  }
  __device__ __forceinline__ ge_cached fetch() {
    wait_staged();
    int32_t t[4 * kEntryPieces];
#pragma unroll
    for (int q = 0; q < kEntryPieces; q++) {
      const int4 v = reinterpret_cast<const int4*>(lds + q * 256)[lane];
      t[4 * q] = v.x; t[4 * q + 1] = v.y; t[4 * q + 2] = v.z; t[4 * q + 3] = v.w;
    }
    ge_cached c;
#pragma unroll
    for (int l = 0; l < 10; l++) {
      c.YpX.v[l] = t[l]; c.YmX.v[l] = t[10 + l]; c.Z.v[l] = t[20 + l]; c.T2d.v[l] = t[30 + l];
    }
    return c;
  }
};
// Phase 2: V8 multi-scalar walk and the identity check.  The window count is
// the wave's maximum over its live lanes, so the loop stays wave-uniform.
// The main kernel's body, shared by edv_main_kernel and the split pipeline's
// edv_main_kernel_prio as a macro (text, not a function), so the plain kernel
// compiles exactly as it did alone: an inlined-function form measured 2 %
// slower at C2 (other register assignment; profiles/r04/ab_refactor_s11.jsonl).
// (In the body: the digit loads are settled once, through opaque_i32, before
// the window loop: the digit registers are shifted inside the loop, and the
// waitcnt pass, merging the loop's back edge with loads still pending from the
// preheader, otherwise inserts vmcnt waits at the loop head and right after
// the table stages.)
#define EDV_MAIN_BODY \
  const uint64_t j = uint64_t(blockIdx.x) * kBlock + threadIdx.x; \
  const bool live = j < a.n && a.st.alive[j] && a.st.alive[a.st.cap + j] && a.st.alive[2 * a.st.cap + j]; \
  const uint32_t* d = a.st.dig + j; \
  const uint64_t cap = a.st.cap; \
  const uint32_t wf = live ? d[uint64_t(kDigNwin) * cap] : 0; \
  int nwin = int(wf & 0xff); \
_Pragma("unroll") \
  for (int o = 32; o > 0; o >>= 1) nwin = max(nwin, __shfl_xor(nwin, o)); \
  nwin = __builtin_amdgcn_readfirstlane(nwin); \
  if (!live) return; \
  const uint64_t i = a.base + (a.st.perm ? a.st.perm[j] : j); \
  uint32_t da[8], db[8]; \
_Pragma("unroll") \
  for (int k = 0; k < 8; k++) { \
    da[k] = d[uint64_t(k) * cap]; \
    db[k] = d[uint64_t(8 + k) * cap]; \
  } \
_Pragma("unroll") \
  for (int k = 0; k < 8; k++) { \
    da[k] = uint32_t(opaque_i32(int32_t(da[k]))); \
    db[k] = uint32_t(opaque_i32(int32_t(db[k]))); \
  } \
  int32_t* wl = lds_main + (threadIdx.x >> 6) * kLdsWaveWords; \
  const int lane = int(threadIdx.x & 63); \
  LdsATab at{a.st.atab + j * kAWords, wl, lane}, rt{a.st.rtab + j * kAWords, wl + kLdsAWords, lane}; \
  a.accept[i] = main_one(da, db, nwin, (wf >> 8) & 1, at, rt) ? 1 : 0;

__global__ __launch_bounds__(kBlock) void edv_main_kernel(VerifyArgs a) {
  __shared__ int32_t lds_main[(kBlock / 64) * kLdsWaveWords];
  EDV_MAIN_BODY
}

// The split pipeline's main kernel (EDV_FLAG_SPLIT_PREP): the same walk at a
// raised issue priority, so the next batch's hash-side waves sharing its SIMDs
// (latency-bound SHA-512 chains) take the cycles it leaves, instead of
// round-robin turns; in the plain paths the raised priority only costs (C2
// sequential 0.698 against 0.678 ms, profiles/r04/ab_prio_s8.jsonl).
constexpr int kSplitMainPrio = 2;
__global__ __launch_bounds__(kBlock) void edv_main_kernel_prio(VerifyArgs a) {
  __shared__ int32_t lds_main[(kBlock / 64) * kLdsWaveWords];
  __builtin_amdgcn_s_setprio(kSplitMainPrio);
  EDV_MAIN_BODY
}

// Comb rows for the batch signer, in global memory (528 KB, L2-resident).
struct GlobalComb {
  const int32_t* w;
  __device__ __forceinline__ ge_precomp entry(int i, int j) const {
    const int4* p = reinterpret_cast<const int4*>(w + (i * kCombEntries + j) * kBStride);
    int32_t t[32];
#pragma unroll
    for (int k = 0; k < 8; k++) {
      const int4 v = p[k];
      t[4 * k] = v.x; t[4 * k + 1] = v.y; t[4 * k + 2] = v.z; t[4 * k + 3] = v.w;
    }
    return precomp_from_words(t);
  }
};

// Batch signer (row f-4: synthetic load generation): seeds -> (pk, sig) over M.
__global__ __launch_bounds__(kBlock) void edv_sign_kernel(const uint32_t* seeds, const uint8_t* msgs,
                                                          const uint64_t* off, uint64_t msg_base, uint64_t n,
                                                          uint32_t* pks, uint32_t* sigs, const int32_t* comb) {
  const uint64_t i = uint64_t(blockIdx.x) * kBlock + threadIdx.x;
  if (i >= n) return;
  uint32_t seed[8], pk[8], sig[16];
  load_words(seed, seeds + 8 * i, 2);
  const uint64_t o0 = off[i] - msg_base, o1 = off[i + 1] - msg_base;
  sign_one(pk, sig, seed, msgs + o0, o1 - o0, GlobalComb{comb});
  uint4* po = reinterpret_cast<uint4*>(pks + 8 * i);
  uint4* so = reinterpret_cast<uint4*>(sigs + 16 * i);
  po[0] = make_uint4(pk[0], pk[1], pk[2], pk[3]);
  po[1] = make_uint4(pk[4], pk[5], pk[6], pk[7]);
#pragma unroll
  for (int k = 0; k < 4; k++) so[k] = make_uint4(sig[4 * k], sig[4 * k + 1], sig[4 * k + 2], sig[4 * k + 3]);
}

__global__ void edv_comb_kernel(int32_t* out) {
  const int t = threadIdx.x + blockIdx.x * blockDim.x;
  if (t < kCombRows * kCombEntries) comb_entry(out + t * kBStride, t / kCombEntries, t % kCombEntries);
}

// ---- length buckets (config C4): group the chunk's requests by SHA-512 block
// count so every wave of the prep kernel runs the same number of compression
// rounds (a wave otherwise pays for its longest message).  Counting sort on
// min(blocks, 63): histogram, then scatter with per-bucket atomic cursors; a
// chunk whose requests all share one bucket keeps the identity order.
__device__ __forceinline__ uint32_t sha_bucket(const uint64_t* off, uint64_t i) {
  const uint64_t nb = (64 + (off[i + 1] - off[i]) + 17 + 127) / 128;
  return nb < kBuckets - 1 ? uint32_t(nb) : uint32_t(kBuckets - 1);
}
// Histogram: per-workgroup counts in LDS, then one global add per non-empty
// bucket per workgroup (a fixed-length batch would otherwise send every lane's
// atomic to the same word).
__global__ __launch_bounds__(kBlock) void edv_bucket_hist_kernel(const uint64_t* off, uint64_t base, uint64_t n,
                                                                 uint32_t* hist) {
  __shared__ uint32_t h[kBuckets];
  if (threadIdx.x < kBuckets) h[threadIdx.x] = 0;
  __syncthreads();
  const uint64_t j = uint64_t(blockIdx.x) * kBlock + threadIdx.x;
  if (j < n) atomicAdd(&h[sha_bucket(off, base + j)], 1u);
  __syncthreads();
  if (threadIdx.x < kBuckets && h[threadIdx.x]) atomicAdd(&hist[threadIdx.x], h[threadIdx.x]);
}
// Scatter: bucket start offsets from the global histogram; each workgroup
// reserves its range per bucket with one global add, then ranks its lanes
// within the range through LDS.
__global__ __launch_bounds__(kBlock) void edv_bucket_scatter_kernel(const uint64_t* off, uint64_t base, uint64_t n,
                                                                    const uint32_t* hist, uint32_t* cursor,
                                                                    uint32_t* perm) {
  __shared__ uint32_t start[kBuckets], cnt[kBuckets], wbase[kBuckets];
  __shared__ int nonempty;
  if (threadIdx.x == 0) {
    uint32_t acc = 0;
    int ne = 0;
    for (int b = 0; b < kBuckets; b++) { start[b] = acc; acc += hist[b]; ne += hist[b] != 0; }
    nonempty = ne;
  }
  if (threadIdx.x < kBuckets) cnt[threadIdx.x] = 0;
  __syncthreads();
  const uint64_t j = uint64_t(blockIdx.x) * kBlock + threadIdx.x;
  if (nonempty <= 1) {
    if (j < n) perm[j] = uint32_t(j);
    return;
  }
  uint32_t b = 0, rank = 0;
  if (j < n) {
    b = sha_bucket(off, base + j);
    rank = atomicAdd(&cnt[b], 1u);
  }
  __syncthreads();
  if (threadIdx.x < kBuckets && cnt[threadIdx.x])
    wbase[threadIdx.x] = start[threadIdx.x] + atomicAdd(&cursor[threadIdx.x], cnt[threadIdx.x]);
  __syncthreads();
  if (j < n) perm[wbase[b] + rank] = uint32_t(j);
}

// Accept bytes -> accept bitmask (bit i % 8 of byte i / 8, little-endian bit
// order): what a multi-GPU run gathers, N/8 bytes per shard.
// One output byte per thread, its eight accept bytes read as two words when
// they are whole.
__global__ __launch_bounds__(kBlock) void edv_pack_bits_kernel(const uint8_t* acc, uint64_t n, uint8_t* bits) {
  const uint64_t k = uint64_t(blockIdx.x) * kBlock + threadIdx.x;
  if (8 * k >= n) return;
  uint32_t b = 0;
  if (8 * k + 8 <= n && !(reinterpret_cast<uintptr_t>(acc) & 3)) {
    const uint32_t lo = reinterpret_cast<const uint32_t*>(acc)[2 * k], hi = reinterpret_cast<const uint32_t*>(acc)[2 * k + 1];
#pragma unroll
    for (int t = 0; t < 4; t++) b |= (((lo >> (8 * t)) & 0xff) != 0 ? 1u : 0u) << t;
#pragma unroll
    for (int t = 0; t < 4; t++) b |= (((hi >> (8 * t)) & 0xff) != 0 ? 1u : 0u) << (4 + t);
  } else {
    for (uint64_t i = 8 * k; i < n && i < 8 * k + 8; i++) b |= (acc[i] != 0 ? 1u : 0u) << (i - 8 * k);
  }
  bits[k] = uint8_t(b);
}

// An [S]B table set, once per GPU: the base points 2^(bits t) B first (one
// lane each), then j x base t for t = 0..tables-1, j = 0..2^(bits-1), affine
// precomp form, one entry per lane.
__global__ void edv_bbase_kernel(ge_p3* bases, SbShape sh) {
  if (int(threadIdx.x) < sh.tables) bases[threadIdx.x] = base_point(int(threadIdx.x) * sh.bits);
}
__global__ void edv_btab_kernel(int32_t* out, const ge_p3* bases, SbShape sh) {
  const uint32_t t = threadIdx.x + blockIdx.x * blockDim.x;
  if (t < uint32_t(sh.tables * sh.entries))
    btab_entry(out + size_t(t) * kBStride, int(t % uint32_t(sh.entries)), bases[t / uint32_t(sh.entries)]);
}

// Row f-3: SHA-256 of n messages, one per lane -> 32-byte digests (out: n x 8 words).
__global__ __launch_bounds__(kBlock) void edv_sha256_kernel(const uint8_t* msgs, const uint64_t* off, uint64_t msg_base,
                                                            uint64_t n, uint32_t* out) {
  const uint64_t i = uint64_t(blockIdx.x) * kBlock + threadIdx.x;
  if (i >= n) return;
  const uint64_t o0 = off[i] - msg_base, o1 = off[i + 1] - msg_base;
  uint32_t d[8];
  sha256_msg(d, msgs + o0, o1 - o0);
  uint4* po = reinterpret_cast<uint4*>(out + 8 * i);
  po[0] = make_uint4(d[0], d[1], d[2], d[3]);
  po[1] = make_uint4(d[4], d[5], d[6], d[7]);
}

}  // namespace

// ------------------------------------------------------------ launch wrappers
namespace edv {

hipError_t launch_main_kernel(unsigned blocks, hipStream_t s, const VerifyArgs& va, bool prio) {
  if (prio) edv_main_kernel_prio<<<dim3(blocks), dim3(kBlock), 0, s>>>(va);
  else edv_main_kernel<<<dim3(blocks), dim3(kBlock), 0, s>>>(va);
  return hipGetLastError();
}
hipError_t launch_bucket_kernels(unsigned blocks, hipStream_t s, const uint64_t* off, uint64_t base, uint64_t n,
                                 uint32_t* ctr, uint32_t* perm) {
  edv_bucket_hist_kernel<<<dim3(blocks), dim3(kBlock), 0, s>>>(off, base, n, ctr);
  edv_bucket_scatter_kernel<<<dim3(blocks), dim3(kBlock), 0, s>>>(off, base, n, ctr, ctr + kBuckets, perm);
  return hipGetLastError();
}
hipError_t launch_btab_kernel(hipStream_t s, int32_t* out, SbShape sh) {
  ge_p3* bases = reinterpret_cast<ge_p3*>(out + sb_words(sh));
  edv_bbase_kernel<<<1, 64, 0, s>>>(bases, sh);
  edv_btab_kernel<<<(sh.tables * sh.entries + 63) / 64, 64, 0, s>>>(out, bases, sh);
  return hipGetLastError();
}
hipError_t launch_comb_kernel(hipStream_t s, int32_t* out) {
  edv_comb_kernel<<<(kCombRows * kCombEntries + 63) / 64, 64, 0, s>>>(out);
  return hipGetLastError();
}
hipError_t launch_sign_kernel(unsigned blocks, hipStream_t s, const uint32_t* seeds, const uint8_t* msgs,
                              const uint64_t* off, uint64_t msg_base, uint64_t n, uint32_t* pks, uint32_t* sigs,
                              const int32_t* comb) {
  edv_sign_kernel<<<dim3(blocks), dim3(kBlock), 0, s>>>(seeds, msgs, off, msg_base, n, pks, sigs, comb);
  return hipGetLastError();
}
hipError_t launch_pack_bits_kernel(hipStream_t s, const uint8_t* acc, uint64_t n, uint8_t* bits) {
  const uint64_t nb = (n + 7) / 8;
  edv_pack_bits_kernel<<<dim3(unsigned((nb + kBlock - 1) / kBlock)), dim3(kBlock), 0, s>>>(acc, n, bits);
  return hipGetLastError();
}
hipError_t launch_sha256_kernel(unsigned blocks, hipStream_t s, const uint8_t* msgs, const uint64_t* off,
                                uint64_t msg_base, uint64_t n, uint32_t* out) {
  edv_sha256_kernel<<<dim3(blocks), dim3(kBlock), 0, s>>>(msgs, off, msg_base, n, out);
  return hipGetLastError();
}

}  // namespace edv
