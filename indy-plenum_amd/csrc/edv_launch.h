// edv_launch.h -- launch wrappers of the kernels in edv_verify.hip and
// edv_prep.hip, for the host runtime (edv_runtime.hip): each launches on
// stream s and returns hipGetLastError().
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "edv_kernels.h"

namespace edv {

// main walk over va.n slots (blocks = ceil(n / kBlock)); prio: the split
// pipeline's issue-priority variant
hipError_t launch_main_kernel(unsigned blocks, hipStream_t s, const VerifyArgs& va, bool prio);
// length buckets of requests [base, base + n): histogram into ctr[0, kBuckets),
// scatter with cursors ctr[kBuckets, 2 kBuckets) into perm (ctr zeroed by the caller)
hipError_t launch_bucket_kernels(unsigned blocks, hipStream_t s, const uint64_t* off, uint64_t base, uint64_t n,
                                 uint32_t* ctr, uint32_t* perm);
// a shared [S]B table set of shape sh (large or compact), once per GPU:
// sb_words(sh) words at out, then the tables' base points 2^(bits t) B
// (sh.tables ge_p3) as scratch; out holds sb_alloc_bytes(sh) bytes
hipError_t launch_btab_kernel(hipStream_t s, int32_t* out, SbShape sh);
// the batch signer's comb rows (kCombRows x kCombEntries x kBStride words)
hipError_t launch_comb_kernel(hipStream_t s, int32_t* out);
hipError_t launch_sign_kernel(unsigned blocks, hipStream_t s, const uint32_t* seeds, const uint8_t* msgs,
                              const uint64_t* off, uint64_t msg_base, uint64_t n, uint32_t* pks, uint32_t* sigs,
                              const int32_t* comb);
// the latency path (edv_quad.hip): requests base .. base + n - 1 of va in one
// launch, four lanes per signature; qtab: n x kQSigWords words of scratch
hipError_t launch_quad_kernel(hipStream_t s, const VerifyArgs& va, int32_t* qtab);
// the right-to-left latency kernel (no table scratch); at most kRtlMax requests
hipError_t launch_rtl_kernel(hipStream_t s, const VerifyArgs& va);
constexpr uint64_t kRtlMax = 4096;
// accept bytes -> bitmask (ceil(n / 8) bytes)
hipError_t launch_pack_bits_kernel(hipStream_t s, const uint8_t* acc, uint64_t n, uint8_t* bits);
hipError_t launch_sha256_kernel(unsigned blocks, hipStream_t s, const uint8_t* msgs, const uint64_t* off,
                                uint64_t msg_base, uint64_t n, uint32_t* out);

}  // namespace edv
