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
// the shared [S]B tables, once per device: kBTabWords words at out, then the
// tables' base points 2^(kBBits t) B (kBTables ge_p3) as scratch
constexpr size_t kBTabWords = size_t(kBTables) * kBEntries * kBStride;
constexpr size_t kBTabAllocBytes = 4 * kBTabWords + kBTables * sizeof(ge_p3);
hipError_t launch_btab_kernel(hipStream_t s, int32_t* out);
// the batch signer's comb rows (kCombRows x kCombEntries x kBStride words)
hipError_t launch_comb_kernel(hipStream_t s, int32_t* out);
hipError_t launch_sign_kernel(unsigned blocks, hipStream_t s, const uint32_t* seeds, const uint8_t* msgs,
                              const uint64_t* off, uint64_t msg_base, uint64_t n, uint32_t* pks, uint32_t* sigs,
                              const int32_t* comb);
// accept bytes -> bitmask (ceil(n / 8) bytes)
hipError_t launch_pack_bits_kernel(hipStream_t s, const uint8_t* acc, uint64_t n, uint8_t* bits);
hipError_t launch_sha256_kernel(unsigned blocks, hipStream_t s, const uint8_t* msgs, const uint64_t* off,
                                uint64_t msg_base, uint64_t n, uint32_t* out);
// measurement helper: read and rewrite `bytes` (a multiple of 16) at p
hipError_t launch_flush_kernel(hipStream_t s, void* p, uint64_t bytes);

}  // namespace edv
