// Counter calibration for the main kernel's table gathers.
//
// The guide calibrates FETCH_SIZE only for wide coalesced streaming reads
// (MI355X_MICROARCH.md "HBM": FETCH_SIZE = 1/2 of the bytes there).  The main
// kernel reads each table entry as 160 contiguous bytes PER LANE (ten
// global_load_lds_dwordx4, 16 B per lane each), from per-signature tables
// 1,440 B apart.  This program runs that exact access pattern on known byte
// counts, so rocprofv3 --pmc on it says what the counters report for it:
//
//   stream   coalesced 16 B/lane reads of a buffer (the guide's calibrated case)
//   once     every lane reads its whole 1,440-B table once, entry by entry,
//            160 B at a time through LDS (each table byte read exactly once)
//   walk     the main kernel's gather: 33 windows, per window one 160-B entry
//            of each of two per-lane tables at a random digit 0..8, through LDS
//
// Sizes: L lanes (tables L x 1,440 B each).  Per launch the program prints the
// requested bytes and the distinct 128-B lines touched.
//
// Build:  hipcc --offload-arch=gfx950 -O3 tools/ubench_gather.hip -o tools/ubench_gather
// Run:    tools/ubench_gather [stream_MiB] [once_lanes] [walk_lanes ...]
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "HIP %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); exit(1);} } while (0)

constexpr int kEntryWords = 40;             // 160 B
constexpr int kEntries = 9;                 // 0..8
constexpr int kTabWords = kEntryWords * kEntries;  // 360 words = 1,440 B
constexpr int kWindows = 33;

__device__ __forceinline__ void wait_vm() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// coalesced 16 B per lane, grid-stride
__global__ __launch_bounds__(256) void k_stream(const int4* __restrict__ p, uint64_t n16, int* sink) {
  int acc = 0;
  for (uint64_t i = uint64_t(blockIdx.x) * 256 + threadIdx.x; i < n16; i += uint64_t(gridDim.x) * 256) {
    const int4 v = p[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x7fffffff) sink[0] = acc;  // practically never: keeps the loads alive
}

// one entry of this lane's table through the wave's LDS slice, as LdsATab does
__device__ __forceinline__ int entry_via_lds(const int32_t* slot, int e, int32_t* lds, int lane) {
  const int32_t* g = slot + e * kEntryWords;
#pragma unroll
  for (int q = 0; q < 10; q++)
    __builtin_amdgcn_global_load_lds(const_cast<int32_t*>(g + 4 * q), lds + q * 256, 16, 0, 0);
  wait_vm();
  int acc = 0;
#pragma unroll
  for (int q = 0; q < 10; q++) {
    const int4 v = reinterpret_cast<const int4*>(lds + q * 256)[lane];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  return acc;
}

__global__ __launch_bounds__(256) void k_once(const int32_t* __restrict__ tab, uint64_t lanes, int* sink) {
  __shared__ int32_t lds[4 * 10 * 256];
  const uint64_t j = uint64_t(blockIdx.x) * 256 + threadIdx.x;
  if (j >= lanes) return;
  int32_t* wl = lds + (threadIdx.x >> 6) * 10 * 256;
  const int lane = threadIdx.x & 63;
  int acc = 0;
  for (int e = 0; e < kEntries; e++) acc ^= entry_via_lds(tab + j * kTabWords, e, wl, lane);
  if (acc == 0x7fffffff) sink[0] = acc;
}

__global__ __launch_bounds__(256) void k_walk(const int32_t* __restrict__ atab, const int32_t* __restrict__ rtab,
                                              const uint8_t* __restrict__ dig, uint64_t lanes, int* sink) {
  __shared__ int32_t lds[4 * 20 * 256];
  const uint64_t j = uint64_t(blockIdx.x) * 256 + threadIdx.x;
  if (j >= lanes) return;
  int32_t* wl = lds + (threadIdx.x >> 6) * 20 * 256;
  const int lane = threadIdx.x & 63;
  int acc = 0;
  for (int w = 0; w < kWindows; w++) {
    const uint8_t d = dig[uint64_t(w) * lanes + j];
    acc ^= entry_via_lds(atab + j * kTabWords, d & 15, wl, lane);
    acc ^= entry_via_lds(rtab + j * kTabWords, d >> 4, wl + 10 * 256, lane);
  }
  if (acc == 0x7fffffff) sink[0] = acc;
}

int main(int argc, char** argv) {
  const uint64_t stream_mib = argc > 1 ? strtoull(argv[1], nullptr, 10) : 1024;
  const uint64_t once_lanes = argc > 2 ? strtoull(argv[2], nullptr, 10) : (1u << 20);
  std::vector<uint64_t> walk;
  for (int a = 3; a < argc; a++) walk.push_back(strtoull(argv[a], nullptr, 10));
  if (walk.empty()) walk = {65536, 262144};
  int* sink;
  CHECK(hipMalloc(&sink, 64));
  // stream: 3 launches
  {
    const uint64_t bytes = stream_mib << 20;
    int4* p;
    CHECK(hipMalloc(&p, bytes));
    CHECK(hipMemset(p, 1, bytes));
    for (int r = 0; r < 3; r++) {
      k_stream<<<4096, 256>>>(p, bytes / 16, sink);
      CHECK(hipDeviceSynchronize());
      printf("{\"kernel\": \"k_stream\", \"launch\": %d, \"requested_bytes\": %llu, \"lines_128\": %llu}\n", r,
             (unsigned long long)bytes, (unsigned long long)(bytes / 128));
    }
    CHECK(hipFree(p));
  }
  // once: 2 launches over L x 1,440 B
  {
    const uint64_t bytes = once_lanes * kTabWords * 4;
    int32_t* t;
    CHECK(hipMalloc(&t, bytes));
    CHECK(hipMemset(t, 2, bytes));
    for (int r = 0; r < 2; r++) {
      k_once<<<unsigned((once_lanes + 255) / 256), 256>>>(t, once_lanes, sink);
      CHECK(hipDeviceSynchronize());
      printf("{\"kernel\": \"k_once\", \"launch\": %d, \"lanes\": %llu, \"requested_bytes\": %llu, "
             "\"lines_128\": %llu}\n", r, (unsigned long long)once_lanes, (unsigned long long)bytes,
             (unsigned long long)((bytes + 127) / 128));
    }
    CHECK(hipFree(t));
  }
  // walk: per size, 3 launches over two L x 1,440-B tables, random digits
  for (uint64_t L : walk) {
    const uint64_t tb = L * kTabWords * 4;
    int32_t *a, *r;
    uint8_t* d;
    CHECK(hipMalloc(&a, tb));
    CHECK(hipMalloc(&r, tb));
    CHECK(hipMalloc(&d, L * kWindows));
    CHECK(hipMemset(a, 3, tb));
    CHECK(hipMemset(r, 4, tb));
    std::vector<uint8_t> hd(L * kWindows);
    uint64_t x = 0x9E3779B97F4A7C15ull, distinct = 0;
    std::vector<uint16_t> seen(L);
    for (uint64_t i = 0; i < L * kWindows; i++) {
      x ^= x << 13; x ^= x >> 7; x ^= x << 17;
      hd[i] = uint8_t((x % 9) | (((x >> 8) % 9) << 4));
    }
    // distinct 128-B lines a launch touches: per lane, the entries its digits select
    for (uint64_t j = 0; j < L; j++) {
      uint32_t ma = 0, mr = 0;
      for (int w = 0; w < kWindows; w++) {
        const uint8_t v = hd[uint64_t(w) * L + j];
        ma |= 1u << (v & 15);
        mr |= 1u << (v >> 4);
      }
      for (int t = 0; t < 2; t++) {
        const uint64_t base = (t == 0 ? 0 : tb) + j * kTabWords * 4;
        std::vector<uint64_t> lines;
        const uint32_t m = t == 0 ? ma : mr;
        for (int e = 0; e < kEntries; e++)
          if ((m >> e) & 1)
            for (uint64_t b = base + e * 160; b < base + e * 160 + 160; b += 16) {
              const uint64_t ln = b / 128;
              if (lines.empty() || lines.back() != ln) lines.push_back(ln);
            }
        distinct += lines.size();
      }
    }
    CHECK(hipMemcpy(d, hd.data(), hd.size(), hipMemcpyHostToDevice));
    for (int rep = 0; rep < 3; rep++) {
      k_walk<<<unsigned((L + 255) / 256), 256>>>(a, r, d, L, sink);
      CHECK(hipDeviceSynchronize());
      printf("{\"kernel\": \"k_walk\", \"launch\": %d, \"lanes\": %llu, \"tables_bytes\": %llu, "
             "\"requested_bytes\": %llu, \"gather_lines_128\": %llu, \"digit_bytes\": %llu, "
             "\"distinct_lines_128\": %llu}\n", rep, (unsigned long long)L, (unsigned long long)(2 * tb),
             (unsigned long long)(L * kWindows * 2 * 160), (unsigned long long)(L * kWindows * 2 * 2),
             (unsigned long long)(L * kWindows), (unsigned long long)distinct);
    }
    CHECK(hipFree(a));
    CHECK(hipFree(r));
    CHECK(hipFree(d));
  }
  CHECK(hipFree(sink));
  return 0;
}
