// Field/point-op throughput on gfx950: cycles per operation per SIMD at a fixed
// occupancy, for the product fe_mul/fe_sq and candidate carry-chain variants.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I indy-plenum_amd/csrc tools/ubench_field.hip -o tools/ubench_field
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include "edv_verify_core.h"

using namespace edv;
#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); exit(1);} } while (0)

// ---- variant B: rounding carry with the 2^(w-1) bias folded into the 64-bit
// carry value and the new limb taken from 32-bit halves (alignbit for the
// carry's low word, arithmetic shift for its high word).
template <int W>
__device__ __forceinline__ int32_t carry_b(int64_t h, int64_t& next) {
  const int64_t t = h + (int64_t(1) << (W - 1));
  const uint32_t lo = uint32_t(t), hi = uint32_t(uint64_t(t) >> 32);
  const uint32_t clo = __builtin_amdgcn_alignbit(hi, lo, W);
  const int32_t chi = int32_t(hi) >> W;
  next += int64_t((uint64_t(uint32_t(chi)) << 32) | clo);
  return int32_t(lo & ((1u << W) - 1)) - (1 << (W - 1));
}
__device__ __forceinline__ fe carry64_b(int64_t h0, int64_t h1, int64_t h2, int64_t h3, int64_t h4, int64_t h5,
                                        int64_t h6, int64_t h7, int64_t h8, int64_t h9) {
  h0 = carry_b<26>(h0, h1); h4 = carry_b<26>(h4, h5);
  h1 = carry_b<25>(h1, h2); h5 = carry_b<25>(h5, h6);
  h2 = carry_b<26>(h2, h3); h6 = carry_b<26>(h6, h7);
  h3 = carry_b<25>(h3, h4); h7 = carry_b<25>(h7, h8);
  h4 = carry_b<26>(h4, h5); h8 = carry_b<26>(h8, h9);
  int64_t c9 = 0;
  h9 = carry_b<25>(h9, c9);
  h0 += c9 * 19;
  h0 = carry_b<26>(h0, h1);
  return fe{{int32_t(h0), int32_t(h1), int32_t(h2), int32_t(h3), int32_t(h4), int32_t(h5), int32_t(h6), int32_t(h7),
             int32_t(h8), int32_t(h9)}};
}
// ---- variant C: sequential single-pass order 0..9 then 0,1 (each column carried
// once; ILP comes from other waves), same carry_step as the product.
__device__ __forceinline__ fe carry64_c(int64_t h0, int64_t h1, int64_t h2, int64_t h3, int64_t h4, int64_t h5,
                                        int64_t h6, int64_t h7, int64_t h8, int64_t h9) {
  h0 = carry_b<26>(h0, h1); h1 = carry_b<25>(h1, h2); h2 = carry_b<26>(h2, h3); h3 = carry_b<25>(h3, h4);
  h4 = carry_b<26>(h4, h5); h5 = carry_b<25>(h5, h6); h6 = carry_b<26>(h6, h7); h7 = carry_b<25>(h7, h8);
  h8 = carry_b<26>(h8, h9);
  int64_t c9 = 0;
  h9 = carry_b<25>(h9, c9);
  h0 += c9 * 19;
  h0 = carry_b<26>(h0, h1);
  return fe{{int32_t(h0), int32_t(h1), int32_t(h2), int32_t(h3), int32_t(h4), int32_t(h5), int32_t(h6), int32_t(h7),
             int32_t(h8), int32_t(h9)}};
}

template <int V>
__device__ __forceinline__ fe mul_v(const fe& f, const fe& g) {
  if constexpr (V == 0) return fe_mul(f, g);
  sched_fence();
  int32_t g19[10], f2[10];
#pragma unroll
  for (int i = 0; i < 10; i++) { g19[i] = 19 * g.v[i]; f2[i] = (i & 1) ? 2 * f.v[i] : f.v[i]; }
  int64_t h[10];
#pragma unroll
  for (int k = 0; k < 10; k++) {
    int64_t acc = 0;
#pragma unroll
    for (int i = 0; i < 10; i++) {
      const int j = k - i;
      acc += int64_t(((k & 1) == 0) ? f2[i] : f.v[i]) * int64_t((j >= 0) ? g.v[j] : g19[j + 10]);
    }
    h[k] = acc;
  }
  fe r = (V == 1) ? carry64_b(h[0], h[1], h[2], h[3], h[4], h[5], h[6], h[7], h[8], h[9])
                  : carry64_c(h[0], h[1], h[2], h[3], h[4], h[5], h[6], h[7], h[8], h[9]);
  sched_fence();
  return r;
}
template <int V>
__device__ __forceinline__ fe sq_v(const fe& f) {
  if constexpr (V == 0) return fe_sq(f);
  sched_fence();
  int64_t h[10];
  fe_sq_cols<false>(f, h);
  fe r = (V == 1) ? carry64_b(h[0], h[1], h[2], h[3], h[4], h[5], h[6], h[7], h[8], h[9])
                  : carry64_c(h[0], h[1], h[2], h[3], h[4], h[5], h[6], h[7], h[8], h[9]);
  sched_fence();
  return r;
}

constexpr int NOPS = 512;

template <int OP, int V>
__global__ __launch_bounds__(256) void kop(fe* io) {
  const int t = blockIdx.x * 256 + threadIdx.x;
  fe x = io[t], y = io[t + gridDim.x * 256];
  if constexpr (OP == 0) {
#pragma unroll 1
    for (int i = 0; i < NOPS; i++) x = mul_v<V>(x, y);
  } else if constexpr (OP == 1) {
#pragma unroll 1
    for (int i = 0; i < NOPS; i++) x = sq_v<V>(x);
  } else {
    ge_p2 p{x, y, fe_add(x, y)};
#pragma unroll 1
    for (int i = 0; i < NOPS / 8; i++) p = ge_p1p1_to_p2(ge_p2_dbl(p));
    x = p.X; y = p.Z;
  }
  io[t] = fe_add(x, y);
}

__global__ void kclock(unsigned long long* out) {
  unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  uint32_t x = threadIdx.x;
  for (int i = 0; i < (1 << 20); i++) asm volatile("v_add_u32 %0, %0, %0" : "+v"(x));
  unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0 && blockIdx.x == 0) { out[0] = t1 - t0; out[1] = r1 - r0; out[2] = x; }
}

template <int OP, int V>
void run(const char* name, int blocks_per_cu, fe* dbuf, double ghz) {
  const int blocks = 256 * blocks_per_cu;
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a)); CHECK(hipEventCreate(&b));
  kop<OP, V><<<blocks, 256>>>(dbuf);
  CHECK(hipDeviceSynchronize());
  float best = 1e30f;
  for (int r = 0; r < 5; r++) {
    CHECK(hipEventRecord(a));
    kop<OP, V><<<blocks, 256>>>(dbuf);
    CHECK(hipEventRecord(b));
    CHECK(hipEventSynchronize(b));
    float ms; CHECK(hipEventElapsedTime(&ms, a, b));
    if (ms < best) best = ms;
  }
  // ops per SIMD: waves per SIMD (= blocks_per_cu * 4 waves / 4 SIMDs) * NOPS
  const double ops_per_simd = double(blocks_per_cu) * NOPS / (OP == 2 ? 8.0 : 1.0);
  printf("{\"op\": \"%s\", \"waves_per_simd\": %d, \"ms\": %.3f, \"cycles_per_op_per_simd\": %.1f}\n", name,
         blocks_per_cu, best, best * 1e-3 * ghz * 1e9 / ops_per_simd);
}

int main() {
  fe* dbuf;
  const size_t n = 256 * 8 * 256 * 2;
  CHECK(hipMalloc(&dbuf, n * sizeof(fe)));
  fe* h = (fe*)malloc(n * sizeof(fe));
  for (size_t i = 0; i < n; i++)
    for (int l = 0; l < 10; l++) h[i].v[l] = int32_t((i * 2654435761u + l * 40503u) & 0x1ffffff) - (1 << 24);
  CHECK(hipMemcpy(dbuf, h, n * sizeof(fe), hipMemcpyHostToDevice));
  unsigned long long* dc; CHECK(hipMalloc(&dc, 64));
  kop<0, 0><<<2048, 256>>>(dbuf);
  kclock<<<2048, 256>>>(dc);
  CHECK(hipDeviceSynchronize());
  unsigned long long hc[3]; CHECK(hipMemcpy(hc, dc, sizeof hc, hipMemcpyDeviceToHost));
  const double ghz = double(hc[0]) / double(hc[1]) * 0.1;
  printf("{\"clock_ghz_under_load\": %.3f}\n", ghz);
  for (int w : {1, 2, 3, 4}) {
    run<0, 0>("mul_product", w, dbuf, ghz);
    run<0, 1>("mul_carry_b", w, dbuf, ghz);
    run<0, 2>("mul_carry_c", w, dbuf, ghz);
    run<1, 0>("sq_product", w, dbuf, ghz);
    run<1, 1>("sq_carry_b", w, dbuf, ghz);
    run<1, 2>("sq_carry_c", w, dbuf, ghz);
    run<2, 0>("dbl_p2_product", w, dbuf, ghz);
  }
  return 0;
}
