// VALU instruction-throughput microbenchmark for gfx950 (MI355X).
//
// Measures, for each integer/FP instruction the Ed25519 field arithmetic could
// be built on, the issue cost in cycles per wave64 instruction per SIMD when
// every SIMD holds 8 waves and each lane runs 8 independent chains (so the
// numbers are throughput, not latency).  The result decides the limb radix of
// the field multiply ("Field arithmetic").
//
// Build:  hipcc --offload-arch=gfx950 -O3 tools/ubench_valu.hip -o tools/ubench_valu
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "HIP %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); exit(1);} } while (0)

enum Op { ADD, MAD64, MULLO, MULHI, MAD24, MULHI24, FMA64, ADDC, DOT2, ALIGNBIT, ADD3, LSHLADD64, FMA32, BFI, XOR, CNDMASK, ADDCO3, MADMIX, LSHR, ASHR64, MADI64, BITOP3, CND64, MULI24 };
static const char* kNames[] = {"v_add_u32", "v_mad_u64_u32", "v_mul_lo_u32", "v_mul_hi_u32",
  "v_mad_u32_u24", "v_mul_hi_u32_u24", "v_fma_f64", "v_add_co+v_addc_co (2 instr)",
  "v_dot2_u32_u16", "v_alignbit_b32", "v_add3_u32", "v_lshl_add_u64", "v_fma_f32", "v_bfi_b32", "v_xor_b32", "v_cndmask_b32", "v_add_co_u32(vop3 sdst)", "v_mad_u64_u32+v_add_u32 (2 instr)", "v_lshrrev_b32",
  "v_ashrrev_i64", "v_mad_i64_i32", "v_bitop3_b32", "v_cndmask_b32_e64 (sgpr mask)", "v_mul_i32_i24"};
static const int kInstrPerStep[] = {1,1,1,1,1,1,1,2,1,1,1,1,1,1,1,1,1,2,1,1,1,1,1,1};

constexpr int ITERS = 4096;   // loop trips
constexpr int UNR_MAX = 8;   // chains per lane (independent)

template <int OP, int UNR = UNR_MAX>
__global__ __launch_bounds__(256) void kbench(uint32_t* out, uint32_t seed) {
  uint32_t x = seed ^ threadIdx.x, y = seed * 3u + blockIdx.x;
  uint32_t r[UNR];
  uint64_t q[UNR];
  double d[UNR];
  float f[UNR];
#pragma unroll
  for (int i = 0; i < UNR; i++) { r[i] = x + i; q[i] = ((uint64_t)y << 32) | (x + i); d[i] = (double)(x + i); f[i] = (float)(x + i); }
  double dx = (double)x * 1e-9, dy = (double)y * 1e-9;
  float fx = (float)x * 1e-9f, fy = (float)y * 1e-9f;
  const uint64_t mask = __builtin_amdgcn_read_exec() & 0x5555555555555555ull;
  for (int it = 0; it < ITERS; it++) {
#pragma unroll
    for (int rep = 0; rep < 4; rep++) {
#pragma unroll
      for (int i = 0; i < UNR; i++) {
        if constexpr (OP == ADD) asm volatile("v_add_u32 %0, %0, %1" : "+v"(r[i]) : "v"(x));
        if constexpr (OP == MAD64) asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(q[i]) : "v"(x), "v"(y) : "vcc");
        if constexpr (OP == MULLO) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(r[i]) : "v"(x));
        if constexpr (OP == MULHI) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(r[i]) : "v"(x));
        if constexpr (OP == MAD24) asm volatile("v_mad_u32_u24 %0, %1, %2, %0" : "+v"(r[i]) : "v"(x), "v"(y));
        if constexpr (OP == MULHI24) asm volatile("v_mul_hi_u32_u24 %0, %0, %1" : "+v"(r[i]) : "v"(x));
        if constexpr (OP == FMA64) asm volatile("v_fma_f64 %0, %1, %2, %0" : "+v"(d[i]) : "v"(dx), "v"(dy));
        if constexpr (OP == ADDC) asm volatile("v_add_co_u32 %0, vcc, %0, %1\n\tv_addc_co_u32 %0, vcc, %0, %1, vcc" : "+v"(r[i]) : "v"(x) : "vcc");
        if constexpr (OP == DOT2) asm volatile("v_dot2_u32_u16 %0, %1, %2, %0" : "+v"(r[i]) : "v"(x), "v"(y));
        if constexpr (OP == ALIGNBIT) asm volatile("v_alignbit_b32 %0, %0, %1, 13" : "+v"(r[i]) : "v"(x));
        if constexpr (OP == ADD3) asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(r[i]) : "v"(x), "v"(y));
        if constexpr (OP == LSHLADD64) asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(q[i]) : "v"(dx));
        if constexpr (OP == FMA32) asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(f[i]) : "v"(fx), "v"(fy));
        if constexpr (OP == BFI) asm volatile("v_bfi_b32 %0, %0, %1, %2" : "+v"(r[i]) : "v"(x), "v"(y));
        if constexpr (OP == XOR) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(r[i]) : "v"(x));
        if constexpr (OP == CNDMASK) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(r[i]) : "v"(x) : "vcc");
        if constexpr (OP == ADDCO3) asm volatile("v_add_co_u32 %0, s[0:1], %0, %1" : "+v"(r[i]) : "v"(x) : "s0", "s1");
        if constexpr (OP == MADMIX) asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0\n\tv_add_u32 %3, %3, %1" : "+v"(q[i]), "+v"(r[i]) : "v"(x), "v"(y) : "vcc");
        if constexpr (OP == LSHR) asm volatile("v_lshrrev_b32 %0, 7, %0" : "+v"(r[i]));
        if constexpr (OP == ASHR64) asm volatile("v_ashrrev_i64 %0, 26, %0" : "+v"(q[i]));
        if constexpr (OP == MADI64) asm volatile("v_mad_i64_i32 %0, vcc, %1, %2, %0" : "+v"(q[i]) : "v"(x), "v"(y) : "vcc");
        if constexpr (OP == BITOP3) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x6c" : "+v"(r[i]) : "v"(x), "v"(y));
        if constexpr (OP == CND64) asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(r[i]) : "v"(x), "s"(mask));
        if constexpr (OP == MULI24) asm volatile("v_mul_i32_i24 %0, %0, %1" : "+v"(r[i]) : "v"(x));
      }
    }
  }
  uint32_t acc = 0;
#pragma unroll
  for (int i = 0; i < UNR; i++) acc += r[i] + (uint32_t)q[i] + (uint32_t)(q[i] >> 32) + (uint32_t)d[i] + (uint32_t)f[i];
  if (acc == 0x12345678u) out[0] = acc;  // keep everything live
}

// In-kernel clock: ticks of s_memtime (shader clock) vs s_memrealtime (100 MHz).
__global__ void kclock(unsigned long long* out, int spin) {
  unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  uint32_t x = threadIdx.x;
  for (int i = 0; i < spin; i++) asm volatile("v_add_u32 %0, %0, %0" : "+v"(x));
  unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0 && blockIdx.x == 0) { out[0] = t1 - t0; out[1] = r1 - r0; out[2] = x; }
}

// wps waves per SIMD (blocks of 256 threads: one wave per SIMD each), UNR
// independent chains per lane: wps 8 / UNR 8 is throughput, wps 1 is what one
// wave alone sustains (the main kernel's regime), UNR 1 the dependent latency.
template <int OP, int UNR = UNR_MAX>
static void run(int ncu, uint32_t* dout, double clk_ghz, int wps = 8) {
  const int blocks = ncu * wps;
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a)); CHECK(hipEventCreate(&b));
  kbench<OP, UNR><<<blocks, 256>>>(dout, 1);  // warm-up
  CHECK(hipDeviceSynchronize());
  float best = 1e30f;
  for (int rep = 0; rep < 5; rep++) {
    CHECK(hipEventRecord(a));
    kbench<OP, UNR><<<blocks, 256>>>(dout, rep + 2);
    CHECK(hipEventRecord(b));
    CHECK(hipEventSynchronize(b));
    float ms; CHECK(hipEventElapsedTime(&ms, a, b));
    if (ms < best) best = ms;
  }
  double wave_instr = (double)blocks * 4 /*waves per block*/ * ITERS * 4 * UNR * kInstrPerStep[OP];
  double per_simd = wave_instr / (ncu * 4.0);
  double cycles = best * 1e-3 * clk_ghz * 1e9;
  double lane_ops = wave_instr * 64 / (best * 1e-3);
  printf("{\"op\": \"%s\", \"waves_per_simd\": %d, \"chains\": %d, \"ms\": %.4f, "
         "\"cyc_per_wave_instr_per_simd\": %.3f, \"cyc_per_instr_per_wave\": %.3f, \"lane_Gops\": %.1f}\n",
         kNames[OP], wps, UNR, best, cycles / per_simd, cycles / per_simd * wps, lane_ops / 1e9);
  CHECK(hipEventDestroy(a)); CHECK(hipEventDestroy(b));
}

int main() {
  hipDeviceProp_t p; CHECK(hipGetDeviceProperties(&p, 0));
  printf("{\"device\": \"%s\", \"gcn\": \"%s\", \"cus\": %d, \"clock_khz\": %d}\n", p.name, p.gcnArchName,
         p.multiProcessorCount, p.clockRate);
  uint32_t* dout; CHECK(hipMalloc(&dout, 64));
  unsigned long long* dclk; CHECK(hipMalloc(&dclk, 64));
  // busy the chip briefly so DVFS settles, then read the in-kernel clock
  for (int i = 0; i < 20; i++) kbench<MAD64><<<p.multiProcessorCount * 8, 256>>>(dout, i);
  kclock<<<p.multiProcessorCount * 8, 256>>>(dclk, 1 << 20);
  CHECK(hipDeviceSynchronize());
  unsigned long long h[3]; CHECK(hipMemcpy(h, dclk, sizeof h, hipMemcpyDeviceToHost));
  double ghz = (double)h[0] / (double)h[1] * 0.1;
  printf("{\"in_kernel_clock_ghz\": %.3f}\n", ghz);
  int ncu = p.multiProcessorCount;
  run<ADD>(ncu, dout, ghz); run<MAD64>(ncu, dout, ghz); run<MULLO>(ncu, dout, ghz);
  run<MULHI>(ncu, dout, ghz); run<MAD24>(ncu, dout, ghz); run<MULHI24>(ncu, dout, ghz);
  run<FMA64>(ncu, dout, ghz); run<ADDC>(ncu, dout, ghz); run<DOT2>(ncu, dout, ghz);
  run<ALIGNBIT>(ncu, dout, ghz); run<ADD3>(ncu, dout, ghz); run<LSHLADD64>(ncu, dout, ghz);
  run<FMA32>(ncu, dout, ghz); run<BFI>(ncu, dout, ghz);
  run<XOR>(ncu, dout, ghz); run<CNDMASK>(ncu, dout, ghz); run<ADDCO3>(ncu, dout, ghz); run<MADMIX>(ncu, dout, ghz); run<LSHR>(ncu, dout, ghz);
  run<ASHR64>(ncu, dout, ghz); run<MADI64>(ncu, dout, ghz); run<BITOP3>(ncu, dout, ghz); run<CND64>(ncu, dout, ghz); run<MULI24>(ncu, dout, ghz);
  // one wave per SIMD (the main kernel at 64k), and dependent chains (latency)
  for (int wps : {1, 2}) {
    run<MADI64>(ncu, dout, ghz, wps); run<ADD>(ncu, dout, ghz, wps); run<ASHR64>(ncu, dout, ghz, wps);
    run<LSHLADD64>(ncu, dout, ghz, wps); run<MULLO>(ncu, dout, ghz, wps); run<MADMIX>(ncu, dout, ghz, wps);
  }
  run<MADI64, 1>(ncu, dout, ghz, 1); run<MADI64, 2>(ncu, dout, ghz, 1); run<MADI64, 4>(ncu, dout, ghz, 1);
  run<ADD, 1>(ncu, dout, ghz, 1); run<ASHR64, 1>(ncu, dout, ghz, 1); run<LSHLADD64, 1>(ncu, dout, ghz, 1);
  run<MULLO, 1>(ncu, dout, ghz, 1);
  return 0;
}
