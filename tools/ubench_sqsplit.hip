// ubench_sqsplit.hip -- how fast can one chain of field squarings run when the
// columns of each squaring are split over ten lanes of a wave, against the one-
// lane chain (fe_sqn, edv_math.h) that the latency kernels' phase 1 runs?
// ("One request in <= 0.2 ms": the exponentiations of the two
// decompressions are that phase's serial part.)
//
// Split squaring, lane k < 10 owns limb k and column k:
//   column k = sum_r f_r * f_((k - r) mod 10) * c(r, k),
//   c = 19 when r > k (the 2^255 = 19 fold), x 2 when both indices are odd
//   (radix 2^25.5); f_r uniform (v_readlane), f_((k-r) mod 10) fetched with
//   ds_bpermute (the rotation is over ten lanes, DPP rotates over sixteen);
// then two floor-carry rounds between neighbouring lanes (lane 9 -> lane 0
// times 19).  Limbs stay inside fe_sq_floor's input bounds.
//
// Both chains run N squarings from the same input; the canonical encodings
// must agree.  One workgroup of 64 threads, one wave: latency, not throughput.
//
//   hipcc -O3 --offload-arch=gfx950 tools/ubench_sqsplit.hip -o /tmp/ubench_sqsplit && /tmp/ubench_sqsplit
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include "../indy-plenum_amd/csrc/edv_math.h"

using namespace edv;

#define CHECK(x)                                                               \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                  \
      return 1;                                                                \
    }                                                                          \
  } while (0)

// every lane runs the chain on its own copy of the input (64 copies): with one
// uniform input the compiler would run the chain on the scalar unit
__global__ void k_one(const uint32_t* in, uint32_t* out, int n, long long* cyc) {
  fe f = fe_frombytes(in + 8 * threadIdx.x);
  const long long t0 = clock64();
  f = fe_sqn(f, n);
  const long long t1 = clock64();
  if (threadIdx.x != 0) return;
  uint32_t w[8];
  fe_tobytes(w, f);
  for (int i = 0; i < 8; i++) out[i] = w[i];
  cyc[0] = t1 - t0;
}

__device__ __forceinline__ int32_t perm32(int src_lane, int32_t v) {
  return __builtin_amdgcn_ds_bpermute(src_lane << 2, v);
}

__global__ void k_split(const uint32_t* in, uint32_t* out, int n, long long* cyc) {
  const int lane = threadIdx.x;
  const int k = lane % 10;
  const int W = (k & 1) ? 25 : 26;
  const int64_t mask = (int64_t(1) << W) - 1;
  const int from = (k + 9) % 10;  // the lane whose carry lands here
  // per-lane rotation sources and coefficients, fixed for the whole chain
  int src[10], coef[10];
#pragma unroll
  for (int r = 0; r < 10; r++) {
    const int j = (k - r + 10) % 10;
    src[r] = j;
    coef[r] = (r > k ? 19 : 1) * (((r & 1) && (j & 1)) ? 2 : 1);
  }
  const fe f0 = fe_frombytes(in);
  int32_t mine = f0.v[0];
#pragma unroll
  for (int i = 1; i < 10; i++)
    if (k == i) mine = f0.v[i];
  const long long t0 = clock64();
#pragma unroll 1
  for (int it = 0; it < n; it++) {
    int64_t col = 0;
#pragma unroll
    for (int r = 0; r < 10; r++) {
      const int32_t fr = __builtin_amdgcn_readlane(mine, r);
      const int32_t b = perm32(src[r], mine) * coef[r];
      col += int64_t(fr) * int64_t(b);
    }
    // round 1: column -> limb + carry (< 2^36) to the next lane
    int32_t limb = int32_t(col & mask);
    int64_t c = col >> W;
    int64_t cin = int64_t(uint32_t(perm32(from, int32_t(c)))) | (int64_t(perm32(from, int32_t(c >> 32))) << 32);
    if (k == 0) cin *= 19;
    int64_t t = int64_t(limb) + cin;
    // round 2: what is left (< 2^16 before the fold) lands on the next limb
    limb = int32_t(t & mask);
    int32_t c2 = int32_t(t >> W);
    int32_t c2in = perm32(from, c2);
    if (k == 0) c2in *= 19;
    mine = limb + c2in;
  }
  const long long t1 = clock64();
  fe f;
#pragma unroll
  for (int i = 0; i < 10; i++) f.v[i] = __builtin_amdgcn_readlane(mine, i);
  if (lane == 0) {
    uint32_t w[8];
    fe_tobytes(w, f);
    for (int i = 0; i < 8; i++) out[i] = w[i];
    cyc[0] = t1 - t0;
  }
}

int main() {
  const int N = 2540;  // ten exponentiations' worth of squarings
  uint32_t h_in[64 * 8];
  for (int i = 0; i < 8; i++) h_in[i] = 0x9e3779b9u * (i + 1) ^ 0x7f4a7c15u;
  h_in[7] &= 0x7fffffffu;
  for (int l = 1; l < 64; l++) memcpy(h_in + 8 * l, h_in, 32);
  uint32_t *d_in, *d_out;
  long long* d_cyc;
  CHECK(hipMalloc(&d_in, sizeof h_in));
  CHECK(hipMalloc(&d_out, 64));
  CHECK(hipMalloc(&d_cyc, 16));
  CHECK(hipMemcpy(d_in, h_in, sizeof h_in, hipMemcpyHostToDevice));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  float ms[2] = {0, 0};
  long long cyc[2] = {0, 0};
  uint32_t res[2][8];
  for (int v = 0; v < 2; v++) {
    for (int rep = 0; rep < 3; rep++) {  // the last of three (warm)
      CHECK(hipEventRecord(e0, 0));
      if (v == 0)
        k_one<<<1, 64>>>(d_in, d_out, N, d_cyc);
      else
        k_split<<<1, 64>>>(d_in, d_out, N, d_cyc);
      CHECK(hipGetLastError());
      CHECK(hipEventRecord(e1, 0));
      CHECK(hipEventSynchronize(e1));
      CHECK(hipEventElapsedTime(&ms[v], e0, e1));
    }
    CHECK(hipMemcpy(res[v], d_out, 32, hipMemcpyDeviceToHost));
    CHECK(hipMemcpy(&cyc[v], d_cyc, 8, hipMemcpyDeviceToHost));
  }
  const bool same = memcmp(res[0], res[1], 32) == 0;
  printf("{\"squarings\": %d, \"one_lane_ns_per_sq\": %.1f, \"split_ns_per_sq\": %.1f, "
         "\"one_lane_clk_per_sq\": %.1f, \"split_clk_per_sq\": %.1f, \"same_result\": %s}\n",
         N, 1e6 * ms[0] / N, 1e6 * ms[1] / N, double(cyc[0]) / N, double(cyc[1]) / N, same ? "true" : "false");
  return same ? 0 : 2;
}
