// edv_verify.hip -- gfx950 batch Ed25519 verification kernel and the C-ABI of
// include/edv.h.
//
// One signature per lane, 256-thread workgroups, grid-stride over the batch.
// Per lane (libsodium 1.0.18 semantics):
//   V2-V4  strictness predicates on S, R, A (bytes only)
//   V5     decompress -A (one sqrt exponentiation)
//   V6/V7  SHA-512(R || A || M) straight from the caller's message buffer
//          (arbitrary byte offsets, padding built in registers), h mod L
//   V8     R' = [h](-A) + [S]B with FIXED windows so all 64 lanes of a wave
//          stay in lock-step: h in 64 signed 4-bit digits against a per-lane
//          table 1..8 x (-A) (cached form, in a coalesced global scratch
//          buffer), S in 32 signed 8-bit digits against a shared 129-entry
//          affine table of j*B held in LDS; 252 doublings, 64 + 32 additions
//   V9     encode R' (one inversion) and compare its 32 bytes with R
// No MFMA: this is scalar bignum integer work (v_mad_i64_i32 chains).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>
#include <stdio.h>
#include <mutex>
#include <thread>
#include <vector>
#include <string>

#include "edv_verify_core.h"
#include "../../include/edv.h"

using namespace edv;

namespace {

constexpr int kBlock = 256;
constexpr int kAWords = kAEntries * 40;   // cached point = 4 x 10 limbs

struct VerifyArgs {
  const uint32_t* sigs;   // n x 16 words
  const uint32_t* pks;    // n x 8 words
  const uint8_t* msgs;
  const uint64_t* off;    // n + 1
  uint64_t msg_base;
  uint64_t n;
  uint8_t* accept;
  int32_t* atab;          // per-thread A tables: [kAWords][total threads]
  const int32_t* btab;    // kBEntries x kBStride
};

// ---------------------------------------------------------------- kernels
// Per-thread A table in a global scratch buffer: word w of thread g at
// slot[w * nthreads], so each load/store of a wave touches 64 consecutive words.
struct GlobalATab {
  int32_t* slot;
  uint64_t stride;
  __device__ __forceinline__ void store(int e, const ge_cached& c) const {
    store_fe(e * 40 + 0, c.YpX); store_fe(e * 40 + 10, c.YmX);
    store_fe(e * 40 + 20, c.Z); store_fe(e * 40 + 30, c.T2d);
  }
  __device__ __forceinline__ ge_cached load(int e) const {
    return ge_cached{load_fe(e * 40 + 0), load_fe(e * 40 + 10), load_fe(e * 40 + 20), load_fe(e * 40 + 30)};
  }
  __device__ __forceinline__ void store_fe(int word, const fe& f) const {
#pragma unroll
    for (int l = 0; l < 10; l++) slot[uint64_t(word + l) * stride] = f.v[l];
  }
  __device__ __forceinline__ fe load_fe(int word) const {
    fe f;
#pragma unroll
    for (int l = 0; l < 10; l++) f.v[l] = slot[uint64_t(word + l) * stride];
    return f;
  }
};
// Shared B table in LDS, read as 16-byte vectors.
struct LdsBTab {
  const int32_t* lds;
  __device__ __forceinline__ ge_precomp entry(int j) const {
    const int4* p = reinterpret_cast<const int4*>(lds + j * kBStride);
    int32_t w[32];
#pragma unroll
    for (int i = 0; i < 8; i++) {
      const int4 v = p[i];
      w[4 * i] = v.x; w[4 * i + 1] = v.y; w[4 * i + 2] = v.z; w[4 * i + 3] = v.w;
    }
    return precomp_from_words(w);
  }
};

__global__ __launch_bounds__(kBlock) void edv_verify_kernel(VerifyArgs a) {
  __shared__ __attribute__((aligned(16))) int32_t btab[kBEntries * kBStride];
  for (int i = threadIdx.x; i < kBEntries * kBStride / 4; i += kBlock)
    reinterpret_cast<int4*>(btab)[i] = reinterpret_cast<const int4*>(a.btab)[i];
  __syncthreads();

  const uint64_t nthreads = uint64_t(gridDim.x) * kBlock;
  const uint64_t gtid = uint64_t(blockIdx.x) * kBlock + threadIdx.x;
  GlobalATab at{a.atab + gtid, nthreads};
  const LdsBTab bt{btab};

  for (uint64_t i = gtid; i < a.n; i += nthreads) {
    uint32_t R[8], S[8], A[8];
    const uint4* sp = reinterpret_cast<const uint4*>(a.sigs + 16 * i);
    const uint4* pp = reinterpret_cast<const uint4*>(a.pks + 8 * i);
#pragma unroll
    for (int k = 0; k < 2; k++) {
      const uint4 r = sp[k], s = sp[2 + k], p = pp[k];
      R[4 * k] = r.x; R[4 * k + 1] = r.y; R[4 * k + 2] = r.z; R[4 * k + 3] = r.w;
      S[4 * k] = s.x; S[4 * k + 1] = s.y; S[4 * k + 2] = s.z; S[4 * k + 3] = s.w;
      A[4 * k] = p.x; A[4 * k + 1] = p.y; A[4 * k + 2] = p.z; A[4 * k + 3] = p.w;
    }
    const uint64_t o0 = a.off[i] - a.msg_base, o1 = a.off[i + 1] - a.msg_base;
    a.accept[i] = verify_one(R, S, A, a.msgs + o0, o1 - o0, at, bt) ? 1 : 0;
  }
}

// j * B for j = 0..128 in affine precomp form, once per device
__global__ void edv_btab_kernel(int32_t* out) {
  const int j = threadIdx.x + blockIdx.x * blockDim.x;
  if (j < kBEntries) btab_entry(out + j * kBStride, j);
}

// ------------------------------------------------------------ host runtime
thread_local std::string g_err;

int set_err(int code, const char* what, hipError_t e = hipSuccess) {
  char buf[256];
  if (e != hipSuccess) snprintf(buf, sizeof buf, "%s: %s", what, hipGetErrorString(e));
  else snprintf(buf, sizeof buf, "%s", what);
  g_err = buf;
  return code;
}
#define HIPOK(call, what)                                  \
  do {                                                     \
    hipError_t e_ = (call);                                \
    if (e_ != hipSuccess) return set_err(EDV_E_HIP, what, e_); \
  } while (0)

struct DevBuf {
  void* p = nullptr;
  uint64_t cap = 0;
  int ensure(uint64_t bytes) {
    if (bytes <= cap) return 0;
    if (p) (void)hipFree(p);
    p = nullptr; cap = 0;
    if (hipMalloc(&p, bytes) != hipSuccess) { p = nullptr; return set_err(EDV_E_OOM, "hipMalloc"); }
    cap = bytes;
    return 0;
  }
};

struct DevCtx {
  std::mutex mu;
  bool ready = false;
  int dev = -1;
  hipStream_t stream = nullptr;
  int32_t* btab = nullptr;
  int max_blocks = 0;   // grid cap: resident blocks on the whole device
  DevBuf atab;          // per-thread A tables (grid cap x 256 x 1280 B)
  DevBuf sigs, pks, msgs, off, acc;
};

std::mutex g_mu;
std::vector<DevCtx*> g_ctx;
int g_ndev = -1;

int device_count_locked() {
  if (g_ndev >= 0) return g_ndev;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
  g_ndev = n;
  g_ctx.resize(n, nullptr);
  for (int i = 0; i < n; i++) g_ctx[i] = new DevCtx();
  return n;
}

int ctx_init(DevCtx& c, int dev) {
  if (c.ready) return 0;
  c.dev = dev;
  HIPOK(hipSetDevice(dev), "hipSetDevice");
  hipDeviceProp_t prop;
  HIPOK(hipGetDeviceProperties(&prop, dev), "hipGetDeviceProperties");
  if (strncmp(prop.gcnArchName, "gfx950", 6) != 0) return set_err(EDV_E_NODEV, "device is not gfx950");
  HIPOK(hipStreamCreateWithFlags(&c.stream, hipStreamNonBlocking), "hipStreamCreate");
  int per_cu = 0;
  HIPOK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, edv_verify_kernel, kBlock, 0), "occupancy");
  if (per_cu < 1) per_cu = 1;
  c.max_blocks = per_cu * prop.multiProcessorCount;
  if (c.atab.ensure(uint64_t(c.max_blocks) * kBlock * kAWords * 4)) return EDV_E_OOM;
  HIPOK(hipMalloc(&c.btab, kBEntries * kBStride * 4), "hipMalloc btab");
  edv_btab_kernel<<<(kBEntries + 63) / 64, 64, 0, c.stream>>>(c.btab);
  HIPOK(hipGetLastError(), "btab launch");
  HIPOK(hipStreamSynchronize(c.stream), "btab sync");
  c.ready = true;
  return 0;
}

DevCtx* get_ctx(int dev, int* err) {
  std::lock_guard<std::mutex> lk(g_mu);
  const int n = device_count_locked();
  if (dev < 0 || dev >= n) { *err = set_err(EDV_E_NODEV, "no such device"); return nullptr; }
  *err = 0;
  return g_ctx[dev];
}

// launch on ctx stream or the given stream; caller holds c.mu
int launch(DevCtx& c, const uint8_t* d_sigs, const uint8_t* d_pks, const uint8_t* d_msgs, const uint64_t* d_off,
           uint64_t msg_base, uint64_t n, uint8_t* d_accept, hipStream_t s) {
  if (n == 0) return 0;
  uint64_t blocks = (n + kBlock - 1) / kBlock;
  if (blocks > uint64_t(c.max_blocks)) blocks = c.max_blocks;
  VerifyArgs va;
  va.sigs = reinterpret_cast<const uint32_t*>(d_sigs);
  va.pks = reinterpret_cast<const uint32_t*>(d_pks);
  va.msgs = d_msgs;
  va.off = d_off;
  va.msg_base = msg_base;
  va.n = n;
  va.accept = d_accept;
  va.atab = static_cast<int32_t*>(c.atab.p);
  va.btab = c.btab;
  edv_verify_kernel<<<dim3(unsigned(blocks)), dim3(kBlock), 0, s>>>(va);
  HIPOK(hipGetLastError(), "verify launch");
  return 0;
}

// one shard on one device, host buffers
int run_shard(int dev, const uint8_t* sigs, const uint8_t* pks, const uint8_t* msgs, const uint64_t* off, uint64_t lo,
              uint64_t hi, uint8_t* accept) {
  int err = 0;
  DevCtx* c = get_ctx(dev, &err);
  if (!c) return err;
  std::lock_guard<std::mutex> lk(c->mu);
  if ((err = ctx_init(*c, dev))) return err;
  HIPOK(hipSetDevice(dev), "hipSetDevice");
  const uint64_t n = hi - lo;
  if (n == 0) return 0;
  const uint64_t mbase = off[lo], mbytes = off[hi] - off[lo];
  if (c->sigs.ensure(n * 64) || c->pks.ensure(n * 32) || c->msgs.ensure(mbytes + 64) ||
      c->off.ensure((n + 1) * 8) || c->acc.ensure(n))
    return EDV_E_OOM;
  HIPOK(hipMemcpyAsync(c->sigs.p, sigs + 64 * lo, n * 64, hipMemcpyHostToDevice, c->stream), "h2d sigs");
  HIPOK(hipMemcpyAsync(c->pks.p, pks + 32 * lo, n * 32, hipMemcpyHostToDevice, c->stream), "h2d pks");
  if (mbytes) HIPOK(hipMemcpyAsync(c->msgs.p, msgs + mbase, mbytes, hipMemcpyHostToDevice, c->stream), "h2d msgs");
  HIPOK(hipMemcpyAsync(c->off.p, off + lo, (n + 1) * 8, hipMemcpyHostToDevice, c->stream), "h2d off");
  if ((err = launch(*c, static_cast<uint8_t*>(c->sigs.p), static_cast<uint8_t*>(c->pks.p),
                    static_cast<uint8_t*>(c->msgs.p), static_cast<uint64_t*>(c->off.p), mbase, n,
                    static_cast<uint8_t*>(c->acc.p), c->stream)))
    return err;
  HIPOK(hipMemcpyAsync(accept + lo, c->acc.p, n, hipMemcpyDeviceToHost, c->stream), "d2h accept");
  HIPOK(hipStreamSynchronize(c->stream), "stream sync");
  return 0;
}

}  // namespace

// ------------------------------------------------------------------ C-ABI
extern "C" {

const char* edv_version(void) { return "edv 0.1.0 gfx950"; }
const char* edv_last_error(void) { return g_err.c_str(); }

int edv_device_count(void) {
  std::lock_guard<std::mutex> lk(g_mu);
  return device_count_locked();
}

int edv_verify_batch(const uint8_t* sigs, const uint8_t* pks, const uint8_t* msgs, const uint64_t* msg_off,
                     uint64_t n, uint8_t* accept, uint32_t device_mask) {
  g_err.clear();
  if (n == 0) return 0;
  if (!sigs || !pks || !msg_off || !accept) return set_err(EDV_E_ARG, "null pointer");
  if (!msgs && msg_off[n] != msg_off[0]) return set_err(EDV_E_ARG, "null msgs");
  for (uint64_t i = 0; i < n; i++)
    if (msg_off[i + 1] < msg_off[i]) return set_err(EDV_E_ARG, "msg_off not non-decreasing");
  int ndev;
  {
    std::lock_guard<std::mutex> lk(g_mu);
    ndev = device_count_locked();
  }
  std::vector<int> devs;
  for (int d = 0; d < ndev && d < 32; d++)
    if (device_mask == 0 || (device_mask >> d) & 1u) devs.push_back(d);
  if (devs.empty()) return set_err(EDV_E_NODEV, "no device selected / visible");
  const uint64_t g = devs.size();
  if (g == 1) return run_shard(devs[0], sigs, pks, msgs, msg_off, 0, n, accept);
  std::vector<int> rc(g, 0);
  std::vector<std::string> errs(g);
  std::vector<std::thread> th;
  for (uint64_t k = 0; k < g; k++) {
    th.emplace_back([&, k]() {
      rc[k] = run_shard(devs[k], sigs, pks, msgs, msg_off, n * k / g, n * (k + 1) / g, accept);
      errs[k] = g_err;
    });
  }
  for (auto& t : th) t.join();
  for (uint64_t k = 0; k < g; k++)
    if (rc[k]) { g_err = errs[k]; return rc[k]; }
  return 0;
}

int edv_verify_batch_dev(const uint8_t* d_sigs, const uint8_t* d_pks, const uint8_t* d_msgs,
                         const uint64_t* d_msg_off, uint64_t msg_base, uint64_t n, uint8_t* d_accept, int device,
                         void* stream) {
  g_err.clear();
  int err = 0;
  DevCtx* c = get_ctx(device, &err);
  if (!c) return err;
  std::lock_guard<std::mutex> lk(c->mu);
  if ((err = ctx_init(*c, device))) return err;
  HIPOK(hipSetDevice(device), "hipSetDevice");
  hipStream_t s = stream ? static_cast<hipStream_t>(stream) : c->stream;
  if ((err = launch(*c, d_sigs, d_pks, d_msgs, d_msg_off, msg_base, n, d_accept, s))) return err;
  if (!stream) HIPOK(hipStreamSynchronize(s), "stream sync");
  return 0;
}

int edv_time_batch_dev(const uint8_t* d_sigs, const uint8_t* d_pks, const uint8_t* d_msgs,
                       const uint64_t* d_msg_off, uint64_t msg_base, uint64_t n, uint8_t* d_accept, int device,
                       int iters, float* ms_out) {
  g_err.clear();
  int err = 0;
  DevCtx* c = get_ctx(device, &err);
  if (!c) return err;
  std::lock_guard<std::mutex> lk(c->mu);
  if ((err = ctx_init(*c, device))) return err;
  HIPOK(hipSetDevice(device), "hipSetDevice");
  hipEvent_t e0, e1;
  HIPOK(hipEventCreate(&e0), "event");
  HIPOK(hipEventCreate(&e1), "event");
  HIPOK(hipEventRecord(e0, c->stream), "record");
  for (int it = 0; it < iters; it++)
    if ((err = launch(*c, d_sigs, d_pks, d_msgs, d_msg_off, msg_base, n, d_accept, c->stream))) return err;
  HIPOK(hipEventRecord(e1, c->stream), "record");
  HIPOK(hipEventSynchronize(e1), "event sync");
  float ms = 0;
  HIPOK(hipEventElapsedTime(&ms, e0, e1), "elapsed");
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  if (ms_out) *ms_out = ms;
  return 0;
}

int edv_dev_alloc(int device, uint64_t bytes, void** out) {
  HIPOK(hipSetDevice(device), "hipSetDevice");
  HIPOK(hipMalloc(out, bytes ? bytes : 1), "hipMalloc");
  return 0;
}
int edv_dev_free(int device, void* p) {
  HIPOK(hipSetDevice(device), "hipSetDevice");
  HIPOK(hipFree(p), "hipFree");
  return 0;
}
int edv_h2d(int device, void* dst, const void* src, uint64_t bytes) {
  HIPOK(hipSetDevice(device), "hipSetDevice");
  HIPOK(hipMemcpy(dst, src, bytes, hipMemcpyHostToDevice), "hipMemcpy h2d");
  return 0;
}
int edv_d2h(int device, void* dst, const void* src, uint64_t bytes) {
  HIPOK(hipSetDevice(device), "hipSetDevice");
  HIPOK(hipMemcpy(dst, src, bytes, hipMemcpyDeviceToHost), "hipMemcpy d2h");
  return 0;
}

}  // extern "C"
