// edv_runtime.hip -- host runtime and C-ABI of libedv.so (include/edv.h):
// device contexts, streams and scratch, the device-resident, host-buffer
// (synchronous, field-ordered), asynchronous and pipelined paths, sharding and
// placement over devices.  Host code only: the kernels are in edv_verify.hip
// and edv_prep.hip, launched through edv_launch.h.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>
#include <stdlib.h>
#include <stdio.h>
#include <algorithm>
#include <atomic>
#include <mutex>
#include <thread>
#include <unistd.h>
#include <vector>
#include <string>

#include "edv_kernels.h"
#include "edv_launch.h"
#include "edv_ledger.h"
#include "../../include/edv.h"

using namespace edv;

namespace {

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

// Pinned (page-locked, portable) host memory: staging of pageable inputs
struct PinnedBuf {
  void* p = nullptr;
  void* dev = nullptr;  // its device-side address (zero-copy), looked up once per allocation
  uint64_t cap = 0;
  int ensure(uint64_t bytes) {
    if (bytes <= cap) return 0;
    if (p) (void)hipHostFree(p);
    p = nullptr; dev = nullptr; cap = 0;
    bytes = bytes + bytes / 4 + 4096;  // headroom: message bytes vary from call to call
    if (hipHostMalloc(&p, bytes, hipHostMallocPortable) != hipSuccess) {
      p = nullptr;
      return set_err(EDV_E_OOM, "hipHostMalloc");
    }
    cap = bytes;
    if (hipHostGetDevicePointer(&dev, p, 0) != hipSuccess) {
      (void)hipGetLastError();
      dev = nullptr;
    }
    return 0;
  }
};

// Host path: a shard is walked in sub-batches, round-robin over kQ streams,
// so the H2D copy of one sub-batch overlaps the kernels of the others and
// several sub-batches share the chip at once (a 64k batch split 4 ways still
// fills every SIMD).  Sub-batch stream q uses scratch slots [q*P, (q+1)*P) of
// the chunk state.
constexpr int kQ = 4;
// Message slices of the synchronous field-ordered path (run_shard_fields): the
// hash side of slice k runs while slice k+1 copies.  edv_set_host_slices.
constexpr int kSlices = 8;
constexpr uint64_t kMinSliceReqs = 65536;
// In-flight batches of the asynchronous host path per device: a Node keeps one
// per prod in flight, and a pool of nodes in one process (C5) one per node, so
// eight slots let up to eight callers overlap before a submission has to wait.
constexpr int kAsyncSlots = 8;
// An asynchronous batch of at most this many requests (a Node's prod carries a
// few hundred) runs on its slot's own stream with its slot's own scratch
// (~25 MB), so the small batches of several callers execute side by side on
// the GPU instead of queueing behind each other on one stream: a batch that
// small is one wave per SIMD on a few SIMDs, and its latency (one main-kernel
// walk, ~0.45 ms) is all it costs.  Larger batches share the chunk scratch.
constexpr uint64_t kSmallAsync = 8192;
// The latency path (edv_quad.hip: one launch, sixteen lanes per signature up to
// 4,096 requests, eight above) takes every batch of at most this many requests
// on the host paths and the device-resident path (edv_set_latency_path changes
// it per device; 0 = off).  Below one wave per SIMD the batch kernels' time is
// one lane's serial chain whatever n is; the latency kernels split each point
// operation over a quad of lanes.
// profiles/r06/latency_paths_s3.jsonl: faster than the batch kernels at every n up to 8,192;
// profiles/r06/quad_limit_s51.jsonl: the two-walk kernel at 12,288 / 16,384 requests 386 / 392 us
// against 569 / 567 for the batch kernels (two waves per SIMD), level at 20,480, behind at 32,768
constexpr uint64_t kQuadMaxDefault = 16384;
constexpr uint64_t kQuadMaxLimit = 16384;  // the quad kernel's per-signature table scratch grows with n (57 MB here)

// One set of per-chunk state buffers (ChunkState storage + bucket permutation)
// for `cap` signatures (~5.5 kB each: ~1.4 GB for a whole 2^18 chunk).  Sized
// by use, not up front: a set grows to the largest batch it has served (in
// steps of powers of two from 4,096, at most the chunk), so a Node verifying
// prods of a few hundred requests holds ~25 MB of it, not 1.4 GB.  The caller
// guarantees that no queued kernel still uses a set it grows (grow_state).
struct ChunkBufs {
  DevBuf atab, rtab, dig, alive;  // ChunkState storage
  DevBuf perm, bucket_ctr;  // length-bucket permutation of a chunk; histogram + cursors (one set per stream)
  uint64_t cap = 0;         // signatures the set holds (the row stride of dig / alive)
  bool fits(uint64_t need) const { return need <= cap; }
  int ensure(uint64_t need, uint64_t limit) {
    if (need <= cap) return 0;
    uint64_t c = 4096;
    while (c < need) c <<= 1;
    if (c > limit) c = limit > need ? limit : need;
    if (atab.ensure(c * kAWords * 4) || rtab.ensure(c * kAWords * 4) || dig.ensure(c * kDigWords * 4) ||
        alive.ensure(3 * c) || perm.ensure(c * 4) || bucket_ctr.ensure(uint64_t(kQ) * 2 * kBuckets * 4)) {
      cap = 0;
      return EDV_E_OOM;
    }
    cap = c;
    return 0;
  }
  uint64_t bytes() const { return atab.cap + rtab.cap + dig.cap + alive.cap + perm.cap + bucket_ctr.cap; }
};

struct DevCtx {
  std::mutex mu;
  bool ready = false;
  std::atomic<bool> live{false};   // ready, readable without mu (placement, edv_context_count)
  std::atomic<int> running{0};     // synchronous calls placed here and not yet returned
  int dev = -1;                    // logical device (edv_* device index)
  int phys = -1;                   // HIP device it runs on
  hipStream_t stream = nullptr;    // the library stream (edv_stream)
  const int32_t* sb_compact = nullptr;  // the GPU's [S]B table sets (shared_tables), when built
  const int32_t* sb_large = nullptr;
  int32_t* comb = nullptr;         // signer comb table, built on first edv_sign_* call
  uint64_t chunk = kChunkDefault;  // EDV_CHUNK overrides (tests exercise chunk seams)
  int length_buckets = 2;          // 0 never, 1 always, 2 auto (edv_set_length_buckets)
  uint64_t quad_max = kQuadMaxDefault;  // latency path up to this batch size (edv_set_latency_path)
  ChunkBufs st;                    // scratch of the ordinary paths
  // st_done: recorded after the last kernel that used `st`, on whatever stream
  // that was; every later user waits for it first, so launches on different
  // caller streams never share the scratch concurrently.
  hipEvent_t st_done = nullptr;
  // host path (edv_verify_batch)
  hipStream_t hs[kQ] = {};
  hipEvent_t hs_staged[kQ] = {};   // pinned slot q may be refilled once its H2D copies are done
  hipEvent_t hs_end[kQ] = {};
  // split-prep host path (run_shard_split): copies on hcp, part q's prep on hs[q]
  hipStream_t hcp = nullptr;
  hipEvent_t part_copied[kQ] = {}, part_prepped[kQ] = {};
  hipEvent_t slice_copied[kSlices] = {}, slice_hashed[kSlices] = {};
  int host_slices = 0;              // 0 = one slice per kMinSliceReqs requests
  // asynchronous host path (edv_verify_batch_async): kAsyncSlots slots used in turn,
  // H2D copies on hcp, kernels and the verdicts' D2H on hac, so the copies of
  // batch k+1 run while batch k computes
  struct AsyncSlot {
    DevBuf sigs, pks, msgs, off, acc, dig;
    PinnedBuf stage, acc_host, dig_host;
    hipEvent_t copied = nullptr, done = nullptr;
    int64_t ticket = -1;         // batch held by the slot, -1 = none
    uint8_t* accept = nullptr;   // the caller's verdict buffer
    uint8_t* digests = nullptr;  // the caller's SHA-256 buffer (null: none asked for)
    uint64_t n = 0;
    bool acc_pinned = false;     // verdicts DMA'd straight into `accept`
    bool dig_pinned = false;     // digests DMA'd straight into `digests`
    hipStream_t st = nullptr;    // small batches: copies, kernels and D2H all on this stream
    ChunkBufs cb;                // small batches: the slot's own chunk scratch (grown to the batch)
    DevBuf qtab;                 // latency-path batches: the quad kernel's table scratch
#ifdef EDV_MEASUREMENT_API
    bool injected = false;       // edv_test_fail_async: this batch launched nothing and fails
#endif
  };
  AsyncSlot as[kAsyncSlots];
  hipStream_t hac = nullptr;
  // tickets issued and failed (edv_ledger.h); a failed batch's slot drops it,
  // so nothing is copied into the caller's buffers afterwards
  AsyncLedger ledger;
  DevBuf sigs, pks, msgs, off, acc;
  DevBuf fblob;  // the field path's signatures | keys | offsets block when they arrive in one copy
  // latency path of the synchronous and device-resident calls: packed inputs
  // (one DMA) and the quad kernel's table scratch (ordered by st_done, like
  // the chunk scratch)
  DevBuf qblob, qtab;
  PinnedBuf qstage;
  PinnedBuf stage[kQ], acc_host;
  // Pipelined submission (edv_verify_batch_dev_pipelined): two state sets, a
  // prep stream and a main stream, so the prep kernel of batch k+1 runs on the
  // SIMDs beside the main kernel of batch k.  prep_done[b] orders main after its
  // prep; main_done[b] keeps the next prep from overwriting state set b early.
  bool pipe_ready = false;
  ChunkBufs pst[2];
  hipStream_t sp = nullptr, sm = nullptr;
  hipEvent_t prep_done[2] = {nullptr, nullptr}, main_done[2] = {nullptr, nullptr}, inputs_ready = nullptr;
  hipEvent_t perm_done[2] = {nullptr, nullptr};  // split prep: state set b's bucket permutation is written
  bool pending[2] = {false, false};
  int next = 0;
#ifdef EDV_MEASUREMENT_API
  int64_t inject_fail = -1;        // edv_test_fail_async (libedv_measure.so only)
#endif
};

std::mutex g_mu;
std::vector<DevCtx*> g_ctx;
int g_ndev = -1;

// ---- the [S]B tables (the prep kernel's R side): one copy per GPU and shape
// in a process, shared by every logical device (EDV_VIRTUAL_DEVICES) mapped
// onto that GPU.  Which shapes a context builds (EDV_SB_TABLES):
//   auto (default)  the compact set (64 MiB) at context creation; the large
//                   set (3 GiB, 4 fewer additions per verify, +1 % at C2) once
//                   a batch of at least kLargeTablesMin requests arrives -- a
//                   Node verifying prods of a few hundred requests never
//                   allocates it (footprint)
//   compact         never the large set
//   large           the large set at context creation (the compact one never)
// A failed allocation of the large set leaves the compact one in use.
constexpr uint64_t kLargeTablesMin = 65536;  // one wave per SIMD of a whole MI355X
enum SbPolicy { kSbAuto, kSbCompact, kSbLarge };
SbPolicy sb_policy() {
  static const SbPolicy p = [] {
    const char* e = getenv("EDV_SB_TABLES");
    if (e && !strcmp(e, "compact")) return kSbCompact;
    if (e && !strcmp(e, "large")) return kSbLarge;
    return kSbAuto;
  }();
  return p;
}
struct SbSet {
  int phys;
  int bits;
  int32_t* p;
  uint64_t bytes;
};
std::mutex g_sb_mu;
std::vector<SbSet> g_sb;
// The table set of shape sh on GPU phys (current device = phys), built on
// first use; nullptr (with the error set) if it cannot be allocated or built.
const int32_t* shared_tables(int phys, SbShape sh, hipStream_t s, int* err) {
  std::lock_guard<std::mutex> lk(g_sb_mu);
  for (const SbSet& t : g_sb)
    if (t.phys == phys && t.bits == sh.bits) return t.p;
  const uint64_t bytes = sb_alloc_bytes(sh);
  int32_t* p = nullptr;
  if (hipMalloc(&p, bytes) != hipSuccess) {
    (void)hipGetLastError();
    *err = set_err(EDV_E_OOM, "hipMalloc [S]B tables");
    return nullptr;
  }
  hipError_t e = launch_btab_kernel(s, p, sh);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  if (e != hipSuccess) {
    (void)hipFree(p);
    *err = set_err(EDV_E_HIP, "[S]B table build", e);
    return nullptr;
  }
  g_sb.push_back({phys, sh.bits, p, bytes});
  return p;
}
uint64_t shared_tables_bytes(int phys) {
  std::lock_guard<std::mutex> lk(g_sb_mu);
  uint64_t b = 0;
  for (const SbSet& t : g_sb)
    if (t.phys == phys) b += t.bytes;
  return b;
}

// Logical devices.  Normally one per visible HIP device.  EDV_VIRTUAL_DEVICES=k
// (testing knob) presents k logical devices mapped round-robin onto the
// physical ones, each with its own context, streams and buffers, so the
// multi-device host path (one thread per device, shard split, error
// propagation) runs on a one-GPU box exactly as it does on eight GPUs.
int device_count_locked() {
  if (g_ndev >= 0) return g_ndev;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) { (void)hipGetLastError(); n = 0; }
  int logical = n;
  if (const char* e = getenv("EDV_VIRTUAL_DEVICES")) {
    const long v = strtol(e, nullptr, 10);
    if (n > 0 && v > 0 && v <= 32) logical = int(v);
  }
  g_ndev = logical;
  g_ctx.resize(logical, nullptr);
  for (int i = 0; i < logical; i++) {
    g_ctx[i] = new DevCtx();
    g_ctx[i]->dev = i;
    g_ctx[i]->phys = n > 0 ? i % n : 0;
  }
  return logical;
}

// Idempotent: a failure part-way leaves what was created in place and the next
// call resumes from there (no second stream or table per retry).
int ctx_init(DevCtx& c) {
  if (c.ready) return 0;
  HIPOK(hipSetDevice(c.phys), "hipSetDevice");
  hipDeviceProp_t prop;
  HIPOK(hipGetDeviceProperties(&prop, c.phys), "hipGetDeviceProperties");
  if (strncmp(prop.gcnArchName, "gfx950", 6) != 0) return set_err(EDV_E_NODEV, "device is not gfx950");
  if (!c.stream) HIPOK(hipStreamCreateWithFlags(&c.stream, hipStreamNonBlocking), "hipStreamCreate");
  for (int q = 0; q < kQ; q++) {
    if (!c.hs[q]) HIPOK(hipStreamCreateWithFlags(&c.hs[q], hipStreamNonBlocking), "hipStreamCreate");
    if (!c.hs_staged[q]) HIPOK(hipEventCreateWithFlags(&c.hs_staged[q], hipEventDisableTiming), "event");
    if (!c.hs_end[q]) HIPOK(hipEventCreateWithFlags(&c.hs_end[q], hipEventDisableTiming), "event");
    if (!c.part_copied[q]) HIPOK(hipEventCreateWithFlags(&c.part_copied[q], hipEventDisableTiming), "event");
    if (!c.part_prepped[q]) HIPOK(hipEventCreateWithFlags(&c.part_prepped[q], hipEventDisableTiming), "event");
  }
  for (int k = 0; k < kSlices; k++) {
    if (!c.slice_copied[k]) HIPOK(hipEventCreateWithFlags(&c.slice_copied[k], hipEventDisableTiming), "event");
    if (!c.slice_hashed[k]) HIPOK(hipEventCreateWithFlags(&c.slice_hashed[k], hipEventDisableTiming), "event");
  }
  if (!c.hcp) HIPOK(hipStreamCreateWithFlags(&c.hcp, hipStreamNonBlocking), "hipStreamCreate");
  if (!c.hac) HIPOK(hipStreamCreateWithFlags(&c.hac, hipStreamNonBlocking), "hipStreamCreate");
  for (auto& s : c.as) {
    if (!s.copied) HIPOK(hipEventCreateWithFlags(&s.copied, hipEventDisableTiming), "event");
    if (!s.done) HIPOK(hipEventCreateWithFlags(&s.done, hipEventDisableTiming), "event");
  }
  if (!c.st_done) HIPOK(hipEventCreateWithFlags(&c.st_done, hipEventDisableTiming), "event");
  if (const char* e = getenv("EDV_CHUNK")) {
    const uint64_t v = strtoull(e, nullptr, 10);
    if (v >= kBlock && v <= (uint64_t(1) << 24)) c.chunk = (v / kBlock) * kBlock;
  }
  // the scratch grows by use (ChunkBufs); the [S]B tables: see sb_policy
  int err = 0;
  if (sb_policy() == kSbLarge) {
    if (!c.sb_large && !(c.sb_large = shared_tables(c.phys, sb_large(), c.stream, &err))) return err;
  } else if (!c.sb_compact && !(c.sb_compact = shared_tables(c.phys, sb_compact(), c.stream, &err))) {
    return err;
  }
  c.ready = true;
  c.live.store(true);
  return 0;
}

DevCtx* get_ctx(int dev, int* err) {
  std::lock_guard<std::mutex> lk(g_mu);
  const int n = device_count_locked();
  if (dev < 0 || dev >= n) { *err = set_err(EDV_E_NODEV, "no such device"); return nullptr; }
  *err = 0;
  return g_ctx[dev];
}

// Lock a device's context, initialise it and make its HIP device current.
struct CtxLock {
  DevCtx* c = nullptr;
  std::unique_lock<std::mutex> lk;
  int err = 0;
  explicit CtxLock(int device) {
    c = get_ctx(device, &err);
    if (!c) return;
    lk = std::unique_lock<std::mutex>(c->mu);
    if ((err = ctx_init(*c))) return;
    if (hipSetDevice(c->phys) != hipSuccess) err = set_err(EDV_E_HIP, "hipSetDevice");
  }
};

int phys_of(int device, int* phys) {
  int err = 0;
  DevCtx* c = get_ctx(device, &err);
  if (!c) return err;
  *phys = c->phys;
  return 0;
}

// The [S]B table set a batch of n requests runs against (sb_policy): the
// large set once built (or once a batch this large asks for it), else the
// compact one.  Caller holds c.mu; the current device is c.phys.
void pick_tables(DevCtx& c, uint64_t n, const int32_t** t, SbShape* sh) {
  if (!c.sb_large && sb_policy() == kSbAuto && n >= kLargeTablesMin) {
    int err = 0;
    c.sb_large = shared_tables(c.phys, sb_large(), c.stream, &err);  // stays compact if this fails
    if (!c.sb_large) g_err.clear();
  }
  if (c.sb_large) {
    *t = c.sb_large;
    *sh = sb_large();
  } else {
    *t = c.sb_compact;
    *sh = sb_compact();
  }
}

// Grow the context's ordinary chunk scratch to `need` signatures (at most one
// chunk's worth is ever used at once), after every queued user of it is done.
int grow_state(DevCtx& c, uint64_t need) {
  if (need > c.chunk) need = c.chunk;
  if (c.st.fits(need)) return 0;
  HIPOK(hipEventSynchronize(c.st_done), "scratch sync");
  return c.st.ensure(need, c.chunk);
}

VerifyArgs make_args(DevCtx& c, ChunkBufs& b, const uint8_t* d_sigs, const uint8_t* d_pks,
                     const uint8_t* d_msgs, const uint64_t* d_off, uint64_t msg_base, uint8_t* d_accept, bool bucket,
                     uint64_t slot0 = 0, uint64_t batch = 0) {
  VerifyArgs va;
  va.sigs = reinterpret_cast<const uint32_t*>(d_sigs);
  va.pks = reinterpret_cast<const uint32_t*>(d_pks);
  va.msgs = d_msgs;
  va.off = d_off;
  va.msg_base = msg_base;
  va.accept = d_accept;
  // slots [slot0, slot0 + n) of the chunk scratch (dig stays indexed w * cap + slot)
  va.st = ChunkState{static_cast<int32_t*>(b.atab.p) + slot0 * kAWords, static_cast<int32_t*>(b.rtab.p) + slot0 * kAWords,
                     static_cast<uint32_t*>(b.dig.p) + slot0,
                     static_cast<uint8_t*>(b.alive.p) + slot0, b.cap,
                     bucket ? static_cast<uint32_t*>(b.perm.p) + slot0 : nullptr};
  pick_tables(c, batch, &va.btab, &va.sb);
  va.base = 0;
  va.n = 0;
  va.side0 = 0;
  va.nsides = 3;
  return va;
}

// length buckets of one chunk on stream s (ctr: this stream's histogram + cursors)
int launch_buckets(uint32_t* ctr, const VerifyArgs& va, const uint64_t* d_off, hipStream_t s) {
  const unsigned blocks = unsigned((va.n + kBlock - 1) / kBlock);
  HIPOK(hipMemsetAsync(ctr, 0, 2 * kBuckets * 4, s), "memset buckets");
  HIPOK(launch_bucket_kernels(blocks, s, d_off, va.base, va.n, ctr, const_cast<uint32_t*>(va.st.perm)),
        "bucket launch");
  return 0;
}
// the prep kernel over the sides va.side0 .. va.side0 + va.nsides - 1
int launch_prep_sides(const VerifyArgs& va, hipStream_t s) {
#ifdef EDV_MEASURE_NO_VERIFY
  return 0;  // measurement build: see launch_main
#endif
  const unsigned blocks = unsigned((va.n + kBlock - 1) / kBlock);
  HIPOK(launch_prep_kernel(unsigned(va.nsides) * blocks, s, va), "prep launch");
  return 0;
}
// [length buckets,] prep kernel (all three sides) of one chunk on stream s
int launch_prep(uint32_t* ctr, const VerifyArgs& va, const uint64_t* d_off, bool bucket, hipStream_t s) {
#ifdef EDV_MEASURE_NO_VERIFY
  return 0;  // measurement build: see launch_main
#endif
  int err;
  if (bucket && (err = launch_buckets(ctr, va, d_off, s))) return err;
  return launch_prep_sides(va, s);  // hash, A and R sides
}
int launch_main(const VerifyArgs& va, hipStream_t s, bool prio = false) {
#ifdef EDV_MEASURE_NO_VERIFY
  // Measurement build only (variants/libedv_noverify.so, loaded by bench.py's
  // C5 leg through EDV_LIB in a separate process, never the product library):
  // every request of the chunk is reported valid without the verify kernels,
  // so a pool run can tell what verification costs from what everything around
  // it costs.  (A chunk's slots map onto accept[base, base + n), in any order.)
  HIPOK(hipMemsetAsync(va.accept + va.base, 1, va.n, s), "memset accept");
  return 0;
#endif
  const unsigned blocks = unsigned((va.n + kBlock - 1) / kBlock);
  HIPOK(launch_main_kernel(blocks, s, va, prio), "main launch");
  return 0;
}
uint32_t* bucket_ctr(ChunkBufs& b, int q) { return static_cast<uint32_t*>(b.bucket_ctr.p) + q * 2 * kBuckets; }

// Length buckets cost three small launches per chunk (memset, histogram,
// scatter).  Per call: EDV_FLAG_UNIFORM_LENGTH turns them off,
// EDV_FLAG_BUCKETS forces them; otherwise the device mode decides
// (edv_set_length_buckets).  Verdicts never depend on it.
bool bucketing_enabled(const DevCtx& c, uint32_t flags) {
  if (flags & EDV_FLAG_UNIFORM_LENGTH) return false;
  if (flags & EDV_FLAG_BUCKETS) return true;
  return c.length_buckets != 0;
}

// ---- the latency path (edv_quad.hip)
// The quad kernel over n requests whose inputs are device pointers (offsets
// absolute, minus msg_base), verdicts to d_acc[0, n); qtab is this launch's
// scratch (the caller orders it against its previous user).
int launch_quad(DevCtx& c, DevBuf& qtab, const uint8_t* d_sigs, const uint8_t* d_pks, const uint8_t* d_msgs,
                const uint64_t* d_off, uint64_t msg_base, uint64_t n, uint8_t* d_acc, hipStream_t s) {
  if (n == 0) return 0;
  // up to kRtlMax requests (one workgroup per CU): the right-to-left kernel, no
  // table scratch; above: the two-walk kernel over per-signature tables
  const bool rtl = n <= kRtlMax;
  // the last workgroup's 64 quads all write their tables, in range or not
  if (!rtl && qtab.ensure((n + 63) / 64 * 64 * kQSigWords * 4)) return EDV_E_OOM;
  VerifyArgs va;
  memset(&va, 0, sizeof va);
  va.sigs = reinterpret_cast<const uint32_t*>(d_sigs);
  va.pks = reinterpret_cast<const uint32_t*>(d_pks);
  va.msgs = d_msgs;
  va.off = d_off;
  va.msg_base = msg_base;
  va.base = 0;
  va.n = n;
  va.accept = d_acc;
  pick_tables(c, n, &va.btab, &va.sb);
#ifdef EDV_MEASURE_NO_VERIFY
  HIPOK(hipMemsetAsync(d_acc, 1, n, s), "memset accept");  // measurement build: see launch_main
  return 0;
#endif
  if (rtl) HIPOK(launch_rtl_kernel(s, va), "rtl launch");
  else HIPOK(launch_quad_kernel(s, va, static_cast<int32_t*>(qtab.p)), "quad launch");
  return 0;
}

// Ordinary device path: launch on stream s; caller holds c.mu.  The batch is
// walked in chunks of c.chunk signatures: [length buckets,] prep kernel, main
// kernel, all in stream order, after every earlier user of the scratch.
int launch(DevCtx& c, const uint8_t* d_sigs, const uint8_t* d_pks, const uint8_t* d_msgs, const uint64_t* d_off,
           uint64_t msg_base, uint64_t n, uint8_t* d_accept, hipStream_t s, uint32_t flags) {
  if (n == 0) return 0;
  const bool bucket = bucketing_enabled(c, flags);
  int err;
  if (n <= c.quad_max) {  // the latency path, its scratch ordered like the chunk scratch
    HIPOK(hipStreamWaitEvent(s, c.st_done, 0), "wait scratch");
    if ((err = launch_quad(c, c.qtab, d_sigs, d_pks, d_msgs, d_off, msg_base, n, d_accept, s))) return err;
    HIPOK(hipEventRecord(c.st_done, s), "record scratch");
    return 0;
  }
  if ((err = grow_state(c, n))) return err;
  HIPOK(hipStreamWaitEvent(s, c.st_done, 0), "wait scratch");
  VerifyArgs va = make_args(c, c.st, d_sigs, d_pks, d_msgs, d_off, msg_base, d_accept, bucket, 0, n);
  for (uint64_t base = 0; base < n; base += c.chunk) {
    va.base = base;
    va.n = (n - base) < c.chunk ? (n - base) : c.chunk;
    if ((err = launch_prep(bucket_ctr(c.st, 0), va, d_off, bucket, s)) || (err = launch_main(va, s))) return err;
  }
  HIPOK(hipEventRecord(c.st_done, s), "record scratch");
  return 0;
}

// A small asynchronous batch on its slot's own scratch (cb, grown to the
// batch by the caller once the slot's previous batch is complete) and stream:
// no ordering against the shared scratch, so batches of different slots run
// concurrently.  Chunks of at most c.chunk, as launch() walks them.
int launch_own(DevCtx& c, ChunkBufs& cb, const uint8_t* d_sigs, const uint8_t* d_pks, const uint8_t* d_msgs,
               const uint64_t* d_off, uint64_t msg_base, uint64_t n, uint8_t* d_accept, hipStream_t s,
               uint32_t flags) {
  if (n == 0) return 0;
  const bool bucket = bucketing_enabled(c, flags);
  VerifyArgs va = make_args(c, cb, d_sigs, d_pks, d_msgs, d_off, msg_base, d_accept, bucket, 0, n);
  const uint64_t step = c.chunk < cb.cap ? c.chunk : cb.cap;
  int err;
  for (uint64_t base = 0; base < n; base += step) {
    va.base = base;
    va.n = (n - base) < step ? (n - base) : step;
    if ((err = launch_prep(bucket_ctr(cb, 0), va, d_off, bucket, s)) || (err = launch_main(va, s))) return err;
  }
  return 0;
}

int pipe_init(DevCtx& c) {
  if (c.pipe_ready) return 0;
  if (!c.sp) HIPOK(hipStreamCreateWithFlags(&c.sp, hipStreamNonBlocking), "hipStreamCreate");
  if (!c.sm) HIPOK(hipStreamCreateWithFlags(&c.sm, hipStreamNonBlocking), "hipStreamCreate");
  for (int b = 0; b < 2; b++) {
    if (!c.prep_done[b]) HIPOK(hipEventCreateWithFlags(&c.prep_done[b], hipEventDisableTiming), "event");
    if (!c.main_done[b]) HIPOK(hipEventCreateWithFlags(&c.main_done[b], hipEventDisableTiming), "event");
    if (!c.perm_done[b]) HIPOK(hipEventCreateWithFlags(&c.perm_done[b], hipEventDisableTiming), "event");
  }
  if (!c.inputs_ready) HIPOK(hipEventCreateWithFlags(&c.inputs_ready, hipEventDisableTiming), "event");
  c.pipe_ready = true;
  return 0;
}

// Pipelined path: chunk k's prep goes on stream sp into state set k%2 (after
// the main kernel that last read that set), its main on stream sm after that
// prep.  Work already queued on the library stream (e.g. the batch signer)
// is ordered before the first prep.  Caller holds c.mu.
int launch_pipelined(DevCtx& c, const uint8_t* d_sigs, const uint8_t* d_pks, const uint8_t* d_msgs,
                     const uint64_t* d_off, uint64_t msg_base, uint64_t n, uint8_t* d_accept, uint32_t flags) {
  int err;
  if ((err = pipe_init(c))) return err;
  const bool bucket = bucketing_enabled(c, flags);
  const bool split = (flags & EDV_FLAG_SPLIT_PREP) != 0;
  HIPOK(hipEventRecord(c.inputs_ready, c.stream), "record");
  HIPOK(hipStreamWaitEvent(c.sp, c.inputs_ready, 0), "wait");
  if (split) HIPOK(hipStreamWaitEvent(c.sm, c.inputs_ready, 0), "wait");
  for (uint64_t base = 0; base < n; base += c.chunk) {
    const int b = c.next;
    c.next ^= 1;
    ChunkBufs& cb = c.pst[b];
    const uint64_t cn = (n - base) < c.chunk ? (n - base) : c.chunk;
    if (!cb.fits(cn)) {  // state set b grows: its last main kernel must be done
      if (c.pending[b]) HIPOK(hipEventSynchronize(c.main_done[b]), "pipeline sync");
      if (cb.ensure(cn, c.chunk)) return EDV_E_OOM;
    }
    VerifyArgs va = make_args(c, cb, d_sigs, d_pks, d_msgs, d_off, msg_base, d_accept, bucket, 0, n);
    va.base = base;
    va.n = cn;
    if (c.pending[b]) HIPOK(hipStreamWaitEvent(c.sp, c.main_done[b], 0), "wait");
    if (split) {
      // Split prep: the hash side (one latency-bound SHA-512 chain per lane,
      // light on issue) goes on sp, where it runs beside the main kernel of the
      // previous chunk; the two point sides (issue-bound exponentiations) go on
      // sm in front of this chunk's main kernel, which waits for the hash side.
      // State set b's previous main kernel ran on sm, so sm needs no wait for
      // it; sp waited for it above.
      if (bucket) {
        if ((err = launch_buckets(bucket_ctr(cb, 0), va, d_off, c.sp))) return err;
        HIPOK(hipEventRecord(c.perm_done[b], c.sp), "record");
        HIPOK(hipStreamWaitEvent(c.sm, c.perm_done[b], 0), "wait");
      }
      VerifyArgs vh = va, vp = va;
      vh.side0 = 0;
      vh.nsides = 1;
      vp.side0 = 1;
      vp.nsides = 2;
      if ((err = launch_prep_sides(vh, c.sp))) return err;
      HIPOK(hipEventRecord(c.prep_done[b], c.sp), "record");
      if ((err = launch_prep_sides(vp, c.sm))) return err;
      HIPOK(hipStreamWaitEvent(c.sm, c.prep_done[b], 0), "wait");
      if ((err = launch_main(va, c.sm, true))) return err;
      HIPOK(hipEventRecord(c.main_done[b], c.sm), "record");
      c.pending[b] = true;
      continue;
    }
    if ((err = launch_prep(bucket_ctr(cb, 0), va, d_off, bucket, c.sp))) return err;
    HIPOK(hipEventRecord(c.prep_done[b], c.sp), "record");
    HIPOK(hipStreamWaitEvent(c.sm, c.prep_done[b], 0), "wait");
    if ((err = launch_main(va, c.sm))) return err;
    HIPOK(hipEventRecord(c.main_done[b], c.sm), "record");
    c.pending[b] = true;
  }
  return 0;
}

// Drain every stream of the context (before scratch is reallocated).
int drain(DevCtx& c) {
  HIPOK(hipStreamSynchronize(c.stream), "stream sync");
  HIPOK(hipEventSynchronize(c.st_done), "scratch sync");
  for (int q = 0; q < kQ; q++) HIPOK(hipStreamSynchronize(c.hs[q]), "stream sync");
  if (c.hcp) HIPOK(hipStreamSynchronize(c.hcp), "stream sync");
  if (c.hac) HIPOK(hipStreamSynchronize(c.hac), "stream sync");  // async batches stay pending until edv_wait_async
  for (auto& s : c.as)
    if (s.st) HIPOK(hipStreamSynchronize(s.st), "stream sync");
  if (c.pipe_ready) {
    HIPOK(hipStreamSynchronize(c.sp), "pipeline sync");
    HIPOK(hipStreamSynchronize(c.sm), "pipeline sync");
    c.pending[0] = c.pending[1] = false;
  }
  return 0;
}

// Best effort after a failed host-path call: wait for whatever was already
// queued on the context's streams (copies may still read the caller's pinned
// buffers), so no DMA touches them after the error is returned.
void quiesce(DevCtx& c) {
  hipStream_t ss[] = {c.stream, c.hcp, c.hac, c.sp, c.sm};
  for (hipStream_t x : ss)
    if (x) (void)hipStreamSynchronize(x);
  for (int q = 0; q < kQ; q++)
    if (c.hs[q]) (void)hipStreamSynchronize(c.hs[q]);
  (void)hipGetLastError();
}

// ---- host memory: pinned detection and a parallel staging copy
bool is_pinned(const void* p) {
  if (!p) return false;
  hipPointerAttribute_t attr;
  if (hipPointerGetAttributes(&attr, p) != hipSuccess) {
    (void)hipGetLastError();  // pageable memory: not an error for us
    return false;
  }
  return attr.type == hipMemoryTypeHost;
}

struct Seg {
  uint8_t* dst;
  const uint8_t* src;
  uint64_t n;
};
int copy_threads() {
  static const int t = [] {
    if (const char* e = getenv("EDV_COPY_THREADS")) {
      const long v = strtol(e, nullptr, 10);
      if (v >= 1 && v <= 64) return int(v);
    }
    const unsigned hw = std::thread::hardware_concurrency();
    return int(hw >= 16 ? 8 : (hw >= 2 ? hw / 2 : 1));
  }();
  return t;
}
// memcpy of several segments, split evenly by bytes over up to copy_threads()
// threads (a single thread below 4 MiB)
void par_copy(const std::vector<Seg>& segs) {
  uint64_t total = 0;
  for (const Seg& s : segs) total += s.n;
  const int T = total < (uint64_t(4) << 20) ? 1 : copy_threads();
  auto part = [&](int t) {
    const uint64_t lo = total * t / T, hi = total * (t + 1) / T;
    uint64_t pos = 0;
    for (const Seg& s : segs) {
      const uint64_t a = lo > pos ? lo - pos : 0, b = hi - pos < s.n ? hi - pos : s.n;
      if (hi > pos && a < b && a < s.n) memcpy(s.dst + a, s.src + a, b - a);
      pos += s.n;
      if (pos >= hi) break;
    }
  };
  if (T == 1) { part(0); return; }
  std::vector<std::thread> th;
  for (int t = 1; t < T; t++) th.emplace_back(part, t);
  part(0);
  for (auto& x : th) x.join();
}

// One pinned block per batch: signatures | keys | offsets | messages (+ 64
// bytes of read slack), copied to the device in ONE DMA (each separate copy
// costs the DMA engine a gap, trace_sync); signatures and keys stay 16-byte
// aligned, offsets 8-byte aligned.
uint64_t quad_pack_bytes(uint64_t n, uint64_t mbytes) { return 96 * n + 8 * (n + 1) + mbytes + 64; }
void quad_pack(uint8_t* dst, const uint8_t* sigs, const uint8_t* pks, const uint8_t* msgs, const uint64_t* off,
               uint64_t lo, uint64_t hi) {
  const uint64_t n = hi - lo, mbase = off[lo], mbytes = off[hi] - mbase;
  par_copy({{dst, sigs + 64 * lo, 64 * n},
            {dst + 64 * n, pks + 32 * lo, 32 * n},
            {dst + 96 * n, reinterpret_cast<const uint8_t*>(off + lo), 8 * (n + 1)},
            {dst + 96 * n + 8 * (n + 1), mbytes ? msgs + mbase : nullptr, mbytes}});
  memset(dst + 96 * n + 8 * (n + 1) + mbytes, 0, 64);
}
// Pageable inputs of a latency-path batch are packed into page-locked staging
// anyway; the quad kernel then reads them from there over PCIe (its phase 1
// reads each input once, at its start) instead of waiting for a DMA of them:
// EDV_QUAD_ZERO_COPY=0 turns that off (A/B).
bool quad_zero_copy() {
  static const bool on = [] {
    const char* e = getenv("EDV_QUAD_ZERO_COPY");
    return !(e && !strcmp(e, "0"));
  }();
  return on;
}
// Device pointers of a latency-path batch
struct QuadIn {
  const uint8_t *sigs, *pks, *msgs;
  const uint64_t* off;
};
// Requests [lo, hi) into device buffer `blob` on stream s for the quad kernel.
// Pinned inputs (the native authenticator's page-locked arena, edv_host_alloc)
// are DMA'd straight from the caller's memory -- signatures, keys and offsets
// in one copy when they lie in one host region in that order, then the
// messages: no host copy on the Node's thread; pageable inputs are packed into
// the pinned `stage` (quad_pack) and copied in one DMA.
int quad_upload(DevBuf& blob, PinnedBuf& stage, const uint8_t* sigs, const uint8_t* pks, const uint8_t* msgs,
                const uint64_t* off, uint64_t lo, uint64_t hi, hipStream_t s, QuadIn* d) {
  const uint64_t n = hi - lo, mbase = off[lo], mbytes = off[hi] - mbase;
  const uint8_t *src_s = sigs + 64 * lo, *src_p = pks + 32 * lo, *src_m = msgs + mbase;
  const uint8_t* src_o = reinterpret_cast<const uint8_t*>(off + lo);
  const bool pinned = is_pinned(src_s) && is_pinned(src_p) && is_pinned(src_o) && (mbytes == 0 || is_pinned(src_m));
  if (!pinned) {
    const uint64_t bytes = quad_pack_bytes(n, mbytes);
    if (stage.ensure(bytes)) return EDV_E_OOM;
    quad_pack(static_cast<uint8_t*>(stage.p), sigs, pks, msgs, off, lo, hi);
    if (quad_zero_copy() && stage.dev) {
      uint8_t* b = static_cast<uint8_t*>(stage.dev);  // read in place (the staging's previous user is done)
      *d = {b, b + 64 * n, b + 96 * n + 8 * (n + 1), reinterpret_cast<const uint64_t*>(b + 96 * n)};
      return 0;
    }
    if (blob.ensure(bytes)) return EDV_E_OOM;
    HIPOK(hipMemcpyAsync(blob.p, stage.p, bytes, hipMemcpyHostToDevice, s), "h2d packed");
    uint8_t* b = static_cast<uint8_t*>(blob.p);
    *d = {b, b + 64 * n, b + 96 * n + 8 * (n + 1), reinterpret_cast<const uint64_t*>(b + 96 * n)};
    return 0;
  }
  const uintptr_t as = reinterpret_cast<uintptr_t>(src_s), ap = reinterpret_cast<uintptr_t>(src_p),
                  ao = reinterpret_cast<uintptr_t>(src_o);
  const bool one = ap >= as + 64 * n && ao >= ap + 32 * n && ao + 8 * (n + 1) - as <= 104 * n + 8 + 4096 &&
                   (ap - as) % 16 == 0 && (ao - as) % 8 == 0;
  const uint64_t span = one ? ao + 8 * (n + 1) - as : 96 * n + 8 * (n + 1);
  const uint64_t moff = (span + 15) / 16 * 16;
  if (blob.ensure(moff + mbytes + 64)) return EDV_E_OOM;
  uint8_t* b = static_cast<uint8_t*>(blob.p);
  if (one) {
    HIPOK(hipMemcpyAsync(b, src_s, span, hipMemcpyHostToDevice, s), "h2d sigs+pks+off");
    *d = {b, b + (ap - as), b + moff, reinterpret_cast<const uint64_t*>(b + (ao - as))};
  } else {
    HIPOK(hipMemcpyAsync(b, src_s, 64 * n, hipMemcpyHostToDevice, s), "h2d sigs");
    HIPOK(hipMemcpyAsync(b + 64 * n, src_p, 32 * n, hipMemcpyHostToDevice, s), "h2d pks");
    HIPOK(hipMemcpyAsync(b + 96 * n, src_o, 8 * (n + 1), hipMemcpyHostToDevice, s), "h2d off");
    *d = {b, b + 64 * n, b + moff, reinterpret_cast<const uint64_t*>(b + 96 * n)};
  }
  if (mbytes) HIPOK(hipMemcpyAsync(b + moff, src_m, mbytes, hipMemcpyHostToDevice, s), "h2d msgs");
  return 0;
}
// memcpy of src[0, bounds[K]) into pinned staging over copy_threads() threads,
// part by part (part k = [bounds[k], bounds[k+1])), with part k's DMA to the
// device queued on stream s -- and ev[k], if given, recorded after it -- as
// soon as every thread has copied its share of it, so the staging of part k+1
// overlaps the DMA of part k (pageable inputs of a synchronous call: the
// messages, 71 % of a C2 batch's bytes).  A copy below 8 MiB is staged by one
// par_copy per part.
int stage_and_send(uint8_t* dev, uint8_t* stage, const uint8_t* src, const uint64_t* bounds, int K, hipStream_t s,
                   const hipEvent_t* ev) {
  const uint64_t bytes = bounds[K] - bounds[0];
  auto send = [&](int k) -> int {
    const uint64_t c0 = bounds[k], c1 = bounds[k + 1];
    if (c1 > c0) HIPOK(hipMemcpyAsync(dev + c0, stage + c0, c1 - c0, hipMemcpyHostToDevice, s), "h2d part");
    if (ev) HIPOK(hipEventRecord(ev[k], s), "record");
    return 0;
  };
  if (bytes < (uint64_t(8) << 20)) {
    int err;
    for (int k = 0; k < K; k++) {
      par_copy({{stage + bounds[k], src + bounds[k], bounds[k + 1] - bounds[k]}});
      if ((err = send(k))) return err;
    }
    return 0;
  }
  const int T = copy_threads();
  std::vector<std::atomic<int>> done(K);
  for (auto& d : done) d.store(0);
  auto part = [&](int t) {
    for (int k = 0; k < K; k++) {
      const uint64_t c0 = bounds[k], c1 = bounds[k + 1];
      const uint64_t a = c0 + (c1 - c0) * t / T, b = c0 + (c1 - c0) * (t + 1) / T;
      memcpy(stage + a, src + a, b - a);
      done[k].fetch_add(1, std::memory_order_release);
    }
  };
  std::vector<std::thread> th;
  for (int t = 1; t < T; t++) th.emplace_back(part, t);
  int err = 0;
  for (int k = 0; k < K; k++) {
    const uint64_t c0 = bounds[k], c1 = bounds[k + 1];
    memcpy(stage + c0, src + c0, (c1 - c0) / T);  // thread 0's share of part k
    while (done[k].load(std::memory_order_acquire) < T - 1) std::this_thread::yield();
    if (!err) err = send(k);
  }
  for (auto& x : th) x.join();
  return err;
}

uint64_t sha512_blocks(const uint64_t* off, uint64_t i) { return (64 + (off[i + 1] - off[i]) + 17 + 127) / 128; }
// One branch-free pass over the offsets of requests [lo, hi): are they
// non-decreasing, and do all messages have request lo's SHA-512 block count?
// (It vectorises: at C2 the two early-exit loops it replaces took ~0.1 ms of a
// synchronous call's host time before the first copy.)
struct OffScan {
  bool ok, uniform;
};
// Built twice (target_clones): an AVX2 clone, picked at load time on hosts
// that have it (the C2 scan in ~20 us), and the x86-64 baseline for the rest;
// the rest of the library's host code is baseline x86-64.
#if defined(__HIP_DEVICE_COMPILE__)
#define EDV_HOST_CLONES
#else
#define EDV_HOST_CLONES __attribute__((target_clones("avx2", "default")))
#endif
EDV_HOST_CLONES OffScan scan_offsets(const uint64_t* off, uint64_t lo,
                                                                        uint64_t hi) {
  const uint64_t nb0 = sha512_blocks(off, lo);
  uint64_t bad = 0, diff = 0;
  for (uint64_t i = lo; i < hi; i++) {
    const uint64_t a = off[i], b = off[i + 1];
    bad |= uint64_t(b < a);
    diff |= ((64 + (b - a) + 17 + 127) >> 7) ^ nb0;  // garbage when b < a: then bad is set
  }
  return {bad == 0, diff == 0};
}

// A shard of one chunk, copied field by field (the default host path for a
// shard that fits one chunk).  Splitting the copy by requests cannot help: a
// sub-batch's kernels take a whole batch's time (latency-bound lanes, DESIGN.md
// section 3).  Splitting it by input field can: the two point sides need only
// the signatures (R) and keys (A), 27 % of the bytes, and the hash side only
// the messages (71 %) besides.  So: H2D of sigs, pks and offsets (one copy
// when they are contiguous), then of the messages in `slices` slices by request,
// on the copy stream; the point sides (and the length buckets) start on stream
// hs[0] as soon as the first part is in, while the messages still copy; the
// hash side of each slice as soon as its messages are in (one slice: in order
// on hs[0]; several: on hs[1..3] in turn), so only the last slice's hash side
// is left after the copy; the main kernel on hs[0] after all of them, writing
// the verdicts straight into page-locked host memory.  Length-bucketed shards
// (messages of several SHA-512 block counts) hash in one piece after the whole
// copy: the bucket permutation spans the shard.  Anatomy of a C2 call:
// DESIGN.md section 3, "The synchronous call".  Caller holds c.mu.
// uniform: 1 / 0 = the offsets were checked and every message has (not) one
// SHA-512 block count; -1 = not checked yet: the check runs here, on the host,
// while the first copy (whose size depends on n only) is already on its way,
// and a failed check returns EDV_E_ARG before anything reads the offsets.
int run_shard_fields(DevCtx& c, const uint8_t* sigs, const uint8_t* pks, const uint8_t* msgs, const uint64_t* off,
                     uint64_t lo, uint64_t hi, bool pinned, int uniform, uint8_t* d_sigs, uint8_t* d_pks,
                     uint8_t* d_msgs, uint64_t* d_off, uint8_t* d_acc, uint8_t* h_acc) {
  const uint64_t n = hi - lo, mbase = off[lo], mbytes = off[hi] - mbase;
  const hipStream_t cp = c.hcp, s0 = c.hs[0];
  int err;
  if ((err = grow_state(c, n))) return err;
  // the scratch's previous users (any stream) finish before the kernels write it,
  // and the copies follow the previous call's (nothing to wait for when its
  // last user is already done, e.g. the previous synchronous call)
  if (hipEventQuery(c.st_done) != hipSuccess) {
    (void)hipGetLastError();
    HIPOK(hipStreamWaitEvent(cp, c.st_done, 0), "wait scratch");
    for (int q = 0; q < kQ; q++) HIPOK(hipStreamWaitEvent(c.hs[q], c.st_done, 0), "wait scratch");
  }
  const uint8_t *src_s = sigs + 64 * lo, *src_p = pks + 32 * lo, *src_m = msgs + mbase;
  const uint8_t* src_o = reinterpret_cast<const uint8_t*>(off + lo);
  PinnedBuf& sl = c.stage[0];
  if (!pinned) {
    HIPOK(hipEventSynchronize(c.hs_staged[0]), "stage wait");  // the slot's previous H2D is done
    if (sl.ensure(n * 96 + (n + 1) * 8 + mbytes)) return EDV_E_OOM;
    uint8_t* p = static_cast<uint8_t*>(sl.p);
    par_copy({{p, src_s, 64 * n}, {p + 64 * n, src_p, 32 * n}, {p + 96 * n, src_o, 8 * (n + 1)}});
    src_s = p; src_p = p + 64 * n; src_o = p + 96 * n;
  }
  // Signatures, keys and offsets that lie in one host region in that order
  // (always so once staged; so for a caller that packs a batch into one
  // pinned buffer) go in ONE copy into a device block of the same layout: each
  // separate copy costs the DMA engine a gap (~12 us each, trace_sync).
  const uintptr_t as = reinterpret_cast<uintptr_t>(src_s), ap = reinterpret_cast<uintptr_t>(src_p),
                  ao = reinterpret_cast<uintptr_t>(src_o);
  const uint64_t gp = ap - as, go = ao - as, span = go + 8 * (n + 1);
  if (ap >= as + 64 * n && ao >= ap + 32 * n && span <= 104 * n + 8 + 4096 && gp % 16 == 0 && go % 8 == 0) {
    if (c.fblob.ensure(span)) return EDV_E_OOM;
    uint8_t* blob = static_cast<uint8_t*>(c.fblob.p);
    d_sigs = blob;
    d_pks = blob + gp;
    d_off = reinterpret_cast<uint64_t*>(blob + go);
    HIPOK(hipMemcpyAsync(blob, src_s, span, hipMemcpyHostToDevice, cp), "h2d sigs+pks+off");
  } else {
    HIPOK(hipMemcpyAsync(d_sigs, src_s, n * 64, hipMemcpyHostToDevice, cp), "h2d sigs");
    HIPOK(hipMemcpyAsync(d_pks, src_p, n * 32, hipMemcpyHostToDevice, cp), "h2d pks");
    HIPOK(hipMemcpyAsync(d_off, src_o, (n + 1) * 8, hipMemcpyHostToDevice, cp), "h2d off");
  }
  if (uniform < 0) {
    const OffScan sc = scan_offsets(off, lo, hi);
    if (!sc.ok) {
      HIPOK(hipStreamSynchronize(cp), "stream sync");  // nothing may read the caller's buffers after we return
      return set_err(EDV_E_ARG, "msg_off not non-decreasing");
    }
    uniform = sc.uniform ? 1 : 0;
  }
  const bool bucket = bucketing_enabled(c, uniform ? EDV_FLAG_UNIFORM_LENGTH : EDV_FLAG_BUCKETS);
  // one slice per 65,536 requests (a slice's hash side takes a whole wave's
  // latency at any size below that, so smaller slices only add copy gaps:
  // profiles/r05/trace_sync_s1.json), at most kSlices; edv_set_host_slices
  // overrides; a bucketed shard is one slice
  int K = bucket ? 1 : (c.host_slices ? c.host_slices : int(n / kMinSliceReqs));
  if (K < 1) K = 1;
  if (K > kSlices) K = kSlices;
  if (uint64_t(K) * kBlock > n) K = int(n / kBlock) > 1 ? int(n / kBlock) : 1;
  uint64_t rb[kSlices + 1], mb[kSlices + 1];  // request / message-byte bounds of the slices (shard-relative)
  for (int k = 0; k <= K; k++) {
    rb[k] = k == K ? n : (n * k / K) / kBlock * kBlock;
    mb[k] = off[lo + rb[k]] - mbase;
  }
  HIPOK(hipEventRecord(c.part_copied[0], cp), "record");
  // The kernels write the verdicts straight into the page-locked host buffer
  // (one 64-byte PCIe write per wave), so no D2H copy and its launch gap follow
  // the main kernel (C2 pinned 1.075 -> 1.046 ms, with the in-stream hash side
  // below 1.033-1.048 ms: profiles/r05/ab_sync_s4.jsonl).
  void* zc = nullptr;
  if (hipHostGetDevicePointer(&zc, h_acc, 0) == hipSuccess && zc) d_acc = static_cast<uint8_t*>(zc);
  else (void)hipGetLastError();
  const bool zc_acc = zc != nullptr;
  // the point sides first: they need only what has just been queued
  VerifyArgs va = make_args(c, c.st, d_sigs, d_pks, d_msgs, d_off, mbase, d_acc, bucket, 0, n);
  va.n = n;
  HIPOK(hipStreamWaitEvent(s0, c.part_copied[0], 0), "wait copy");
  if (bucket && (err = launch_buckets(bucket_ctr(c.st, 0), va, d_off, s0))) return err;
  HIPOK(hipEventRecord(c.part_prepped[0], s0), "record");  // the bucket permutation is written
  VerifyArgs vp = va;
  vp.side0 = 1;
  vp.nsides = 2;
  if ((err = launch_prep_sides(vp, s0))) return err;
  // then the messages, slice by slice (staged in the same slices when pageable)
  if (!pinned) {
    uint8_t* pm = static_cast<uint8_t*>(sl.p) + 96 * n + 8 * (n + 1);
    if (mbytes && (err = stage_and_send(d_msgs, pm, src_m, mb, K, cp, c.slice_copied))) return err;
    if (!mbytes)
      for (int k = 0; k < K; k++) HIPOK(hipEventRecord(c.slice_copied[k], cp), "record");
    HIPOK(hipEventRecord(c.hs_staged[0], cp), "record");
  } else {
    for (int k = 0; k < K; k++) {
      if (mb[k + 1] > mb[k])
        HIPOK(hipMemcpyAsync(d_msgs + mb[k], src_m + mb[k], mb[k + 1] - mb[k], hipMemcpyHostToDevice, cp), "h2d msgs");
      HIPOK(hipEventRecord(c.slice_copied[k], cp), "record");
    }
  }
  for (int k = 0; k < K; k++) {
    // one slice: the hash side in order behind the point sides on s0 (they are
    // done long before the messages land), so main follows it in-stream with no
    // cross-stream event between them
    const hipStream_t hk = K == 1 ? s0 : c.hs[1 + k % (kQ - 1)];
    // requests [rb[k], rb[k+1]) of the shard: scratch slots and request index
    // both start at rb[k] (a bucketed shard is one slice, over the permutation)
    VerifyArgs vh = make_args(c, c.st, d_sigs, d_pks, d_msgs, d_off, mbase, d_acc, bucket, rb[k]);
    vh.base = rb[k];
    vh.n = rb[k + 1] - rb[k];
    vh.side0 = 0;
    vh.nsides = 1;
    HIPOK(hipStreamWaitEvent(hk, c.slice_copied[k], 0), "wait copy");
    if (bucket) HIPOK(hipStreamWaitEvent(hk, c.part_prepped[0], 0), "wait buckets");
    if ((err = launch_prep_sides(vh, hk))) return err;
    HIPOK(hipEventRecord(c.slice_hashed[k], hk), "record");
  }
  if (K > 1)
    for (int k = 0; k < K; k++) HIPOK(hipStreamWaitEvent(s0, c.slice_hashed[k], 0), "wait hash side");
  if ((err = launch_main(va, s0))) return err;
  if (!zc_acc) HIPOK(hipMemcpyAsync(h_acc, d_acc, n, hipMemcpyDeviceToHost, s0), "d2h accept");
  HIPOK(hipEventRecord(c.st_done, s0), "record scratch");
  HIPOK(hipStreamWaitEvent(c.stream, c.st_done, 0), "join");
  HIPOK(hipStreamSynchronize(s0), "stream sync");
  return 0;
}

// The latency path of a synchronous call (a shard of at most c.quad_max
// requests): inputs DMA'd straight from pinned caller memory, or packed into
// the pinned staging block and read there by the kernel (quad_upload), the
// quad kernel, verdicts written straight into page-locked host memory.
// Caller holds c.mu.
int run_shard_quad(DevCtx& c, const uint8_t* sigs, const uint8_t* pks, const uint8_t* msgs, const uint64_t* off,
                   uint64_t lo, uint64_t hi, uint8_t* accept) {
  const uint64_t n = hi - lo, mbase = off[lo];
  const hipStream_t s = c.hs[0];
  // the table-free kernel (n <= kRtlMax) touches no device scratch, so it need
  // not be ordered after (nor before) the scratch's other users; the qblob /
  // qstage / acc buffers are this call's alone while it holds c.mu
  const bool scratch = n > kRtlMax;
  if (scratch && hipEventQuery(c.st_done) != hipSuccess) {  // the scratch's previous user (any stream)
    (void)hipGetLastError();
    HIPOK(hipStreamWaitEvent(s, c.st_done, 0), "wait scratch");
  }
  int err;
  QuadIn d;
  if ((err = quad_upload(c.qblob, c.qstage, sigs, pks, msgs, off, lo, hi, s, &d))) return err;
  const bool acc_pinned = is_pinned(accept + lo);
  if (!acc_pinned && c.acc_host.ensure(n)) return EDV_E_OOM;
  uint8_t* h_acc = acc_pinned ? accept + lo : static_cast<uint8_t*>(c.acc_host.p);
  void* zc = acc_pinned ? nullptr : c.acc_host.dev;
  if (acc_pinned && (hipHostGetDevicePointer(&zc, h_acc, 0) != hipSuccess || !zc)) {
    (void)hipGetLastError();
    zc = nullptr;
  }
  if (!zc && c.acc.ensure(n)) return EDV_E_OOM;
  uint8_t* d_acc = zc ? static_cast<uint8_t*>(zc) : static_cast<uint8_t*>(c.acc.p);
  if ((err = launch_quad(c, c.qtab, d.sigs, d.pks, d.msgs, d.off, mbase, n, d_acc, s))) return err;
  if (!zc) HIPOK(hipMemcpyAsync(h_acc, d_acc, n, hipMemcpyDeviceToHost, s), "d2h accept");
  if (scratch) HIPOK(hipEventRecord(c.st_done, s), "record scratch");
  HIPOK(hipStreamSynchronize(s), "stream sync");
  if (!acc_pinned) memcpy(accept + lo, h_acc, n);
  return 0;
}

// One shard on one device, host buffers: sub-batches of P requests go round
// robin over the kQ host-path streams; per sub-batch: H2D copies (straight
// from the caller's memory when it is pinned, else through this stream's
// pinned slot, filled by a parallel memcpy while earlier sub-batches run),
// [length buckets,] prep, main, D2H of its accept bytes.  Caller holds c.mu.
// uniform: 1 = every message of the whole batch has one SHA-512 block count
// (known from the argument check), 0 = not, so the shard is scanned for it;
// -1 = the offsets are not checked yet (a large one-shard call: the field path
// checks them while its first copy runs, the other paths first thing).
int run_shard(DevCtx& c, const uint8_t* sigs, const uint8_t* pks, const uint8_t* msgs, const uint64_t* off, uint64_t lo,
              uint64_t hi, uint8_t* accept, int uniform) {
  const uint64_t n = hi - lo;
  if (n == 0) return 0;
  if (n <= c.quad_max) return run_shard_quad(c, sigs, pks, msgs, off, lo, hi, accept);
  // A shard that fits one chunk is one sub-batch (the field path): split 2 or
  // 4 ways at 64k it measured 1.6x / 1.9x slower (profiles/r02/e2e_probe_s4.json),
  // as a 16k sub-batch still takes a whole batch's latency at one wave per
  // SIMD.  A larger shard alternates two streams of half-chunk sub-batches, so
  // the H2D copy of one overlaps the kernels of the other.
  const int Q = (n > c.chunk && c.chunk >= 2 * uint64_t(kBlock)) ? 2 : 1;
  const uint64_t pmax = c.chunk / Q;
  uint64_t P = (n + Q - 1) / Q;
  P = ((P + 63) / 64) * 64;
  if (P > pmax) P = pmax;
  const uint64_t nsub = (n + P - 1) / P;
  if (uniform < 0 && nsub != 1) {
    const OffScan sc = scan_offsets(off, lo, hi);
    if (!sc.ok) return set_err(EDV_E_ARG, "msg_off not non-decreasing");
    uniform = sc.uniform ? 1 : 0;
  }
  if (uniform == 0) uniform = scan_offsets(off, lo, hi).uniform ? 1 : 0;  // this shard may be uniform
  const uint64_t mbase = off[lo], mbytes = off[hi] - off[lo];
  if (c.sigs.ensure(n * 64) || c.pks.ensure(n * 32) || c.msgs.ensure(mbytes + 64) ||
      c.off.ensure((n + nsub) * 8) || c.acc.ensure(n))
    return EDV_E_OOM;
  const bool pinned = is_pinned(sigs + 64 * lo) && is_pinned(pks + 32 * lo) && is_pinned(off + lo) &&
                      (mbytes == 0 || is_pinned(msgs + mbase));
  const bool acc_pinned = is_pinned(accept + lo);
  if (!acc_pinned && c.acc_host.ensure(n)) return EDV_E_OOM;
  // bucket by SHA block count only when the shard's messages differ in block count
  const uint32_t flags = uniform == 0 ? EDV_FLAG_BUCKETS : EDV_FLAG_UNIFORM_LENGTH;
  uint8_t* d_sigs = static_cast<uint8_t*>(c.sigs.p);
  uint8_t* d_pks = static_cast<uint8_t*>(c.pks.p);
  uint8_t* d_msgs = static_cast<uint8_t*>(c.msgs.p);
  uint64_t* d_off = static_cast<uint64_t*>(c.off.p);
  uint8_t* d_acc = static_cast<uint8_t*>(c.acc.p);
  uint8_t* h_acc = acc_pinned ? accept + lo : static_cast<uint8_t*>(c.acc_host.p);
  int err;
  // One chunk: copied field by field, the point sides starting before the
  // messages are in.
  if (nsub == 1) {
    if ((err = run_shard_fields(c, sigs, pks, msgs, off, lo, hi, pinned, uniform, d_sigs, d_pks, d_msgs, d_off,
                                d_acc, h_acc)))
      return err;
    if (!acc_pinned) memcpy(accept + lo, h_acc, n);
    return 0;
  }
  hipStream_t* hs = c.hs;
  if ((err = grow_state(c, uint64_t(Q) * pmax))) return err;  // sub-batch stream q uses slots [q pmax, (q + 1) pmax)
  for (int q = 0; q < Q; q++) HIPOK(hipStreamWaitEvent(hs[q], c.st_done, 0), "wait scratch");
  for (uint64_t k = 0; k < nsub; k++) {
    const int q = int(k % Q);
    hipStream_t s = hs[q];
    const uint64_t a = lo + k * P, b = (a + P) < hi ? (a + P) : hi, cnt = b - a;
    const uint64_t mA = off[a], mB = off[b];
    // sub-batch k's offsets live at d_off + (a - lo) + k: one private n+1 window each
    uint64_t* d_o = d_off + (a - lo) + k;
    const uint8_t *src_s = sigs + 64 * a, *src_p = pks + 32 * a, *src_m = msgs + mA;
    const uint64_t* src_o = off + a;
    if (!pinned) {
      // pageable: staged through this stream's pinned slot (a parallel memcpy),
      // then copied by DMA.  (Staging in four parts with each part's H2D queued
      // as soon as it was staged measured slower at C2, 2.43 vs 1.78 ms per 64k:
      // profiles/r02/e2e_probe_s6.json.)
      PinnedBuf& sl = c.stage[q];
      HIPOK(hipEventSynchronize(c.hs_staged[q]), "stage wait");  // the slot's previous H2D is done
      if (sl.ensure(cnt * 96 + (cnt + 1) * 8 + (mB - mA))) return EDV_E_OOM;
      uint8_t* p = static_cast<uint8_t*>(sl.p);
      uint8_t *ps = p, *pp = p + cnt * 64, *po = p + cnt * 96, *pm = p + cnt * 96 + (cnt + 1) * 8;
      par_copy({{ps, src_s, 64 * cnt}, {pp, src_p, 32 * cnt}, {po, reinterpret_cast<const uint8_t*>(src_o), 8 * (cnt + 1)},
                {pm, src_m, mB - mA}});
      HIPOK(hipMemcpyAsync(d_sigs + 64 * (a - lo), ps, 64 * cnt, hipMemcpyHostToDevice, s), "h2d sigs");
      HIPOK(hipMemcpyAsync(d_pks + 32 * (a - lo), pp, 32 * cnt, hipMemcpyHostToDevice, s), "h2d pks");
      HIPOK(hipMemcpyAsync(d_o, po, 8 * (cnt + 1), hipMemcpyHostToDevice, s), "h2d off");
      if (mB > mA) HIPOK(hipMemcpyAsync(d_msgs + (mA - mbase), pm, mB - mA, hipMemcpyHostToDevice, s), "h2d msgs");
    } else {
      HIPOK(hipMemcpyAsync(d_sigs + 64 * (a - lo), src_s, cnt * 64, hipMemcpyHostToDevice, s), "h2d sigs");
      HIPOK(hipMemcpyAsync(d_pks + 32 * (a - lo), src_p, cnt * 32, hipMemcpyHostToDevice, s), "h2d pks");
      HIPOK(hipMemcpyAsync(d_o, src_o, (cnt + 1) * 8, hipMemcpyHostToDevice, s), "h2d off");
      if (mB > mA)
        HIPOK(hipMemcpyAsync(d_msgs + (mA - mbase), src_m, mB - mA, hipMemcpyHostToDevice, s), "h2d msgs");
    }
    if (!pinned) HIPOK(hipEventRecord(c.hs_staged[q], s), "record");
    const bool bucket = bucketing_enabled(c, flags);
    VerifyArgs va = make_args(c, c.st, d_sigs + 64 * (a - lo), d_pks + 32 * (a - lo), d_msgs, d_o, mbase,
                              d_acc + (a - lo), bucket, uint64_t(q) * pmax, n);
    va.n = cnt;
    if ((err = launch_prep(bucket_ctr(c.st, q), va, d_o, bucket, s)) || (err = launch_main(va, s))) return err;
    HIPOK(hipMemcpyAsync(h_acc + (a - lo), d_acc + (a - lo), cnt, hipMemcpyDeviceToHost, s), "d2h accept");
  }
  // join the sub-batch streams into the library stream: the scratch's next user waits for all of them
  for (int q = 0; q < Q; q++) {
    HIPOK(hipEventRecord(c.hs_end[q], hs[q]), "record");
    HIPOK(hipStreamWaitEvent(c.stream, c.hs_end[q], 0), "wait");
  }
  HIPOK(hipEventRecord(c.st_done, c.stream), "record scratch");
  HIPOK(hipStreamSynchronize(c.stream), "stream sync");
  if (!acc_pinned) memcpy(accept + lo, h_acc, n);
  return 0;
}

int launch_sha256(const uint8_t* d_msgs, const uint64_t* d_off, uint64_t msg_base, uint64_t n, uint8_t* d_out,
                  hipStream_t s) {
  if (n == 0) return 0;
  const unsigned blocks = unsigned((n + kBlock - 1) / kBlock);
  HIPOK(launch_sha256_kernel(blocks, s, d_msgs, d_off, msg_base, n, reinterpret_cast<uint32_t*>(d_out)),
        "sha256 launch");
  return 0;
}

// SHA-256 digests of messages [lo, hi) on one device, host buffers; caller holds c.mu
int run_digest_shard(DevCtx& c, const uint8_t* msgs, const uint64_t* off, uint64_t lo, uint64_t hi, uint8_t* out) {
  const uint64_t n = hi - lo;
  if (n == 0) return 0;
  const uint64_t mbase = off[lo], mbytes = off[hi] - off[lo];
  if (c.msgs.ensure(mbytes + 64) || c.off.ensure((n + 1) * 8) || c.sigs.ensure(n * 32)) return EDV_E_OOM;
  // the host verify path shares these buffers; it finishes (synchronously) under the same lock
  if (mbytes) HIPOK(hipMemcpyAsync(c.msgs.p, msgs + mbase, mbytes, hipMemcpyHostToDevice, c.stream), "h2d msgs");
  HIPOK(hipMemcpyAsync(c.off.p, off + lo, (n + 1) * 8, hipMemcpyHostToDevice, c.stream), "h2d off");
  int err;
  if ((err = launch_sha256(static_cast<uint8_t*>(c.msgs.p), static_cast<uint64_t*>(c.off.p), mbase, n,
                           static_cast<uint8_t*>(c.sigs.p), c.stream)))
    return err;
  HIPOK(hipMemcpyAsync(out + 32 * lo, c.sigs.p, n * 32, hipMemcpyDeviceToHost, c.stream), "d2h digests");
  HIPOK(hipStreamSynchronize(c.stream), "stream sync");
  return 0;
}

// Asynchronous host path.  Wait for a slot's batch and hand over its verdicts.
void async_fail(DevCtx& c, DevCtx::AsyncSlot& s) {
  c.ledger.fail(s.ticket);
  s.ticket = -1;
}
int async_complete(DevCtx& c, DevCtx::AsyncSlot& s) {
  if (s.ticket < 0) return 0;
  if (const hipError_t e = hipEventSynchronize(s.done); e != hipSuccess) {
    async_fail(c, s);
    return set_err(EDV_E_HIP, "async wait", e);
  }
#ifdef EDV_MEASUREMENT_API
  if (s.injected) {
    s.injected = false;
    async_fail(c, s);
    return set_err(EDV_E_HIP, "async batch failed (injected by edv_test_fail_async)");
  }
#endif
  if (!s.acc_pinned) memcpy(s.accept, s.acc_host.p, s.n);
  if (s.digests && !s.dig_pinned) memcpy(s.digests, s.dig_host.p, 32 * s.n);
  s.ticket = -1;
  return 0;
}

// An asynchronous latency-path batch on slot s (ticket t, the slot's previous
// batch complete): packed into the slot's pinned staging, one DMA and the quad
// kernel on the slot's own stream, verdicts (and digests) as submit_async's.
int submit_async_quad(DevCtx& c, DevCtx::AsyncSlot& s, int64_t t, const uint8_t* sigs, const uint8_t* pks,
                      const uint8_t* msgs, const uint64_t* off, uint64_t n, uint8_t* accept, uint8_t* digests,
                      int64_t* ticket) {
  const uint64_t mbase = off[0];
  if (!s.st) HIPOK(hipStreamCreateWithFlags(&s.st, hipStreamNonBlocking), "hipStreamCreate");
  if (s.acc.ensure(n) || (digests && s.dig.ensure(32 * n))) return EDV_E_OOM;
  s.dig_pinned = digests && is_pinned(digests);
  if (digests && !s.dig_pinned && s.dig_host.ensure(32 * n)) return EDV_E_OOM;
  s.acc_pinned = is_pinned(accept);
  if (!s.acc_pinned && s.acc_host.ensure(n)) return EDV_E_OOM;
  int err;
  QuadIn d;
  if ((err = quad_upload(s.msgs, s.stage, sigs, pks, msgs, off, 0, n, s.st, &d))) return err;
  uint8_t* h_acc = s.acc_pinned ? accept : static_cast<uint8_t*>(s.acc_host.p);
  void* zc = nullptr;
  if (hipHostGetDevicePointer(&zc, h_acc, 0) != hipSuccess || !zc) {
    (void)hipGetLastError();
    zc = nullptr;
  }
  uint8_t* d_acc = zc ? static_cast<uint8_t*>(zc) : static_cast<uint8_t*>(s.acc.p);
  bool skip = false;  // edv_test_fail_async (measurement build): no kernels, and the wait fails
#ifdef EDV_MEASUREMENT_API
  skip = s.injected = (t == c.inject_fail);
#endif
  if (!skip && (err = launch_quad(c, s.qtab, d.sigs, d.pks, d.msgs, d.off, mbase, n, d_acc, s.st))) return err;
  if (!zc) HIPOK(hipMemcpyAsync(h_acc, d_acc, n, hipMemcpyDeviceToHost, s.st), "d2h accept");
  if (digests && !skip) {
    // Request.getDigest of requests whose signing bytes ARE the message (the
    // caller decides which): SHA-256 of the message bytes already on the device
    uint8_t* d_dig = static_cast<uint8_t*>(s.dig.p);
    if ((err = launch_sha256(d.msgs, d.off, mbase, n, d_dig, s.st)))
      return err;
    uint8_t* h_dig = s.dig_pinned ? digests : static_cast<uint8_t*>(s.dig_host.p);
    HIPOK(hipMemcpyAsync(h_dig, d_dig, 32 * n, hipMemcpyDeviceToHost, s.st), "d2h digests");
  }
  HIPOK(hipEventRecord(s.done, s.st), "record");
  s.ticket = t;
  s.accept = accept;
  s.digests = digests;
  s.n = n;
  *ticket = c.ledger.issue();
  return 0;
}

// Queue one host batch: H2D copies on hcp (from the caller's memory when it is
// pinned, else through the slot's pinned staging, filled here while the
// previous batch computes), then on hac the kernels and the D2H of the
// verdicts; a batch of at most kSmallAsync requests does all of that on its
// slot's own stream and scratch instead.  A slot is reused kAsyncSlots
// submissions later, after its batch is complete.  Caller holds c.mu.
int submit_async(DevCtx& c, const uint8_t* sigs, const uint8_t* pks, const uint8_t* msgs, const uint64_t* off,
                 uint64_t n, uint8_t* accept, uint8_t* digests, bool uniform, int64_t* ticket) {
  const int64_t t = c.ledger.next;
  DevCtx::AsyncSlot& s = c.as[t % kAsyncSlots];
  int err;
  if ((err = async_complete(c, s))) return err;  // the batch of kAsyncSlots submissions ago
  // an unfilled verdict buffer rejects: whatever happens to this batch, no stale
  // byte of a reused buffer can read as "accept"
  memset(accept, 0, n);
  const uint64_t mbase = off[0], mbytes = off[n] - mbase;
  if (s.sigs.ensure(n * 64) || s.pks.ensure(n * 32) || s.msgs.ensure(mbytes + 64) || s.off.ensure((n + 1) * 8) ||
      s.acc.ensure(n) || (digests && s.dig.ensure(32 * n)))
    return EDV_E_OOM;
  // the latency path: the slot's pinned staging packed, one DMA, the quad kernel
  if (n <= c.quad_max) return submit_async_quad(c, s, t, sigs, pks, msgs, off, n, accept, digests, ticket);
  // small batch: everything on the slot's stream and scratch (see kSmallAsync)
  const bool own = n <= kSmallAsync;
  if (own) {
    if (!s.st) HIPOK(hipStreamCreateWithFlags(&s.st, hipStreamNonBlocking), "hipStreamCreate");
    if (s.cb.ensure(n, kSmallAsync)) return EDV_E_OOM;  // the slot's previous batch is complete
  }
  const hipStream_t cs = own ? s.st : c.hcp, ks = own ? s.st : c.hac;
  s.dig_pinned = digests && is_pinned(digests);
  if (digests && !s.dig_pinned && s.dig_host.ensure(32 * n)) return EDV_E_OOM;
  const bool pinned = is_pinned(sigs) && is_pinned(pks) && is_pinned(off) && (mbytes == 0 || is_pinned(msgs + mbase));
  s.acc_pinned = is_pinned(accept);
  if (!s.acc_pinned && s.acc_host.ensure(n)) return EDV_E_OOM;
  const bool varied = !uniform;
  const uint32_t lflags = varied ? EDV_FLAG_BUCKETS : EDV_FLAG_UNIFORM_LENGTH;
  const uint8_t *src_s = sigs, *src_p = pks, *src_m = msgs + mbase;
  const uint8_t* src_o = reinterpret_cast<const uint8_t*>(off);
  if (!pinned) {
    if (s.stage.ensure(n * 96 + (n + 1) * 8 + mbytes)) return EDV_E_OOM;
    uint8_t* p = static_cast<uint8_t*>(s.stage.p);
    par_copy({{p, sigs, 64 * n}, {p + 64 * n, pks, 32 * n}, {p + 96 * n, src_o, 8 * (n + 1)},
              {p + 96 * n + 8 * (n + 1), src_m, mbytes}});
    src_s = p; src_p = p + 64 * n; src_o = p + 96 * n; src_m = p + 96 * n + 8 * (n + 1);
  }
  uint8_t* d_sigs = static_cast<uint8_t*>(s.sigs.p);
  uint8_t* d_pks = static_cast<uint8_t*>(s.pks.p);
  uint8_t* d_msgs = static_cast<uint8_t*>(s.msgs.p);
  uint64_t* d_off = static_cast<uint64_t*>(s.off.p);
  uint8_t* d_acc = static_cast<uint8_t*>(s.acc.p);
  HIPOK(hipMemcpyAsync(d_sigs, src_s, n * 64, hipMemcpyHostToDevice, cs), "h2d sigs");
  HIPOK(hipMemcpyAsync(d_pks, src_p, n * 32, hipMemcpyHostToDevice, cs), "h2d pks");
  HIPOK(hipMemcpyAsync(d_off, src_o, (n + 1) * 8, hipMemcpyHostToDevice, cs), "h2d off");
  if (mbytes) HIPOK(hipMemcpyAsync(d_msgs, src_m, mbytes, hipMemcpyHostToDevice, cs), "h2d msgs");
  if (!own) {
    HIPOK(hipEventRecord(s.copied, c.hcp), "record");
    HIPOK(hipStreamWaitEvent(c.hac, s.copied, 0), "wait copy");
  }
  uint8_t* h_acc = s.acc_pinned ? accept : static_cast<uint8_t*>(s.acc_host.p);
  // verdicts written by the kernels straight into page-locked host memory, as
  // in the synchronous path: no D2H between this batch's main kernel and the
  // next batch's prep on the stream (a C2 stream of batches 0.945 -> 0.965x
  // device-resident, profiles/r05/ab_async_s7.jsonl)
  void* zc = nullptr;
  if (hipHostGetDevicePointer(&zc, h_acc, 0) == hipSuccess && zc) d_acc = static_cast<uint8_t*>(zc);
  else (void)hipGetLastError();
  bool skip = false;  // edv_test_fail_async (measurement build): no kernels, and the wait fails
#ifdef EDV_MEASUREMENT_API
  skip = s.injected = (t == c.inject_fail);
#endif
  if (!skip && (err = own ? launch_own(c, s.cb, d_sigs, d_pks, d_msgs, d_off, mbase, n, d_acc, ks, lflags)
                          : launch(c, d_sigs, d_pks, d_msgs, d_off, mbase, n, d_acc, ks, lflags)))
    return err;
  if (!zc) HIPOK(hipMemcpyAsync(h_acc, d_acc, n, hipMemcpyDeviceToHost, ks), "d2h accept");
  if (digests && !skip) {
    // Request.getDigest of requests whose signing bytes ARE the message (the
    // caller decides which): SHA-256 of the same resident message bytes
    uint8_t* d_dig = static_cast<uint8_t*>(s.dig.p);
    if ((err = launch_sha256(d_msgs, d_off, mbase, n, d_dig, ks))) return err;
    uint8_t* h_dig = s.dig_pinned ? digests : static_cast<uint8_t*>(s.dig_host.p);
    HIPOK(hipMemcpyAsync(h_dig, d_dig, 32 * n, hipMemcpyDeviceToHost, ks), "d2h digests");
  }
  HIPOK(hipEventRecord(s.done, ks), "record");
  s.ticket = t;
  s.accept = accept;
  s.digests = digests;
  s.n = n;
  *ticket = c.ledger.issue();
  return 0;
}

// Per-verify cost in SHA-512-block units for the shard split: W(m) of SURVEY.md
// section 8d is 217,600 + 5,500 * blocks INT32 ops, i.e. ~40 blocks' worth of
// fixed work (decompress, scalar multiplication, encode) per signature.
constexpr uint64_t kVerifyBlocks = 40;

// Split [0, n) into g contiguous shards by request index: equal counts when
// every message has the same SHA-512 block count (C2/C3), else equal estimated
// cost, sum over the shard of (kVerifyBlocks + blocks_i) (C4).
void shard_bounds(const uint64_t* off, uint64_t n, uint32_t g, uint64_t* b, int uniform = -1) {
  b[0] = 0;
  b[g] = n;
  if (g == 1) return;
  if (n == 0 || uniform == 1 || (uniform < 0 && scan_offsets(off, 0, n).uniform)) {
    for (uint32_t k = 1; k < g; k++) b[k] = uint64_t((unsigned __int128)n * k / g);
    return;
  }
  // total cost = kVerifyBlocks * n + sum of blocks; shard k starts at the first
  // request whose prefix cost reaches total * k / g
  unsigned __int128 total = 0;
  for (uint64_t i = 0; i < n; i++) total += kVerifyBlocks + sha512_blocks(off, i);
  unsigned __int128 pre = 0;
  uint32_t k = 1;
  for (uint64_t i = 0; i < n && k < g; i++) {
    while (k < g && pre * g >= total * k) b[k++] = i;
    pre += kVerifyBlocks + sha512_blocks(off, i);
  }
  while (k < g) b[k++] = n;
}

// ---- device placement (several GPUs in one process)
// A shard smaller than one wave per SIMD of a whole MI355X (256 CUs x 4 SIMDs x
// 64 lanes) takes as long as a full one: prep and main run one serial chain per
// lane and a lane's latency, not the lane count, sets the time (profiles/r03/
// e2e_host_parts_s36.jsonl, profiles/r04/latency_vs_n_*.jsonl).  So a batch is
// split only into shards of at least that many requests; a smaller batch (a
// Node's prod: a few hundred, or a single Verifier.verify) runs whole on ONE
// device, with no thread spawned and no other device touched.
// EDV_MIN_SHARD overrides (tests split small batches on purpose).
constexpr uint64_t kMinShard = 65536;
uint64_t min_shard() {
  static const uint64_t v = [] {
    if (const char* e = getenv("EDV_MIN_SHARD")) {
      const long long x = strtoll(e, nullptr, 10);
      if (x >= 1) return uint64_t(x);
    }
    return kMinShard;
  }();
  return v;
}

// Asynchronous batches of a context still running on the GPU: slots holding a
// ticket whose done event has not completed (a batch stops counting as soon as
// it is finished, waited for or not).  If another thread holds the context's
// lock, a call is running there: count it as one.
int async_running(DevCtx& c) {
  std::unique_lock<std::mutex> lk(c.mu, std::try_to_lock);
  if (!lk.owns_lock()) return 1;
  int k = 0;
  for (auto& s : c.as)
    if (s.ticket >= 0 && s.done && hipEventQuery(s.done) == hipErrorNotReady) k++;
  (void)hipGetLastError();  // hipErrorNotReady is not an error of ours
  return k;
}
int device_load(int d) {
  DevCtx& c = *g_ctx[d];
  return c.running.load() + (c.live.load() ? async_running(c) : 0);
}

// Placement of the g shards of a batch on g of the devices `devs` (g == 1: a
// batch that runs on one device).  Preference: initialised devices whose load is
// below `busy_at` (1 for synchronous calls: nothing running; so a process that
// verifies one batch at a time stays on its contexts); then devices not yet
// initialised, in an order that starts at pid mod ndev (the processes of a node
// spread over its GPUs); then the least-loaded busy devices.  Load = synchronous calls placed on the device + its asynchronous
// batches still running.  Chosen devices are reserved (running + 1) under one
// placement lock, so concurrent callers see each other's choices; the caller
// releases them (Placed).
std::mutex g_place_mu;
std::vector<int> place(const std::vector<int>& devs, uint32_t g, int busy_at = 1) {
  const int k = int(devs.size());
  std::vector<int> out;
  std::lock_guard<std::mutex> lk(g_place_mu);
  if (uint32_t(k) <= g) {
    out = devs;
  } else {
    const int start = int(uint64_t(getpid()) % uint64_t(k));
    std::vector<std::pair<int, int>> busy;  // (load, device)
    std::vector<int> idle, fresh;
    for (int j = 0; j < k; j++) {
      const int d = devs[(start + j) % k];
      if (!g_ctx[d]->live.load()) {
        if (g_ctx[d]->running.load()) busy.push_back({g_ctx[d]->running.load(), d});  // being initialised
        else fresh.push_back(d);
        continue;
      }
      const int load = device_load(d);
      if (load < busy_at) idle.push_back(d);
      else busy.push_back({load, d});
    }
    std::stable_sort(busy.begin(), busy.end(), [](const auto& x, const auto& y) { return x.first < y.first; });
    for (int d : idle) out.push_back(d);
    for (int d : fresh) out.push_back(d);
    for (auto& b : busy) out.push_back(b.second);
    out.resize(g);
  }
  for (int d : out) g_ctx[d]->running.fetch_add(1);
  return out;
}
// The asynchronous path's pick (edv_pick_device): an initialised device with
// fewer than two batches running still counts as free -- a Node that keeps one
// prod's batch in flight while it submits the next stays on its context (small
// batches run side by side on their slots' own streams, kSmallAsync), while
// several nodes' prods in flight together spread over the GPUs.
constexpr int kAsyncBusyAt = 2;
int pick_device(const std::vector<int>& devs) {
  if (devs.size() == 1) return devs[0];
  const int d = place(devs, 1, kAsyncBusyAt)[0];
  g_ctx[d]->running.fetch_sub(1);  // a pick only advises (edv_pick_device): no reservation kept
  return d;
}
// Releases a device reserved by place() when the shard on it returns.
struct Placed {
  DevCtx* c;
  ~Placed() { c->running.fetch_sub(1); }
};

std::vector<int> devices_of(uint32_t device_mask, int* err) {
  int ndev;
  {
    std::lock_guard<std::mutex> lk(g_mu);
    ndev = device_count_locked();
  }
  std::vector<int> devs;
  for (int d = 0; d < ndev && d < 32; d++)
    if (device_mask == 0 || (device_mask >> d) & 1u) devs.push_back(d);
  *err = devs.empty() ? set_err(EDV_E_NODEV, "no device selected / visible") : 0;
  return devs;
}

// Validate a host batch and split [0, n) over the devices of device_mask (at
// most one shard per min_shard() requests), one host thread per shard; a batch
// that is one shard runs on the calling thread.  The devices are place()'s
// choice.  shard(ctx, lo, hi) does the work under the context lock.
template <class Shard>
int for_each_shard(const uint64_t* off, uint64_t n, uint32_t device_mask, Shard shard, int uniform = -1) {
  int err;
  std::vector<int> devs = devices_of(device_mask, &err);
  if (err) return err;
  const uint64_t most = n / min_shard();
  const uint32_t g = uint32_t(most < devs.size() ? (most > 1 ? most : 1) : devs.size());
  const std::vector<int> on = place(devs, g);
  auto one = [&](int dev, uint64_t lo, uint64_t hi) {
    Placed placed{g_ctx[dev]};
    CtxLock cl(dev);
    if (cl.err) return cl.err;
    const int rc = shard(*cl.c, lo, hi);
    if (rc) quiesce(*cl.c);
    return rc;
  };
  if (g == 1) return one(on[0], 0, n);
  std::vector<uint64_t> bounds(g + 1);
  shard_bounds(off, n, g, bounds.data(), uniform);
  std::vector<int> rc(g, 0);
  std::vector<std::string> errs(g);
  std::vector<std::thread> th;
  for (uint32_t k = 0; k < g; k++) {
    th.emplace_back([&, k]() {
      rc[k] = one(on[k], bounds[k], bounds[k + 1]);
      errs[k] = g_err;
    });
  }
  for (auto& t : th) t.join();
  for (uint32_t k = 0; k < g; k++)
    if (rc[k]) { g_err = errs[k]; return rc[k]; }
  return 0;
}

// One pass over the offsets: valid (non-decreasing), and -- into *uniform if
// asked -- whether every message has the same SHA-512 block count.
constexpr uint64_t kDeferScanMin = 16384;  // see edv_verify_batch
int check_offsets(const uint64_t* msg_off, uint64_t n, bool* uniform = nullptr) {
  const OffScan sc = scan_offsets(msg_off, 0, n);
  if (!sc.ok) return set_err(EDV_E_ARG, "msg_off not non-decreasing");
  if (uniform) *uniform = sc.uniform;
  return 0;
}

// device pointers the kernels read as 16-byte vectors must be 16-byte aligned
int check_dev_align(const void* d_sigs, const void* d_pks, const void* d_off) {
  if ((reinterpret_cast<uintptr_t>(d_sigs) & 15) || (reinterpret_cast<uintptr_t>(d_pks) & 15) ||
      (reinterpret_cast<uintptr_t>(d_off) & 7))
    return set_err(EDV_E_ARG, "d_sigs / d_pks must be 16-byte and d_msg_off 8-byte aligned");
  return 0;
}

}  // namespace

// ------------------------------------------------------------------ C-ABI
extern "C" {

// Builds whose verdicts are not libsodium's say so in their version string;
// edv.lib() refuses them unless EDV_ALLOW_MEASUREMENT_LIB=1.
#if defined(EDV_MEASURE_NO_VERIFY)
const char* edv_version(void) { return "edv 0.2.0 gfx950 MEASUREMENT-ONLY: verification skipped"; }
#else
const char* edv_version(void) { return "edv 0.2.0 gfx950"; }
#endif
const char* edv_last_error(void) { return g_err.c_str(); }

int edv_device_count(void) {
  std::lock_guard<std::mutex> lk(g_mu);
  return device_count_locked();
}

int edv_context_count(void) {
  std::lock_guard<std::mutex> lk(g_mu);
  const int n = device_count_locked();
  int k = 0;
  for (int d = 0; d < n; d++) k += g_ctx[d]->live.load() ? 1 : 0;
  return k;
}

int edv_context_memory(int device, uint64_t out[7]) {
  g_err.clear();
  if (!out) return set_err(EDV_E_ARG, "null pointer");
  for (int k = 0; k < 7; k++) out[k] = 0;
  int err = 0;
  DevCtx* c = get_ctx(device, &err);
  if (!c) return err;
  std::lock_guard<std::mutex> lk(c->mu);
  if (!c->ready) return 0;
  out[1] = shared_tables_bytes(c->phys);
  out[2] = c->st.bytes();
  for (const auto& a : c->as)
    out[3] += a.sigs.cap + a.pks.cap + a.msgs.cap + a.off.cap + a.acc.cap + a.dig.cap + a.cb.bytes() + a.qtab.cap;
  out[4] = c->pst[0].bytes() + c->pst[1].bytes();
  out[5] = c->sigs.cap + c->pks.cap + c->msgs.cap + c->off.cap + c->acc.cap + c->fblob.cap + c->qblob.cap +
           c->qtab.cap;
  out[6] = c->comb ? uint64_t(kCombRows) * kCombEntries * kBStride * 4 : 0;
  for (int k = 1; k < 7; k++) out[0] += out[k];
  return 0;
}

int edv_pick_device(uint32_t device_mask) {
  g_err.clear();
  int err;
  const std::vector<int> devs = devices_of(device_mask, &err);
  if (err) return err;
  return pick_device(devs);
}

int edv_shard_split(const uint64_t* msg_off, uint64_t n, uint32_t g, uint64_t* bounds) {
  g_err.clear();
  if (!bounds || g == 0 || (n > 0 && !msg_off)) return set_err(EDV_E_ARG, "null pointer / zero shards");
  int err;
  if (n > 0 && (err = check_offsets(msg_off, n))) return err;
  shard_bounds(msg_off, n, g, bounds);
  return 0;
}

int edv_verify_batch(const uint8_t* sigs, const uint8_t* pks, const uint8_t* msgs, const uint64_t* msg_off,
                     uint64_t n, uint8_t* accept, uint32_t device_mask) {
  g_err.clear();
  if (n == 0) return 0;
  if (!sigs || !pks || !msg_off || !accept) return set_err(EDV_E_ARG, "null pointer");
  if (!msgs && msg_off[n] != msg_off[0]) return set_err(EDV_E_ARG, "null msgs");
  int err;
  // A batch that runs as one shard (below 2 x min_shard()) has its offsets
  // checked by the shard path itself, while its first copy is in flight (the
  // scan of a C2 batch's 65,537 offsets is a few tens of microseconds of host
  // time before the first byte would otherwise move); a small batch, or one
  // that is split over devices (the split needs the scan), is checked here.
  int uniform = -1;
  if (msg_off[n] < msg_off[0]) return set_err(EDV_E_ARG, "msg_off not non-decreasing");
  if (n < kDeferScanMin || n / min_shard() >= 2) {
    bool u = false;
    if ((err = check_offsets(msg_off, n, &u))) return err;
    uniform = u ? 1 : 0;
  }
  memset(accept, 0, n);  // fail closed: a call that fails part-way leaves rejections
  return for_each_shard(
      msg_off, n, device_mask,
      [&](DevCtx& c, uint64_t lo, uint64_t hi) { return run_shard(c, sigs, pks, msgs, msg_off, lo, hi, accept, uniform); },
      uniform);
}

int edv_verify_batch_async(const uint8_t* sigs, const uint8_t* pks, const uint8_t* msgs, const uint64_t* msg_off,
                           uint64_t n, uint8_t* accept, int device, int64_t* ticket) {
  return edv_verify_digest_batch_async(sigs, pks, msgs, msg_off, n, accept, nullptr, device, ticket);
}

int edv_verify_digest_batch_async(const uint8_t* sigs, const uint8_t* pks, const uint8_t* msgs,
                                  const uint64_t* msg_off, uint64_t n, uint8_t* accept, uint8_t* digests, int device,
                                  int64_t* ticket) {
  g_err.clear();
  if (!ticket) return set_err(EDV_E_ARG, "null ticket");
  if (n > 0 && (!sigs || !pks || !msg_off || !accept)) return set_err(EDV_E_ARG, "null pointer");
  if (n > 0 && !msgs && msg_off[n] != msg_off[0]) return set_err(EDV_E_ARG, "null msgs");
  int err;
  bool uniform = false;
  if (n > 0 && (err = check_offsets(msg_off, n, &uniform))) return err;
  CtxLock cl(device);
  if (cl.err) return cl.err;
  if (n == 0) {
    *ticket = cl.c->ledger.issue();
    return 0;
  }
  if ((err = submit_async(*cl.c, sigs, pks, msgs, msg_off, n, accept, digests, uniform, ticket))) {
    // whatever was queued before the failure may still read the caller's
    // buffers: let it finish before the caller gets the error back
    (void)hipStreamSynchronize(cl.c->hcp);
    (void)hipStreamSynchronize(cl.c->hac);
    for (auto& s : cl.c->as)
      if (s.st) (void)hipStreamSynchronize(s.st);
    (void)hipGetLastError();
  }
  return err;
}

int edv_wait_async(int device, int64_t ticket) {
  g_err.clear();
  CtxLock cl(device);
  if (cl.err) return cl.err;
  if (!cl.c->ledger.known(ticket)) return set_err(EDV_E_ARG, "unknown ticket");
  for (auto& s : cl.c->as) {
    if (s.ticket != ticket) continue;
    // wait without holding the device lock (other threads keep submitting);
    // a submission that reuses the slot meanwhile completes this batch itself
    const hipEvent_t done = s.done;
    cl.lk.unlock();
    const hipError_t e = hipEventSynchronize(done);
    cl.lk.lock();
    if (e != hipSuccess) {
      if (s.ticket == ticket) async_fail(*cl.c, s);
      return set_err(EDV_E_HIP, "async wait", e);
    }
    if (s.ticket == ticket) return async_complete(*cl.c, s);
    break;  // a submission reusing the slot completed it meanwhile: its outcome is in the ledger
  }
  // already complete (waited for, or its slot was reused) -- unless a batch at
  // or after it failed (sticky, edv_ledger.h)
  if (cl.c->ledger.settled(ticket) != 0) return set_err(EDV_E_HIP, "async batch failed earlier");
  return 0;
}

int edv_query_async(int device, int64_t ticket) {
  g_err.clear();
  CtxLock cl(device);
  if (cl.err) return cl.err;
  if (!cl.c->ledger.known(ticket)) return set_err(EDV_E_ARG, "unknown ticket");
  for (auto& s : cl.c->as) {
    if (s.ticket != ticket) continue;
    const hipError_t e = hipEventQuery(s.done);
    if (e == hipErrorNotReady) {
      (void)hipGetLastError();
      return EDV_PENDING;
    }
    if (e != hipSuccess) {
      async_fail(*cl.c, s);
      return set_err(EDV_E_HIP, "async query", e);
    }
    return async_complete(*cl.c, s);  // done: hand over as edv_wait_async would, without blocking
  }
  if (cl.c->ledger.settled(ticket) != 0) return set_err(EDV_E_HIP, "async batch failed earlier");
  return 0;
}

int edv_sha256_batch(const uint8_t* msgs, const uint64_t* msg_off, uint64_t n, uint8_t* out, uint32_t device_mask) {
  g_err.clear();
  if (n == 0) return 0;
  if (!msg_off || !out) return set_err(EDV_E_ARG, "null pointer");
  if (!msgs && msg_off[n] != msg_off[0]) return set_err(EDV_E_ARG, "null msgs");
  int err;
  if ((err = check_offsets(msg_off, n))) return err;
  return for_each_shard(msg_off, n, device_mask, [&](DevCtx& c, uint64_t lo, uint64_t hi) {
    return run_digest_shard(c, msgs, msg_off, lo, hi, out);
  });
}

int edv_pack_bits_dev(const uint8_t* d_accept, uint64_t n, uint8_t* d_bits, int device, void* stream) {
  g_err.clear();
  if (n == 0) return 0;
  if (!d_accept || !d_bits) return set_err(EDV_E_ARG, "null pointer");
  CtxLock cl(device);
  if (cl.err) return cl.err;
  DevCtx* c = cl.c;
  hipStream_t s = stream ? static_cast<hipStream_t>(stream) : c->stream;
  // after every verify launched on this device so far, on whatever stream:
  // the ordinary paths record st_done after their last kernel, the pipelined
  // path main_done per state set
  HIPOK(hipStreamWaitEvent(s, c->st_done, 0), "wait verdicts");
  if (c->pipe_ready)
    for (int b = 0; b < 2; b++)
      if (c->pending[b]) HIPOK(hipStreamWaitEvent(s, c->main_done[b], 0), "wait verdicts");
  HIPOK(launch_pack_bits_kernel(s, d_accept, n, d_bits), "pack bits launch");
  if (!stream) HIPOK(hipStreamSynchronize(s), "stream sync");
  return 0;
}

int edv_sha256_batch_dev(const uint8_t* d_msgs, const uint64_t* d_msg_off, uint64_t msg_base, uint64_t n,
                         uint8_t* d_out, int device, void* stream) {
  g_err.clear();
  CtxLock cl(device);
  if (cl.err) return cl.err;
  hipStream_t s = stream ? static_cast<hipStream_t>(stream) : cl.c->stream;
  int err;
  if ((err = launch_sha256(d_msgs, d_msg_off, msg_base, n, d_out, s))) return err;
  if (!stream) HIPOK(hipStreamSynchronize(s), "stream sync");
  return 0;
}

int edv_verify_batch_dev_flags(const uint8_t* d_sigs, const uint8_t* d_pks, const uint8_t* d_msgs,
                               const uint64_t* d_msg_off, uint64_t msg_base, uint64_t n, uint8_t* d_accept, int device,
                               void* stream, uint32_t flags) {
  g_err.clear();
  int err;
  if ((err = check_dev_align(d_sigs, d_pks, d_msg_off))) return err;
  CtxLock cl(device);
  if (cl.err) return cl.err;
  hipStream_t s = stream ? static_cast<hipStream_t>(stream) : cl.c->stream;
  if ((err = launch(*cl.c, d_sigs, d_pks, d_msgs, d_msg_off, msg_base, n, d_accept, s, flags))) return err;
  if (!stream) HIPOK(hipStreamSynchronize(s), "stream sync");
  return 0;
}

int edv_verify_batch_dev(const uint8_t* d_sigs, const uint8_t* d_pks, const uint8_t* d_msgs,
                         const uint64_t* d_msg_off, uint64_t msg_base, uint64_t n, uint8_t* d_accept, int device,
                         void* stream) {
  return edv_verify_batch_dev_flags(d_sigs, d_pks, d_msgs, d_msg_off, msg_base, n, d_accept, device, stream, 0);
}

int edv_verify_batch_dev_pipelined(const uint8_t* d_sigs, const uint8_t* d_pks, const uint8_t* d_msgs,
                                   const uint64_t* d_msg_off, uint64_t msg_base, uint64_t n, uint8_t* d_accept,
                                   int device, uint32_t flags) {
  g_err.clear();
  int err;
  if ((err = check_dev_align(d_sigs, d_pks, d_msg_off))) return err;
  CtxLock cl(device);
  if (cl.err) return cl.err;
  if (n == 0) return 0;
  return launch_pipelined(*cl.c, d_sigs, d_pks, d_msgs, d_msg_off, msg_base, n, d_accept, flags);
}

int edv_pipeline_sync(int device) {
  g_err.clear();
  CtxLock cl(device);
  if (cl.err) return cl.err;
  DevCtx* c = cl.c;
  if (!c->pipe_ready) return 0;
  HIPOK(hipStreamSynchronize(c->sp), "pipeline sync");
  HIPOK(hipStreamSynchronize(c->sm), "pipeline sync");
  c->pending[0] = c->pending[1] = false;
  return 0;
}


static int ensure_comb(DevCtx& c) {
  if (c.comb) return 0;
  int32_t* p = nullptr;
  HIPOK(hipMalloc(&p, uint64_t(kCombRows) * kCombEntries * kBStride * 4), "hipMalloc comb");
  hipError_t e = launch_comb_kernel(c.stream, p);
  if (e == hipSuccess) e = hipStreamSynchronize(c.stream);
  if (e != hipSuccess) {
    (void)hipFree(p);
    return set_err(EDV_E_HIP, "comb table", e);
  }
  c.comb = p;
  return 0;
}

int edv_sign_batch_dev(const uint8_t* d_seeds, const uint8_t* d_msgs, const uint64_t* d_msg_off, uint64_t msg_base,
                       uint64_t n, uint8_t* d_pks, uint8_t* d_sigs, int device, void* stream) {
  g_err.clear();
  if ((reinterpret_cast<uintptr_t>(d_seeds) & 15) || (reinterpret_cast<uintptr_t>(d_pks) & 15) ||
      (reinterpret_cast<uintptr_t>(d_sigs) & 15))
    return set_err(EDV_E_ARG, "d_seeds / d_pks / d_sigs must be 16-byte aligned");
  CtxLock cl(device);
  if (cl.err) return cl.err;
  DevCtx* c = cl.c;
  int err;
  if ((err = ensure_comb(*c))) return err;
  if (n == 0) return 0;
  hipStream_t s = stream ? static_cast<hipStream_t>(stream) : c->stream;
  const unsigned blocks = unsigned((n + kBlock - 1) / kBlock);
  HIPOK(launch_sign_kernel(blocks, s, reinterpret_cast<const uint32_t*>(d_seeds), d_msgs, d_msg_off, msg_base, n,
                           reinterpret_cast<uint32_t*>(d_pks), reinterpret_cast<uint32_t*>(d_sigs), c->comb),
        "sign launch");
  if (!stream) HIPOK(hipStreamSynchronize(s), "stream sync");
  return 0;
}

int edv_stream(int device, void** out) {
  g_err.clear();
  CtxLock cl(device);
  if (cl.err) return cl.err;
  *out = static_cast<void*>(cl.c->stream);
  return 0;
}

int edv_sync(int device) {
  g_err.clear();
  CtxLock cl(device);
  if (cl.err) return cl.err;
  HIPOK(hipStreamSynchronize(cl.c->stream), "stream sync");
  return 0;
}

int edv_set_chunk(int device, uint64_t chunk) {
  g_err.clear();
  CtxLock cl(device);
  if (cl.err) return cl.err;
  DevCtx* c = cl.c;
  if (chunk == 0) chunk = kChunkDefault;
  if (chunk < kBlock || chunk > (uint64_t(1) << 24)) return set_err(EDV_E_ARG, "chunk out of range");
  int err;
  if ((err = drain(*c))) return err;  // nothing may still use the scratch being reallocated
  c->chunk = (chunk / kBlock) * kBlock;  // the scratch grows to it by use
  return 0;
}

int edv_set_host_slices(int device, int slices) {
  g_err.clear();
  int err = 0;
  DevCtx* c = get_ctx(device, &err);
  if (!c) return err;
  if (slices < 0 || slices > kSlices) return set_err(EDV_E_ARG, "slices must be 0..8");
  std::lock_guard<std::mutex> lk(c->mu);
  c->host_slices = slices;
  return 0;
}

int edv_set_latency_path(int device, uint64_t max_requests) {
  g_err.clear();
  int err = 0;
  DevCtx* c = get_ctx(device, &err);
  if (!c) return err;
  if (max_requests > kQuadMaxLimit) return set_err(EDV_E_ARG, "latency path is for batches of at most 16,384");
  std::lock_guard<std::mutex> lk(c->mu);
  c->quad_max = max_requests;
  return 0;
}

int edv_set_length_buckets(int device, int mode) {
  g_err.clear();
  int err = 0;
  DevCtx* c = get_ctx(device, &err);
  if (!c) return err;
  if (mode < 0 || mode > 2) return set_err(EDV_E_ARG, "length-bucket mode must be 0, 1 or 2");
  std::lock_guard<std::mutex> lk(c->mu);
  c->length_buckets = mode;
  return 0;
}



int edv_dev_alloc(int device, uint64_t bytes, void** out) {
  int phys, err;
  if ((err = phys_of(device, &phys))) return err;
  HIPOK(hipSetDevice(phys), "hipSetDevice");
  HIPOK(hipMalloc(out, bytes ? bytes : 1), "hipMalloc");
  return 0;
}
int edv_dev_free(int device, void* p) {
  int phys, err;
  if ((err = phys_of(device, &phys))) return err;
  HIPOK(hipSetDevice(phys), "hipSetDevice");
  HIPOK(hipFree(p), "hipFree");
  return 0;
}
int edv_h2d(int device, void* dst, const void* src, uint64_t bytes) {
  int phys, err;
  if ((err = phys_of(device, &phys))) return err;
  HIPOK(hipSetDevice(phys), "hipSetDevice");
  HIPOK(hipMemcpy(dst, src, bytes, hipMemcpyHostToDevice), "hipMemcpy h2d");
  return 0;
}
int edv_d2h(int device, void* dst, const void* src, uint64_t bytes) {
  int phys, err;
  if ((err = phys_of(device, &phys))) return err;
  HIPOK(hipSetDevice(phys), "hipSetDevice");
  HIPOK(hipMemcpy(dst, src, bytes, hipMemcpyDeviceToHost), "hipMemcpy d2h");
  return 0;
}

int edv_host_alloc(uint64_t bytes, void** out) {
  g_err.clear();
  if (!out) return set_err(EDV_E_ARG, "null pointer");
  int n;
  {
    std::lock_guard<std::mutex> lk(g_mu);
    n = device_count_locked();
  }
  if (n == 0) return set_err(EDV_E_NODEV, "no device visible");
  HIPOK(hipSetDevice(g_ctx[0]->phys), "hipSetDevice");
  if (hipHostMalloc(out, bytes ? bytes : 1, hipHostMallocPortable) != hipSuccess) {
    *out = nullptr;
    return set_err(EDV_E_OOM, "hipHostMalloc");
  }
  return 0;
}
int edv_host_free(void* p) {
  g_err.clear();
  if (p) HIPOK(hipHostFree(p), "hipHostFree");
  return 0;
}

}  // extern "C"

#ifdef EDV_MEASUREMENT_API
#include "edv_measure.inc"
#endif
