// edv_hostcheck.cpp -- TEST HARNESS ONLY.  Builds the kernel's own math and
// per-signature algorithm (edv_math.h, edv_verify_core.h) as plain C++ so the
// CPU test suite can check them against the oracle and Python big integers
// without a GPU.  Nothing in the product path (libedv.so, the Python shim)
// loads this library; it is not a fallback.
#include <stdint.h>
#include <string.h>
#include <vector>
#include "edv_verify_core.h"
#include "edv_sha256.h"
#include "edv_ledger.h"

using namespace edv;

namespace {
struct HostATab {
  ge_cached t[kAEntries];
  int staged = 0;
  void store(int e, const ge_cached& c) { t[e] = c; }
  ge_cached load(int e) const { return t[e]; }
  void stage(int e) { staged = e; }
  ge_cached fetch() const { return t[staged]; }
};
// The R side's view of an [S]B table set (large or compact): each entry
// computed when asked for, by the device table's own btab_entry (the sets'
// millions of entries would take minutes to build on one core; a verify needs
// 12 or 16 of them).
struct HostBTab {
  SbShape sh;
  ge_p3 base[kBTablesCompact];
  explicit HostBTab(SbShape s) : sh(s) {
    for (int t = 0; t < sh.tables; t++) base[t] = base_point(t * sh.bits);
  }
  ge_precomp entry(int t, int j) const {
    int32_t w[kBStride];
    btab_entry(w, j, base[t]);
    return precomp_from_words(w);
  }
};
struct HostBStage {
  const HostBTab& b;
  int t = 0, j = 0;
  ge_cached stash;
  SbShape shape() const { return b.sh; }
  void stage(int tt, int jj) { t = tt; j = jj; }
  ge_precomp fetch() const { return b.entry(t, j); }
  void put(const ge_cached& c) { stash = c; }
  ge_cached get() const { return stash; }
};
struct HostComb {
  std::vector<int32_t> w;
  HostComb() : w(kCombRows * kCombEntries * kBStride) {
    for (int i = 0; i < kCombRows; i++)
      for (int j = 0; j < kCombEntries; j++) comb_entry(w.data() + (i * kCombEntries + j) * kBStride, i, j);
  }
  ge_precomp entry(int i, int j) const { return precomp_from_words(w.data() + (i * kCombEntries + j) * kBStride); }
};
const HostComb& comb() {
  static HostComb c;
  return c;
}
static_assert(kBTablesCompact >= kBTables, "base[] holds the larger table count");
const HostBTab& btab(int bits = kBBits) {
  static HostBTab large(sb_large()), compact(sb_compact());
  return bits == kBBitsCompact ? compact : large;
}
void load_words(uint32_t* w, const uint8_t* b, int n) {
  for (int i = 0; i < n; i++) w[i] = uint32_t(b[4 * i]) | uint32_t(b[4 * i + 1]) << 8 | uint32_t(b[4 * i + 2]) << 16 | uint32_t(b[4 * i + 3]) << 24;
}
void store_words(uint8_t* b, const uint32_t* w, int n) {
  for (int i = 0; i < n; i++)
    for (int j = 0; j < 4; j++) b[4 * i + j] = uint8_t(w[i] >> (8 * j));
}
fe to_fe(const int32_t* l) { fe f; for (int i = 0; i < 10; i++) f.v[i] = l[i]; return f; }
void from_fe(int32_t* l, const fe& f) { for (int i = 0; i < 10; i++) l[i] = f.v[i]; }
}  // namespace

extern "C" {
void hc_fe_mul(const int32_t* f, const int32_t* g, int32_t* h) { from_fe(h, fe_mul(to_fe(f), to_fe(g))); }
void hc_fe_sq(const int32_t* f, int32_t* h) { from_fe(h, fe_sq(to_fe(f))); }
void hc_fe_sq_floor(const int32_t* f, int32_t* h) { from_fe(h, fe_sq_floor(to_fe(f))); }
void hc_fe_sq2(const int32_t* f, int32_t* h) { from_fe(h, fe_sq2(to_fe(f))); }
void hc_fe_carry32(const int32_t* f, int32_t* h) { from_fe(h, fe_carry32(to_fe(f))); }
void hc_fe_invert(const int32_t* f, int32_t* h) { from_fe(h, fe_invert(to_fe(f))); }
void hc_fe_invert_safegcd(const int32_t* f, int32_t* h) { from_fe(h, fe_invert_safegcd(to_fe(f))); }
void hc_fe_pow22523(const int32_t* f, int32_t* h) { from_fe(h, fe_pow22523(to_fe(f))); }
void hc_fe_tobytes(const int32_t* f, uint8_t* out) { uint32_t w[8]; fe_tobytes(w, to_fe(f)); store_words(out, w, 8); }
void hc_fe_frombytes(const uint8_t* in, int32_t* h) { uint32_t w[8]; load_words(w, in, 8); from_fe(h, fe_frombytes(w)); }
void hc_sc_reduce(const uint8_t* in64, uint8_t* out32) {
  uint32_t w[16], o[8];
  load_words(w, in64, 16);
  sc_reduce(o, w);
  store_words(out32, o, 8);
}
void hc_hram(const uint8_t* R, const uint8_t* A, const uint8_t* m, uint64_t mlen, uint8_t* out64) {
  uint32_t r[8], a[8], o[16];
  load_words(r, R, 8);
  load_words(a, A, 8);
  // msg_word reads whole aligned words up to 12 bytes past the end: pad a copy
  std::vector<uint8_t> buf(mlen + 32, 0);
  if (mlen) memcpy(buf.data() + 16, m, mlen);
  hram(o, r, a, buf.data() + 16, mlen);
  store_words(out64, o, 16);
}
int hc_decompress_negate(const uint8_t* in, uint8_t* out) {
  uint32_t w[8], o[8];
  load_words(w, in, 8);
  ge_p3 p;
  const bool ok = ge_frombytes_negate(p, w);
  ge_p2_tobytes(o, ge_p3_to_p2(p));
  store_words(out, o, 8);
  return ok ? 0 : -1;
}
// SHA-256 of m at a chosen misalignment of the copy (the kernel reads aligned words)
void hc_sha256(const uint8_t* m, uint64_t mlen, int misalign, uint8_t* out32) {
  std::vector<uint8_t> buf(mlen + 48, 0xA5);
  if (mlen) memcpy(buf.data() + 16 + misalign, m, mlen);
  uint32_t o[8];
  sha256_msg(o, buf.data() + 16 + misalign, mlen);
  store_words(out32, o, 8);
}
// edv_sha256_batch's signature, the kernel's SHA-256 on the CPU (tests hand its
// address to _edvhost.request_digests)
int hc_sha256_batch(const uint8_t* msgs, const uint64_t* off, uint64_t n, uint8_t* out, uint32_t) {
  for (uint64_t i = 0; i < n; i++) {
    const uint64_t mlen = off[i + 1] - off[i];
    std::vector<uint8_t> buf(mlen + 48, 0);
    if (mlen) memcpy(buf.data() + 16, msgs + off[i], mlen);
    uint32_t o[8];
    sha256_msg(o, buf.data() + 16, mlen);
    store_words(out + 32 * i, o, 8);
  }
  return 0;
}
// entries js[0..nj) of table t (j x 2^(bits t) B) of the set with `bits`
// (22 large, 16 compact), kBStride words each
int hc_btab_entries_of_bits(int bits, int t, const int32_t* js, int nj, int32_t* out) {
  if (bits != kBBits && bits != kBBitsCompact) return -1;
  const HostBTab& b = btab(bits);
  if (t < 0 || t >= b.sh.tables) return -1;
  for (int k = 0; k < nj; k++) {
    if (js[k] < 0 || js[k] >= b.sh.entries) return -1;
    btab_entry(out + size_t(k) * kBStride, js[k], b.base[t]);
  }
  return 0;
}
int hc_btab_entries_of(int t, const int32_t* js, int nj, int32_t* out) {
  return hc_btab_entries_of_bits(kBBits, t, js, nj, out);
}
// the R side's Q = [S]B - R against the table set with `bits`, encoded (0),
// or -1 if R is rejected
int hc_rside_point_bits(int bits, const uint8_t* R32, const uint8_t* S32, uint8_t* out32) {
  struct Keep {  // keeps entry 1 of the table: Q itself
    ge_cached q;
    void store(int e, const ge_cached& c) { if (e == 1) q = c; }
  } tab;
  uint32_t R[8], S[8], o[8];
  load_words(R, R32, 8);
  load_words(S, S32, 8);
  if (bits != kBBits && bits != kBBitsCompact) return -1;
  HostBStage bs{btab(bits)};
  if (!prep_rpoint(R, S, tab, bs)) return -1;
  // cached (Y+X, Y-X, Z, 2dT) -> (X : Y : Z)
  const fe two_y = fe_carry32(fe_add(tab.q.YpX, tab.q.YmX)), two_x = fe_carry32(fe_sub(tab.q.YpX, tab.q.YmX));
  ge_p2 p{two_x, two_y, fe_carry32(fe_add(tab.q.Z, tab.q.Z))};
  ge_p2_tobytes(o, p);
  store_words(out32, o, 8);
  return 0;
}
int hc_rside_point(const uint8_t* R32, const uint8_t* S32, uint8_t* out32) {
  return hc_rside_point_bits(kBBits, R32, S32, out32);
}
// the lattice reduction of the prep kernel: (a, u, neg) for h (32-byte scalars)
int hc_half_scalars(const uint8_t* h32, uint8_t* a32, uint8_t* u32) {
  uint32_t h[8], a[8], u[8];
  load_words(h, h32, 8);
  bool neg = false;
  half_scalars(h, a, u, neg);
  store_words(a32, a, 8);
  store_words(u32, u, 8);
  return neg ? 1 : 0;
}
// the walk's layout constants: kAWin, kAEntries, kBBits, kBTables
void hc_layout(int32_t* out4) {
  const int32_t v[4] = {kAWin, kAEntries, kBBits, kBTables};
  memcpy(out4, v, sizeof v);
}
int hc_btab_entries() { return kBEntries; }
// the asynchronous path's ticket ledger (edv_ledger.h): issue n tickets, fail
// the listed ones, then report settled() for each query
void hc_ledger(int64_t n, const int64_t* failed, int nf, const int64_t* queries, int nq, int* out) {
  AsyncLedger l;
  for (int64_t i = 0; i < n; i++) l.issue();
  for (int k = 0; k < nf; k++) l.fail(failed[k]);
  for (int k = 0; k < nq; k++) out[k] = l.settled(queries[k]);
}
// windows the packed radix-2^kAWin digits need (the prep kernel's per-lane count)
int hc_digits_windows(const uint32_t* d8) { return digits5_windows(d8); }
// packed signed digits of a 32-byte scalar at radix 2^bits: 4 (64 digits: the main
// loop's windows at kAWin = 4), 5 (51 digits), 8 -> recode8 (signer)
int hc_recode(const uint8_t* in32, int bits, uint32_t* out8) {
  uint32_t w[8];
  load_words(w, in32, 8);
  if (bits == 4) recode4(out8, w);
  else if (bits == 5) recode5_fixed(out8, w);
  else if (bits == 8) recode8(out8, w);
  else return -1;
  return 0;
}
int hc_sign_batch(const uint8_t* seeds, const uint8_t* msgs, const uint64_t* off, uint64_t n, uint8_t* pks,
                  uint8_t* sigs) {
  const HostComb& ct = comb();
  for (uint64_t i = 0; i < n; i++) {
    uint32_t seed[8], pk[8], sig[16];
    load_words(seed, seeds + 32 * i, 8);
    const uint64_t mlen = off[i + 1] - off[i];
    std::vector<uint8_t> buf(mlen + 32, 0);
    if (mlen) memcpy(buf.data() + 16, msgs + off[i], mlen);
    sign_one(pk, sig, seed, buf.data() + 16, mlen, ct);
    store_words(pks + 32 * i, pk, 8);
    store_words(sigs + 64 * i, sig, 16);
  }
  return 0;
}
int hc_verify_batch(const uint8_t* sigs, const uint8_t* pks, const uint8_t* msgs, const uint64_t* off, uint64_t n,
                    uint8_t* accept) {
  const HostBTab& bt = btab();
  for (uint64_t i = 0; i < n; i++) {
    uint32_t R[8], S[8], A[8];
    load_words(R, sigs + 64 * i, 8);
    load_words(S, sigs + 64 * i + 32, 8);
    load_words(A, pks + 32 * i, 8);
    const uint64_t mlen = off[i + 1] - off[i];
    std::vector<uint8_t> buf(mlen + 32, 0);
    if (mlen) memcpy(buf.data() + 16, msgs + off[i], mlen);
    HostATab at, rt;
    HostBStage bs{bt};
    accept[i] = verify_one(R, S, A, buf.data() + 16, mlen, at, rt, bs) ? 1 : 0;
  }
  return 0;
}
}
