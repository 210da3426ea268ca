// edv_sha256.h -- batch SHA-256 for the request-digest / state-key hashing on
// the same path, one message per lane.
//
// Replaces, per request:
//   plenum/common/request.py:71-72  Request.getDigest
//       = sha256(serialize_msg_for_signing(signingState())).hexdigest()
//   plenum/server/domain_req_handler.py:166-167  nym_to_state_key
//       = sha256(nym.encode()).digest()
// FIPS 180-4 SHA-256; __host__ __device__ so the identical code is checked
// against hashlib on the CPU (tests/test_math_host.py) before it runs on gfx950.
#pragma once
#include <stdint.h>

#include "edv_math.h"  // EDV_HD, bswap32, funnel32

namespace edv {

EDV_HD uint32_t rotr32(uint32_t x, int n) { return funnel32(x, x, n); }

EDV_HD void sha256_compress(uint32_t H[8], uint32_t W[16]) {
  const uint32_t K[64] = {
      0x428a2f98u, 0x71374491u, 0xb5c0fbcfu, 0xe9b5dba5u, 0x3956c25bu, 0x59f111f1u, 0x923f82a4u, 0xab1c5ed5u,
      0xd807aa98u, 0x12835b01u, 0x243185beu, 0x550c7dc3u, 0x72be5d74u, 0x80deb1feu, 0x9bdc06a7u, 0xc19bf174u,
      0xe49b69c1u, 0xefbe4786u, 0x0fc19dc6u, 0x240ca1ccu, 0x2de92c6fu, 0x4a7484aau, 0x5cb0a9dcu, 0x76f988dau,
      0x983e5152u, 0xa831c66du, 0xb00327c8u, 0xbf597fc7u, 0xc6e00bf3u, 0xd5a79147u, 0x06ca6351u, 0x14292967u,
      0x27b70a85u, 0x2e1b2138u, 0x4d2c6dfcu, 0x53380d13u, 0x650a7354u, 0x766a0abbu, 0x81c2c92eu, 0x92722c85u,
      0xa2bfe8a1u, 0xa81a664bu, 0xc24b8b70u, 0xc76c51a3u, 0xd192e819u, 0xd6990624u, 0xf40e3585u, 0x106aa070u,
      0x19a4c116u, 0x1e376c08u, 0x2748774cu, 0x34b0bcb5u, 0x391c0cb3u, 0x4ed8aa4au, 0x5b9cca4fu, 0x682e6ff3u,
      0x748f82eeu, 0x78a5636fu, 0x84c87814u, 0x8cc70208u, 0x90befffau, 0xa4506cebu, 0xbef9a3f7u, 0xc67178f2u};
  uint32_t a = H[0], b = H[1], c = H[2], d = H[3], e = H[4], f = H[5], g = H[6], h = H[7];
#pragma unroll 1
  for (int r = 0; r < 64; r += 16) {
    if (r > 0) {
#pragma unroll
      for (int t = 0; t < 16; t++) {
        const uint32_t w15 = W[(t + 1) & 15], w2 = W[(t + 14) & 15];
        const uint32_t s0 = xor3_32(rotr32(w15, 7), rotr32(w15, 18), w15 >> 3);
        const uint32_t s1 = xor3_32(rotr32(w2, 17), rotr32(w2, 19), w2 >> 10);
        W[t] += s0 + W[(t + 9) & 15] + s1;
      }
    }
#pragma unroll
    for (int t = 0; t < 16; t++) {
      const uint32_t S1 = xor3_32(rotr32(e, 6), rotr32(e, 11), rotr32(e, 25));
      const uint32_t ch = (e & f) ^ (~e & g);
      const uint32_t t1 = h + S1 + ch + K[r + t] + W[t];
      const uint32_t S0 = xor3_32(rotr32(a, 2), rotr32(a, 13), rotr32(a, 22));
      const uint32_t mj = maj32(a, b, c);
      h = g; g = f; f = e; e = d + t1;
      d = c; c = b; b = a; a = t1 + S0 + mj;
    }
  }
  H[0] += a; H[1] += b; H[2] += c; H[3] += d; H[4] += e; H[5] += f; H[6] += g; H[7] += h;
}

// The 16 big-endian words of a 64-byte block [q0, q0 + 64) that reaches past the
// message end (0x80 pad byte at mlen, zeros after): every dword address clamped
// to the one holding byte mlen (the buffer is readable 8 bytes past the message),
// so the 17 loads issue together, and the masks come from shifts, not selects
// (msg_word32 per word compiled to a load + wait per word).
EDV_HD void msg_words32_tail(uint32_t W[16], const uint8_t* m, uint64_t mlen, uint64_t q0) {
  const uintptr_t a = reinterpret_cast<uintptr_t>(m) + q0;
  const uint32_t sh = uint32_t(a & 3);
  const uintptr_t base = a - sh;
  const uintptr_t last = (reinterpret_cast<uintptr_t>(m) + mlen) & ~uintptr_t(3);
  const int32_t lim = int32_t(int64_t(last) - int64_t(base));  // < 0 for a block wholly past the end
  uint32_t d[17];
#pragma unroll
  for (int t = 0; t < 17; t++) {
    // min(base + 4t, last) as last - max(lim - 4t, 0): one v_max_i32 instead of
    // a 64-bit compare and two VCC-mask selects
    const int32_t back = lim - 4 * t;
    d[t] = *reinterpret_cast<const uint32_t*>(last - uintptr_t(uint32_t(back > 0 ? back : 0)));
  }
  const int32_t rem0 = int32_t(int64_t(mlen) - int64_t(q0));
#pragma unroll
  for (int t = 0; t < 16; t++) {
    const int32_t r = rem0 - 4 * t;
    const int32_t nv = r < 0 ? 0 : (r > 4 ? 4 : r);
    const int32_t nv1 = r + 1 < 0 ? 0 : (r + 1 > 4 ? 4 : r + 1);
    const uint32_t keep = ((1u << (4 * nv)) << (4 * nv)) - 1u;   // low nv bytes (nv = 4: all)
    const uint32_t keep1 = ((1u << (4 * nv1)) << (4 * nv1)) - 1u;
    uint32_t v = uint32_t(((uint64_t(d[t + 1]) << 32) | d[t]) >> (8 * sh));  // little-endian byte order
    v = (v & keep) | ((keep ^ keep1) & 0x80808080u);
    W[t] = bswap32(v);
  }
}

// SHA-256(M) -> 8 big-endian-order words of the digest, stored as bytes by the caller.
EDV_HD void sha256_msg(uint32_t out[8], const uint8_t* m, uint64_t mlen) {
  uint32_t H[8] = {0x6a09e667u, 0xbb67ae85u, 0x3c6ef372u, 0xa54ff53au,
                   0x510e527fu, 0x9b05688cu, 0x1f83d9abu, 0x5be0cd19u};
  const uint64_t nb = (mlen + 8 + 1 + 63) / 64;
  uint32_t W[16];
#pragma unroll 1
  for (uint64_t b = 0; b < nb; b++) {
    if (64 * b + 64 <= mlen) {
      // whole block inside the message (every block but the last one or two):
      // plain funnel-shifted loads, none of the clamp/pad selects, which lower
      // to v_cndmask_b32 with a VCC mask (~23 cycles each on gfx950)
      const uintptr_t a = reinterpret_cast<uintptr_t>(m + 64 * b);
      const uint32_t sh = uint32_t(a & 3);
      const uint32_t* p = reinterpret_cast<const uint32_t*>(a - sh);
      uint32_t d[17];
#pragma unroll
      for (int t = 0; t < 17; t++) d[t] = p[t];
#pragma unroll
      for (int t = 0; t < 16; t++) W[t] = bswap32(uint32_t(((uint64_t(d[t + 1]) << 32) | d[t]) >> (8 * sh)));
    } else {
      msg_words32_tail(W, m, mlen, 64 * b);
    }
    if (b == nb - 1) {
      W[14] = uint32_t(mlen >> 29);
      W[15] = uint32_t(mlen << 3);
    }
    sha256_compress(H, W);
  }
#pragma unroll
  for (int i = 0; i < 8; i++) out[i] = bswap32(H[i]);  // little-endian words of the digest bytes
}

}  // namespace edv
