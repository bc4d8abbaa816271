// sha256.h -- SHA-256 of a message, one lane per message.
//
// Request.digest (plenum/common/request.py:51-52) is
//   sha256(serialize_msg_for_signing(request.signingState)).hexdigest(),
// computed for every request at construction (request.py:24).  SURVEY §8(f)
// row 3: an adjacent hash over the same signing bytes the verify path already
// holds in HBM.  The message is read with the 16-byte chunk scheme of
// sha512.h (only chunks holding message bytes; per-lane word-shift selects).
#pragma once
#include "sha512.h"

namespace edv {

#if defined(__HIPCC__)
__device__ __constant__ uint32_t SHA256_K[64] = {
#else
static const uint32_t SHA256_K[64] = {
#endif
    0x428a2f98u, 0x71374491u, 0xb5c0fbcfu, 0xe9b5dba5u, 0x3956c25bu, 0x59f111f1u, 0x923f82a4u, 0xab1c5ed5u,
    0xd807aa98u, 0x12835b01u, 0x243185beu, 0x550c7dc3u, 0x72be5d74u, 0x80deb1feu, 0x9bdc06a7u, 0xc19bf174u,
    0xe49b69c1u, 0xefbe4786u, 0x0fc19dc6u, 0x240ca1ccu, 0x2de92c6fu, 0x4a7484aau, 0x5cb0a9dcu, 0x76f988dau,
    0x983e5152u, 0xa831c66du, 0xb00327c8u, 0xbf597fc7u, 0xc6e00bf3u, 0xd5a79147u, 0x06ca6351u, 0x14292967u,
    0x27b70a85u, 0x2e1b2138u, 0x4d2c6dfcu, 0x53380d13u, 0x650a7354u, 0x766a0abbu, 0x81c2c92eu, 0x92722c85u,
    0xa2bfe8a1u, 0xa81a664bu, 0xc24b8b70u, 0xc76c51a3u, 0xd192e819u, 0xd6990624u, 0xf40e3585u, 0x106aa070u,
    0x19a4c116u, 0x1e376c08u, 0x2748774cu, 0x34b0bcb5u, 0x391c0cb3u, 0x4ed8aa4au, 0x5b9cca4fu, 0x682e6ff3u,
    0x748f82eeu, 0x78a5636fu, 0x84c87814u, 0x8cc70208u, 0x90befffau, 0xa4506cebu, 0xbef9a3f7u, 0xc67178f2u};

EDV_HD uint32_t rotr32(uint32_t x, int n) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_alignbit(x, x, n);
#else
  return (x >> n) | (x << (32 - n));
#endif
}

#define EDV_SHA256_ROUND(KI, WI)                                          \
  {                                                                       \
    const uint32_t S1 = rotr32(e, 6) ^ rotr32(e, 11) ^ rotr32(e, 25);     \
    const uint32_t ch = (e & f) ^ (~e & g);                               \
    const uint32_t t1 = h + S1 + ch + (KI) + (WI);                        \
    const uint32_t S0 = rotr32(a, 2) ^ rotr32(a, 13) ^ rotr32(a, 22);     \
    const uint32_t mj = (a & b) ^ (a & c) ^ (b & c);                      \
    h = g;                                                                \
    g = f;                                                                \
    f = e;                                                                \
    e = d + t1;                                                           \
    d = c;                                                                \
    c = b;                                                                \
    b = a;                                                                \
    a = t1 + S0 + mj;                                                     \
  }

EDV_HD void sha256_compress(uint32_t st[8], uint32_t w[16]) {
  uint32_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], h = st[7];
#pragma unroll
  for (int i = 0; i < 16; ++i) EDV_SHA256_ROUND(SHA256_K[i], w[i])
#pragma unroll 1
  for (int r = 16; r < 64; r += 16) {
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const uint32_t w15 = w[(i + 1) & 15], w2 = w[(i + 14) & 15];
      const uint32_t s0 = rotr32(w15, 7) ^ rotr32(w15, 18) ^ (w15 >> 3);
      const uint32_t s1 = rotr32(w2, 17) ^ rotr32(w2, 19) ^ (w2 >> 10);
      w[i] += s0 + w[(i + 9) & 15] + s1;
      EDV_SHA256_ROUND(SHA256_K[r + i], w[i])
    }
  }
  st[0] += a;
  st[1] += b;
  st[2] += c;
  st[3] += d;
  st[4] += e;
  st[5] += f;
  st[6] += g;
  st[7] += h;
}
#undef EDV_SHA256_ROUND

// Block b (64 bytes) of msg || 0x80 || 0... as 16 big-endian words.
EDV_HD void sha256_block_words(uint32_t w[16], uint64_t b, const Chunk16* c16, uint64_t nq, uint32_t d16,
                               uint64_t mlen) {
  constexpr int NCH = 5;  // 64 bytes at any misalignment
  const uint64_t pos = d16 + 64 * b;
  const uint64_t q0 = pos >> 4;
  const uint32_t s4 = (uint32_t)(pos >> 2) & 3u, sh = d16 & 3u;
  uint32_t W[4 * NCH];
  const int avail = chunks_left(nq, q0);
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    Chunk16 v = {0u, 0u, 0u, 0u};
    if (c < avail) v = c16[q0 + c];
    W[4 * c] = v.x;
    W[4 * c + 1] = v.y;
    W[4 * c + 2] = v.z;
    W[4 * c + 3] = v.w;
  }
  uint32_t V[17];
#pragma unroll
  for (int j = 0; j <= 16; ++j) {
    const uint32_t a0 = W[j], a1 = W[j + 1], a2 = W[j + 2], a3 = W[j + 3];
    V[j] = s4 == 0 ? a0 : s4 == 1 ? a1 : s4 == 2 ? a2 : a3;
  }
  uint32_t le[16];
#pragma unroll
  for (int t = 0; t < 16; ++t) le[t] = funnel8(V[t + 1], V[t], sh);
  const int64_t u0 = 16 * (int64_t)b;
  if (4 * (u0 + 16) > (int64_t)mlen) {
    const int32_t rb = bytes_left(mlen, u0);
#pragma unroll
    for (int t = 0; t < 16; ++t) le[t] = tail_word(le[t], rb - 4 * t);
  }
#pragma unroll
  for (int t = 0; t < 16; ++t) w[t] = bswap32(le[t]);
}

// SHA-256(msg); digest: 8 little-endian u32 words = the 32 digest bytes in order.
EDV_HD void sha256_msg(uint32_t digest[8], const uint8_t* msg, uint64_t mlen) {
  uint32_t st[8] = {0x6a09e667u, 0xbb67ae85u, 0x3c6ef372u, 0xa54ff53au,
                    0x510e527fu, 0x9b05688cu, 0x1f83d9abu, 0x5be0cd19u};
  const uint64_t nblocks = (mlen + 8) / 64 + 1;  // incl. 0x80 and the 64-bit length
  const uint32_t d16 = (uint32_t)((uintptr_t)msg & 15);
  const Chunk16* c16 = (const Chunk16*)(msg - d16);
  const uint64_t nq = (d16 + mlen + 15) / 16;
  const uint64_t bitlen = mlen * 8;
#pragma unroll 1
  for (uint64_t b = 0; b < nblocks; ++b) {
    uint32_t w[16];
    sha256_block_words(w, b, c16, nq, d16, mlen);
    if (b == nblocks - 1) {
      w[14] = (uint32_t)(bitlen >> 32);
      w[15] = (uint32_t)bitlen;
    }
    sha256_compress(st, w);
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) digest[j] = bswap32(st[j]);
}

}  // namespace edv
