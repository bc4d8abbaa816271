// sha512.h -- SHA-512 of (prefix || message), one lane per message.
//
// Restates the hashing inside libsodium 1.0.18's ed25519 verify
// (crypto_hash_sha512 over R || A || M), reached from
// stp_core/crypto/nacl_wrappers.py:108.  The prefix (R||A for verify,
// az[32..64] for the signer's nonce) lives in registers; the message is read
// from global memory as aligned 32-bit words funnel-shifted into place, so any
// byte offset works and no byte past the message end is needed beyond the
// containing aligned word.
#pragma once
#include "fe25519.h"

namespace edv {

#if defined(__HIPCC__)
__device__ __constant__ uint64_t SHA512_K[80] = {
#else
static const uint64_t SHA512_K[80] = {
#endif
    0x428a2f98d728ae22ULL, 0x7137449123ef65cdULL, 0xb5c0fbcfec4d3b2fULL, 0xe9b5dba58189dbbcULL, 0x3956c25bf348b538ULL,
    0x59f111f1b605d019ULL, 0x923f82a4af194f9bULL, 0xab1c5ed5da6d8118ULL, 0xd807aa98a3030242ULL, 0x12835b0145706fbeULL,
    0x243185be4ee4b28cULL, 0x550c7dc3d5ffb4e2ULL, 0x72be5d74f27b896fULL, 0x80deb1fe3b1696b1ULL, 0x9bdc06a725c71235ULL,
    0xc19bf174cf692694ULL, 0xe49b69c19ef14ad2ULL, 0xefbe4786384f25e3ULL, 0x0fc19dc68b8cd5b5ULL, 0x240ca1cc77ac9c65ULL,
    0x2de92c6f592b0275ULL, 0x4a7484aa6ea6e483ULL, 0x5cb0a9dcbd41fbd4ULL, 0x76f988da831153b5ULL, 0x983e5152ee66dfabULL,
    0xa831c66d2db43210ULL, 0xb00327c898fb213fULL, 0xbf597fc7beef0ee4ULL, 0xc6e00bf33da88fc2ULL, 0xd5a79147930aa725ULL,
    0x06ca6351e003826fULL, 0x142929670a0e6e70ULL, 0x27b70a8546d22ffcULL, 0x2e1b21385c26c926ULL, 0x4d2c6dfc5ac42aedULL,
    0x53380d139d95b3dfULL, 0x650a73548baf63deULL, 0x766a0abb3c77b2a8ULL, 0x81c2c92e47edaee6ULL, 0x92722c851482353bULL,
    0xa2bfe8a14cf10364ULL, 0xa81a664bbc423001ULL, 0xc24b8b70d0f89791ULL, 0xc76c51a30654be30ULL, 0xd192e819d6ef5218ULL,
    0xd69906245565a910ULL, 0xf40e35855771202aULL, 0x106aa07032bbd1b8ULL, 0x19a4c116b8d2d0c8ULL, 0x1e376c085141ab53ULL,
    0x2748774cdf8eeb99ULL, 0x34b0bcb5e19b48a8ULL, 0x391c0cb3c5c95a63ULL, 0x4ed8aa4ae3418acbULL, 0x5b9cca4f7763e373ULL,
    0x682e6ff3d6b2b8a3ULL, 0x748f82ee5defb2fcULL, 0x78a5636f43172f60ULL, 0x84c87814a1f0ab72ULL, 0x8cc702081a6439ecULL,
    0x90befffa23631e28ULL, 0xa4506cebde82bde9ULL, 0xbef9a3f7b2c67915ULL, 0xc67178f2e372532bULL, 0xca273eceea26619cULL,
    0xd186b8c721c0c207ULL, 0xeada7dd6cde0eb1eULL, 0xf57d4f7fee6ed178ULL, 0x06f067aa72176fbaULL, 0x0a637dc5a2c898a6ULL,
    0x113f9804bef90daeULL, 0x1b710b35131c471bULL, 0x28db77f523047d84ULL, 0x32caab7b40c72493ULL, 0x3c9ebe0a15c9bebcULL,
    0x431d67c49c100d4cULL, 0x4cc5d4becb3e42b6ULL, 0x597f299cfc657e2aULL, 0x5fcb6fab3ad6faecULL, 0x6c44198c4a475817ULL};

// 64-bit rotate / shift on the 32-bit halves: two v_alignbit_b32 per rotate
// (the compiler's i64 rotate is two 64-bit shifts + two ors).  n is a
// compile-time constant at every call, so the branches fold.
EDV_HD uint64_t rotr64(uint64_t x, int n) {
#if defined(__HIP_DEVICE_COMPILE__)
  const uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
  if (n < 32)
    return ((uint64_t)__builtin_amdgcn_alignbit(lo, hi, n) << 32) | __builtin_amdgcn_alignbit(hi, lo, n);
  return ((uint64_t)__builtin_amdgcn_alignbit(hi, lo, n - 32) << 32) | __builtin_amdgcn_alignbit(lo, hi, n - 32);
#else
  return (x >> n) | (x << (64 - n));
#endif
}
EDV_HD uint64_t shr64(uint64_t x, int n) {  // 0 < n < 32
#if defined(__HIP_DEVICE_COMPILE__)
  const uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
  return ((uint64_t)(hi >> n) << 32) | __builtin_amdgcn_alignbit(hi, lo, n);
#else
  return x >> n;
#endif
}
EDV_HD uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }

// Three-input bitwise functions as one gfx950 v_bitop3_b32 per 32-bit half
// (truth table over x = 0xf0, y = 0xcc, z = 0xaa).  The compiler lowers
// x ^ y ^ z to two v_xor_b32 per half and Maj to xor + bfi; with bitop3 a
// round's Sigma0/Sigma1/sigma0/sigma1/Maj take 10 instructions instead of 20.
template <int TT>
EDV_HD uint64_t bitop3_64(uint64_t x, uint64_t y, uint64_t z) {
#if defined(__HIP_DEVICE_COMPILE__)
  const uint32_t lo = __builtin_amdgcn_bitop3_b32((uint32_t)x, (uint32_t)y, (uint32_t)z, TT);
  const uint32_t hi = __builtin_amdgcn_bitop3_b32((uint32_t)(x >> 32), (uint32_t)(y >> 32), (uint32_t)(z >> 32), TT);
  // The empty asm makes the pair opaque: otherwise the optimizer splits the
  // 64-bit adds that consume it into a 32-bit add of the high halves plus a
  // 64-bit add of the zero-extended low half (+1 v_mov and +1 add per use).
  uint64_t r = ((uint64_t)hi << 32) | lo;
  asm("" : "+v"(r));
  return r;
#else
  static_assert(TT == 0x96 || TT == 0xca || TT == 0xe8, "host form of this table");
  if (TT == 0x96) return x ^ y ^ z;
  if (TT == 0xca) return (x & y) ^ (~x & z);
  return (x & y) | (z & (x | y));
#endif
}
EDV_HD uint64_t xor3_64(uint64_t x, uint64_t y, uint64_t z) { return bitop3_64<0x96>(x, y, z); }

#define EDV_SHA_ROUND(KI, WI)                                                        \
  {                                                                                \
    const uint64_t S1 = xor3_64(rotr64(e, 14), rotr64(e, 18), rotr64(e, 41));      \
    const uint64_t ch = bitop3_64<0xca>(e, f, g);                                  \
    const uint64_t t1 = h + S1 + ch + (KI) + (WI);                                 \
    const uint64_t S0 = xor3_64(rotr64(a, 28), rotr64(a, 34), rotr64(a, 39));      \
    const uint64_t mj = bitop3_64<0xe8>(a, b, c);                                  \
    h = g;                                                                         \
    g = f;                                                                         \
    f = e;                                                                         \
    e = d + t1;                                                                    \
    d = c;                                                                         \
    c = b;                                                                         \
    b = a;                                                                         \
    a = t1 + S0 + mj;                                                              \
  }

// Rounds 0..15 on the block words, then 64 rounds with the message schedule
// in place (w[i] <- sigma1(w[i-2]) + w[i-7] + sigma0(w[i-15]) + w[i-16]).
// No per-round branch: a conditional schedule made the compiler copy the
// whole w[16] array every round.
EDV_HD void sha512_compress(uint64_t st[8], uint64_t w[16]) {
  uint64_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], h = st[7];
#pragma unroll
  for (int i = 0; i < 16; ++i) EDV_SHA_ROUND(SHA512_K[i], w[i])
#pragma unroll 1
  for (int r = 16; r < 80; r += 16) {
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const uint64_t w15 = w[(i + 1) & 15], w2 = w[(i + 14) & 15];
      const uint64_t s0 = xor3_64(rotr64(w15, 1), rotr64(w15, 8), shr64(w15, 7));
      const uint64_t s1 = xor3_64(rotr64(w2, 19), rotr64(w2, 61), shr64(w2, 6));
      w[i] += s0 + w[(i + 9) & 15] + s1;
      EDV_SHA_ROUND(SHA512_K[r + i], w[i])
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
#undef EDV_SHA_ROUND

// (hi:lo) >> (8 * sh) low word: message word from two aligned words.
EDV_HD uint32_t funnel8(uint32_t hi, uint32_t lo, uint32_t sh) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_alignbit(hi, lo, 8 * sh);
#else
  return (uint32_t)((((uint64_t)hi << 32) | lo) >> (8 * sh));
#endif
}

// One 128-byte block of the stream prefix || msg || 0x80 || 0... as 16
// big-endian words.  The message is read as 16-byte chunks of its 16-byte
// aligned base (c16[q], q < nq: only chunks holding message bytes, so no read
// can leave the pages the message lies in): at most 9 dwordx4 loads per block
// instead of 33 dword loads.  Message word t of the block is the byte funnel
// (sh = msg & 3) of window words V[j], V[j+1], where V is the loaded window
// shifted by s4 = 0..3 words (per-lane selects).  Blocks that reach the end of
// the message get the tail masked and the 0x80 pad byte placed.
struct Chunk16 {
  uint32_t x, y, z, w;
};

// Chunks of this block that hold message bytes: nq - q0 clamped to [0, 16]
// (one 64-bit compare per block; the per-chunk guards are then 32-bit).
EDV_HD int chunks_left(uint64_t nq, uint64_t q0) {
  return nq <= q0 ? 0 : (nq - q0 >= 16 ? 16 : (int)(nq - q0));
}

// Message bytes left at a block's first word, clamped to [-1024, 1024] so the
// per-word tail arithmetic is 32-bit.
EDV_HD int32_t bytes_left(uint64_t mlen, int64_t word0) {
  const int64_t r = (int64_t)mlen - 4 * word0;
  return r < -1024 ? -1024 : r > 1024 ? 1024 : (int32_t)r;
}

// Word with `rem` message bytes left at it: keep min(rem, 4) bytes, put the
// 0x80 pad byte at byte rem when 0 <= rem < 4.
EDV_HD uint32_t tail_word(uint32_t v, int32_t rem) {
  const uint32_t keep = rem >= 4 ? 0xffffffffu : rem <= 0 ? 0u : (0xffffffffu >> (32 - 8 * rem));
  const uint32_t pad = (uint32_t)rem < 4u ? (0x80u << (8 * rem)) : 0u;
  return (v & keep) | pad;
}
template <int NP, bool FIRST>
EDV_HD void sha512_block_words(uint64_t w[16], uint64_t b, const uint32_t* prefix, const Chunk16* c16, uint64_t nq,
                               uint32_t d16, uint64_t mlen) {
  constexpr int T0 = FIRST ? NP : 0;          // first message word of the block
  constexpr int NW = 32 - T0;                 // message words in the block
  constexpr int NCH = (NW * 4 + 15 + 15) / 16;  // chunks covering them at any misalignment
  const int64_t u0 = 32 * (int64_t)b - NP;    // message word index of stream word 0
  const uint64_t pos = d16 + 4 * (uint64_t)(u0 + T0);  // base16 byte of the block's first message byte
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
  uint32_t V[NW + 1];
#pragma unroll
  for (int j = 0; j <= NW; ++j) {
    const uint32_t a0 = W[j], a1 = j + 1 < 4 * NCH ? W[j + 1] : 0u, a2 = j + 2 < 4 * NCH ? W[j + 2] : 0u,
                   a3 = j + 3 < 4 * NCH ? W[j + 3] : 0u;
    V[j] = s4 == 0 ? a0 : s4 == 1 ? a1 : s4 == 2 ? a2 : a3;
  }
  uint32_t le[32];
#pragma unroll
  for (int t = 0; t < 32; ++t) le[t] = t < T0 ? prefix[t < NP ? t : 0] : funnel8(V[t - T0 + 1], V[t - T0], sh);
  if (4 * (u0 + 32) > (int64_t)mlen) {
    const int32_t rb = bytes_left(mlen, u0);  // bytes left at stream word 0 of the block
#pragma unroll
    for (int t = T0; t < 32; ++t) le[t] = tail_word(le[t], rb - 4 * t);
  }
#pragma unroll
  for (int j = 0; j < 16; ++j) w[j] = ((uint64_t)bswap32(le[2 * j]) << 32) | bswap32(le[2 * j + 1]);
}

// SHA-512(prefix || msg).  prefix: NP little-endian u32 words (NP = 8 or 16).
// digest: 16 little-endian u32 words = the 64 digest bytes in order.
template <int NP>
EDV_HD void sha512_prefixed(uint32_t digest[16], const uint32_t prefix[NP], const uint8_t* msg, uint64_t mlen) {
  static_assert(NP <= 16, "the prefix must fit block 0");
  uint64_t st[8] = {0x6a09e667f3bcc908ULL, 0xbb67ae8584caa73bULL, 0x3c6ef372fe94f82bULL, 0xa54ff53a5f1d36f1ULL,
                    0x510e527fade682d1ULL, 0x9b05688c2b3e6c1fULL, 0x1f83d9abfb41bd6bULL, 0x5be0cd19137e2179ULL};
  const uint64_t total = 4 * NP + mlen;            // stream bytes before padding
  const uint64_t nblocks = (total + 16) / 128 + 1;  // incl. 0x80 and 128-bit length
  const uint64_t bitlen = total * 8;
  const uint32_t d16 = (uint32_t)((uintptr_t)msg & 15);
  const Chunk16* c16 = (const Chunk16*)(msg - d16);  // pointer arithmetic keeps the address space
  const uint64_t nq = (d16 + mlen + 15) / 16;
  uint64_t w[16];
  sha512_block_words<NP, true>(w, 0, prefix, c16, nq, d16, mlen);
  if (nblocks == 1) {
    w[14] = 0;
    w[15] = bitlen;
  }
  sha512_compress(st, w);
#pragma unroll 1
  for (uint64_t b = 1; b < nblocks; ++b) {
    sha512_block_words<NP, false>(w, b, prefix, c16, nq, d16, mlen);
    if (b == nblocks - 1) {
      w[14] = 0;
      w[15] = bitlen;
    }
    sha512_compress(st, w);
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    digest[2 * j] = bswap32((uint32_t)(st[j] >> 32));
    digest[2 * j + 1] = bswap32((uint32_t)st[j]);
  }
}

// ---- Length-bucketed SoA message layout (north_star (1)).
//
// For a 64-byte prefix (R || A) the SHA-512 stream is R || A || M || 0x80 ||
// 0... || bitlen, and M starts exactly at stream word 8: the message part of
// the stream is (SHA-512 blocks) * 128 - 64 bytes = 8 * nblocks - 4 "units"
// of 16 bytes (two big-endian stream words).  pack_lane_units writes a lane's
// units, already byte-swapped, padded and carrying the bit length, at
// out[p * stride]; with stride 64 and lane-interleaved groups (edverify.hip
// edv_pack_units_kernel) the hash kernel's unit loads are one coalesced 1 KiB
// access per wave and need no funnel, select or tail masking.
EDV_HD uint64_t sha512_nblocks64(uint64_t mlen) { return (64 + mlen + 16) / 128 + 1; }
EDV_HD uint64_t sha512_units64(uint64_t mlen) { return 8 * sha512_nblocks64(mlen) - 4; }

EDV_HD void pack_lane_units(Chunk16* out, uint64_t stride, const uint8_t* msg, uint64_t mlen) {
  const uint64_t nunits = sha512_units64(mlen);
  const uint32_t d16 = (uint32_t)((uintptr_t)msg & 15);
  const Chunk16* c16 = (const Chunk16*)(msg - d16);
  const uint64_t nq = (d16 + mlen + 15) / 16;  // chunks holding message bytes
  const uint32_t s4 = d16 >> 2, sh = d16 & 3u;
  const uint64_t bitlen = (64 + mlen) * 8;
  Chunk16 cur = {0u, 0u, 0u, 0u};
  if (nq > 0) cur = c16[0];
#pragma unroll 1
  for (uint64_t p = 0; p < nunits; ++p) {
    Chunk16 nxt = {0u, 0u, 0u, 0u};
    if (p + 1 < nq) nxt = c16[p + 1];
    // message bytes [16p, 16p + 16) = bytes d16.. of the 32-byte window cur || nxt
    const uint32_t W[8] = {cur.x, cur.y, cur.z, cur.w, nxt.x, nxt.y, nxt.z, nxt.w};
    uint32_t V[5];
#pragma unroll
    for (int j = 0; j < 5; ++j) V[j] = s4 == 0 ? W[j] : s4 == 1 ? W[j + 1] : s4 == 2 ? W[j + 2] : W[j + 3];
    uint32_t le[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) le[k] = funnel8(V[k + 1], V[k], sh);
    if (16 * (p + 1) > mlen) {
      const int32_t rb = bytes_left(mlen, (int64_t)(4 * p));  // message bytes left at the unit's first byte
#pragma unroll
      for (int k = 0; k < 4; ++k) le[k] = tail_word(le[k], rb - 4 * k);
    }
    uint64_t w0 = ((uint64_t)bswap32(le[0]) << 32) | bswap32(le[1]);
    uint64_t w1 = ((uint64_t)bswap32(le[2]) << 32) | bswap32(le[3]);
    if (p + 1 == nunits) w1 = bitlen;  // the high length word (w0) is zero padding
    out[p * stride] = {(uint32_t)w0, (uint32_t)(w0 >> 32), (uint32_t)w1, (uint32_t)(w1 >> 32)};
    cur = nxt;
  }
}

// SHA-512(prefix || M) from the unit layout above: prefix = 16 little-endian
// u32 words (R || A), units[p * stride] = unit p of M's stream.
EDV_HD void sha512_prefixed_units(uint32_t digest[16], const uint32_t prefix[16], const Chunk16* units, uint64_t stride,
                                  uint64_t mlen) {
  uint64_t st[8] = {0x6a09e667f3bcc908ULL, 0xbb67ae8584caa73bULL, 0x3c6ef372fe94f82bULL, 0xa54ff53a5f1d36f1ULL,
                    0x510e527fade682d1ULL, 0x9b05688c2b3e6c1fULL, 0x1f83d9abfb41bd6bULL, 0x5be0cd19137e2179ULL};
  const uint64_t nblocks = sha512_nblocks64(mlen);
  uint64_t w[16];
#pragma unroll
  for (int j = 0; j < 8; ++j) w[j] = ((uint64_t)bswap32(prefix[2 * j]) << 32) | bswap32(prefix[2 * j + 1]);
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const Chunk16 u = units[q * stride];
    w[8 + 2 * q] = ((uint64_t)u.y << 32) | u.x;
    w[9 + 2 * q] = ((uint64_t)u.w << 32) | u.z;
  }
  sha512_compress(st, w);
#pragma unroll 1
  for (uint64_t b = 1; b < nblocks; ++b) {
    const Chunk16* ub = units + (8 * b - 4) * stride;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const Chunk16 u = ub[q * stride];
      w[2 * q] = ((uint64_t)u.y << 32) | u.x;
      w[2 * q + 1] = ((uint64_t)u.w << 32) | u.z;
    }
    sha512_compress(st, w);
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    digest[2 * j] = bswap32((uint32_t)(st[j] >> 32));
    digest[2 * j + 1] = bswap32((uint32_t)st[j]);
  }
}

}  // namespace edv
