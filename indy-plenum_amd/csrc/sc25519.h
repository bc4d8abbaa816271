// sc25519.h -- scalars modulo L = 2^252 + 27742317777372353535851937790883648493.
//
// Restates the scalar half of libsodium 1.0.18's verify
// (sc25519_is_canonical on S; sc25519_reduce on SHA-512(R||A||M)), reached from
// stp_core/crypto/nacl_wrappers.py:108.  The reduction is our own: 21-bit
// signed limbs in int64, folding 2^252 == -c (mod L), then an exact final
// correction into [0, L).  h MUST be the canonical residue: for a mixed-order
// public key [h]A depends on h mod 8L, and libsodium uses the canonical h.
#pragma once
#include "fe25519.h"

namespace edv {

// c = L - 2^252 in 21-bit limbs.
EDV_HD constexpr int64_t sc_c(int j) {
  return j == 0 ? 1430509 : j == 1 ? 1626855 : j == 2 ? 1442968 : j == 3 ? 997804 : j == 4 ? 1960495 : 683900;
}
EDV_HD constexpr uint32_t sc_L(int k) {
  return k == 0 ? 0x5cf5d3edu : k == 1 ? 0x5812631au : k == 2 ? 0xa2f79cd6u : k == 3 ? 0x14def9deu : k == 7 ? 0x10000000u : 0u;
}

// s < L ?  (sc25519_is_canonical)
EDV_HD bool sc_is_canonical(const uint32_t s[8]) {
  // borrow out of s - L: set iff s < L
  uint64_t borrow = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    uint64_t t = (uint64_t)s[k] - sc_L(k) - borrow;
    borrow = (t >> 63) & 1;
  }
  return borrow != 0;
}

EDV_HD void sc_fold(int64_t s[25], int i) {
#pragma unroll
  for (int j = 0; j < 6; ++j) s[i - 12 + j] -= s[i] * sc_c(j);
  s[i] = 0;
}
EDV_HD void sc_carry_round(int64_t s[25], int k) {
  int64_t c = (s[k] + (1 << 20)) >> 21;
  s[k + 1] += c;
  s[k] -= c * (int64_t)(1 << 21);
}

// out = in mod L, canonical.  in: 16 LE u32 words (512 bits); out: 8 LE u32 words.
EDV_HDNI void sc_reduce(uint32_t out[8], const uint32_t in[16]) {
  int64_t s[25];
#pragma unroll
  for (int i = 0; i < 25; ++i) {
    const int bit = 21 * i, w = bit >> 5, sh = bit & 31;
    uint64_t lo = in[w];
    uint64_t hi = (w + 1 < 16) ? in[w + 1] : 0;
    uint64_t v = ((hi << 32) | lo) >> sh;
    s[i] = (int64_t)(v & ((1u << 21) - 1));
  }
  // Stage A: fold limbs 24..18 into 6..17 (|s| <= 2^21 + 6 * 2^42).
#pragma unroll
  for (int i = 24; i >= 18; --i) sc_fold(s, i);
  // Stage B: carry 6..17 (into 18).
#pragma unroll
  for (int k = 6; k <= 17; ++k) sc_carry_round(s, k);
  // Stage C: fold 18..12 into 0..11.
#pragma unroll
  for (int i = 18; i >= 12; --i) sc_fold(s, i);
  // Stage D: carry 0..11 (into 12), fold 12, carry again, fold 12.
#pragma unroll
  for (int k = 0; k <= 11; ++k) sc_carry_round(s, k);
  sc_fold(s, 12);
#pragma unroll
  for (int k = 0; k <= 11; ++k) sc_carry_round(s, k);
  sc_fold(s, 12);
  // Floor carries: limbs 0..11 in [0, 2^21), s[12] a small signed top.
#pragma unroll
  for (int k = 0; k <= 11; ++k) {
    int64_t c = s[k] >> 21;  // arithmetic
    s[k] -= c * (int64_t)(1 << 21);
    s[k + 1] += c;
  }
  // Pack 252 bits + signed top into 8 words (two's complement).
  uint32_t w[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) w[k] = 0;
#pragma unroll
  for (int i = 0; i < 12; ++i) {
    const int bit = 21 * i, wi = bit >> 5, sh = bit & 31;
    uint64_t v = (uint64_t)s[i] << sh;
    w[wi] |= (uint32_t)v;
    if (wi + 1 < 8) w[wi + 1] |= (uint32_t)(v >> 32);
  }
  w[7] += (uint32_t)s[12] << 28;
  // Exact correction into [0, L): add L while negative, subtract L while >= L.
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    const bool neg = (w[7] >> 31) != 0;
    uint64_t carry = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      uint64_t t = (uint64_t)w[k] + (neg ? sc_L(k) : 0u) + carry;
      w[k] = (uint32_t)t;
      carry = t >> 32;
    }
  }
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    uint32_t t[8];
    uint64_t borrow = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      uint64_t d = (uint64_t)w[k] - sc_L(k) - borrow;
      t[k] = (uint32_t)d;
      borrow = (d >> 63) & 1;
    }
    const bool ge = borrow == 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) w[k] = ge ? t[k] : w[k];
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) out[k] = w[k];
}

// Signed radix-16 recoding without a digit array: with y = x + 0x8888...88
// (x < 2^253, so no overflow), digit_i = nibble_i(y) - 8 in [-8, 7] and
// x = sum digit_i 16^i.
EDV_HD void sc_recode16(uint32_t y[8], const uint32_t x[8]) {
  uint64_t carry = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    uint64_t t = (uint64_t)x[k] + 0x88888888u + carry;
    y[k] = (uint32_t)t;
    carry = t >> 32;
  }
}

// (a * b + c) mod L for 8-word scalars (a, b, c < 2^256).  Used by the signer.
EDV_HDNI void sc_muladd(uint32_t out[8], const uint32_t a[8], const uint32_t b[8], const uint32_t c[8]) {
  uint32_t prod[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) prod[k] = 0;
  for (int i = 0; i < 8; ++i) {
    uint64_t carry = 0;
    for (int j = 0; j < 8; ++j) {
      uint64_t t = (uint64_t)a[i] * b[j] + prod[i + j] + carry;
      prod[i + j] = (uint32_t)t;
      carry = t >> 32;
    }
    prod[i + 8] = (uint32_t)carry;
  }
  uint64_t carry = 0;
  for (int k = 0; k < 16; ++k) {
    uint64_t t = (uint64_t)prod[k] + (k < 8 ? c[k] : 0u) + carry;
    prod[k] = (uint32_t)t;
    carry = t >> 32;
  }
  // a*b + c < 2^512 + 2^256 only if a, b are near 2^256; callers pass a, b < 2^256 with
  // a*b + c < 2^512 (clamped secret scalar < 2^255).
  sc_reduce(out, prod);
}

}  // namespace edv
