// fe25519.h -- GF(2^255 - 19) arithmetic for gfx950 VALU.
//
// Part of the MI355X Ed25519 verify path that replaces libsodium's
// crypto_sign_open (reached from stp_core/crypto/nacl_wrappers.py:108).
//
// Representation: 10 unsigned 32-bit limbs, radix 2^25.5 (widths 26,25,26,...),
// value = sum v[k] * 2^ceil(25.5 k).  Products are 32x32->64 multiply-adds, which
// hipcc lowers to v_mad_u64_u32 (measured half-rate on gfx950: 58.7 of 64
// lane-ops/clk/CU, tools/microbench).  Carries use 64-bit shifts/adds only on
// the accumulators.
//
// Bound classes (checked by tests/test_fe_bounds.py and, in the host self-test
// build, by EDV_BOUND_CHECK assertions):
//   C  "carried":  even limbs < 2^26, odd limbs <= 2^25 + 2^18   (mul/sq/carry output)
//   L  "loose":    even <= 3*2^26, odd <= 3*2^25 + 2^18          (C+C, C+C+C, C+2p-C)
//   W  "wide":     even <= 5*2^26, odd <= 5*2^25 + 2^18          (C+4p-L, ...)
// fe_mul(h, f, g): f in W, g in L  (worst accumulator 2^62.87 < 2^64)
// fe_sq(h, f):     f in L          (worst accumulator 2^62.13)
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define EDV_HD __host__ __device__ __forceinline__
#define EDV_HDNI __host__ __device__ __forceinline__
#define EDV_HDM __host__ __device__ __forceinline__
#else
#define EDV_HD static inline
#define EDV_HDNI static
#define EDV_HDM inline
#endif

#ifdef EDV_BOUND_CHECK
#include <assert.h>
#define EDV_ASSERT(x) assert(x)
#else
#define EDV_ASSERT(x) ((void)0)
#endif

namespace edv {

struct fe {
  uint32_t v[10];
};

constexpr uint32_t M26 = (1u << 26) - 1;
constexpr uint32_t M25 = (1u << 25) - 1;
EDV_HD constexpr int fe_width(int k) { return (k & 1) ? 25 : 26; }
EDV_HD constexpr uint32_t fe_mask(int k) { return (k & 1) ? M25 : M26; }

// 2p and 4p in this radix (limbwise >= any C / L value respectively).
EDV_HD constexpr uint32_t two_p(int k) { return k == 0 ? (1u << 27) - 38 : ((k & 1) ? (1u << 26) - 2 : (1u << 27) - 2); }
EDV_HD constexpr uint32_t four_p(int k) { return k == 0 ? (1u << 28) - 76 : ((k & 1) ? (1u << 27) - 4 : (1u << 28) - 4); }

EDV_HD void fe_0(fe& h) {
#pragma unroll
  for (int k = 0; k < 10; ++k) h.v[k] = 0;
}
EDV_HD void fe_1(fe& h) {
  fe_0(h);
  h.v[0] = 1;
}
EDV_HD void fe_add(fe& h, const fe& f, const fe& g) {
#pragma unroll
  for (int k = 0; k < 10; ++k) h.v[k] = f.v[k] + g.v[k];
}
// h = f - g, for g in C (adds 2p).
EDV_HD void fe_sub(fe& h, const fe& f, const fe& g) {
#pragma unroll
  for (int k = 0; k < 10; ++k) h.v[k] = f.v[k] + (two_p(k) - g.v[k]);
}
// h = f - g, for g in L (adds 4p); result class W when f in C.
EDV_HD void fe_sub4(fe& h, const fe& f, const fe& g) {
#pragma unroll
  for (int k = 0; k < 10; ++k) h.v[k] = f.v[k] + (four_p(k) - g.v[k]);
}
EDV_HD void fe_neg(fe& h, const fe& f) {
#pragma unroll
  for (int k = 0; k < 10; ++k) h.v[k] = two_p(k) - f.v[k];
}
// Conditional move: h = b ? f : h   (b is 0 or 1; lowered to v_cndmask).
EDV_HD void fe_cmov(fe& h, const fe& f, bool b) {
#pragma unroll
  for (int k = 0; k < 10; ++k) h.v[k] = b ? f.v[k] : h.v[k];
}

// 64-bit accumulator carry chain, final limbs in class C.
EDV_HD void fe_carry64(fe& out, uint64_t h[10]) {
#define EDV_C(k)                                 \
  {                                              \
    uint64_t c = h[k] >> fe_width(k);            \
    h[k] &= fe_mask(k);                          \
    h[k + 1] += c;                               \
  }
  EDV_C(0) EDV_C(4) EDV_C(1) EDV_C(5) EDV_C(2) EDV_C(6) EDV_C(3) EDV_C(7) EDV_C(4) EDV_C(8)
  {
    uint64_t c = h[9] >> 25;
    h[9] &= M25;
    h[0] += c * 19;
  }
  EDV_C(0)
#undef EDV_C
#pragma unroll
  for (int k = 0; k < 10; ++k) out.v[k] = (uint32_t)h[k];
}

#ifdef EDV_BOUND_CHECK
static inline bool fe_in_class(const fe& f, uint32_t even_max, uint32_t odd_max) {
  for (int k = 0; k < 10; ++k)
    if (f.v[k] > ((k & 1) ? odd_max : even_max)) return false;
  return true;
}
#define EDV_IS_W(f) fe_in_class(f, 5u << 26, (5u << 25) + (1u << 18))
#define EDV_IS_L(f) fe_in_class(f, 3u << 26, (3u << 25) + (1u << 18))
#define EDV_IS_C(f) fe_in_class(f, (1u << 26) - 1, (1u << 25) + (1u << 18))
#endif

// acc += a * b as one v_mad_u64_u32 in program order (EDV_MAD_CHAIN): inline
// asm keeps the compiler from re-associating a carry-started chain into a
// zero-started chain plus a 64-bit add of the carry.
#ifndef EDV_MAD_CHAIN
#define EDV_MAD_CHAIN 1  // +3.5% on the keyed step (tools/ab_libs.py, profiles/r02b)
#endif
#if defined(__HIP_DEVICE_COMPILE__) && EDV_MAD_CHAIN
__device__ __forceinline__ void mad_acc(uint64_t& acc, uint32_t a, uint32_t b) {
  uint64_t carry_out;  // VOP3b sdst (unused)
  asm("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(acc), "=s"(carry_out) : "v"(a), "v"(b));
}
// acc += sum_i a[i] * b[i], ten MADs in one asm block (one serial chain)
__device__ __forceinline__ void mad_acc10(uint64_t& acc, const uint32_t a[10], const uint32_t b[10]) {
  uint64_t co;
  asm("v_mad_u64_u32 %0, %1, %2, %12, %0\n\t"
      "v_mad_u64_u32 %0, %1, %3, %13, %0\n\t"
      "v_mad_u64_u32 %0, %1, %4, %14, %0\n\t"
      "v_mad_u64_u32 %0, %1, %5, %15, %0\n\t"
      "v_mad_u64_u32 %0, %1, %6, %16, %0\n\t"
      "v_mad_u64_u32 %0, %1, %7, %17, %0\n\t"
      "v_mad_u64_u32 %0, %1, %8, %18, %0\n\t"
      "v_mad_u64_u32 %0, %1, %9, %19, %0\n\t"
      "v_mad_u64_u32 %0, %1, %10, %20, %0\n\t"
      "v_mad_u64_u32 %0, %1, %11, %21, %0"
      : "+v"(acc), "=s"(co)
      : "v"(a[0]), "v"(a[1]), "v"(a[2]), "v"(a[3]), "v"(a[4]), "v"(a[5]), "v"(a[6]), "v"(a[7]), "v"(a[8]),
        "v"(a[9]), "v"(b[0]), "v"(b[1]), "v"(b[2]), "v"(b[3]), "v"(b[4]), "v"(b[5]), "v"(b[6]), "v"(b[7]),
        "v"(b[8]), "v"(b[9]));
}
// the squaring chains: 6 (even limbs) or 5 (odd limbs) products
__device__ __forceinline__ void mad_acc6(uint64_t& acc, const uint32_t a[6], const uint32_t b[6]) {
  uint64_t co;
  asm("v_mad_u64_u32 %0, %1, %2, %8, %0\n\t"
      "v_mad_u64_u32 %0, %1, %3, %9, %0\n\t"
      "v_mad_u64_u32 %0, %1, %4, %10, %0\n\t"
      "v_mad_u64_u32 %0, %1, %5, %11, %0\n\t"
      "v_mad_u64_u32 %0, %1, %6, %12, %0\n\t"
      "v_mad_u64_u32 %0, %1, %7, %13, %0"
      : "+v"(acc), "=s"(co)
      : "v"(a[0]), "v"(a[1]), "v"(a[2]), "v"(a[3]), "v"(a[4]), "v"(a[5]), "v"(b[0]), "v"(b[1]), "v"(b[2]),
        "v"(b[3]), "v"(b[4]), "v"(b[5]));
}
__device__ __forceinline__ void mad_acc5(uint64_t& acc, const uint32_t a[5], const uint32_t b[5]) {
  uint64_t co;
  asm("v_mad_u64_u32 %0, %1, %2, %7, %0\n\t"
      "v_mad_u64_u32 %0, %1, %3, %8, %0\n\t"
      "v_mad_u64_u32 %0, %1, %4, %9, %0\n\t"
      "v_mad_u64_u32 %0, %1, %5, %10, %0\n\t"
      "v_mad_u64_u32 %0, %1, %6, %11, %0"
      : "+v"(acc), "=s"(co)
      : "v"(a[0]), "v"(a[1]), "v"(a[2]), "v"(a[3]), "v"(a[4]), "v"(b[0]), "v"(b[1]), "v"(b[2]), "v"(b[3]),
        "v"(b[4]));
}
#else
EDV_HD void mad_acc(uint64_t& acc, uint32_t a, uint32_t b) { acc += (uint64_t)a * b; }
EDV_HD void mad_acc10(uint64_t& acc, const uint32_t a[10], const uint32_t b[10]) {
  for (int i = 0; i < 10; ++i) acc += (uint64_t)a[i] * b[i];
}
EDV_HD void mad_acc6(uint64_t& acc, const uint32_t a[6], const uint32_t b[6]) {
  for (int i = 0; i < 6; ++i) acc += (uint64_t)a[i] * b[i];
}
EDV_HD void mad_acc5(uint64_t& acc, const uint32_t a[5], const uint32_t b[5]) {
  for (int i = 0; i < 5; ++i) acc += (uint64_t)a[i] * b[i];
}
#endif

// h = f * g.  f in W, g in L; h in C.  100 multiply-adds.
// EDV_FE_MUL_ORDER 1 emits the products operand-major (for each f_i, one
// product into each of the 10 accumulators), so consecutive v_mad_u64_u32 go
// to different accumulators; 0 emits them accumulator-major.
// EDV_FE_MUL_ORDER 2 computes the accumulators in order with the previous
// limb's carry as the chain's initial addend (no separate 64-bit carry adds;
// one accumulator live; a serial chain per multiply).
#ifndef EDV_FE_MUL_ORDER
#define EDV_FE_MUL_ORDER 2  // 2: -3% comb time vs 0 and 1 (tools/ab_keyed.py)
#endif
// EDV ORDER 3 (latency: one wave, one request): as 2, but limbs 0-4 and 5-9 run as two
// independent carry-started chains (limb 5's starts from 0), so a lone wave can overlap them;
// then the first chain's carry ripples through limbs 5-9 (32-bit steps) and the wrap adds
// 19 x (both chains' final carries) to limb 0.  Output class C, as ORDER 2.
EDV_HD void fe_join_halves(uint32_t o[10], uint64_t ca, uint64_t cb) {
  uint64_t t = (uint64_t)o[5] + ca;
  o[5] = (uint32_t)t & M25;
  uint32_t c = (uint32_t)(t >> 25);  // < 2^14
#pragma unroll
  for (int k = 6; k < 10; ++k) {
    const uint32_t u = o[k] + c;
    o[k] = u & fe_mask(k);
    c = u >> fe_width(k);
  }
  t = (uint64_t)o[0] + (cb + c) * 19u;  // carry out of limb 9 wraps as 19 * 2^0
  o[0] = (uint32_t)t & M26;
  o[1] += (uint32_t)(t >> 26);
}
template <int ORDER>
EDV_HD void fe_mul_o(fe& h, const fe& f, const fe& g) {
  EDV_ASSERT(EDV_IS_W(f) && EDV_IS_L(g));
  uint32_t g19[10], f2[10];
#pragma unroll
  for (int k = 0; k < 10; ++k) {
    g19[k] = 19u * g.v[k];
    f2[k] = (k & 1) ? 2u * f.v[k] : f.v[k];
  }
  if constexpr (ORDER == 2 || ORDER == 3) {
    uint64_t c = 0, ca = 0;
    uint32_t o[10];  // h may alias f or g
#pragma unroll
    for (int k = 0; k < 10; ++k) {
      if (ORDER == 3 && k == 5) {
        ca = c;
        c = 0;
      }
#if EDV_MAD_CHAIN
      // the chain starts from the carry of limb k - 1 (one v_mad_u64_u32 per
      // product, no separate 64-bit add of the carry, which the compiler's
      // reassociation otherwise emits)
      uint64_t a = c;
      uint32_t fa[10], gb[10];
#pragma unroll
      for (int i = 0; i < 10; ++i) {
        const int j = k - i;
        fa[i] = ((i & 1) && (j & 1)) ? f2[i] : f.v[i];
        gb[i] = j >= 0 ? g.v[j] : g19[j + 10];
      }
      mad_acc10(a, fa, gb);
#else
      uint64_t a = c;
#pragma unroll
      for (int i = 0; i < 10; ++i) {
        const int j = k - i;
        const uint32_t fi = ((i & 1) && (j & 1)) ? f2[i] : f.v[i];
        const uint32_t gj = j >= 0 ? g.v[j] : g19[j + 10];
        a += (uint64_t)fi * gj;
      }
#endif
      o[k] = (uint32_t)a & fe_mask(k);
      c = a >> fe_width(k);
    }
    if constexpr (ORDER == 3) {
      fe_join_halves(o, ca, c);
    } else {
      const uint64_t t = (uint64_t)o[0] + c * 19u;  // carry out of limb 9 wraps as 19 * 2^0
      o[0] = (uint32_t)t & M26;
      o[1] += (uint32_t)(t >> 26);
    }
#pragma unroll
    for (int k = 0; k < 10; ++k) h.v[k] = o[k];
  } else {
    uint64_t acc[10];
    if constexpr (ORDER == 1) {
#pragma unroll
      for (int k = 0; k < 10; ++k) acc[k] = 0;
#pragma unroll
      for (int i = 0; i < 10; ++i) {
#pragma unroll
        for (int k = 0; k < 10; ++k) {
          const int j = k - i;
          const uint32_t fi = ((i & 1) && (j & 1)) ? f2[i] : f.v[i];
          const uint32_t gj = j >= 0 ? g.v[j] : g19[j + 10];
          acc[k] += (uint64_t)fi * gj;
        }
      }
    } else {
#pragma unroll
      for (int k = 0; k < 10; ++k) {
        uint64_t a = 0;
#pragma unroll
        for (int i = 0; i < 10; ++i) {
          const int j = k - i;
          const uint32_t fi = ((i & 1) && (j & 1)) ? f2[i] : f.v[i];
          const uint32_t gj = j >= 0 ? g.v[j] : g19[j + 10];
          a += (uint64_t)fi * gj;
        }
        acc[k] = a;
      }
    }
    fe_carry64(h, acc);
  }
}
EDV_HD void fe_mul(fe& h, const fe& f, const fe& g) { fe_mul_o<EDV_FE_MUL_ORDER>(h, f, g); }

// h = f^2.  f in L; h in C.  55 multiply-adds.  With EDV_FE_MUL_ORDER 2 the
// carry of limb k-1 is the initial addend of limb k's chain (as fe_mul).
template <int ORDER>
EDV_HD void fe_sq_o(fe& h, const fe& f) {
  EDV_ASSERT(EDV_IS_L(f));
  uint32_t d[10], d2[10], d19[10], d38[10];
#pragma unroll
  for (int k = 0; k < 10; ++k) {
    d[k] = f.v[k];
    d2[k] = 2u * f.v[k];
    d19[k] = 19u * f.v[k];
    d38[k] = 38u * f.v[k];
  }
  constexpr bool kChain = ORDER == 2 || ORDER == 3;
  uint64_t acc[10];
  uint64_t c = 0, ca = 0;
  uint32_t o[10];
#pragma unroll
  for (int k = 0; k < 10; ++k) {
    if (ORDER == 3 && k == 5) {
      ca = c;
      c = 0;
    }
    uint64_t a = kChain ? c : 0;
    uint32_t pa[6], pb[6];
    int np = 0;
#pragma unroll
    for (int i = 0; i < 10; ++i) {
#pragma unroll
      for (int j = i; j < 10; ++j) {
        if ((i + j) % 10 != k) continue;
        const bool both_odd = (i & 1) && (j & 1);
        const bool wrap = i + j >= 10;
        const uint32_t fi = (i != j) ? d2[i] : d[i];
        const uint32_t fj = wrap ? (both_odd ? d38[j] : d19[j]) : (both_odd ? d2[j] : d[j]);
        if (kChain && EDV_MAD_CHAIN) {
          pa[np] = fi;  // carry-started chain, one asm block per limb
          pb[np] = fj;
          ++np;
        } else {
          a += (uint64_t)fi * fj;
        }
      }
    }
    if (kChain && EDV_MAD_CHAIN) {
      if (k & 1)
        mad_acc5(a, pa, pb);
      else
        mad_acc6(a, pa, pb);
    }
    acc[k] = a;
    if (kChain) {
      o[k] = (uint32_t)a & fe_mask(k);
      c = a >> fe_width(k);
    }
  }
  if (kChain) {
    if (ORDER == 3) {
      fe_join_halves(o, ca, c);
    } else {
      const uint64_t t = (uint64_t)o[0] + c * 19u;
      o[0] = (uint32_t)t & M26;
      o[1] += (uint32_t)(t >> 26);
    }
#pragma unroll
    for (int k = 0; k < 10; ++k) h.v[k] = o[k];
  } else {
    fe_carry64(h, acc);
  }
}
EDV_HD void fe_sq(fe& h, const fe& f) { fe_sq_o<EDV_FE_MUL_ORDER>(h, f); }

// h = f^(2^n), n >= 1.
template <int ORDER = EDV_FE_MUL_ORDER>
EDV_HDNI void fe_sqn(fe& h, const fe& f, int n) {
  fe_sq_o<ORDER>(h, f);
#pragma unroll 1
  for (int i = 1; i < n; ++i) fe_sq_o<ORDER>(h, h);
}

// One 32-bit carry pass: any class up to 2^31 per limb -> C.
EDV_HD void fe_carry(fe& h) {
  uint32_t c;
#pragma unroll
  for (int k = 0; k < 9; ++k) {
    c = h.v[k] >> fe_width(k);
    h.v[k] &= fe_mask(k);
    h.v[k + 1] += c;
  }
  c = h.v[9] >> 25;
  h.v[9] &= M25;
  h.v[0] += 19u * c;
  c = h.v[0] >> 26;
  h.v[0] &= M26;
  h.v[1] += c;
}

// Fully reduce into [0, p) (every limb within its width).
EDV_HD void fe_canon(fe& h) {
  fe_carry(h);
  fe_carry(h);
  fe_carry(h);
  // value now in [0, 2^255); subtract p iff value + 19 >= 2^255.
  uint32_t q = (h.v[0] + 19u) >> 26;
#pragma unroll
  for (int k = 1; k < 10; ++k) q = (h.v[k] + q) >> fe_width(k);
  h.v[0] += 19u * q;
#pragma unroll
  for (int k = 0; k < 9; ++k) {
    uint32_t c = h.v[k] >> fe_width(k);
    h.v[k] &= fe_mask(k);
    h.v[k + 1] += c;
  }
  h.v[9] &= M25;
}

// Little-endian 8 x u32 words of the canonical encoding of h (bit 255 = 0).
EDV_HD void fe_tobytes(uint32_t w[8], const fe& hin) {
  fe h = hin;
  fe_canon(h);
  // limb offsets 0,26,51,77,102,128,153,179,204,230
  w[0] = h.v[0] | (h.v[1] << 26);
  w[1] = (h.v[1] >> 6) | (h.v[2] << 19);
  w[2] = (h.v[2] >> 13) | (h.v[3] << 13);
  w[3] = (h.v[3] >> 19) | (h.v[4] << 6);
  w[4] = h.v[5] | (h.v[6] << 25);
  w[5] = (h.v[6] >> 7) | (h.v[7] << 19);
  w[6] = (h.v[7] >> 13) | (h.v[8] << 12);
  w[7] = (h.v[8] >> 20) | (h.v[9] << 6);
}

// fe25519_frombytes: the low 255 bits of 8 LE words (bit 255 ignored), not reduced.
EDV_HD void fe_frombytes(fe& h, const uint32_t w[8]) {
  h.v[0] = w[0] & M26;
  h.v[1] = ((w[0] >> 26) | (w[1] << 6)) & M25;
  h.v[2] = ((w[1] >> 19) | (w[2] << 13)) & M26;
  h.v[3] = ((w[2] >> 13) | (w[3] << 19)) & M25;
  h.v[4] = (w[3] >> 6) & M26;
  h.v[5] = w[4] & M25;
  h.v[6] = ((w[4] >> 25) | (w[5] << 7)) & M26;
  h.v[7] = ((w[5] >> 19) | (w[6] << 13)) & M25;
  h.v[8] = ((w[6] >> 12) | (w[7] << 20)) & M26;
  h.v[9] = (w[7] >> 6) & M25;
}

EDV_HD bool fe_iszero(const fe& f) {
  fe h = f;
  fe_canon(h);
  uint32_t acc = 0;
#pragma unroll
  for (int k = 0; k < 10; ++k) acc |= h.v[k];
  return acc == 0;
}
EDV_HD uint32_t fe_isnegative(const fe& f) {
  fe h = f;
  fe_canon(h);
  return h.v[0] & 1;
}

// z^(2^255 - 21) = z^-1 (ref10 addition chain: 254 squarings, 11 multiplies).
// ORDER as fe_mul_o: 1 gives ten independent accumulator chains per product
// (for latency-bound callers at low occupancy, e.g. the batched encode).
template <int ORDER = EDV_FE_MUL_ORDER>
EDV_HDNI void fe_invert(fe& out, const fe& z) {
  fe t0, t1, t2, t3;
  fe_sq_o<ORDER>(t0, z);
  fe_sqn<ORDER>(t1, t0, 2);
  fe_mul_o<ORDER>(t1, z, t1);
  fe_mul_o<ORDER>(t0, t0, t1);
  fe_sq_o<ORDER>(t2, t0);
  fe_mul_o<ORDER>(t1, t1, t2);
  fe_sqn<ORDER>(t2, t1, 5);
  fe_mul_o<ORDER>(t1, t2, t1);
  fe_sqn<ORDER>(t2, t1, 10);
  fe_mul_o<ORDER>(t2, t2, t1);
  fe_sqn<ORDER>(t3, t2, 20);
  fe_mul_o<ORDER>(t2, t3, t2);
  fe_sqn<ORDER>(t2, t2, 10);
  fe_mul_o<ORDER>(t1, t2, t1);
  fe_sqn<ORDER>(t2, t1, 50);
  fe_mul_o<ORDER>(t2, t2, t1);
  fe_sqn<ORDER>(t3, t2, 100);
  fe_mul_o<ORDER>(t2, t3, t2);
  fe_sqn<ORDER>(t2, t2, 50);
  fe_mul_o<ORDER>(t1, t2, t1);
  fe_sqn<ORDER>(t1, t1, 5);
  fe_mul_o<ORDER>(out, t1, t0);
}

// z^(2^252 - 3) (for square roots; 250 squarings, 11 multiplies).
EDV_HDNI void fe_pow22523(fe& out, const fe& z) {
  fe t0, t1, t2;
  fe_sq(t0, z);
  fe_sqn(t1, t0, 2);
  fe_mul(t1, z, t1);
  fe_mul(t0, t0, t1);
  fe_sq(t0, t0);
  fe_mul(t0, t1, t0);
  fe_sqn(t1, t0, 5);
  fe_mul(t0, t1, t0);
  fe_sqn(t1, t0, 10);
  fe_mul(t1, t1, t0);
  fe_sqn(t2, t1, 20);
  fe_mul(t1, t2, t1);
  fe_sqn(t1, t1, 10);
  fe_mul(t0, t1, t0);
  fe_sqn(t1, t0, 50);
  fe_mul(t1, t1, t0);
  fe_sqn(t2, t1, 100);
  fe_mul(t1, t2, t1);
  fe_sqn(t1, t1, 50);
  fe_mul(t0, t1, t0);
  fe_sqn(t0, t0, 2);
  fe_mul(out, t0, z);
}

}  // namespace edv
