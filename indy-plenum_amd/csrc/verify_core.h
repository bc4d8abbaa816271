// verify_core.h -- one Ed25519 verification per lane, libsodium 1.0.18 predicate.
//
// The per-request arithmetic Plenum runs in
//   NaclAuthNr.authenticate (plenum/server/client_authn.py:99-102)
//     -> DidVerifier.verify (plenum/common/verifier.py:48-49)
//     -> Verifier.verify (stp_core/crypto/nacl_wrappers.py:232-242)
//     -> libnacl.crypto_sign_open (nacl_wrappers.py:108)
//     -> libsodium crypto_sign_verify_detached.
// Accept iff ALL of (libsodium 1.0.18, non-ED25519_COMPAT):
//   S < L;  R not in the small-order blacklist;  A canonical (y < p);
//   A not in the blacklist;  A decodes;  encode([h](-A) + [S]B) == R  byte-exact,
// with h = SHA-512(R || A || M) mod L.  Cofactorless, so mixed-order A with a
// cofactorless-valid signature is accepted and R + T8 is rejected.
//
// The same code is compiled for gfx950 (the product kernels) and for the host
// (csrc/host_selftest.cpp) so the arithmetic can be checked on a CPU.
#pragma once
#include "comb.h"
#include "ge25519.h"
#include "sc25519.h"
#include "sha512.h"

namespace edv {

// ge25519_has_small_order blacklist (31 bytes exact, last byte sign-masked),
// as LE u32 words.
EDV_HD bool has_small_order(const uint32_t s[8]) {
  const uint32_t top = s[7] & 0x7fffffffu;
  bool mid_zero = true, mid_ff = true;
#pragma unroll
  for (int k = 1; k < 7; ++k) {
    mid_zero = mid_zero && s[k] == 0;
    mid_ff = mid_ff && s[k] == 0xffffffffu;
  }
  // 0 and 1
  if (mid_zero && top == 0 && (s[0] == 0 || s[0] == 1)) return true;
  // p-1, p, p+1
  if (mid_ff && top == 0x7fffffffu && (s[0] == 0xffffffecu || s[0] == 0xffffffedu || s[0] == 0xffffffeeu))
    return true;
  // the two order-8 points
  const uint32_t o8a[8] = {0x8f95e826u, 0xb027b2c2u, 0x89f4c345u, 0xf098eff2u,
                           0x05acdfd5u, 0x3933c6d3u, 0x880238b1u, 0x05fc536du};
  const uint32_t o8b[8] = {0x706a17c7u, 0x4fd84d3du, 0x760b3cbau, 0x0f67100du,
                           0xfa53202au, 0xc6cc392cu, 0x77fdc74eu, 0x7a03ac92u};
  bool ea = top == o8a[7], eb = top == o8b[7];
#pragma unroll
  for (int k = 0; k < 7; ++k) {
    ea = ea && s[k] == o8a[k];
    eb = eb && s[k] == o8b[k];
  }
  return ea || eb;
}

// ge25519_is_canonical: y (sign bit masked) < p.
EDV_HD bool is_canonical_point(const uint32_t s[8]) {
  bool all_ff = (s[7] & 0x7fffffffu) == 0x7fffffffu;
#pragma unroll
  for (int k = 1; k < 7; ++k) all_ff = all_ff && s[k] == 0xffffffffu;
  return !(all_ff && s[0] >= 0xffffffedu);
}

EDV_HD int recode_digit(const uint32_t y[8], int i) {
  const int w = i >> 3;
  uint32_t v = y[0];
#pragma unroll
  for (int k = 1; k < 8; ++k) v = (w == k) ? y[k] : v;
  return (int)((v >> (4 * (i & 7))) & 15u) - 8;
}

// Phase 1: libsodium's prechecks and h = SHA-512(R || A || M) mod L.
EDV_HD bool verify_phase_hash(uint32_t h[8], const uint32_t sig[16], const uint32_t pk[8], const uint8_t* msg,
                              uint64_t mlen) {
  const uint32_t* R = sig;
  const uint32_t* S = sig + 8;
  const bool ok = sc_is_canonical(S) && !has_small_order(R) && is_canonical_point(pk) && !has_small_order(pk);
  uint32_t prefix[16], digest[16];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    prefix[k] = R[k];
    prefix[8 + k] = pk[k];
  }
  sha512_prefixed<16>(digest, prefix, msg, mlen);
  sc_reduce(h, digest);
  return ok;
}
// The same with M in the packed unit layout (sha512.h pack_lane_units).
EDV_HD bool verify_phase_hash_units(uint32_t h[8], const uint32_t sig[16], const uint32_t pk[8], const Chunk16* units,
                                    uint64_t stride, uint64_t mlen) {
  const uint32_t* R = sig;
  const uint32_t* S = sig + 8;
  const bool ok = sc_is_canonical(S) && !has_small_order(R) && is_canonical_point(pk) && !has_small_order(pk);
  uint32_t prefix[16], digest[16];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    prefix[k] = R[k];
    prefix[8 + k] = pk[k];
  }
  sha512_prefixed_units(digest, prefix, units, stride, mlen);
  sc_reduce(h, digest);
  return ok;
}

// Phase 2: decode -A and store the cached multiples [1..8](-A) through TA:
//   TA::store(j, const ge_cached&) for j in 0..7 (= (j+1)(-A)); slot 8 holds
//   the identity (TA::load(-1) in phase 3).
template <class TA>
EDV_HD bool verify_phase_table(const uint32_t pk[8], TA& ta) {
  ge_p3 A;
  const bool ok = ge_frombytes(A, pk, true);
  ge_cached c;
  ge_p3 acc = A;
  ge_p1p1 t;
  ge_p3_to_cached(c, acc);
  ta.store(0, c);
  const ge_cached a1 = c;
#pragma unroll 1
  for (int j = 1; j < 8; ++j) {
    ge_add(t, acc, a1);
    ge_p1p1_to_p3_addlike(acc, t);
    ge_p3_to_cached(c, acc);
    ta.store(j, c);
  }
  ge_cached_0(c);
  ta.store(8, c);
  return ok;
}

// Phase 3: R' = [h](-A) + [S]B.  [h](-A): signed radix-16 windows, 4
// doublings per digit, TA::load(j, ge_cached&) gives (j+1)(-A).  [S]B: the
// W = 8 fixed-base comb of B (CB::load(row, j, ge_niels&), comb.h), 32 mixed
// additions and no doublings of its own.
#ifndef EDV_BASE_W
#define EDV_BASE_W 24  // 16: 16 rows (64 MiB); 20: 13 (832 MiB), comb -8% vs 16; 22: 12 (3 GiB), +1.5% vs 20;
                       // 24: 11 rows (11 GiB, 1 GiB row slabs), comb -4..7% vs 22; 26: 10 rows (40 GiB, 4 GiB
                       // slabs), comb +6..15% vs 24 (profiles/r02i/ab_b24, ab_b26)
#endif                  // (tools/gpu_basew.sh, tools/gpu_ab_b22.sh)
constexpr int kBaseW = EDV_BASE_W;  // base-point comb window: 11 rows x 2^23 entries (11 GiB) at W = 24
template <class TA, class CB>
EDV_HD uint32_t verify_phase_dsm_point(ge_p3& Q, const uint32_t h[8], const uint32_t S[8], const TA& ta,
                                       const CB& cb) {
  // radix-16 digits of h, top first: shift the recoded words left 4 bits per
  // digit (static register indexing; see CombDigits)
  uint32_t hy[8];
  sc_recode16(hy, h);
  ge_p3_0(Q);
  ge_p1p1 t;
#pragma unroll 1
  for (int i = 63; i >= 0; --i) {
    if (i != 63) {
      ge_p2 q2;
      ge_p3_to_p2(q2, Q);
      ge_p2_dbl(t, q2);
      ge_dbl_to_p2(q2, t);
      ge_p2_dbl(t, q2);
      ge_dbl_to_p2(q2, t);
      ge_p2_dbl(t, q2);
      ge_dbl_to_p2(q2, t);
      ge_p2_dbl(t, q2);
      ge_dbl_to_p3(Q, t);
    }
    const int e = (int)(hy[7] >> 28) - 8;  // = recode_digit(hy, i) of the unshifted words
#pragma unroll
    for (int k = 7; k > 0; --k) hy[k] = funnel32(hy[k], hy[k - 1], 28);
    hy[0] <<= 4;
    const int m = e < 0 ? -e : e;
    ge_cached c;
    ta.load(m - 1, c);  // m = 0: the identity (an address select in the accessor)
    ge_add_signed(Q, Q, c, e < 0);
  }
  return comb_mul_add<kBaseW>(Q, S, cb);  // the base comb's prefetch sink (comb.h)
}

// Split tables for keys shared by many requests (the general path's distinct
// keys, edverify.hip): h = sum_t h_t 2^(256 t / K), t < K, and table t holds
// [1..8] 2^(256 t / K)(-A), so the ladder runs 256 / K - 4 doublings instead
// of 252 and the same 64 additions; the K - 1 extra tables cost 256 (K-1)/K
// doublings once per key.  TAS::store(t, j, c) / TAS::load(t, j, c) address
// table t (j = -1: the identity).  Same point as verify_phase_dsm_point
// (another order of the same group operations).
template <int K, class TAS>
EDV_HD bool verify_phase_table_split(const uint32_t pk[8], const TAS& tas) {
  ge_p3 P;
  const bool ok = ge_frombytes(P, pk, true);
#pragma unroll 1
  for (int t = 0; t < K; ++t) {
    if (t > 0) {  // P = 2^(256/K) P
      ge_p2 q2;
      ge_p1p1 d;
      ge_p3_to_p2(q2, P);
#pragma unroll 1
      for (int k = 0; k < 256 / K - 1; ++k) {
        ge_p2_dbl(d, q2);
        ge_dbl_to_p2(q2, d);
      }
      ge_p2_dbl(d, q2);
      ge_dbl_to_p3(P, d);
    }
    ge_cached c;
    ge_p3 acc = P;
    ge_p1p1 u;
    ge_p3_to_cached(c, acc);
    tas.store(t, 0, c);
    const ge_cached a1 = c;
#pragma unroll 1
    for (int j = 1; j < 8; ++j) {
      ge_add(u, acc, a1);
      ge_p1p1_to_p3_addlike(acc, u);
      ge_p3_to_cached(c, acc);
      tas.store(t, j, c);
    }
    ge_cached_0(c);
    tas.store(t, 8, c);
  }
  return ok;
}

template <int K, class TAS, class CB>
EDV_HD uint32_t verify_phase_dsm_split_point(ge_p3& Q, const uint32_t h[8], const uint32_t S[8], const TAS& tas,
                                             const CB& cb) {
  constexpr int kWords = 8 / K;       // recoded words per table
  constexpr int kDigits = 8 * kWords;  // radix-16 digits per table
  uint32_t hy[8];
  sc_recode16(hy, h);
  ge_p3_0(Q);
  ge_p1p1 t;
#pragma unroll 1
  for (int i = kDigits - 1; i >= 0; --i) {
    if (i != kDigits - 1) {
      ge_p2 q2;
      ge_p3_to_p2(q2, Q);
      ge_p2_dbl(t, q2);
      ge_dbl_to_p2(q2, t);
      ge_p2_dbl(t, q2);
      ge_dbl_to_p2(q2, t);
      ge_p2_dbl(t, q2);
      ge_dbl_to_p2(q2, t);
      ge_p2_dbl(t, q2);
      ge_dbl_to_p3(Q, t);
    }
#pragma unroll
    for (int s = K - 1; s >= 0; --s) {
      uint32_t* w = hy + s * kWords;
      const int e = (int)(w[kWords - 1] >> 28) - 8;  // digit s * kDigits + i
#pragma unroll
      for (int k = kWords - 1; k > 0; --k) w[k] = funnel32(w[k], w[k - 1], 28);
      w[0] <<= 4;
      const int m = e < 0 ? -e : e;
      ge_cached c;
      tas.load(s, m - 1, c);
      ge_add_signed(Q, Q, c, e < 0);
    }
  }
  return comb_mul_add<kBaseW>(Q, S, cb);
}

// encode(R') == R byte for byte (per-request inversion; the kernels batch it).
EDV_HD bool encode_equals(const ge_p3& Q, const uint32_t R[8]) {
  ge_p2 r2;
  ge_p3_to_p2(r2, Q);
  uint32_t rcheck[8];
  ge_tobytes(rcheck, r2);
  bool eq = true;
#pragma unroll
  for (int k = 0; k < 8; ++k) eq = eq && rcheck[k] == R[k];
  return eq;
}

template <class TA, class CB>
EDV_HD bool verify_phase_dsm(const uint32_t h[8], const uint32_t S[8], const uint32_t R[8], const TA& ta,
                             const CB& cb) {
  ge_p3 Q;
  verify_phase_dsm_point(Q, h, S, ta, cb);
  return encode_equals(Q, R);
}

// All three phases for one request (host self-test and the fused kernel).
template <class TA, class TB>
EDV_HD bool verify_one(const uint32_t sig[16], const uint32_t pk[8], const uint8_t* msg, uint64_t mlen, TA& ta,
                       const TB& tb) {
  uint32_t h[8];
  bool ok = verify_phase_hash(h, sig, pk, msg, mlen);
  ok = verify_phase_table(pk, ta) && ok;
  return verify_phase_dsm(h, sig + 8, sig, ta, tb) && ok;
}

}  // namespace edv
