// batch_encode.h -- encode M projective results with ONE field inversion.
//
// libsodium's verify ends with ge25519_tobytes(R') (one inversion, ~265 field
// multiplications) and a byte compare with R.  Inversions of M independent
// requests share one inversion by Montgomery's trick: prefix products
// P_j = Z_0 ... Z_j, inv = P_{M-1}^-1, then walking back
// Z_j^-1 = inv * P_{j-1} and inv <- inv * Z_j: 3 multiplications per request
// plus 265/M.  The encodings are bit-identical to per-request tobytes.
//
// Z = 0 cannot arise from the complete a = -1 formulas on curve points, but a
// zero would poison the whole group, so it is replaced by 1 and that request
// is reported as not encodable (libsodium would encode (0, 0) -> 32 zero bytes,
// a blacklisted R that the precheck has already rejected: same verdict).
//
// Accessor A (device or host):
//   bool valid(j)                       request j of this group exists
//   void z(j, fe&), xy(j, fe&, fe&)     its projective Z and X, Y (class C)
//   void put_pre(j, const fe&), get_pre(j, fe&)   prefix-product scratch
//   void emit(j, const uint32_t enc[8], bool zero_z)   called for every j
//                                       in descending order (uniform control flow)
#pragma once
#include "ge25519.h"

namespace edv {

// Product form of the encode (fe_mul_o ORDER).  It runs at about one wave
// per SIMD (M results per lane), but ten independent accumulator chains per
// product (ORDER 1) measured slower than the carry-serial chains (ORDER 2):
// encode 0.148-0.152 -> 0.161-0.166 ms per 1M (profiles/r02o/ab_enc).
#ifndef EDV_ENCODE_ORDER
#define EDV_ENCODE_ORDER 2
#endif

template <int M, class A>
EDV_HD void encode_batch(A& a) {
  uint32_t zero_mask = 0;
  fe acc, z;
#pragma unroll 1
  for (int j = 0; j < M; ++j) {
    fe_1(z);
    if (a.valid(j)) {
      a.z(j, z);
      if (fe_iszero(z)) {
        fe_1(z);
        zero_mask |= 1u << j;
      }
    }
    if (j == 0)
      acc = z;
    else
      fe_mul_o<EDV_ENCODE_ORDER>(acc, acc, z);
    a.put_pre(j, acc);
  }
  fe inv;
  fe_invert<EDV_ENCODE_ORDER>(inv, acc);
#pragma unroll 1
  for (int j = M - 1; j >= 0; --j) {
    fe zinv;
    if (j > 0) {
      fe prev;
      a.get_pre(j - 1, prev);
      fe_mul_o<EDV_ENCODE_ORDER>(zinv, inv, prev);
      fe_1(z);
      if (a.valid(j) && !((zero_mask >> j) & 1u)) a.z(j, z);
      fe_mul_o<EDV_ENCODE_ORDER>(inv, inv, z);
    } else {
      zinv = inv;
    }
    fe X, Y, x, y;
    fe_1(X);
    fe_1(Y);
    if (a.valid(j)) a.xy(j, X, Y);
    fe_mul_o<EDV_ENCODE_ORDER>(x, X, zinv);
    fe_mul_o<EDV_ENCODE_ORDER>(y, Y, zinv);
    uint32_t enc[8];
    fe_tobytes(enc, y);
    enc[7] ^= fe_isnegative(x) << 31;
    a.emit(j, enc, (zero_mask >> j) & 1u);
  }
}

}  // namespace edv
