// ge25519.h -- edwards25519 group arithmetic (a = -1) on top of fe25519.h.
//
// Restates the point half of libsodium 1.0.18's verify, reached from
// stp_core/crypto/nacl_wrappers.py:108: decoding A with
// ge25519_frombytes_negate_vartime, the double-scalar multiplication
// [h](-A) + [S]B, and the final encoding compared byte-for-byte with R.
// Coordinates follow the usual extended/completed split:
//   p2 (X:Y:Z), p3 (X:Y:Z:T), p1p1 ((X:Z),(Y:T)), cached (Y+X, Y-X, Z, 2dT),
//   niels (y+x, y-x, 2dxy) for affine precomputed points.
// Bound classes (fe25519.h) are annotated on every intermediate.
#pragma once
#include "fe25519.h"
#include "base_table.h"

namespace edv {

struct ge_p2 {
  fe X, Y, Z;
};
struct ge_p3 {
  fe X, Y, Z, T;
};
struct ge_p1p1 {
  fe X, Y, Z, T;
};
struct ge_cached {
  fe YplusX, YminusX, Z, T2d;
};
struct ge_niels {
  fe ypx, ymx, xy2d;
};

// Curve constants (d, 2d, sqrt(-1)) and base tables: base_table.h, generated
// by tools/gen_constants.py from exact integers.

EDV_HD void ge_p3_0(ge_p3& h) {
  fe_0(h.X);
  fe_1(h.Y);
  fe_1(h.Z);
  fe_0(h.T);
}
EDV_HD void ge_cached_0(ge_cached& h) {
  fe_1(h.YplusX);
  fe_1(h.YminusX);
  fe_1(h.Z);
  fe_0(h.T2d);
}
EDV_HD void ge_niels_0(ge_niels& h) {
  fe_1(h.ypx);
  fe_1(h.ymx);
  fe_0(h.xy2d);
}

EDV_HD void ge_p1p1_to_p2(ge_p2& r, const ge_p1p1& p) {
  fe_mul(r.X, p.X, p.T);
  fe_mul(r.Y, p.Y, p.Z);
  fe_mul(r.Z, p.Z, p.T);
}
EDV_HD void ge_p1p1_to_p3(ge_p3& r, const ge_p1p1& p) {
  fe_mul(r.X, p.X, p.T);
  fe_mul(r.Y, p.Y, p.Z);
  fe_mul(r.Z, p.Z, p.T);
  fe_mul(r.T, p.X, p.Y);
}
EDV_HD void ge_p3_to_p2(ge_p2& r, const ge_p3& p) {
  r.X = p.X;
  r.Y = p.Y;
  r.Z = p.Z;
}
// p3 (all C) -> cached (YplusX L, YminusX L, Z C, T2d C).
// ORDER picks fe_mul_o's product order (fe25519.h): the default for throughput, 1 (ten
// independent accumulators) where one lane's latency is what counts (the small-batch kernel).
template <int ORDER = EDV_FE_MUL_ORDER>
EDV_HD void ge_p3_to_cached(ge_cached& r, const ge_p3& p) {
  fe_add(r.YplusX, p.Y, p.X);
  fe_sub(r.YminusX, p.Y, p.X);
  r.Z = p.Z;
  fe_mul_o<ORDER>(r.T2d, p.T, fe_const_d2());
}

// r = 2p.  p in C.  Output: X W, Y L, Z L, T C.
EDV_HD void ge_p2_dbl(ge_p1p1& r, const ge_p2& p) {
  fe xx, yy, zz, aa, s;
  fe_sq(xx, p.X);
  fe_sq(yy, p.Y);
  fe_sq(zz, p.Z);
  fe_add(s, p.X, p.Y);  // L
  fe_sq(aa, s);
  fe_add(r.Y, yy, xx);        // L
  fe_sub(r.Z, yy, xx);        // L
  fe_sub4(r.X, aa, r.Y);      // W   (AA - YY - XX = 2XY)
  fe t;
  fe_add(t, zz, zz);
  fe_add(t, t, xx);           // 3 C
  fe_sub(r.T, t, yy);         // W   (2ZZ + XX - YY)
  fe_carry(r.T);              // C
}
EDV_HD void ge_p3_dbl(ge_p1p1& r, const ge_p3& p) {
  ge_p2 q;
  ge_p3_to_p2(q, p);
  ge_p2_dbl(r, q);
}

// r = p + q.  p in C, q cached.  Output: X L, Y L, Z L, T W.
template <int ORDER = EDV_FE_MUL_ORDER>
EDV_HD void ge_add(ge_p1p1& r, const ge_p3& p, const ge_cached& q) {
  fe s, a, b, c, d;
  fe_add(s, p.Y, p.X);
  fe_mul_o<ORDER>(a, s, q.YplusX);
  fe_sub(s, p.Y, p.X);
  fe_mul_o<ORDER>(b, s, q.YminusX);
  fe_mul_o<ORDER>(c, p.T, q.T2d);
  fe_mul_o<ORDER>(d, p.Z, q.Z);
  fe_add(d, d, d);            // L
  fe_sub(r.X, a, b);          // L
  fe_add(r.Y, a, b);          // L
  fe_add(r.Z, d, c);          // L (3 C)
  fe_sub(r.T, d, c);          // 2C + 2p: W
}
// r = p - q.  Output: X L, Y L, Z W, T L.
EDV_HD void ge_sub(ge_p1p1& r, const ge_p3& p, const ge_cached& q) {
  fe s, a, b, c, d;
  fe_add(s, p.Y, p.X);
  fe_mul(a, s, q.YminusX);
  fe_sub(s, p.Y, p.X);
  fe_mul(b, s, q.YplusX);
  fe_mul(c, p.T, q.T2d);
  fe_mul(d, p.Z, q.Z);
  fe_add(d, d, d);
  fe_sub(r.X, a, b);
  fe_add(r.Y, a, b);
  fe_sub(r.Z, d, c);          // W
  fe_add(r.T, d, c);          // L
}
// r = p + q for affine q.  Output as ge_add.
EDV_HD void ge_madd(ge_p1p1& r, const ge_p3& p, const ge_niels& q) {
  fe s, a, b, c, d;
  fe_add(s, p.Y, p.X);
  fe_mul(a, s, q.ypx);
  fe_sub(s, p.Y, p.X);
  fe_mul(b, s, q.ymx);
  fe_mul(c, p.T, q.xy2d);
  fe_add(d, p.Z, p.Z);        // L
  fe_sub(r.X, a, b);
  fe_add(r.Y, a, b);
  fe_add(r.Z, d, c);
  fe_sub(r.T, d, c);          // W
}
// r = p - q for affine q.  Output as ge_sub.
EDV_HD void ge_msub(ge_p1p1& r, const ge_p3& p, const ge_niels& q) {
  fe s, a, b, c, d;
  fe_add(s, p.Y, p.X);
  fe_mul(a, s, q.ymx);
  fe_sub(s, p.Y, p.X);
  fe_mul(b, s, q.ypx);
  fe_mul(c, p.T, q.xy2d);
  fe_add(d, p.Z, p.Z);
  fe_sub(r.X, a, b);
  fe_add(r.Y, a, b);
  fe_sub(r.Z, d, c);          // W
  fe_add(r.T, d, c);
}

// r = p + q or p - q (neg) for affine q, straight to p3: ge_madd/ge_msub +
// ge_p1p1_to_p3_*, with the sign folded into selects on p's side so the
// table entry is used exactly as loaded.  -q = (y-x, y+x, -2dxy), so for neg
// the Y+X / Y-X multiplicands swap (a, b come out swapped: X3 = b - a) and
// 2Z +/- T*2dxy swap roles (Z3 = 2Z - c, T3 = 2Z + c).  Classes: a, b, c C;
// X3, Y3, plus L; minus W.
EDV_HD void ge_madd_signed(ge_p3& r, const ge_p3& p, const ge_niels& q, bool neg) {
  fe sp, sm, a, b, c, d, plus, minus, t;
  fe_add(sp, p.Y, p.X);       // L
  fe_sub(sm, p.Y, p.X);       // L
  t = sp;
  fe_cmov(sp, sm, neg);
  fe_cmov(sm, t, neg);
  fe_mul(a, sp, q.ypx);
  fe_mul(b, sm, q.ymx);
  fe_mul(c, p.T, q.xy2d);
  fe_add(d, p.Z, p.Z);        // L
  fe X3, Y3;
  fe_sub(X3, a, b);           // L
  fe_sub(t, b, a);            // L
  fe_cmov(X3, t, neg);
  fe_add(Y3, a, b);           // L
  fe_add(plus, d, c);         // L
  fe_sub(minus, d, c);        // W
  fe zs = plus, ts = minus;   // r.Z-side / r.T-side of the p1p1 point
  fe_cmov(zs, minus, neg);    // W
  fe_cmov(ts, plus, neg);     // W
  fe_mul(r.X, ts, X3);
  fe_mul(r.Y, zs, Y3);
  fe_mul(r.Z, minus, plus);
  fe_mul(r.T, X3, Y3);
}

// r = p + q or p - q (neg) for cached q, straight to p3 (ge_add/ge_sub +
// ge_p1p1_to_p3_*), the sign folded in as in ge_madd_signed.
EDV_HD void ge_add_signed(ge_p3& r, const ge_p3& p, const ge_cached& q, bool neg) {
  fe sp, sm, a, b, c, d, plus, minus, t;
  fe_add(sp, p.Y, p.X);
  fe_sub(sm, p.Y, p.X);
  t = sp;
  fe_cmov(sp, sm, neg);
  fe_cmov(sm, t, neg);
  fe_mul(a, sp, q.YplusX);
  fe_mul(b, sm, q.YminusX);
  fe_mul(c, p.T, q.T2d);
  fe_mul(d, p.Z, q.Z);
  fe_add(d, d, d);            // L
  fe X3, Y3;
  fe_sub(X3, a, b);
  fe_sub(t, b, a);
  fe_cmov(X3, t, neg);
  fe_add(Y3, a, b);
  fe_add(plus, d, c);         // L
  fe_sub(minus, d, c);        // W
  fe zs = plus, ts = minus;
  fe_cmov(zs, minus, neg);
  fe_cmov(ts, plus, neg);
  fe_mul(r.X, ts, X3);
  fe_mul(r.Y, zs, Y3);
  fe_mul(r.Z, minus, plus);
  fe_mul(r.T, X3, Y3);
}

// p1p1 -> p2/p3 need the W operand first (fe_mul's f).  ge_add/madd leave T
// in W, ge_sub/msub leave Z in W; ge_p2_dbl leaves X in W and T carried.
// T3 = Y * X (not X * Y): the four products then need 2 * Y / 2 * T odd limbs
// and 19 * X / 19 * Z premultiplies only (fe_mul's f2 / g19), not three each.
template <int ORDER = EDV_FE_MUL_ORDER>
EDV_HD void ge_p1p1_to_p3_addlike(ge_p3& r, const ge_p1p1& p) {  // T is W
  fe_mul_o<ORDER>(r.X, p.T, p.X);
  fe_mul_o<ORDER>(r.Y, p.Y, p.Z);
  fe_mul_o<ORDER>(r.Z, p.T, p.Z);
  fe_mul_o<ORDER>(r.T, p.Y, p.X);
}
EDV_HD void ge_p1p1_to_p3_sublike(ge_p3& r, const ge_p1p1& p) {  // Z is W
  fe_mul(r.X, p.X, p.T);
  fe_mul(r.Y, p.Z, p.Y);
  fe_mul(r.Z, p.Z, p.T);
  fe_mul(r.T, p.X, p.Y);
}
template <int ORDER = EDV_FE_MUL_ORDER>
EDV_HD void ge_p1p1_to_p2_addlike(ge_p2& r, const ge_p1p1& p) {
  fe_mul_o<ORDER>(r.X, p.T, p.X);
  fe_mul_o<ORDER>(r.Y, p.Y, p.Z);
  fe_mul_o<ORDER>(r.Z, p.T, p.Z);
}
EDV_HD void ge_p1p1_to_p2_sublike(ge_p2& r, const ge_p1p1& p) {
  fe_mul(r.X, p.X, p.T);
  fe_mul(r.Y, p.Z, p.Y);
  fe_mul(r.Z, p.Z, p.T);
}
// After ge_p2_dbl: X is W, T is C, Y/Z L.
EDV_HD void ge_dbl_to_p2(ge_p2& r, const ge_p1p1& p) {
  fe_mul(r.X, p.X, p.T);
  fe_mul(r.Y, p.Y, p.Z);
  fe_mul(r.Z, p.Z, p.T);
}
EDV_HD void ge_dbl_to_p3(ge_p3& r, const ge_p1p1& p) {
  fe_mul(r.X, p.X, p.T);
  fe_mul(r.Y, p.Y, p.Z);
  fe_mul(r.Z, p.Z, p.T);
  fe_mul(r.T, p.X, p.Y);
}

// Encoding: y with the sign of x in bit 255 (8 LE words).
EDV_HDNI void ge_tobytes(uint32_t s[8], const ge_p2& h) {
  fe recip, x, y;
  fe_invert(recip, h.Z);
  fe_mul(x, h.X, recip);
  fe_mul(y, h.Y, recip);
  fe_tobytes(s, y);
  s[7] ^= fe_isnegative(x) << 31;
}

// libsodium 1.0.18 ge25519_frombytes_negate_vartime restated; negate = false
// gives +P (base point, signer).  Returns false if x^2 has no square root.
EDV_HDNI bool ge_frombytes(ge_p3& h, const uint32_t s[8], bool negate) {
  fe u, v, v3, vxx, chk, one;
  fe_1(one);
  fe_frombytes(h.Y, s);
  fe_1(h.Z);
  fe_sq(u, h.Y);
  fe_mul(v, u, fe_const_d());
  fe_sub(u, u, one);   // y^2 - 1           (L)
  fe_carry(u);         // C
  fe_add(v, v, one);   // d y^2 + 1         (C + 1)
  fe_sq(v3, v);
  fe_mul(v3, v3, v);   // v^3
  fe_sq(h.X, v3);
  fe_mul(h.X, h.X, v);
  fe_mul(h.X, h.X, u); // u v^7
  fe_pow22523(h.X, h.X);
  fe_mul(h.X, h.X, v3);
  fe_mul(h.X, h.X, u); // u v^3 (u v^7)^((p-5)/8)
  fe_sq(vxx, h.X);
  fe_mul(vxx, vxx, v);
  fe_sub(chk, vxx, u); // v x^2 - u
  if (!fe_iszero(chk)) {
    fe_add(chk, vxx, u);
    if (!fe_iszero(chk)) {
      ge_p3_0(h);  // not on the curve: hand back a well-formed point (the verdict is reject)
      return false;
    }
    fe_mul(h.X, h.X, fe_const_sqrtm1());
  }
  const uint32_t sign = s[7] >> 31;
  const bool flip = negate ? (fe_isnegative(h.X) == sign) : (fe_isnegative(h.X) != sign);
  if (flip) {
    fe_neg(h.X, h.X);
    fe_carry(h.X);
  }
  fe_mul(h.T, h.X, h.Y);
  return true;
}

}  // namespace edv
