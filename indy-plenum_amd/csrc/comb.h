// comb.h -- fixed-base comb tables and the comb double-scalar multiplication.
//
// For a point P and window width W, the table holds, for every row
// i < ROWS = ceil(253 / W) and every magnitude j < 2^(W-1), the affine niels
// form (y+x, y-x, 2dxy) of (j+1) * 2^(W*i) * P.  With signed radix-2^W digits
// d_i in [-2^(W-1), 2^(W-1) - 1] of a scalar x < 2^253,
//     [x]P = sum_i d_i * 2^(W*i) * P,
// so the double-scalar multiplication of libsodium's verify,
// [h](-A) + [S]B, becomes ROWS_A + ROWS_B mixed additions and no doublings
// (the a-priori ref10 count: ~253 doublings + ~86 additions).
//   A = a registered public key (client_authn.py SimpleAuthNr.addIdr keys),
//       in HBM; the context's key window picks memory against additions:
//       W = 4: 64 rows x   8 entries x 128 B =  64 KiB per key, 64 additions
//       W = 6: 43 rows x  32 entries x 128 B = 172 KiB per key, 43 additions
//       W = 8: 32 rows x 128 entries x 128 B = 512 KiB per key, 32 additions
//       W = 10: 26 rows x 512 entries x 128 B = 1.6 MiB per key, 26 additions
//       W = 13: 20 rows x 4096 entries x 128 B = 10 MiB per key, 20 additions
//   B = the base point, one table per context (kBaseW, verify_core.h):
//       W = 24: 11 rows x 2^23 entries x 128 B = 11 GiB (a 1 GiB slab per row).
// Entries are 32 u32 words (30 limbs + 2 pad) so one entry is 8 dwordx4 loads.
#pragma once
#include "ge25519.h"

namespace edv {

constexpr int kEntryWords = 32;

template <int W>
struct Window {
  static_assert(W >= 4 && W <= 26, "comb window width 4..26");
  // x < L < 2^253 plus the digit bias must stay below 2^(W * kRows): W * kRows >= 254
  static constexpr int kRows = (254 + W - 1) / W;
  static constexpr int kEntries = 1 << (W - 1);
  static constexpr uint64_t kTableWords = (uint64_t)kRows * kEntries * kEntryWords;
  // word k of bias = sum_{i < kRows} 2^(W-1) * 2^(W*i)   (9 words: W*kRows may exceed 256)
  static constexpr uint32_t bias_word(int k) {
    uint32_t w = 0;
    for (int i = 0; i < kRows; ++i) {
      const int b = W - 1 + W * i;
      if ((b >> 5) == k) w |= 1u << (b & 31);
    }
    return w;
  }
};

// y = x + bias: digit_i = ((y >> W*i) & (2^W - 1)) - 2^(W-1) in [-2^(W-1), 2^(W-1) - 1]
// and x = sum digit_i 2^(W*i) for x < L (x + bias < 2^(W*kRows) since W*kRows >= 254).  Any
// 256-bit x still yields in-range digits (table indices stay in bounds); only
// S >= L reaches that, and it is rejected by the precheck.
template <int W>
EDV_HD void comb_recode(uint32_t y[9], const uint32_t x[8]) {
  uint64_t carry = 0;
#pragma unroll
  for (int k = 0; k < 9; ++k) {
    const uint64_t t = (uint64_t)(k < 8 ? x[k] : 0u) + Window<W>::bias_word(k) + carry;
    y[k] = (uint32_t)t;
    carry = t >> 32;
  }
}

// (hi:lo) >> s, low word (v_alignbit_b32 on the device).
EDV_HD uint32_t funnel32(uint32_t hi, uint32_t lo, uint32_t s) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_alignbit(hi, lo, s);
#else
  return (uint32_t)((((uint64_t)hi << 32) | lo) >> s);
#endif
}

// The digits of comb_recode's y, lowest first, by shifting y right W bits per
// digit: static register indexing only (a per-row select over y, or a
// private array indexed by the row, ends up in scratch memory).
template <int W>
struct CombDigits {
  uint32_t y[9];
  EDV_HDM explicit CombDigits(const uint32_t x[8]) { comb_recode<W>(y, x); }
  EDV_HDM int next() {
    const int d = (int)(y[0] & ((1u << W) - 1)) - (1 << (W - 1));
#pragma unroll
    for (int k = 0; k < 8; ++k) y[k] = funnel32(y[k + 1], y[k], W);
    y[8] >>= W;
    return d;
  }
};

template <int W>
EDV_HD int comb_digit(const uint32_t y[9], int i) {
  const int b = W * i;
  const int w = b >> 5, s = b & 31;
  uint32_t lo = y[0], hi = y[1];
#pragma unroll
  for (int k = 1; k < 8; ++k) {
    lo = (w == k) ? y[k] : lo;
    hi = (w == k) ? y[k + 1] : hi;
  }
  const uint32_t v = (uint32_t)((((uint64_t)hi << 32) | lo) >> s);
  return (int)(v & ((1u << W) - 1)) - (1 << (W - 1));
}

// Signed-digit entry of row `row` for digit e: T::load(row, j, ge_niels&)
// gives entry j (= (j+1) * 2^(W*row) * P), or the identity for j = -1 (an
// address select in the accessors, so no data is shuffled); the sign is
// applied by ge_madd_signed on Q's side.  A conditional swap of whole fe
// structs is lowered through scratch memory, so none is done here.
template <class T>
EDV_HD void comb_fetch(ge_niels& nb, int e, const T& tab, int row) {
  const int m = e < 0 ? -e : e;
  tab.load(row, m - 1, nb);
}
#ifndef EDV_SIGNED_MADD
#define EDV_SIGNED_MADD 0  // 1: fold the sign into ge_madd_signed (p side) instead of selecting the entry
#endif
EDV_HD void comb_apply(ge_p3& Q, ge_niels& nb, int e) {
#if EDV_SIGNED_MADD
  ge_madd_signed(Q, Q, nb, e < 0);
#else
  // -entry = (y-x, y+x, -2dxy): per-limb selects in place (no struct swap)
  const bool neg = e < 0;
#pragma unroll
  for (int l = 0; l < 10; ++l) {
    const uint32_t p = nb.ypx.v[l], m = nb.ymx.v[l], t = nb.xy2d.v[l];
    nb.ypx.v[l] = neg ? m : p;
    nb.ymx.v[l] = neg ? p : m;
    nb.xy2d.v[l] = neg ? two_p(l) - t : t;
  }
  ge_p1p1 u;
  ge_madd(u, Q, nb);
  ge_p1p1_to_p3_addlike(Q, u);
#endif
}

// The identity as a niels entry (y+x, y-x, 2dxy) = (1, 1, 0), padded to kEntryWords.
#if defined(__HIPCC__)
__device__ __constant__ const uint32_t kNielsIdentity[kEntryWords] = {1, 0, 0, 0, 0, 0, 0, 0, 0, 0,
                                                                      1, 0, 0, 0, 0, 0, 0, 0, 0, 0};
#endif
static const uint32_t kNielsIdentityHost[kEntryWords] = {1, 0, 0, 0, 0, 0, 0, 0, 0, 0, 1, 0, 0, 0, 0, 0, 0, 0, 0, 0};

// Q += [x]P for x < 2^253 by the comb over P's table: kRows mixed additions
// (7 multiplications each).  Row r + 1's entry is fetched before row r's
// addition runs, so the table gather overlaps the arithmetic.
#ifndef EDV_COMB_PREFETCH
#define EDV_COMB_PREFETCH 0  // 0: none (best: the comb is VALU-bound); 1: row r+1 into registers (spills); 2: touch its line (-5%)
#endif
// T::touch(row, j) (optional prefetch): a 4-byte load of entry j's 128-B line
// whose value is folded into `sink` one row later, so the line is in L2/MALL
// when the row's own loads arrive and no wait is placed early.
template <int W, class T>
EDV_HD uint32_t comb_mul_add(ge_p3& Q, const uint32_t x[8], const T& tab) {
  CombDigits<W> dg(x);
  uint32_t sink = 0;
#if EDV_COMB_PREFETCH == 1
  int e = dg.next();
  ge_niels cur;
  comb_fetch(cur, e, tab, 0);
#pragma unroll 1
  for (int r = 0; r < Window<W>::kRows; ++r) {
    ge_niels next;
    int e_next = 0;
    if (r + 1 < Window<W>::kRows) {
      e_next = dg.next();
      comb_fetch(next, e_next, tab, r + 1);
    } else {
      ge_niels_0(next);
    }
    comb_apply(Q, cur, e);
    cur = next;
    e = e_next;
  }
#elif EDV_COMB_PREFETCH == 2
  int e = dg.next();
  uint32_t pf = 0;
#pragma unroll 1
  for (int r = 0; r < Window<W>::kRows; ++r) {
    sink ^= pf;
    int e_next = 0;
    if (r + 1 < Window<W>::kRows) {
      e_next = dg.next();
      const int m = e_next < 0 ? -e_next : e_next;
      pf = tab.touch(r + 1, m - 1);
    }
    ge_niels nb;
    comb_fetch(nb, e, tab, r);
    comb_apply(Q, nb, e);
    e = e_next;
  }
  sink ^= pf;
#else
#pragma unroll 1
  for (int r = 0; r < Window<W>::kRows; ++r) {
    const int e = dg.next();
    ge_niels nb;
    comb_fetch(nb, e, tab, r);
    comb_apply(Q, nb, e);  // nb is consumed
  }
#endif
  return sink;
}

// Q = signed entry e of row 0 as an extended point (Q += entry from the
// identity, without the mixed addition): (y+x) - (y-x) = 2x, (y+x) + (y-x) =
// 2y, Z = 2, T = XY / Z = 2xy = 2dxy / d -- one multiplication instead of 7.
// -entry = (y-x, y+x, -2dxy) gives (-2x, 2y, 2, -2xy); the identity entry
// (1, 1, 0) gives (0, 2, 2, 0).  Output classes: X, Y, Z, T all C.
template <int ORDER = EDV_FE_MUL_ORDER>
EDV_HD void comb_set_entry(ge_p3& Q, const ge_niels& nb, int e) {
  const bool neg = e < 0;
  fe p, m, t;
#pragma unroll
  for (int l = 0; l < 10; ++l) {
    p.v[l] = neg ? nb.ymx.v[l] : nb.ypx.v[l];
    m.v[l] = neg ? nb.ypx.v[l] : nb.ymx.v[l];
    t.v[l] = neg ? two_p(l) - nb.xy2d.v[l] : nb.xy2d.v[l];
  }
  fe_sub(Q.X, p, m);  // L
  fe_carry(Q.X);
  fe_add(Q.Y, p, m);  // L
  fe_carry(Q.Y);
  fe_0(Q.Z);
  Q.Z.v[0] = 2;
  fe_mul_o<ORDER>(Q.T, t, fe_const_dinv());
}
template <class T>
EDV_HD void comb_set(ge_p3& Q, int e, const T& tab) {
  ge_niels nb;
  comb_fetch(nb, e, tab, 0);
  comb_set_entry(Q, nb, e);
}

// Q = [x]P by the comb over P's table: row 0 by comb_set, then kRows - 1
// mixed additions.
template <int W, class T>
EDV_HD void comb_mul_set(ge_p3& Q, const uint32_t x[8], const T& tab) {
  CombDigits<W> dg(x);
  comb_set(Q, dg.next(), tab);
#pragma unroll 1
  for (int r = 1; r < Window<W>::kRows; ++r) {
    const int e = dg.next();
    ge_niels nb;
    comb_fetch(nb, e, tab, r);
    comb_apply(Q, nb, e);
  }
}

EDV_HD void store_fe(uint32_t* p, const fe& f) {
#pragma unroll
  for (int l = 0; l < 10; ++l) p[l] = f.v[l];
}
EDV_HD void load_fe(fe& f, const uint32_t* p) {
#pragma unroll
  for (int l = 0; l < 10; ++l) f.v[l] = p[l];
}
EDV_HD void store_fe_canon(uint32_t* p, const fe& f) {
  fe c = f;
  fe_canon(c);
  store_fe(p, c);
}

// Row bases 2^(W*i) * P, i < ROWS, as p3 points (40 words each).
template <int W>
EDV_HD void comb_rows(uint32_t* rows, ge_p3 P) {
#pragma unroll 1
  for (int i = 0; i < Window<W>::kRows; ++i) {
    store_fe(rows + i * 40, P.X);
    store_fe(rows + i * 40 + 10, P.Y);
    store_fe(rows + i * 40 + 20, P.Z);
    store_fe(rows + i * 40 + 30, P.T);
    ge_p2 q2;
    ge_p1p1 t;
    ge_p3_to_p2(q2, P);
#pragma unroll 1
    for (int d = 0; d < W - 1; ++d) {
      ge_p2_dbl(t, q2);
      ge_dbl_to_p2(q2, t);
    }
    ge_p2_dbl(t, q2);
    ge_dbl_to_p3(P, t);
  }
}

// Entries j = c + nch * t (t < count) of one row -- the multiples (j+1) * base
// -- with one shared inversion (Montgomery's trick; prefix product t at
// pre + t * pre_stride, 10 words), affine niels out.  Lane c of a row starts
// at (c+1) * base (double-and-add) and steps by nch * base (log2(nch)
// doublings; nch a power of two), so the nch lanes of a row write
// consecutive entries at every step (edv_comb_fill_kernel).
EDV_HD void comb_fill_strided(uint32_t* entries, uint32_t* pre, uint64_t pre_stride, const uint32_t* base_words,
                              int c, int nch, int count) {
  ge_p3 base, m, step;
  load_fe(base.X, base_words);
  load_fe(base.Y, base_words + 10);
  load_fe(base.Z, base_words + 20);
  load_fe(base.T, base_words + 30);
  ge_cached cb, cs;
  ge_p3_to_cached(cb, base);
  step = base;
#pragma unroll 1
  for (int s = nch; s > 1; s >>= 1) {
    ge_p1p1 t;
    ge_p3_dbl(t, step);
    ge_dbl_to_p3(step, t);
  }
  ge_p3_to_cached(cs, step);
  // m = (c + 1) * base, most significant bit first
  const uint32_t k = (uint32_t)c + 1u;
  const int top = 31 - __builtin_clz(k);
  m = base;
#pragma unroll 1
  for (int bit = top - 1; bit >= 0; --bit) {
    ge_p1p1 t;
    ge_p3_dbl(t, m);
    ge_dbl_to_p3(m, t);
    if ((k >> bit) & 1u) {
      ge_add(t, m, cb);
      ge_p1p1_to_p3_addlike(m, t);
    }
  }
  fe acc;
#pragma unroll 1
  for (int t = 0; t < count; ++t) {
    if (t > 0) {
      ge_p1p1 u;
      ge_add(u, m, cs);
      ge_p1p1_to_p3_addlike(m, u);
    }
    uint32_t* e = entries + (uint64_t)(c + nch * t) * kEntryWords;
    store_fe(e, m.X);
    store_fe(e + 10, m.Y);
    store_fe(e + 20, m.Z);
    if (t == 0)
      acc = m.Z;
    else
      fe_mul(acc, acc, m.Z);
    store_fe(pre + t * pre_stride, acc);
  }
  fe inv;
  fe_invert(inv, acc);
#pragma unroll 1
  for (int t = count - 1; t >= 0; --t) {
    uint32_t* e = entries + (uint64_t)(c + nch * t) * kEntryWords;
    fe zinv, X, Y, Z, x, y, u;
    load_fe(X, e);
    load_fe(Y, e + 10);
    load_fe(Z, e + 20);
    if (t > 0) {
      fe p;
      load_fe(p, pre + (t - 1) * pre_stride);
      fe_mul(zinv, inv, p);
      fe_mul(inv, inv, Z);
    } else {
      zinv = inv;
    }
    fe_mul(x, X, zinv);
    fe_mul(y, Y, zinv);
    fe_add(u, y, x);
    store_fe_canon(e, u);
    fe_sub(u, y, x);
    store_fe_canon(e + 10, u);
    fe_mul(u, x, y);
    fe_mul(u, u, fe_const_d2());
    store_fe_canon(e + 20, u);
    e[30] = 0;
    e[31] = 0;
  }
}

// The whole row (kEntries multiples) in one chunk.
template <int W>
EDV_HD void comb_fill_row(uint32_t* entries, uint32_t* pre, const uint32_t* base_words) {
  comb_fill_strided(entries, pre, 10, base_words, 0, 1, Window<W>::kEntries);
}

}  // namespace edv
