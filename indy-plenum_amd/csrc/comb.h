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
//   A = a registered public key (client_authn.py SimpleAuthNr.addIdr keys):
//       W = 4, 64 rows x 8 entries x 128 B = 64 KiB per key, in HBM.
//   B = the base point: W = 8, 32 rows x 128 entries x 128 B = 512 KiB, one
//       copy per context (L2-resident: 4 MiB per XCD).
// Entries are 32 u32 words (30 limbs + 2 pad) so one entry is 8 dwordx4 loads.
#pragma once
#include "verify_core.h"

namespace edv {

constexpr int kEntryWords = 32;

template <int W>
struct Window {
  static constexpr int kRows = (253 + W - 1) / W;
  static constexpr int kEntries = 1 << (W - 1);
  static constexpr int kTableWords = kRows * kEntries * kEntryWords;
  // sum_i 2^(W-1) * 2^(W*i) restricted to one 32-bit word (W divides 32)
  static constexpr uint32_t kBiasWord = W == 4 ? 0x88888888u : W == 8 ? 0x80808080u : 0u;
  static_assert(W == 4 || W == 8, "window widths that divide 32");
};

// y = x + bias: digit_i = ((y >> W*i) & (2^W - 1)) - 2^(W-1) in [-2^(W-1), 2^(W-1) - 1]
// and x = sum digit_i 2^(W*i); requires x + bias < 2^256 (x < 2^253 suffices).
template <int W>
EDV_HD void comb_recode(uint32_t y[8], const uint32_t x[8]) {
  uint64_t carry = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const uint64_t t = (uint64_t)x[k] + Window<W>::kBiasWord + carry;
    y[k] = (uint32_t)t;
    carry = t >> 32;
  }
}

template <int W>
EDV_HD int comb_digit(const uint32_t y[8], int i) {
  constexpr int per_word = 32 / W;
  const int w = i / per_word;
  uint32_t v = y[0];
#pragma unroll
  for (int k = 1; k < 8; ++k) v = (w == k) ? y[k] : v;
  return (int)((v >> (W * (i % per_word))) & ((1u << W) - 1)) - (1 << (W - 1));
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

// The kEntries multiples of one row base, one shared inversion (Montgomery's
// trick, prefix products in `pre`, kEntries * 10 words), affine niels out.
template <int W>
EDV_HD void comb_fill_row(uint32_t* entries, uint32_t* pre, const uint32_t* base_words) {
  constexpr int E = Window<W>::kEntries;
  ge_p3 base, m;
  load_fe(base.X, base_words);
  load_fe(base.Y, base_words + 10);
  load_fe(base.Z, base_words + 20);
  load_fe(base.T, base_words + 30);
  ge_cached cb;
  ge_p3_to_cached(cb, base);
  m = base;
  fe acc;
#pragma unroll 1
  for (int j = 0; j < E; ++j) {
    if (j > 0) {
      ge_p1p1 t;
      ge_add(t, m, cb);
      ge_p1p1_to_p3_addlike(m, t);
    }
    store_fe(entries + j * kEntryWords, m.X);
    store_fe(entries + j * kEntryWords + 10, m.Y);
    store_fe(entries + j * kEntryWords + 20, m.Z);
    if (j == 0)
      acc = m.Z;
    else
      fe_mul(acc, acc, m.Z);
    store_fe(pre + j * 10, acc);
  }
  fe inv;
  fe_invert(inv, acc);
#pragma unroll 1
  for (int j = E - 1; j >= 0; --j) {
    fe zinv, X, Y, Z, x, y, t;
    load_fe(X, entries + j * kEntryWords);
    load_fe(Y, entries + j * kEntryWords + 10);
    load_fe(Z, entries + j * kEntryWords + 20);
    if (j > 0) {
      fe p;
      load_fe(p, pre + (j - 1) * 10);
      fe_mul(zinv, inv, p);
      fe_mul(inv, inv, Z);
    } else {
      zinv = inv;
    }
    fe_mul(x, X, zinv);
    fe_mul(y, Y, zinv);
    fe_add(t, y, x);
    store_fe_canon(entries + j * kEntryWords, t);
    fe_sub(t, y, x);
    store_fe_canon(entries + j * kEntryWords + 10, t);
    fe_mul(t, x, y);
    fe_mul(t, t, fe_const_d2());
    store_fe_canon(entries + j * kEntryWords + 20, t);
    entries[j * kEntryWords + 30] = 0;
    entries[j * kEntryWords + 31] = 0;
  }
}

}  // namespace edv
