// host_check.cpp -- TEST INFRASTRUCTURE: the kernel arithmetic (verify_core.h
// and friends) compiled for the host CPU with EDV_BOUND_CHECK limb-bound
// assertions, so tests/ can check the exact device code paths against the
// oracle without a GPU.  The product (libplenum_edverify.so) never links this.
#include <string.h>

#include <vector>

#include "comb.h"
#include "verify_core.h"

using namespace edv;

namespace {
struct HostTableA {
  ge_cached e[8];
  void store(int j, const ge_cached& c) { e[j] = c; }
  void load(int j, ge_cached& c) const { c = e[j]; }
};
struct HostTableB {
  void load(int j, ge_niels& n) const {
    const uint32_t* p = BASE_SMALL_U32 + 30 * j;
    memcpy(n.ypx.v, p, 40);
    memcpy(n.ymx.v, p + 10, 40);
    memcpy(n.xy2d.v, p + 20, 40);
  }
};
}  // namespace

extern "C" {

int edv_host_verify(const uint8_t* sig64, const uint8_t* pk32, const uint8_t* msg, uint64_t mlen) {
  uint32_t sig[16], pk[8];
  memcpy(sig, sig64, 64);
  memcpy(pk, pk32, 32);
  HostTableA ta;
  HostTableB tb;
  return verify_one(sig, pk, msg, mlen, ta, tb) ? 0 : -1;
}

void edv_host_sha512_prefixed(uint8_t out[64], const uint8_t prefix64[64], const uint8_t* msg, uint64_t mlen) {
  uint32_t pre[16], dig[16];
  memcpy(pre, prefix64, 64);
  sha512_prefixed<16>(dig, pre, msg, mlen);
  memcpy(out, dig, 64);
}

void edv_host_sc_reduce(uint8_t out[32], const uint8_t in[64]) {
  uint32_t i[16], o[8];
  memcpy(i, in, 64);
  sc_reduce(o, i);
  memcpy(out, o, 32);
}

int edv_host_sc_is_canonical(const uint8_t s[32]) {
  uint32_t w[8];
  memcpy(w, s, 32);
  return sc_is_canonical(w);
}

// out = canonical bytes of (a * b) for field elements given as 32-byte LE
// integers < 2^255 (exercises fe_frombytes, fe_mul, fe_sq, fe_tobytes).
void edv_host_fe_mul(uint8_t out[32], const uint8_t a[32], const uint8_t b[32], int square) {
  uint32_t wa[8], wb[8], wo[8];
  memcpy(wa, a, 32);
  memcpy(wb, b, 32);
  fe fa, fb, fo;
  fe_frombytes(fa, wa);
  fe_frombytes(fb, wb);
  if (square)
    fe_sq(fo, fa);
  else
    fe_mul(fo, fa, fb);
  fe_tobytes(wo, fo);
  memcpy(out, wo, 32);
}

void edv_host_fe_invert(uint8_t out[32], const uint8_t a[32]) {
  uint32_t wa[8], wo[8];
  memcpy(wa, a, 32);
  fe fa, fo;
  fe_frombytes(fa, wa);
  fe_invert(fo, fa);
  fe_tobytes(wo, fo);
  memcpy(out, wo, 32);
}

// Decode (negate = 0) and re-encode a point; -1 if not on the curve.
int edv_host_point_roundtrip(uint8_t out[32], const uint8_t in[32]) {
  uint32_t w[8], o[8];
  memcpy(w, in, 32);
  ge_p3 P;
  if (!ge_frombytes(P, w, false)) return -1;
  ge_p2 p2;
  ge_p3_to_p2(p2, P);
  ge_tobytes(o, p2);
  memcpy(out, o, 32);
  return 0;
}

int edv_host_has_small_order(const uint8_t s[32]) {
  uint32_t w[8];
  memcpy(w, s, 32);
  return has_small_order(w);
}

int edv_host_is_canonical_point(const uint8_t s[32]) {
  uint32_t w[8];
  memcpy(w, s, 32);
  return is_canonical_point(w);
}

// The key-table (comb) path on the CPU: build the W = 4 table of -A and the
// W = 8 table of B with the device code, then [h](-A) + [S]B by the comb.
static std::vector<uint32_t> g_btab;

static void build_table(std::vector<uint32_t>& tab, const ge_p3& P, int W) {
  const int rows = W == 4 ? Window<4>::kRows : Window<8>::kRows;
  const int E = W == 4 ? Window<4>::kEntries : Window<8>::kEntries;
  std::vector<uint32_t> rw(rows * 40), pre(E * 10);
  tab.assign((size_t)rows * E * kEntryWords, 0);
  if (W == 4) comb_rows<4>(rw.data(), P); else comb_rows<8>(rw.data(), P);
  for (int r = 0; r < rows; ++r) {
    if (W == 4) comb_fill_row<4>(&tab[(size_t)r * E * kEntryWords], pre.data(), &rw[r * 40]);
    else comb_fill_row<8>(&tab[(size_t)r * E * kEntryWords], pre.data(), &rw[r * 40]);
  }
}

static void comb_add(ge_p3& Q, int e, const uint32_t* row) {
  const int m = e < 0 ? -e : e;
  ge_niels nb;
  ge_niels_0(nb);
  if (m) {
    const uint32_t* p = row + (m - 1) * kEntryWords;
    load_fe(nb.ypx, p);
    load_fe(nb.ymx, p + 10);
    load_fe(nb.xy2d, p + 20);
  }
  if (e < 0) {
    fe t = nb.ypx;
    nb.ypx = nb.ymx;
    nb.ymx = t;
    fe_neg(nb.xy2d, nb.xy2d);
  }
  ge_p1p1 t;
  ge_madd(t, Q, nb);
  ge_p1p1_to_p3_addlike(Q, t);
}

int edv_host_verify_comb(const uint8_t* sig64, const uint8_t* pk32, const uint8_t* msg, uint64_t mlen) {
  uint32_t sig[16], pk[8], h[8], hy[8], sy[8];
  memcpy(sig, sig64, 64);
  memcpy(pk, pk32, 32);
  if (g_btab.empty()) {
    uint32_t b[8];
    for (int k = 0; k < 8; ++k) b[k] = 0x66666666u;
    b[0] = 0x66666658u;
    ge_p3 B;
    ge_frombytes(B, b, false);
    build_table(g_btab, B, 8);
  }
  bool ok = verify_phase_hash(h, sig, pk, msg, mlen);
  ge_p3 A;
  ok = ge_frombytes(A, pk, true) && is_canonical_point(pk) && !has_small_order(pk) && ok;
  std::vector<uint32_t> atab;
  build_table(atab, A, 4);
  comb_recode<4>(hy, h);
  comb_recode<8>(sy, sig + 8);
  ge_p3 Q;
  ge_p3_0(Q);
  for (int r = 0; r < Window<4>::kRows; ++r) comb_add(Q, comb_digit<4>(hy, r), &atab[(size_t)r * 8 * kEntryWords]);
  for (int r = 0; r < Window<8>::kRows; ++r) comb_add(Q, comb_digit<8>(sy, r), &g_btab[(size_t)r * 128 * kEntryWords]);
  ge_p2 r2;
  ge_p3_to_p2(r2, Q);
  uint32_t rc[8];
  ge_tobytes(rc, r2);
  return (ok && memcmp(rc, sig, 32) == 0) ? 0 : -1;
}

}  // extern "C"
