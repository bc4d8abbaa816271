// host_check.cpp -- TEST INFRASTRUCTURE: the kernel arithmetic (verify_core.h
// and friends) compiled for the host CPU with EDV_BOUND_CHECK limb-bound
// assertions, so tests/ can check the exact device code paths against the
// oracle without a GPU.  The product (libplenum_edverify.so) never links this.
#include <string.h>

#include <vector>

#include "batch_encode.h"
#include "bn254.h"
#include "comb.h"
#include "sha256.h"
#include "verify_core.h"

using namespace edv;

namespace {
struct HostTableA {
  ge_cached e[9];  // slot 8: the identity
  void store(int j, const ge_cached& c) { e[j] = c; }
  void load(int j, ge_cached& c) const { c = e[j >= 0 ? j : 8]; }
};
template <int K>
struct HostTableSplit {
  HostTableA t[K];
  void store(int s, int j, const ge_cached& c) const { const_cast<HostTableA&>(t[s]).store(j, c); }
  void load(int s, int j, ge_cached& c) const { t[s].load(j, c); }
};
// A comb table in host memory (comb.h layout).
template <int W>
struct HostComb {
  const uint32_t* tab;
  void load(int row, int j, ge_niels& n) const {
    const uint32_t* p = j >= 0 ? tab + ((size_t)row * Window<W>::kEntries + j) * kEntryWords : kNielsIdentityHost;
    memcpy(n.ypx.v, p, 40);
    memcpy(n.ymx.v, p + 10, 40);
    memcpy(n.xy2d.v, p + 20, 40);
  }
  uint32_t touch(int, int) const { return 0; }
};

std::vector<uint32_t> g_btab;  // W = 8 comb of B, built by the device code on first use

template <int W>
void build_table(std::vector<uint32_t>& tab, const ge_p3& P) {
  constexpr int rows = Window<W>::kRows, E = Window<W>::kEntries;
  std::vector<uint32_t> rw(rows * 40), pre(32 * 10);
  tab.assign((size_t)rows * E * kEntryWords, 0);
  comb_rows<W>(rw.data(), P);
  // strided lanes of up to 32 entries, as edv_comb_fill_kernel fills them
  const int CH = E < 32 ? E : 32, NCH = E / CH;
  for (int r = 0; r < rows; ++r)
    for (int c = 0; c < NCH; ++c)
      comb_fill_strided(&tab[(size_t)r * E * kEntryWords], pre.data(), 10, &rw[r * 40], c, NCH, CH);
}

const uint32_t* base_comb() {
  if (g_btab.empty()) {
    uint32_t b[8];
    for (int k = 0; k < 8; ++k) b[k] = 0x66666666u;
    b[0] = 0x66666658u;
    ge_p3 B;
    ge_frombytes(B, b, false);
    build_table<kBaseW>(g_btab, B);
  }
  return g_btab.data();
}
}  // namespace

extern "C" {

int edv_host_verify(const uint8_t* sig64, const uint8_t* pk32, const uint8_t* msg, uint64_t mlen) {
  uint32_t sig[16], pk[8];
  memcpy(sig, sig64, 64);
  memcpy(pk, pk32, 32);
  HostTableA ta;
  const HostComb<kBaseW> cb{base_comb()};
  return verify_one(sig, pk, msg, mlen, ta, cb) ? 0 : -1;
}

// The general path's split-table ladder (K tables of 2^(256t/K)(-A)), as
// edv_table_kernel / edv_dsm_kernel run it for keys shared by >= 4 requests.
int edv_host_verify_split(const uint8_t* sig64, const uint8_t* pk32, const uint8_t* msg, uint64_t mlen, int k) {
  uint32_t sig[16], pk[8], h[8];
  memcpy(sig, sig64, 64);
  memcpy(pk, pk32, 32);
  const HostComb<kBaseW> cb{base_comb()};
  bool ok = verify_phase_hash(h, sig, pk, msg, mlen);
  ge_p3 Q;
  if (k == 8) {
    HostTableSplit<8> tas;
    ok = verify_phase_table_split<8>(pk, tas) && ok;
    verify_phase_dsm_split_point<8>(Q, h, sig + 8, tas, cb);
  } else if (k == 4) {
    HostTableSplit<4> tas;
    ok = verify_phase_table_split<4>(pk, tas) && ok;
    verify_phase_dsm_split_point<4>(Q, h, sig + 8, tas, cb);
  } else if (k == 2) {
    HostTableSplit<2> tas;
    ok = verify_phase_table_split<2>(pk, tas) && ok;
    verify_phase_dsm_split_point<2>(Q, h, sig + 8, tas, cb);
  } else {
    HostTableSplit<1> tas;
    ok = verify_phase_table_split<1>(pk, tas) && ok;
    verify_phase_dsm_split_point<1>(Q, h, sig + 8, tas, cb);
  }
  return encode_equals(Q, sig) && ok ? 0 : -1;
}

void edv_host_sha512_prefixed(uint8_t out[64], const uint8_t prefix64[64], const uint8_t* msg, uint64_t mlen) {
  uint32_t pre[16], dig[16];
  memcpy(pre, prefix64, 64);
  sha512_prefixed<16>(dig, pre, msg, mlen);
  memcpy(out, dig, 64);
}

// The packed unit layout: M packed into units at `stride` (a lane of a
// lane-interleaved group), then hashed from them; also hands the units back.
void edv_host_sha512_units(uint8_t out[64], const uint8_t prefix64[64], const uint8_t* msg, uint64_t mlen,
                           uint64_t stride, uint8_t* units_out) {
  uint32_t pre[16], dig[16];
  memcpy(pre, prefix64, 64);
  const uint64_t nu = sha512_units64(mlen);
  std::vector<Chunk16> u(nu * stride, Chunk16{0xdeadbeefu, 0xdeadbeefu, 0xdeadbeefu, 0xdeadbeefu});
  pack_lane_units(u.data(), stride, msg, mlen);
  sha512_prefixed_units(dig, pre, u.data(), stride, mlen);
  memcpy(out, dig, 64);
  if (units_out)
    for (uint64_t p = 0; p < nu; ++p) memcpy(units_out + 16 * p, &u[p * stride], 16);
}
uint64_t edv_host_sha512_units_count(uint64_t mlen) { return sha512_units64(mlen); }

void edv_host_sha256(uint8_t out[32], const uint8_t* msg, uint64_t mlen) {
  uint32_t d[8];
  sha256_msg(d, msg, mlen);
  memcpy(out, d, 32);
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
// mode: bit 0 square; bits 1-2 the product order (0: the default, else fe_mul_o / fe_sq_o<order>)
static void fe_mul_mode(fe& fo, const fe& fa, const fe& fb, int mode) {
  const bool sq = mode & 1;
  switch (mode >> 1) {
    case 1:
      sq ? fe_sq_o<1>(fo, fa) : fe_mul_o<1>(fo, fa, fb);
      break;
    case 2:
      sq ? fe_sq_o<2>(fo, fa) : fe_mul_o<2>(fo, fa, fb);
      break;
    case 3:
      sq ? fe_sq_o<3>(fo, fa) : fe_mul_o<3>(fo, fa, fb);
      break;
    default:
      sq ? fe_sq(fo, fa) : fe_mul(fo, fa, fb);
  }
  EDV_ASSERT(EDV_IS_C(fo));
}
void edv_host_fe_mul(uint8_t out[32], const uint8_t a[32], const uint8_t b[32], int mode) {
  uint32_t wa[8], wb[8], wo[8];
  memcpy(wa, a, 32);
  memcpy(wb, b, 32);
  fe fa, fb, fo;
  fe_frombytes(fa, wa);
  fe_frombytes(fb, wb);
  fe_mul_mode(fo, fa, fb, mode);
  fe_tobytes(wo, fo);
  memcpy(out, wo, 32);
}
// The same on raw limbs (a in W, b in L; a in L when squaring): out = the product's limbs (class C).
void edv_host_fe_mul_limbs(uint32_t out[10], const uint32_t a[10], const uint32_t b[10], int mode) {
  fe fa, fb, fo;
  memcpy(fa.v, a, 40);
  memcpy(fb.v, b, 40);
  fe_mul_mode(fo, fa, fb, mode);
  memcpy(out, fo.v, 40);
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

}  // extern "C"

// The key-table (comb) path on the CPU: build the W-window table of -A and
// the W = 8 table of B with the device code, then [h](-A) + [S]B by the comb
// (comb_mul_add, the kernel's code).  Result point and the combined prechecks.
template <int W>
static bool comb_point(ge_p3& Q, const uint32_t sig[16], const uint32_t pk[8], const uint8_t* msg, uint64_t mlen) {
  uint32_t h[8];
  bool ok = verify_phase_hash(h, sig, pk, msg, mlen);
  ge_p3 A;
  ok = ge_frombytes(A, pk, true) && is_canonical_point(pk) && !has_small_order(pk) && ok;
  std::vector<uint32_t> atab;
  build_table<W>(atab, A);
  comb_mul_set<W>(Q, h, HostComb<W>{atab.data()});
  comb_mul_add<kBaseW>(Q, sig + 8, HostComb<kBaseW>{base_comb()});
  return ok;
}

static bool comb_point_w(int w, ge_p3& Q, const uint32_t sig[16], const uint32_t pk[8], const uint8_t* msg,
                         uint64_t mlen) {
  switch (w) {
    case 4: return comb_point<4>(Q, sig, pk, msg, mlen);
    case 5: return comb_point<5>(Q, sig, pk, msg, mlen);
    case 6: return comb_point<6>(Q, sig, pk, msg, mlen);
    case 7: return comb_point<7>(Q, sig, pk, msg, mlen);
    case 9: return comb_point<9>(Q, sig, pk, msg, mlen);
    case 10: return comb_point<10>(Q, sig, pk, msg, mlen);
    case 11: return comb_point<11>(Q, sig, pk, msg, mlen);
    case 12: return comb_point<12>(Q, sig, pk, msg, mlen);
    default: return comb_point<8>(Q, sig, pk, msg, mlen);
  }
}

extern "C" {

int edv_host_verify_comb_w(const uint8_t* sig64, const uint8_t* pk32, const uint8_t* msg, uint64_t mlen, int w) {
  uint32_t sig[16], pk[8];
  memcpy(sig, sig64, 64);
  memcpy(pk, pk32, 32);
  ge_p3 Q;
  const bool ok = comb_point_w(w, Q, sig, pk, msg, mlen);
  return (ok && encode_equals(Q, sig)) ? 0 : -1;
}

int edv_host_verify_comb(const uint8_t* sig64, const uint8_t* pk32, const uint8_t* msg, uint64_t mlen) {
  return edv_host_verify_comb_w(sig64, pk32, msg, mlen, 4);
}

}  // extern "C"

template <int W>
static int digits_w(const uint32_t x[8], int* out) {
  uint32_t y[9];
  comb_recode<W>(y, x);
  for (int r = 0; r < Window<W>::kRows; ++r) out[r] = comb_digit<W>(y, r);
  return Window<W>::kRows;
}

extern "C" {

// comb.h signed radix-2^W digits of a 32-byte scalar; returns the row count.
int edv_host_comb_digits(const uint8_t x32[32], int w, int* out) {
  uint32_t x[8];
  memcpy(x, x32, 32);
  switch (w) {
    case 4: return digits_w<4>(x, out);
    case 5: return digits_w<5>(x, out);
    case 6: return digits_w<6>(x, out);
    case 7: return digits_w<7>(x, out);
    case 8: return digits_w<8>(x, out);
    case 9: return digits_w<9>(x, out);
    case 10: return digits_w<10>(x, out);
    case 11: return digits_w<11>(x, out);
    case 12: return digits_w<12>(x, out);
    case 13: return digits_w<13>(x, out);
    case 14: return digits_w<14>(x, out);
    default: return -1;
  }
}

}  // extern "C"

// The batched encode (batch_encode.h) over groups of M = 16 consecutive items,
// as edv_encode_kernel runs it per lane.  zero_z[i] != 0 forces item i's Z to
// 0 (exercises the poisoned-group guard).  Bits: 1 = accept.
namespace {
struct HostEncode {
  const std::vector<ge_p3>* Q;
  std::vector<fe>* pre;
  const uint32_t* R;       // 16 words per item (sig)
  const uint8_t* ok;
  uint8_t* bits;
  uint64_t base, n;
  bool valid(int j) const { return base + j < n; }
  void z(int j, fe& f) const { f = (*Q)[base + j].Z; }
  void xy(int j, fe& X, fe& Y) const {
    X = (*Q)[base + j].X;
    Y = (*Q)[base + j].Y;
  }
  void put_pre(int j, const fe& f) const {
    if (valid(j)) (*pre)[base + j] = f;
  }
  void get_pre(int j, fe& f) const {
    if (valid(j)) f = (*pre)[base + j]; else fe_1(f);
  }
  void emit(int j, const uint32_t enc[8], bool zero_z) const {
    if (!valid(j)) return;
    const uint64_t i = base + j;
    const bool acc = !zero_z && ok[i] && memcmp(enc, R + 16 * i, 32) == 0;
    if (acc) bits[i / 8] |= (uint8_t)(1u << (i % 8));
  }
};
}  // namespace

extern "C" {

int edv_host_verify_batch_comb(const uint8_t* sig64, const uint8_t* pk32, const uint8_t* msgs, const uint64_t* off,
                               uint64_t n, int w, const uint8_t* zero_z, uint8_t* bits) {
  std::vector<ge_p3> Q(n);
  std::vector<fe> pre(n);
  std::vector<uint32_t> sig(16 * n);
  std::vector<uint8_t> ok(n);
  memcpy(sig.data(), sig64, 64 * n);
  for (uint64_t i = 0; i < n; ++i) {
    uint32_t pk[8];
    memcpy(pk, pk32 + 32 * i, 32);
    ok[i] = comb_point_w(w, Q[i], &sig[16 * i], pk, msgs + off[i], off[i + 1] - off[i]);
    if (zero_z && zero_z[i]) fe_0(Q[i].Z);
  }
  memset(bits, 0, (n + 7) / 8);
  for (uint64_t g = 0; g < n; g += 16) {
    HostEncode a{&Q, &pre, sig.data(), ok.data(), bits, g, n};
    encode_batch<16>(a);
  }
  return 0;
}

}  // extern "C"

// ---- BLS (bn254.h) on the CPU, for tests/test_bls.py against the oracle.
extern "C" {

// H(m) as 128 G1 bytes
void edv_host_bls_hash(const uint8_t* msg, uint64_t mlen, uint8_t out128[128]) {
  edv::bn::g1 h;
  edv::bn::g1_hash(h, msg, mlen);
  edv::bn::g1_to_bytes(out128, h);
}
// [sk]H(m) (sk 32 big-endian bytes, < r)
void edv_host_bls_sign(const uint8_t sk32[32], const uint8_t* msg, uint64_t mlen, uint8_t out128[128]) {
  uint32_t k[8];
  edv::bn::words_from_be(k, sk32);
  edv::bn::g1 h, s;
  edv::bn::g1_hash(h, msg, mlen);
  edv::bn::g1_mul(s, h, k);
  edv::bn::g1_to_bytes(out128, s);
}
void edv_host_bls_keygen(const uint8_t sk32[32], const uint8_t gen128[128], uint8_t out128[128]) {
  uint32_t k[8];
  edv::bn::words_from_be(k, sk32);
  edv::bn::g2 g, v;
  edv::bn::g2_from_bytes(g, gen128);
  edv::bn::g2_mul(v, g, k);
  edv::bn::g2_to_bytes(out128, v);
}
// the reduced pairing e(P, Q) as 12 Fp values (tower order c0.c0.a, c0.c0.b,
// c0.c1.a, ..., c1.c2.b), 32 big-endian bytes each
int edv_host_bls_pairing(const uint8_t p128[128], const uint8_t q128[128], uint8_t out[384]) {
  using namespace edv::bn;
  g1 P;
  g2 Q;
  g1_from_bytes(P, p128);
  g2_from_bytes(Q, q128);
  if (g1_isinf(P) || g2_isinf(Q)) return -1;
  fp x, y;
  fp2 qx, qy;
  g1_affine(x, y, P);
  g2_affine(qx, qy, Q);
  fp12 f, e;
  fp12_one(f);
  miller_loop_acc(f, x, y, qx, qy);
  final_exp(e, f);
  const fp* c[12] = {&e.c0.c0.a, &e.c0.c0.b, &e.c0.c1.a, &e.c0.c1.b, &e.c0.c2.a, &e.c0.c2.b,
                     &e.c1.c0.a, &e.c1.c0.b, &e.c1.c1.a, &e.c1.c1.b, &e.c1.c2.a, &e.c1.c2.b};
  for (int k = 0; k < 12; ++k) {
    uint32_t w[8];
    fp_to_plain(w, *c[k]);
    words_to_be(out + 32 * k, w);
  }
  return 0;
}
// Bls.verify over wire bytes: 1 accept, 0 reject
int edv_host_bls_verify(const uint8_t sig128[128], const uint8_t* msg, uint64_t mlen, const uint8_t vk128[128],
                        const uint8_t gen128[128]) {
  using namespace edv::bn;
  g1 s, h;
  g2 v, g;
  g1_from_bytes(s, sig128);
  g1_hash(h, msg, mlen);
  g2_from_bytes(v, vk128);
  g2_from_bytes(g, gen128);
  return bls_check(s, h, v, g) ? 1 : 0;
}

}  // extern "C"

// ---- the wave form's program (bls_wave.h) run step by step on the CPU, for tests/test_bls_program.py.
#include "bls_wave.h"
extern "C" {
// Bls.verify over wire bytes through bls_program.h: 1 accept, 0 reject, 2 degenerate (the
// kernel would redo the check on the four-lane form), -1 an input at infinity (rejected by
// the prologue).  vk_n verkeys are summed (verify_multi_sig).
int edv_host_bls_verify_program(const uint8_t sig128[128], const uint8_t* msg, uint64_t mlen, const uint8_t* vk128,
                                uint64_t vk_n, const uint8_t gen128[128]) {
  using namespace edv::bn;
  thread_local fp S[edv::blsp::kSlots];  // per thread: concurrent callers (test workers) never share slots
  for (int k = 0; k < edv::blsp::kConsts; ++k) fp_load(S[edv::blsp::kConstSlot[k]], edv::blsp::kConstVal + 8 * k);
  g1 s, h;
  g2 g, v;
  g1_from_bytes(s, sig128);
  g1_hash(h, msg, mlen);
  g2_from_bytes(g, gen128);
  g2_inf(v);
  for (uint64_t k = 0; k < vk_n; ++k) {
    g2 t;
    g2_from_bytes(t, vk128 + 128 * k);
    g2_add(v, v, t);
  }
  if (g1_isinf(s) || g2_isinf(g) || g2_isinf(v) || g1_isinf(h)) return -1;
  namespace P = edv::blsp;
  S[P::kIn_xP1] = s.X;
  S[P::kIn_yP1] = s.Y;
  S[P::kIn_xP2] = h.X;
  S[P::kIn_yP2] = h.Y;
  const fp* q[12] = {&g.X.a, &g.X.b, &g.Y.a, &g.Y.b, &g.Z.a, &g.Z.b, &v.X.a, &v.X.b, &v.Y.a, &v.Y.b, &v.Z.a, &v.Z.b};
  const int qs[12] = {P::kIn_Q1Xa, P::kIn_Q1Xb, P::kIn_Q1Ya, P::kIn_Q1Yb, P::kIn_Q1Za, P::kIn_Q1Zb,
                      P::kIn_Q2Xa, P::kIn_Q2Xb, P::kIn_Q2Ya, P::kIn_Q2Yb, P::kIn_Q2Za, P::kIn_Q2Zb};
  for (int k = 0; k < 12; ++k) S[qs[k]] = *q[k];
  uint32_t flag = 0;
  thread_local fp res[64];
  bool wr[64];
  uint32_t dst[64];
  for (int st = 0; st < P::kSteps; ++st) {
    const uint32_t o0 = P::kStep[st], o1 = P::kStep[st + 1];
    for (uint32_t o = o0; o < o1; ++o) {  // every lane reads ...
      const uint32_t* w = P::kOp + (size_t)P::kOpWords * o;
      wr[o - o0] = blsp_exec(w, S, res[o - o0], &flag);
      dst[o - o0] = blsp_field(w, 0);
    }
    for (uint32_t o = o0; o < o1; ++o)  // ... then every lane writes
      if (wr[o - o0]) S[dst[o - o0]] = res[o - o0];
  }
  if (flag) return 2;
  return blsp_result_is_one(S) ? 1 : 0;
}
}  // extern "C"
