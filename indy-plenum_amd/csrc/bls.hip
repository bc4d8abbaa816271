// bls.hip -- the BLS multi-signature check of Plenum's COMMIT / state-proof
// path on MI355X, one lane per check, behind include/edverify.h.
//
// Replaces indy-crypto 0.1.6 under crypto/bls/indy_crypto/
// bls_crypto_indy_crypto.py:59-90 (Bls.verify, Bls.verify_multi_sig,
// MultiSignature.new), called from plenum/bls/bls_bft_replica_plenum.py:157,
// :170, :205 and plenum/client/client.py:541.  Arithmetic: bn254.h.
//   edv_bls_verify_kernel   decode sig (G1) and verkeys (G2), sum the verkeys
//                           of a multi-signature, H(m), then
//                           FE(ML(sig, g) * ML(-H, vk)) == 1; wave ballot
//   edv_bls_aggregate_kernel  create_multi_sig: the sum of G1 points
//   edv_bls_sign_kernel / edv_bls_keygen_kernel  [sk]H(m), [sk]g (test data)
#include <hip/hip_runtime.h>
#include <string.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../../include/edverify.h"
#include "bls_wave.h"
#include "bn254.h"
#include "edv_internal.h"

using namespace edv::bn;
namespace blsp = edv::blsp;
using edv::sha256_msg;
using edv_internal::set_err;

#define BLS_TRY(expr)                                                                              \
  do {                                                                                             \
    hipError_t e_ = (expr);                                                                        \
    if (e_ != hipSuccess) return set_err(EDV_EHIP, "%s: %s", #expr, hipGetErrorString(e_));        \
  } while (0)

namespace {

constexpr int kBlsBlock = 64;

__global__ __launch_bounds__(kBlsBlock) void edv_bls_verify_kernel(const uint8_t* __restrict__ sig128,
                                                                  const uint8_t* __restrict__ msgs,
                                                                  const uint64_t* __restrict__ moff,
                                                                  const uint8_t* __restrict__ vk128,
                                                                  const uint64_t* __restrict__ vk_off,
                                                                  const uint8_t* __restrict__ gen128, uint64_t n,
                                                                  unsigned long long* __restrict__ words) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  bool ok = false;
  if (i < n) {
    g1 s, h;
    g2 v, g;
    g1_from_bytes(s, sig128 + 128 * i);
    g1_hash(h, msgs + moff[i], moff[i + 1] - moff[i]);
    const uint64_t k0 = vk_off ? vk_off[i] : i, k1 = vk_off ? vk_off[i + 1] : i + 1;
    g2_inf(v);
    for (uint64_t k = k0; k < k1; ++k) {  // Bls.verify_multi_sig: the verkeys' sum
      g2 t;
      g2_from_bytes(t, vk128 + 128 * k);
      g2_add(v, v, t);
    }
    g2_from_bytes(g, gen128);
    ok = bls_check(s, h, v, g);
  }
  const unsigned long long b = __ballot(ok);  // every lane of the wave takes part
  if ((threadIdx.x & 63) == 0 && i < n) words[i >> 6] = b;
}

// The latency form (batches of at most bls_pair_max checks, e.g. a COMMIT round's ~25): two
// lanes per check, side by side in a wave.  Even lane: the signature and the generator; odd
// lane: H(m) and the verkey sum.  Each runs ONE Miller loop -- the same code on both lanes, so
// the wave runs them together -- then the two Fp12 values are swapped across the pair and both
// lanes form the product and its final exponentiation (the same value on both: no divergence);
// the even lane's verdict is the check's.  Half the serial Miller work of the one-lane form.
// words32[j]: the verdicts of checks 32j..32j+31 (the byte layout of the one-lane form's uint64
// words).
__device__ __forceinline__ void shfl_xor_fp12(fp12& o, const fp12& x) {
  const uint32_t* a = (const uint32_t*)&x;
  uint32_t* b = (uint32_t*)&o;
#pragma unroll
  for (int k = 0; k < (int)(sizeof(fp12) / 4); ++k) b[k] = (uint32_t)__shfl_xor((int)a[k], 1, 64);
}
__global__ __launch_bounds__(kBlsBlock) void edv_bls_verify_pair_kernel(const uint8_t* __restrict__ sig128,
                                                                       const uint8_t* __restrict__ msgs,
                                                                       const uint64_t* __restrict__ moff,
                                                                       const uint8_t* __restrict__ vk128,
                                                                       const uint64_t* __restrict__ vk_off,
                                                                       const uint8_t* __restrict__ gen128, uint64_t n,
                                                                       uint32_t* __restrict__ words32) {
  const uint64_t lane_g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t i = lane_g >> 1;
  const bool odd = lane_g & 1;
  bool live = i < n;  // lanes past the end still take part in the shuffles and the ballot
  const uint64_t ii = live ? i : 0;
  fp x, y;
  fp2 qx, qy;
  bool inf_p = true, inf_q = true;
  if (!odd) {
    g1 s;
    g2 g;
    g1_from_bytes(s, sig128 + 128 * ii);
    g2_from_bytes(g, gen128);
    inf_p = g1_isinf(s);
    inf_q = g2_isinf(g);
    if (!inf_p) g1_affine(x, y, s);
    if (!inf_q) g2_affine(qx, qy, g);
  } else {
    g1 h;
    g2 v;
    g1_hash(h, msgs + moff[ii], moff[ii + 1] - moff[ii]);
    const uint64_t k0 = vk_off ? vk_off[ii] : ii, k1 = vk_off ? vk_off[ii + 1] : ii + 1;
    g2_inf(v);
    for (uint64_t k = k0; k < k1; ++k) {  // Bls.verify_multi_sig: the verkeys' sum
      g2 t;
      g2_from_bytes(t, vk128 + 128 * k);
      g2_add(v, v, t);
    }
    inf_p = g1_isinf(h);
    inf_q = g2_isinf(v);
    if (!inf_p) {
      g1_affine(x, y, h);
      fp_neg(y, y);
    }
    if (!inf_q) g2_affine(qx, qy, v);
  }
  fp12 f;
  fp12_one(f);
  if (live && !inf_p && !inf_q) miller_loop_acc(f, x, y, qx, qy);
  // bls_check's rejections: signature, verkey sum or generator at infinity
  const bool bad_here = odd ? inf_q : (inf_p || inf_q);
  const bool bad = bad_here || __shfl_xor((int)bad_here, 1, 64);
  fp12 other, e;
  shfl_xor_fp12(other, f);
  fp12_mul(f, f, other);
  final_exp(e, f);
  const bool ok = live && !bad && fp12_isone(e) && !odd;
  unsigned long long b = __ballot(ok);  // even lanes' verdicts
  b &= 0x5555555555555555ull;
  b = (b | (b >> 1)) & 0x3333333333333333ull;
  b = (b | (b >> 2)) & 0x0f0f0f0f0f0f0f0full;
  b = (b | (b >> 4)) & 0x00ff00ff00ff00ffull;
  b = (b | (b >> 8)) & 0x0000ffff0000ffffull;
  b = (b | (b >> 16)) & 0x00000000ffffffffull;
  if ((threadIdx.x & 63) == 0 && (lane_g >> 1) < n) words32[lane_g >> 6] = (uint32_t)b;
}

// The four-lane form (batches of at most half of bls_pair_max checks): lanes 0 / 2 of a check's
// quad run the (signature, generator) Miller loop and lanes 1 / 3 the (-H(m), verkeys) one,
// each over its two lanes (LineSplit), then all four hold the product and run the final
// exponentiation together with each cyclotomic squaring spread over lanes 0-2 (one Fp4
// squaring each, the 2 x 2 Fp2 results gathered by shuffles; lane 3 repeats lane 0's), the
// rest of it replicated.  words16[j]: the verdicts of checks 16j..16j+15.
struct CycloSqQuad {
  int q;     // lane within the quad
  int base;  // the quad's first lane in the wave
  __device__ void operator()(fp12& r, const fp12& x) const {
    const fp2& a = q == 1 ? x.c1.c0 : q == 2 ? x.c0.c1 : x.c0.c0;  // (1, w^3) / (w, w^4) / (w^2, w^5)
    const fp2& b = q == 1 ? x.c0.c2 : q == 2 ? x.c1.c2 : x.c1.c1;
    fp2 te[2];
    fp4_sqr(te[0], te[1], a, b);
    fp2 t[6];  // t0..t5 of fp12_cyclo_sqr: lane base + j holds t[2j], t[2j+1]
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const uint32_t* src = (const uint32_t*)te;
      uint32_t* dst = (uint32_t*)&t[2 * j];
#pragma unroll
      for (int k = 0; k < (int)(2 * sizeof(fp2) / 4); ++k) dst[k] = (uint32_t)__shfl((int)src[k], base + j, 64);
    }
    fp2 xt5;
    fp2_mul_xi(xt5, t[5]);
    fp12 o;
    fp2_3t_m2z(o.c0.c0, t[0], x.c0.c0);
    fp2_3t_p2z(o.c1.c1, t[1], x.c1.c1);
    fp2_3t_p2z(o.c1.c0, xt5, x.c1.c0);
    fp2_3t_m2z(o.c0.c2, t[4], x.c0.c2);
    fp2_3t_m2z(o.c0.c1, t[2], x.c0.c1);
    fp2_3t_p2z(o.c1.c2, t[3], x.c1.c2);
    r = o;
  }
};
// The Miller loop of one pairing over two lanes (h = 0 / 1, partners lane ^ 2): each Fp12
// squaring's two Fp6 products (a b; (a + b)(a + v b)) and each line multiply's two sparse Fp6
// products (b (l1, l2); (a + b)(l0 + l1, l2)) go one to each lane -- the same code on both,
// operands chosen by selects -- and are swapped by shuffles; the line evaluation and the twist
// point's doubling / addition stay on both lanes.
__device__ __forceinline__ void fp6_shfl_xor(fp6& o, const fp6& x, int m) {
  const uint32_t* a = (const uint32_t*)&x;
  uint32_t* b = (uint32_t*)&o;
#pragma unroll
  for (int k = 0; k < (int)(sizeof(fp6) / 4); ++k) b[k] = (uint32_t)__shfl_xor((int)a[k], m, 64);
}
__device__ __forceinline__ void fp6_sel(fp6& r, bool c, const fp6& x, const fp6& y) {  // c ? y : x
  const uint32_t* a = (const uint32_t*)&x;
  const uint32_t* b = (const uint32_t*)&y;
  uint32_t* o = (uint32_t*)&r;
#pragma unroll
  for (int k = 0; k < (int)(sizeof(fp6) / 4); ++k) o[k] = c ? b[k] : a[k];
}
struct LineSplit {
  int h;
  __device__ void sqr(fp12& g) const {
    fp6 s, u, t, X, Y, R, O, ab, sq;
    fp6_add(s, g.c0, g.c1);
    fp6_mul_v(t, g.c1);
    fp6_add(u, g.c0, t);
    fp6_sel(X, h, g.c0, s);  // lane 0: a * b; lane 1: (a + b)(a + v b)
    fp6_sel(Y, h, g.c1, u);
    fp6_mul(R, X, Y);
    fp6_shfl_xor(O, R, 2);
    fp6_sel(ab, h, R, O);
    fp6_sel(sq, h, O, R);
    fp6_sub(sq, sq, ab);  // a^2 + v b^2 + v ab
    fp6_mul_v(t, ab);
    fp6_sub(g.c0, sq, t);
    fp6_add(g.c1, ab, ab);
  }
  __device__ void mul_line(fp12& f, const fp2& l0, const fp2& l1, const fp2& l2) const {
    fp6 aA, s, X, R, O, bB, sm;
    fp2_mul(aA.c0, f.c0.c0, l0);  // a * (l0, 0, 0), both lanes
    fp2_mul(aA.c1, f.c0.c1, l0);
    fp2_mul(aA.c2, f.c0.c2, l0);
    fp6_add(s, f.c0, f.c1);
    fp6_sel(X, h, f.c1, s);  // lane 0: b * (l1, l2, 0); lane 1: (a + b)(l0 + l1, l2, 0)
    fp2 m0, b0;
    fp2_add(m0, l0, l1);
    const uint32_t* p0 = (const uint32_t*)&l1;
    const uint32_t* p1 = (const uint32_t*)&m0;
    uint32_t* pb = (uint32_t*)&b0;
#pragma unroll
    for (int k = 0; k < (int)(sizeof(fp2) / 4); ++k) pb[k] = h ? p1[k] : p0[k];
    fp6_mul_01(R, X, b0, l2);
    fp6_shfl_xor(O, R, 2);
    fp6_sel(bB, h, R, O);
    fp6_sel(sm, h, O, R);
    fp6_sub(sm, sm, aA);
    fp6_sub(f.c1, sm, bB);
    fp6_mul_v(bB, bB);
    fp6_add(f.c0, aA, bB);
  }
};

__device__ __forceinline__ void shfl_fp12(fp12& o, const fp12& x, int src_lane) {
  const uint32_t* a = (const uint32_t*)&x;
  uint32_t* b = (uint32_t*)&o;
#pragma unroll
  for (int k = 0; k < (int)(sizeof(fp12) / 4); ++k) b[k] = (uint32_t)__shfl((int)a[k], src_lane, 64);
}
__global__ __launch_bounds__(kBlsBlock) void edv_bls_verify_quad_kernel(const uint8_t* __restrict__ sig128,
                                                                       const uint8_t* __restrict__ msgs,
                                                                       const uint64_t* __restrict__ moff,
                                                                       const uint8_t* __restrict__ vk128,
                                                                       const uint64_t* __restrict__ vk_off,
                                                                       const uint8_t* __restrict__ gen128, uint64_t n,
                                                                       uint16_t* __restrict__ words16) {
  const uint64_t lane_g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t i = lane_g >> 2;
  const int q = (int)(lane_g & 3), base = (int)(threadIdx.x & 63) & ~3;
  const bool live = i < n;  // lanes past the end still take part in the shuffles and the ballot
  const uint64_t ii = live ? i : 0;
  fp x, y;
  fp2 qx, qy;
  bool inf_p = false, inf_q = false, run = false;
  // lanes 0 / 2: the (signature, generator) pairing's two halves; lanes 1 / 3: (-H(m), verkeys)
  if ((q & 1) == 0) {
    g1 s;
    g2 g;
    g1_from_bytes(s, sig128 + 128 * ii);
    g2_from_bytes(g, gen128);
    inf_p = g1_isinf(s);
    inf_q = g2_isinf(g);
    if (!inf_p) g1_affine(x, y, s);
    if (!inf_q) g2_affine(qx, qy, g);
    run = !inf_p && !inf_q;
  } else {
    g1 h;
    g2 v;
    g1_hash(h, msgs + moff[ii], moff[ii + 1] - moff[ii]);
    const uint64_t k0 = vk_off ? vk_off[ii] : ii, k1 = vk_off ? vk_off[ii + 1] : ii + 1;
    g2_inf(v);
    for (uint64_t k = k0; k < k1; ++k) {  // Bls.verify_multi_sig: the verkeys' sum
      g2 t;
      g2_from_bytes(t, vk128 + 128 * k);
      g2_add(v, v, t);
    }
    inf_p = g1_isinf(h);
    inf_q = g2_isinf(v);
    if (!inf_p) {
      g1_affine(x, y, h);
      fp_neg(y, y);
    }
    if (!inf_q) g2_affine(qx, qy, v);
    run = !inf_p && !inf_q;
  }
  fp12 f;
  fp12_one(f);
  if (live && run) miller_loop_acc(f, x, y, qx, qy, LineSplit{q >> 1});
  // bls_check's rejections: signature or generator (lane 0), verkey sum (lane 1) at infinity
  const bool bad_here = q == 0 ? (inf_p || inf_q) : q == 1 ? inf_q : false;
  const bool bad = __shfl((int)bad_here, base, 64) || __shfl((int)bad_here, base + 1, 64);
  fp12 f0, f1, e;
  shfl_fp12(f0, f, base);
  shfl_fp12(f1, f, base + 1);
  fp12_mul(f, f0, f1);
  final_exp(e, f, CycloSqQuad{q == 3 ? 0 : q, base});
  const bool ok = live && !bad && fp12_isone(e) && q == 0;
  unsigned long long b = __ballot(ok);  // lane 0 of each quad
  b &= 0x1111111111111111ull;
  b = (b | (b >> 3)) & 0x0303030303030303ull;
  b = (b | (b >> 6)) & 0x000f000f000f000full;
  b = (b | (b >> 12)) & 0x000000ff000000ffull;
  b = (b | (b >> 24)) & 0x000000000000ffffull;
  if ((threadIdx.x & 63) == 0 && (lane_g >> 2) < n) words16[lane_g >> 6] = (uint16_t)b;
}

// The wave form (batches of at most bls_wave_max checks -- a COMMIT round's ~25): one wave per
// check running bls_program.h, the whole pairing check as a straight-line program of Fp
// operations scheduled over the 64 lanes (tools/gen_bls_program.py).  Prologue (per-lane code,
// as the other forms): H(m) with the try-and-increment's first 61 candidates side by side on every
// lane but 16-18 (candidate c on lane c for c < 16, on lane c + 3 after; the first candidate that is
// a point wins, as in g1_hash's loop), the signature, generator and verkey-sum decodes on lanes
// 16-18.  Per step each lane reads its operation
// (prefetched two steps ahead) and its operand slots, and writes its result after a barrier
// (for a one-wave block the barrier is only the compiler's fence: LDS is in order per wave).
// verdict[i]: 1 accept, 0 reject, 2 redo on the four-lane kernel (a degenerate Miller step
// flagged by the program, or no point among the 61 candidates -- about 2^-61 of messages, so no
// message can be searched for that costs its round the four-lane kernel: bn254.h's branches decide).
constexpr int kHashTries = 16;  // candidates on lanes 0..15; lanes kHashTries..+2 decode; 45 more after
__device__ __forceinline__ bool hash_lane(int lane) { return lane < kHashTries || lane >= kHashTries + 3; }
__device__ __forceinline__ int hash_candidate(int lane) { return lane < kHashTries ? lane : lane - 3; }
__global__ __launch_bounds__(kBlsBlock) void edv_bls_verify_wave_kernel(const uint8_t* __restrict__ sig128,
                                                                       const uint8_t* __restrict__ msgs,
                                                                       const uint64_t* __restrict__ moff,
                                                                       const uint8_t* __restrict__ vk128,
                                                                       const uint64_t* __restrict__ vk_off,
                                                                       const uint8_t* __restrict__ gen128, uint64_t n,
                                                                       uint8_t* __restrict__ verdict,
                                                                       unsigned long long* __restrict__ clk,
                                                                       int tries) {
  __shared__ fp S[blsp::kSlots];
  // clk (EDV_BLS_WAVE_CLOCKS=1, block 0): shader clocks at the start, after the prologue, after
  // the program, and the program's clocks in steps with a product / without one
  const unsigned long long c_start = clock64();
  __shared__ uint32_t bad[4];  // [0] reject (a point at infinity), [1] redo
  const uint64_t i = blockIdx.x;
  const int lane = (int)threadIdx.x;
  if (i >= n) return;  // the whole block
  for (int k = lane; k < blsp::kConsts; k += kBlsBlock) fp_load(S[blsp::kConstSlot[k]], blsp::kConstVal + 8 * k);
  if (lane < 4) bad[lane] = 0;
  // H(m): candidate h + hash_candidate(lane) on the hash lanes
  bool hit = false;
  fp hx, hy;
  if (hash_lane(lane) && hash_candidate(lane) < tries) {
    uint32_t d[8];
    sha256_msg(d, msgs + moff[i], moff[i + 1] - moff[i]);
    uint8_t hb[32];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      hb[4 * k] = (uint8_t)d[k];
      hb[4 * k + 1] = (uint8_t)(d[k] >> 8);
      hb[4 * k + 2] = (uint8_t)(d[k] >> 16);
      hb[4 * k + 3] = (uint8_t)(d[k] >> 24);
    }
    uint32_t x[8];
    words_from_be(x, hb);
    uint64_t c = (uint64_t)hash_candidate(lane);  // h + c, wrapping at 2^256 like g1_hash's h += 1
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const uint64_t t = (uint64_t)x[k] + c;
      x[k] = (uint32_t)t;
      c = t >> 32;
    }
    while (fp_geq_p(x)) {  // mod p (h < 2^256 < 5p)
      fp t;
      fp_reduce_once(t, x);
#pragma unroll
      for (int k = 0; k < 8; ++k) x[k] = t.v[k];
    }
    fp rhs, bb;
    fp_from_plain(hx, x);
    fp_sqr(rhs, hx);
    fp_mul(rhs, rhs, hx);
    fp_load(bb, kB1);
    fp_add(rhs, rhs, bb);
    hit = fp_sqrt(hy, rhs);
  }
  const unsigned long long hits = __ballot(hit);
  __syncthreads();
  // the winner: the lowest candidate that is a point (lanes 0..15 hold candidates 0..15, lanes 19..
  // hold 16..)
  const unsigned long long lo = hits & ((1ull << kHashTries) - 1);
  const int win = lo ? __ffsll((long long)lo) - 1 : (hits ? __ffsll((long long)hits) - 1 : -1);
  if (hits == 0) {
    if (lane == 0) bad[1] = 1;
  } else if (lane == win) {
    S[blsp::kIn_xP2] = hx;
    S[blsp::kIn_yP2] = hy;
  }
  if (lane == kHashTries) {
    g1 s;
    g1_from_bytes(s, sig128 + 128 * i);  // affine (Z = 1) when finite
    if (g1_isinf(s)) {
      bad[0] = 1;
    } else {
      S[blsp::kIn_xP1] = s.X;
      S[blsp::kIn_yP1] = s.Y;
    }
  } else if (lane == kHashTries + 1 || lane == kHashTries + 2) {
    g2 q;
    if (lane == kHashTries + 1) {
      g2_from_bytes(q, gen128);
    } else {
      const uint64_t k0 = vk_off ? vk_off[i] : i, k1 = vk_off ? vk_off[i + 1] : i + 1;
      g2_inf(q);
      for (uint64_t k = k0; k < k1; ++k) {  // Bls.verify_multi_sig: the verkeys' sum
        g2 t;
        g2_from_bytes(t, vk128 + 128 * k);
        g2_add(q, q, t);
      }
    }
    if (g2_isinf(q)) {
      bad[0] = 1;
    } else if (lane == kHashTries + 1) {
      S[blsp::kIn_Q1Xa] = q.X.a;
      S[blsp::kIn_Q1Xb] = q.X.b;
      S[blsp::kIn_Q1Ya] = q.Y.a;
      S[blsp::kIn_Q1Yb] = q.Y.b;
      S[blsp::kIn_Q1Za] = q.Z.a;
      S[blsp::kIn_Q1Zb] = q.Z.b;
    } else {
      S[blsp::kIn_Q2Xa] = q.X.a;
      S[blsp::kIn_Q2Xb] = q.X.b;
      S[blsp::kIn_Q2Ya] = q.Y.a;
      S[blsp::kIn_Q2Yb] = q.Y.b;
      S[blsp::kIn_Q2Za] = q.Z.a;
      S[blsp::kIn_Q2Zb] = q.Z.b;
    }
  }
  __syncthreads();
  if (bad[0] || bad[1]) {  // bls_check's rejections; or no H among the candidates: redo
    if (lane == 0) verdict[i] = bad[0] ? 0 : 2;
    return;
  }
  struct OpW {
    uint32_t w[blsp::kOpWords];
  };
  static_assert(blsp::kOpWords % 4 == 0, "operations load as 16-byte vectors");
  auto load_op = [&](OpW& q, int sn) {
    const uint32_t o = (sn < blsp::kSteps ? blsp::kStep[sn] : 0u) + (uint32_t)lane;
    if (sn < blsp::kSteps && o < blsp::kStep[sn + 1]) {
      const uint4* src = (const uint4*)(blsp::kOp + (size_t)blsp::kOpWords * o);
#pragma unroll
      for (int v = 0; v < blsp::kOpWords / 4; ++v) {
        const uint4 t = src[v];
        q.w[4 * v] = t.x;
        q.w[4 * v + 1] = t.y;
        q.w[4 * v + 2] = t.z;
        q.w[4 * v + 3] = t.w;
      }
    } else {
      q.w[0] = blsp::kNop;
    }
  };
  // two named prefetch registers, ping-pong (an array indexed by the step would live in scratch
  // memory): step s runs while the operation of step s + 2 loads
  OpW qa, qb;
  uint32_t flag = 0;
  const bool timing = clk != nullptr && blockIdx.x == 0;
  const unsigned long long c_prologue = clock64();
  unsigned long long c_prev = c_prologue, c_heavy = 0, c_light = 0;
  auto run_step = [&](OpW& q, int s) __attribute__((always_inline)) {
    const OpW cur = q;
    load_op(q, s + 2);
    fp r;
    bool wr = false;
    if ((cur.w[0] & 15u) != blsp::kNop) wr = blsp_exec(cur.w, S, r, &flag);
    __syncthreads();  // every operand read before any result is written
    if (wr) S[blsp_field(cur.w, 0)] = r;
    __syncthreads();
    if (timing) {
      const unsigned long long c = clock64();
      if (__ballot((cur.w[0] & 15u) == blsp::kMul || (cur.w[0] & 15u) == blsp::kInv))
        c_heavy += c - c_prev;
      else
        c_light += c - c_prev;
      c_prev = c;
    }
  };
  load_op(qa, 0);
  load_op(qb, 1);
  for (int s = 0; s < blsp::kSteps; s += 2) {
    run_step(qa, s);
    if (s + 1 < blsp::kSteps) run_step(qb, s + 1);  // uniform
  }
  const bool degenerate = __ballot(flag != 0) != 0;
  if (lane == 0) verdict[i] = degenerate ? 2 : blsp_result_is_one(S) ? 1 : 0;
  if (timing && lane == 0) {
    clk[0] = c_start;
    clk[1] = c_prologue;
    clk[2] = clock64();
    clk[3] = c_heavy;
    clk[4] = c_light;
  }
}

__global__ __launch_bounds__(kBlsBlock) void edv_bls_aggregate_kernel(const uint8_t* __restrict__ sig128,
                                                                     const uint64_t* __restrict__ off, uint64_t m,
                                                                     uint8_t* __restrict__ out128) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= m) return;
  g1 acc;
  g1_inf(acc);
  for (uint64_t k = off[i]; k < off[i + 1]; ++k) {
    g1 t;
    g1_from_bytes(t, sig128 + 128 * k);
    g1_add(acc, acc, t);
  }
  g1_to_bytes(out128 + 128 * i, acc);
}

__global__ __launch_bounds__(kBlsBlock) void edv_bls_sign_kernel(const uint8_t* __restrict__ sk32,
                                                                const uint8_t* __restrict__ msgs,
                                                                const uint64_t* __restrict__ moff, uint64_t n,
                                                                uint8_t* __restrict__ sig128) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t k[8];
  words_from_be(k, sk32 + 32 * i);
  g1 h, s;
  g1_hash(h, msgs + moff[i], moff[i + 1] - moff[i]);
  g1_mul(s, h, k);
  g1_to_bytes(sig128 + 128 * i, s);
}

__global__ __launch_bounds__(kBlsBlock) void edv_bls_keygen_kernel(const uint8_t* __restrict__ sk32,
                                                                  const uint8_t* __restrict__ gen128, uint64_t n,
                                                                  uint8_t* __restrict__ vk128) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t k[8];
  words_from_be(k, sk32 + 32 * i);
  g2 g, v;
  g2_from_bytes(g, gen128);
  g2_mul(v, g, k);
  g2_to_bytes(vk128 + 128 * i, v);
}

// Device buffers of one host-pointer call, freed on every exit.
struct Scratch {
  std::vector<void*> p;
  ~Scratch() {
    for (void* q : p) (void)hipFree(q);
  }
  template <class T>
  int alloc(T** out, size_t bytes) {
    void* q = nullptr;
    hipError_t e = hipMalloc(&q, bytes ? bytes : 16);
    if (e != hipSuccess) return set_err(EDV_ENOMEM, "hipMalloc(%zu): %s", bytes, hipGetErrorString(e));
    p.push_back(q);
    *out = (T*)q;
    return 0;
  }
};

int check_offsets(const uint64_t* off, uint64_t n, const char* what) {
  if (!off) return set_err(EDV_EINVAL, "null %s", what);
  for (uint64_t i = 0; i < n; ++i)
    if (off[i + 1] < off[i]) return set_err(EDV_EINVAL, "%s[%llu] decreasing", what, (unsigned long long)i);
  return 0;
}

// Messages [off[0], off[n]) to the device, offsets rebased to 0.
int upload_msgs(Scratch& sc, hipStream_t st, const uint8_t* msgs, const uint64_t* off, uint64_t n, uint8_t** d_msgs,
                uint64_t** d_off) {
  const uint64_t m0 = off[0], mbytes = off[n] - m0;
  if (mbytes && !msgs) return set_err(EDV_EINVAL, "null msgs");
  int r;
  if ((r = sc.alloc(d_msgs, mbytes + 16)) || (r = sc.alloc(d_off, 8 * (n + 1)))) return r;
  std::vector<uint64_t> o(n + 1);
  for (uint64_t i = 0; i <= n; ++i) o[i] = off[i] - m0;
  if (mbytes) BLS_TRY(hipMemcpyAsync(*d_msgs, msgs + m0, mbytes, hipMemcpyHostToDevice, st));
  BLS_TRY(hipMemcpyAsync(*d_off, o.data(), 8 * (n + 1), hipMemcpyHostToDevice, st));
  BLS_TRY(hipStreamSynchronize(st));  // o is freed on return
  return 0;
}

uint32_t grid_of(uint64_t n) { return (uint32_t)((n + kBlsBlock - 1) / kBlsBlock); }

}  // namespace

extern "C" {

static int bls_verify(edv_ctx* ctx, const uint8_t* sig128, const uint8_t* msgs, const uint64_t* msg_off,
                      const uint8_t* vk128, const uint64_t* vk_off, const uint8_t* gen128, uint64_t n,
                      uint8_t* accept_bits, bool allow_wave);

int edv_bls_verify_batch(edv_ctx* ctx, const uint8_t* sig128, const uint8_t* msgs, const uint64_t* msg_off,
                         const uint8_t* vk128, const uint64_t* vk_off, const uint8_t* gen128, uint64_t n,
                         uint8_t* accept_bits) {
  return bls_verify(ctx, sig128, msgs, msg_off, vk128, vk_off, gen128, n, accept_bits, true);
}

static int bls_verify(edv_ctx* ctx, const uint8_t* sig128, const uint8_t* msgs, const uint64_t* msg_off,
                      const uint8_t* vk128, const uint64_t* vk_off, const uint8_t* gen128, uint64_t n,
                      uint8_t* accept_bits, bool allow_wave) {
  hipStream_t st;
  int r = edv_internal::begin(ctx, &st);
  if (r) return r;
  if (n == 0) return 0;
  if (!sig128 || !vk128 || !gen128 || !accept_bits) return set_err(EDV_EINVAL, "null pointer");
  if ((r = check_offsets(msg_off, n, "msg_off"))) return r;
  if (vk_off && (r = check_offsets(vk_off, n, "vk_off"))) return r;
  const uint64_t nvk = vk_off ? vk_off[n] - vk_off[0] : n, vk0 = vk_off ? vk_off[0] : 0;
  Scratch sc;
  uint8_t *d_sig, *d_vk, *d_gen, *d_msgs;
  uint64_t *d_off, *d_vkoff = nullptr;
  unsigned long long* d_words;
  const uint64_t nwords = (n + 63) / 64;
  if ((r = sc.alloc(&d_sig, 128 * n)) || (r = sc.alloc(&d_vk, 128 * nvk)) || (r = sc.alloc(&d_gen, 128)) ||
      (r = sc.alloc(&d_words, 8 * nwords)) || (r = upload_msgs(sc, st, msgs, msg_off, n, &d_msgs, &d_off)))
    return r;
  BLS_TRY(hipMemcpyAsync(d_sig, sig128, 128 * n, hipMemcpyHostToDevice, st));
  BLS_TRY(hipMemcpyAsync(d_vk, vk128 + 128 * vk0, 128 * nvk, hipMemcpyHostToDevice, st));
  BLS_TRY(hipMemcpyAsync(d_gen, gen128, 128, hipMemcpyHostToDevice, st));
  std::vector<uint64_t> vo;
  if (vk_off) {
    if ((r = sc.alloc(&d_vkoff, 8 * (n + 1)))) return r;
    vo.resize(n + 1);
    for (uint64_t i = 0; i <= n; ++i) vo[i] = vk_off[i] - vk0;
    BLS_TRY(hipMemcpyAsync(d_vkoff, vo.data(), 8 * (n + 1), hipMemcpyHostToDevice, st));
  }
  std::vector<uint8_t> vb;
  if (allow_wave && n <= edv_internal::bls_wave_max(ctx)) {
    uint8_t* d_verdict;
    if ((r = sc.alloc(&d_verdict, n))) return r;
    unsigned long long* d_clk = nullptr;
    const bool clocks = getenv("EDV_BLS_WAVE_CLOCKS") != nullptr;
    if (clocks && (r = sc.alloc(&d_clk, 8 * 8))) return r;
    // EDV_BLS_HASH_TRIES (tests): fewer side-by-side H(m) candidates than the 61 the wave has lanes for
    const char* te = getenv("EDV_BLS_HASH_TRIES");
    const int tries = te && atoi(te) > 0 && atoi(te) < 61 ? atoi(te) : 61;
    hipLaunchKernelGGL(edv_bls_verify_wave_kernel, dim3((uint32_t)n), dim3(kBlsBlock), 0, st, d_sig, d_msgs, d_off,
                       d_vk, d_vkoff, d_gen, n, d_verdict, d_clk, tries);
    BLS_TRY(hipGetLastError());
    if (clocks) {  // diagnostics: where block 0's shader clocks went
      unsigned long long c[8];
      BLS_TRY(hipMemcpyAsync(c, d_clk, sizeof c, hipMemcpyDeviceToHost, st));
      BLS_TRY(hipStreamSynchronize(st));
      fprintf(stderr, "bls wave clocks: prologue %llu, program %llu (steps with a product %llu, without %llu)\n",
              c[1] - c[0], c[2] - c[1], c[3], c[4]);
    }
    vb.resize(n);
    BLS_TRY(hipMemcpyAsync(vb.data(), d_verdict, n, hipMemcpyDeviceToHost, st));
    BLS_TRY(hipStreamSynchronize(st));
    for (uint64_t b = 0; b < (n + 7) / 8; ++b) accept_bits[b] = 0;
    std::vector<uint64_t> redo;
    for (uint64_t k = 0; k < n; ++k) {
      accept_bits[k / 8] |= (uint8_t)((vb[k] & 1u) << (k % 8));
      if (vb[k] == 2) redo.push_back(k);
    }
    if (redo.empty()) return 0;
    // the checks the wave form could not decide (no point among H(m)'s first candidates -- a message
    // can be searched for that --, a degenerate Miller step): only they, compacted, on the four-lane
    // kernel (one crafted message no longer re-runs its whole COMMIT round)
    const uint64_t m = redo.size();
    std::vector<uint8_t> rs(128 * m), rmsg, rvk;
    std::vector<uint64_t> roff(m + 1, 0), rvoff;
    if (vk_off) rvoff.assign(m + 1, 0);
    for (uint64_t j = 0; j < m; ++j) {
      const uint64_t k = redo[j];
      memcpy(&rs[128 * j], sig128 + 128 * k, 128);
      rmsg.insert(rmsg.end(), msgs + msg_off[k], msgs + msg_off[k + 1]);
      roff[j + 1] = rmsg.size();
      const uint64_t v0 = vk_off ? vk_off[k] : k, v1 = vk_off ? vk_off[k + 1] : k + 1;
      rvk.insert(rvk.end(), vk128 + 128 * v0, vk128 + 128 * v1);
      if (vk_off) rvoff[j + 1] = rvk.size() / 128;
    }
    std::vector<uint8_t> rbits((m + 7) / 8, 0);
    if ((r = bls_verify(ctx, rs.data(), rmsg.empty() ? nullptr : rmsg.data(), roff.data(), rvk.data(),
                        vk_off ? rvoff.data() : nullptr, gen128, m, rbits.data(), false)))
      return r;
    for (uint64_t j = 0; j < m; ++j) {
      const uint64_t k = redo[j];
      const uint8_t bit = (rbits[j / 8] >> (j % 8)) & 1u;
      accept_bits[k / 8] = (uint8_t)((accept_bits[k / 8] & ~(1u << (k % 8))) | (bit << (k % 8)));
    }
    return 0;
  }
  if (!vb.empty() || 2 * n <= edv_internal::bls_pair_max(ctx))
    hipLaunchKernelGGL(edv_bls_verify_quad_kernel, dim3(grid_of(4 * n)), dim3(kBlsBlock), 0, st, d_sig, d_msgs, d_off,
                       d_vk, d_vkoff, d_gen, n, (uint16_t*)d_words);
  else if (n <= edv_internal::bls_pair_max(ctx))
    hipLaunchKernelGGL(edv_bls_verify_pair_kernel, dim3(grid_of(2 * n)), dim3(kBlsBlock), 0, st, d_sig, d_msgs, d_off,
                       d_vk, d_vkoff, d_gen, n, (uint32_t*)d_words);
  else
    hipLaunchKernelGGL(edv_bls_verify_kernel, dim3(grid_of(n)), dim3(kBlsBlock), 0, st, d_sig, d_msgs, d_off, d_vk,
                       d_vkoff, d_gen, n, d_words);
  BLS_TRY(hipGetLastError());
  std::vector<unsigned long long> w(nwords);
  BLS_TRY(hipMemcpyAsync(w.data(), d_words, 8 * nwords, hipMemcpyDeviceToHost, st));
  BLS_TRY(hipStreamSynchronize(st));
  for (uint64_t b = 0; b < (n + 7) / 8; ++b) accept_bits[b] = (uint8_t)(w[b / 8] >> (8 * (b % 8)));
  if (n & 7) accept_bits[n / 8] &= (uint8_t)((1u << (n & 7)) - 1);
  return 0;
}

int edv_bls_aggregate(edv_ctx* ctx, const uint8_t* sig128, const uint64_t* sig_off, uint64_t m, uint8_t* out128) {
  hipStream_t st;
  int r = edv_internal::begin(ctx, &st);
  if (r) return r;
  if (m == 0) return 0;
  if (!sig128 || !out128) return set_err(EDV_EINVAL, "null pointer");
  if ((r = check_offsets(sig_off, m, "sig_off"))) return r;
  const uint64_t s0 = sig_off[0], ns = sig_off[m] - s0;
  Scratch sc;
  uint8_t *d_sig, *d_out;
  uint64_t* d_off;
  if ((r = sc.alloc(&d_sig, 128 * ns)) || (r = sc.alloc(&d_out, 128 * m)) || (r = sc.alloc(&d_off, 8 * (m + 1))))
    return r;
  std::vector<uint64_t> o(m + 1);
  for (uint64_t i = 0; i <= m; ++i) o[i] = sig_off[i] - s0;
  BLS_TRY(hipMemcpyAsync(d_sig, sig128 + 128 * s0, 128 * ns, hipMemcpyHostToDevice, st));
  BLS_TRY(hipMemcpyAsync(d_off, o.data(), 8 * (m + 1), hipMemcpyHostToDevice, st));
  hipLaunchKernelGGL(edv_bls_aggregate_kernel, dim3(grid_of(m)), dim3(kBlsBlock), 0, st, d_sig, d_off, m, d_out);
  BLS_TRY(hipGetLastError());
  BLS_TRY(hipMemcpyAsync(out128, d_out, 128 * m, hipMemcpyDeviceToHost, st));
  BLS_TRY(hipStreamSynchronize(st));
  return 0;
}

int edv_bls_sign_batch(edv_ctx* ctx, const uint8_t* sk32, const uint8_t* msgs, const uint64_t* msg_off, uint64_t n,
                       uint8_t* sig128) {
  hipStream_t st;
  int r = edv_internal::begin(ctx, &st);
  if (r) return r;
  if (n == 0) return 0;
  if (!sk32 || !sig128) return set_err(EDV_EINVAL, "null pointer");
  if ((r = check_offsets(msg_off, n, "msg_off"))) return r;
  Scratch sc;
  uint8_t *d_sk, *d_msgs, *d_sig;
  uint64_t* d_off;
  if ((r = sc.alloc(&d_sk, 32 * n)) || (r = sc.alloc(&d_sig, 128 * n)) ||
      (r = upload_msgs(sc, st, msgs, msg_off, n, &d_msgs, &d_off)))
    return r;
  BLS_TRY(hipMemcpyAsync(d_sk, sk32, 32 * n, hipMemcpyHostToDevice, st));
  hipLaunchKernelGGL(edv_bls_sign_kernel, dim3(grid_of(n)), dim3(kBlsBlock), 0, st, d_sk, d_msgs, d_off, n, d_sig);
  BLS_TRY(hipGetLastError());
  BLS_TRY(hipMemcpyAsync(sig128, d_sig, 128 * n, hipMemcpyDeviceToHost, st));
  BLS_TRY(hipStreamSynchronize(st));
  return 0;
}

int edv_bls_keygen_batch(edv_ctx* ctx, const uint8_t* sk32, const uint8_t* gen128, uint64_t n, uint8_t* vk128) {
  hipStream_t st;
  int r = edv_internal::begin(ctx, &st);
  if (r) return r;
  if (n == 0) return 0;
  if (!sk32 || !gen128 || !vk128) return set_err(EDV_EINVAL, "null pointer");
  Scratch sc;
  uint8_t *d_sk, *d_gen, *d_vk;
  if ((r = sc.alloc(&d_sk, 32 * n)) || (r = sc.alloc(&d_gen, 128)) || (r = sc.alloc(&d_vk, 128 * n))) return r;
  BLS_TRY(hipMemcpyAsync(d_sk, sk32, 32 * n, hipMemcpyHostToDevice, st));
  BLS_TRY(hipMemcpyAsync(d_gen, gen128, 128, hipMemcpyHostToDevice, st));
  hipLaunchKernelGGL(edv_bls_keygen_kernel, dim3(grid_of(n)), dim3(kBlsBlock), 0, st, d_sk, d_gen, n, d_vk);
  BLS_TRY(hipGetLastError());
  BLS_TRY(hipMemcpyAsync(vk128, d_vk, 128 * n, hipMemcpyDeviceToHost, st));
  BLS_TRY(hipStreamSynchronize(st));
  return 0;
}

}  // extern "C"
