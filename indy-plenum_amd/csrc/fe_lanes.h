// GF(2^255 - 19) squarings and products spread over one wave's lanes, for the one dependent chain
// of a single request (edv_verify_small_kernel's R decode: fe_pow22523's 250 squarings and 11
// products).  On one lane that chain issues its 55-100 v_mad_u64_u32 one after another; here the
// element sits in lanes 0..9 (limb k, radix 2^25.5 as fe25519.h) and lane 16r + k forms terms
// 2r, 2r + 1 (a square) or 3r .. 3r + 2 (a product) of column k -- operands fetched with
// ds_bpermute, the x2 (odd x odd, and i != j in a square) and x19 (past 2^255) factors from a
// per-lane table --, the four rows of 16 are summed with permlane32 / permlane16 swaps, and two
// carry rounds pass each limb's carry one lane up (lane 0 takes 19 x lane 9's).  252 dependent
// squarings: 99k shader cycles against 135-170k on one lane (tools/microbench/ubench_lanesq.hip,
// profiles/r09h).
//
// Bounds: inputs with limbs < 2^27 + 2^16 (class C, or a dist_* output: lane_cols_carry); a
// term's operands after the x2 / x4 and x19 scalings < 2^29.1 and < 2^31.3, a column of 10 terms
// < 2^62.6; the carry brings it back inside the input bounds.  dist_to_fe's fe_carry brings a
// result back to class C for the one-lane code.
#pragma once
#include "fe25519.h"

namespace edv {

// EDV_LANE_FORM 1: the distributed element also keeps 19 x its limbs in row 1 (lane 16 + k), made
// by one multiply on each result; a term's b operand is fetched from row 0 or row 1 (ib + 16: the
// x19 past 2^255), its a operand's x2 / x4 is a shift (sa) -- no v_mul_lo on the operands; an
// empty slot reads lane 10 (zero: results are zeroed outside limbs 0-9).  0: the factors from the
// table and v_mul_lo (A/B).
#ifndef EDV_LANE_FORM
#define EDV_LANE_FORM 0  // (form 1: 370-378 cycles per square, but the kernel 51.0-51.6 us: profiles/r10n)
#endif
struct LaneTerms {
  uint32_t ia[3], ib[3], ma[3], mb[3];  // factor 0: an empty slot (form 0)
  uint32_t sa[3];                       // form 1: a-side shift; ib already + 16 where x19
};
struct LaneTab {
  LaneTerms t[64];
};
constexpr LaneTab make_lane_tab(bool square) {
  LaneTab tab{};
  for (int l = 0; l < 64; ++l)
    for (int s = 0; s < 3; ++s) {
      tab.t[l].ia[s] = EDV_LANE_FORM ? 10u : 0u;
      tab.t[l].ib[s] = EDV_LANE_FORM ? 10u : 0u;
    }
  for (int k = 0; k < 10; ++k) {
    int q = 0;
    for (int i = 0; i < 10; ++i)
      for (int j = square ? i : 0; j < 10; ++j) {
        if ((i + j) % 10 != k) continue;
        const int per = square ? 2 : 3, lane = (q / per) * 16 + k, s = q % per;
        const bool odd2 = (i & 1) && (j & 1);
        const uint32_t ma = (square && i != j ? 2u : 1u) * (odd2 ? 2u : 1u);
        tab.t[lane].ia[s] = (uint32_t)i;
        tab.t[lane].ib[s] = (uint32_t)j + (EDV_LANE_FORM && i + j >= 10 ? 16u : 0u);
        tab.t[lane].ma[s] = ma;
        tab.t[lane].mb[s] = i + j >= 10 ? 19u : 1u;
        tab.t[lane].sa[s] = ma == 1 ? 0u : ma == 2 ? 1u : 2u;
        ++q;
      }
  }
  return tab;
}
__constant__ LaneTab c_lane_sq = make_lane_tab(true);
__constant__ LaneTab c_lane_mul = make_lane_tab(false);

__device__ __forceinline__ uint32_t lane_bperm(uint32_t src_lane, uint32_t v) {
  return (uint32_t)__builtin_amdgcn_ds_bpermute((int)(src_lane << 2), (int)v);
}

// the column sums of lanes 16r + k summed into lane k, then carried: limb k in lane k.
// EDV_LANE_CARRY 1 (default): ONE exchange -- each column sum p_k (< 2^62.6) is split at the limb
// widths into a_k (w_k bits), b_k (the next limb's width) and d_k (the rest, < 2^11.6), and limb k
// becomes a_k + b_{k-1} + d_{k-2} (x19 where the source wraps past 2^255: b_9 into limb 0, d_8 into
// limb 0, d_9 into limb 1), both fetched by one pair of ds_bpermute; limb 0's excess (< 2^30.4 in
// all) then moves into limb 1 through v_readlane, not another LDS round trip.  Outputs: limb 0 <
// 2^26, limb 1 < 2^26 + 2^16, other even limbs < 2^27 + 2^12, odd limbs < 2^26 + 2^12 -- inputs
// whose products keep a column of 10 terms below 2^62.6 (x2 and x19 factors included) and whose
// x19 / x4 operand scalings stay below 2^32 (tests/test_fe_lanes_model.py runs this carry on the
// CPU against exact arithmetic at those bounds).  EDV_LANE_CARRY 0: the two carry rounds of three
// ds_bpermute (A/B).
#ifndef EDV_LANE_CARRY
#define EDV_LANE_CARRY 2
#endif
// EDV_LANE_CARRY 2 (default): the one exchange by DPP row moves (row_shr:1 / :2; row_ror:7 / :8
// bring limbs 9 and 8, 9 round to lanes 0, 1) instead of a ds_bpermute pair -- 365 against 378-389
// shader cycles per square (tools/microbench/ubench_lanesq2.hip), the single-request kernel
// 49.4-49.7 against 49.8-50.2 us (profiles/r10n); 1: the ds_bpermute pair (A/B)
template <int kCtrl>
__device__ __forceinline__ uint32_t lane_dpp(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, kCtrl, 0xf, 0xf, false);
}
// EDV_LANE_SCALE 1: no quarter-rate v_mul_lo_u32 on the chain -- 19 x as two v_lshl_add_u32 (the
// compiler folds shift-adds back into a multiply, hence the asm), the operands' x2 / x4 as shifts,
// their x19 selected per lane, limb 0's excess into limb 1 by a DPP row move instead of
// v_readlane.  Measured slower: the single-request kernel 62.4-63.6 against 50.1-51.0 us
// (profiles/r10s); 0 (default): the v_mul_lo forms
#ifndef EDV_LANE_SCALE
#define EDV_LANE_SCALE 0
#endif
__device__ __forceinline__ uint32_t lane_mul19(uint32_t x) {
  uint32_t t, r;
  asm("v_lshl_add_u32 %0, %1, 4, %1" : "=v"(t) : "v"(x));
  asm("v_lshl_add_u32 %0, %1, 1, %2" : "=v"(r) : "v"(x), "v"(t));
  return r;
}
__device__ __forceinline__ uint32_t lane_cols_carry(uint64_t p, uint32_t lane) {
  const uint32_t k = lane & 15;
  uint32_t lo = (uint32_t)p, hi = (uint32_t)(p >> 32);
  auto rl = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);  // [1]: lanes 0-31 <- lanes 32-63
  auto rh = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
  p += ((uint64_t)rh[1] << 32) | rl[1];
  lo = (uint32_t)p, hi = (uint32_t)(p >> 32);
  auto sl = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);  // [1]: row 0 <- row 1; [0]: row 1 <- row 0
  auto sh = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
#if EDV_LANE_FORM
  p += (lane & 16) ? (((uint64_t)sh[0] << 32) | sl[0]) : (((uint64_t)sh[1] << 32) | sl[1]);  // rows 0, 1: the sum
#else
  p += ((uint64_t)sh[1] << 32) | sl[1];
#endif
#if EDV_LANE_CARRY
  const uint32_t w = (k & 1) ? 25 : 26, wn = 51 - w;  // widths of limb k and limb k + 1
  const uint32_t a = (uint32_t)p & ((1u << w) - 1);
  const uint32_t b = (uint32_t)(p >> w) & ((1u << wn) - 1);
  const uint32_t d = (uint32_t)(p >> 51);
  const uint32_t m1 = k == 0 ? 19 : 1, m2 = k <= 1 ? 19 : 1;
#if EDV_LANE_CARRY == 2
  const uint32_t b1 = lane_dpp<0x111>(b), b9 = lane_dpp<0x127>(b), d2 = lane_dpp<0x112>(d), d8 = lane_dpp<0x128>(d);
  const uint32_t bb = k == 0 ? b9 : b1, dd = k <= 1 ? d8 : d2;
#else
  const uint32_t src1 = k == 0 ? 9 : k - 1, src2 = k >= 2 ? k - 2 : k + 8;
  const uint32_t bb = lane_bperm(src1, b), dd = lane_bperm(src2, d);
#endif
#if EDV_LANE_SCALE
  const uint32_t r = a + (k == 0 ? lane_mul19(bb) : bb) + (k <= 1 ? lane_mul19(dd) : dd);
  const uint32_t c0 = lane_dpp<0x111>(r >> 26);  // lane 1 <- lane 0
  const uint32_t out = k == 0 ? (r & ((1u << 26) - 1)) : k == 1 ? r + c0 : r;
#else
  const uint32_t r = a + bb * m1 + dd * m2;
  const uint32_t c0 = (uint32_t)__builtin_amdgcn_readlane((int)(r >> 26), 0);
  const uint32_t out = k == 0 ? (r & ((1u << 26) - 1)) : k == 1 ? r + c0 : r;
#endif
#else
  const uint32_t w = (k & 1) ? 25 : 26, mask = (1u << w) - 1, src = k == 0 ? 9 : k - 1, m = k == 0 ? 19 : 1;
  const uint64_t c = p >> w;
  const uint32_t cl = lane_bperm(src, (uint32_t)c), ch = lane_bperm(src, (uint32_t)(c >> 32));
  const uint64_t s = ((uint64_t)ch << 32 | cl) * m + ((uint32_t)p & mask);
  const uint32_t c2 = lane_bperm(src, (uint32_t)(s >> w));
  const uint32_t out = ((uint32_t)s & mask) + c2 * m;
#endif
#if EDV_LANE_FORM
  return k < 10 ? out * ((lane & 48) == 16 ? 19u : 1u) : 0u;  // row 1: 19 x the limb
#else
  return out;
#endif
}

// f^2; every lane of the wave takes part (t = c_lane_sq.t[lane])
__device__ __forceinline__ uint32_t dist_sq(uint32_t f, const LaneTerms& t, uint32_t lane) {
#if EDV_LANE_FORM
  const uint32_t a0 = lane_bperm(t.ia[0], f) << t.sa[0], b0 = lane_bperm(t.ib[0], f);
  const uint32_t a1 = lane_bperm(t.ia[1], f) << t.sa[1], b1 = lane_bperm(t.ib[1], f);
  uint64_t p = (uint64_t)a0 * b0;
  p += (uint64_t)a1 * b1;
#elif EDV_LANE_SCALE  // (an empty slot: ma = 0 -- its a-side operand zeroed by the select)
  const uint32_t a0 = lane_bperm(t.ia[0], f), b0 = lane_bperm(t.ib[0], f);
  const uint32_t a1 = lane_bperm(t.ia[1], f), b1 = lane_bperm(t.ib[1], f);
  uint64_t p = (uint64_t)(t.ma[0] ? a0 << t.sa[0] : 0u) * (t.mb[0] == 19 ? lane_mul19(b0) : b0);
  p += (uint64_t)(t.ma[1] ? a1 << t.sa[1] : 0u) * (t.mb[1] == 19 ? lane_mul19(b1) : b1);
#else
  const uint32_t a0 = lane_bperm(t.ia[0], f), b0 = lane_bperm(t.ib[0], f);
  const uint32_t a1 = lane_bperm(t.ia[1], f), b1 = lane_bperm(t.ib[1], f);
  uint64_t p = (uint64_t)(a0 * t.ma[0]) * (b0 * t.mb[0]);
  p += (uint64_t)(a1 * t.ma[1]) * (b1 * t.mb[1]);
#endif
  return lane_cols_carry(p, lane);
}
__device__ __forceinline__ uint32_t dist_sqn(uint32_t f, int n, const LaneTerms& t, uint32_t lane) {
#pragma unroll 1
  for (int i = 0; i < n; ++i) f = dist_sq(f, t, lane);
  return f;
}
// f g (t = c_lane_mul.t[lane])
__device__ __forceinline__ uint32_t dist_mul(uint32_t f, uint32_t g, const LaneTerms& t, uint32_t lane) {
  uint64_t p = 0;
#pragma unroll
  for (int s = 0; s < 3; ++s) {
#if EDV_LANE_FORM
    const uint32_t a = lane_bperm(t.ia[s], f) << t.sa[s], b = lane_bperm(t.ib[s], g);
    p += (uint64_t)a * b;
#elif EDV_LANE_SCALE
    const uint32_t a = lane_bperm(t.ia[s], f), b = lane_bperm(t.ib[s], g);
    p += (uint64_t)(t.ma[s] ? a << t.sa[s] : 0u) * (t.mb[s] == 19 ? lane_mul19(b) : b);
#else
    const uint32_t a = lane_bperm(t.ia[s], f), b = lane_bperm(t.ib[s], g);
    p += (uint64_t)(a * t.ma[s]) * (b * t.mb[s]);
#endif
  }
  return lane_cols_carry(p, lane);
}
// a limb value r of lane (limb lane & 15 of row 0) in the distributed form: row 1 takes 19 r
// (EDV_LANE_FORM 1); other lanes' r must be 0 outside limbs 0-9 of rows 0 and 1
__device__ __forceinline__ uint32_t dist_form(uint32_t r, uint32_t lane) {
#if EDV_LANE_FORM
  return (lane & 15) < 10 && lane < 32 ? r * ((lane & 16) ? 19u : 1u) : 0u;
#else
  return r;
#endif
}

// lane 0's f as the distributed form (every lane calls; other lanes' f is ignored)
__device__ __forceinline__ uint32_t dist_from_lane0(const fe& f, uint32_t lane) {
  uint32_t r = 0;
#pragma unroll
  for (int k = 0; k < 10; ++k) {
    const uint32_t v = (uint32_t)__builtin_amdgcn_readlane((int)f.v[k], 0);
    r = (lane & 15) == (uint32_t)k ? v : r;
  }
  return dist_form(EDV_LANE_FORM || lane < 16 ? r : 0u, lane);
}
// the distributed d as an fe (class C) in every lane
__device__ __forceinline__ void dist_to_fe(fe& f, uint32_t d) {
#pragma unroll
  for (int k = 0; k < 10; ++k) f.v[k] = (uint32_t)__builtin_amdgcn_readlane((int)d, k);
  fe_carry(f);
}

}  // namespace edv
