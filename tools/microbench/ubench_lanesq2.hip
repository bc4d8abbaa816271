// Microbenchmark: 252 dependent lane-distributed squarings (fe_lanes.h's dist_sq, the R decode's
// chain in edv_verify_small_kernel) against variants of its two costs besides the operand fetch:
//   V0  fe_lanes.h as built (ds_bpermute operands, v_mul_lo scalings, one-exchange carry by
//       ds_bpermute + v_readlane)
//   V1  V0 with the carry's exchange by DPP row moves (row_shr:1 / :2, row_ror:7 / :8 for the
//       wrap into lanes 0, 1) instead of the second ds_bpermute pair
//   V2  V0 without the operand scalings' v_mul_lo: row 1 keeps 19 x the limbs (one multiply per
//       square on the result), the b-side fetch reads row 0 or row 1 by its lane index, the a-side
//       x2 / x4 are shifts
//   V3  V1 + V2
// s_memtime ticks; each variant's result compared with the one-lane chain as canonical bytes.
// hipcc -O3 --offload-arch=gfx950 -o ubench_lanesq2 ubench_lanesq2.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
#include "../../indy-plenum_amd/csrc/fe_lanes.h"
using namespace edv;

struct SqTerm2 {  // V2: per lane two terms: a-side source lane and shift, b-side source lane (+16: x19)
  uint32_t ia[2], sa[2], ib[2];
};
__constant__ SqTerm2 c_sq2[64];

__device__ __forceinline__ uint32_t dpp_shr1(uint32_t v) {  // lane i <- lane i - 1 (row of 16)
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, false);
}
__device__ __forceinline__ uint32_t dpp_shr2(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, false);
}
__device__ __forceinline__ uint32_t dpp_ror7(uint32_t v) {  // lane i <- lane (i - 7) mod 16: 0 <- 9
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x127, 0xf, 0xf, false);
}
__device__ __forceinline__ uint32_t dpp_ror8(uint32_t v) {  // 0 <- 8, 1 <- 9
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x128, 0xf, 0xf, false);
}

// rows 2, 3 onto 0, 1, then row 1 onto row 0; with ROW1: row 1 also gets the full sum
template <bool ROW1>
__device__ __forceinline__ uint64_t rows_sum(uint64_t p, uint32_t lane) {
  uint32_t lo = (uint32_t)p, hi = (uint32_t)(p >> 32);
  auto rl = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
  auto rh = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
  p += ((uint64_t)rh[1] << 32) | rl[1];
  lo = (uint32_t)p, hi = (uint32_t)(p >> 32);
  auto sl = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
  auto sh = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
  if (ROW1 && (lane & 16)) return p + (((uint64_t)sh[0] << 32) | sl[0]);
  return p + (((uint64_t)sh[1] << 32) | sl[1]);
}

template <bool DPP>
__device__ __forceinline__ uint32_t carry1(uint64_t p, uint32_t k) {
  const uint32_t w = (k & 1) ? 25 : 26, wn = 51 - w;
  const uint32_t a = (uint32_t)p & ((1u << w) - 1);
  const uint32_t b = (uint32_t)(p >> w) & ((1u << wn) - 1);
  const uint32_t d = (uint32_t)(p >> 51);
  uint32_t bb, dd;
  if (DPP) {
    const uint32_t b1 = dpp_shr1(b), b9 = dpp_ror7(b), d2 = dpp_shr2(d), d8 = dpp_ror8(d);
    bb = k == 0 ? b9 : b1;
    dd = k <= 1 ? d8 : d2;
  } else {
    bb = lane_bperm(k == 0 ? 9 : k - 1, b);
    dd = lane_bperm(k >= 2 ? k - 2 : k + 8, d);
  }
  const uint32_t m1 = k == 0 ? 19 : 1, m2 = k <= 1 ? 19 : 1;
  const uint32_t r = a + bb * m1 + dd * m2;
  const uint32_t c0 = (uint32_t)__builtin_amdgcn_readlane((int)(r >> 26), 0);
  return k == 0 ? (r & ((1u << 26) - 1)) : k == 1 ? r + c0 : r;
}

template <bool DPP>
__device__ __forceinline__ uint32_t sq_v01(uint32_t f, const LaneTerms& t, uint32_t lane) {
  const uint32_t k = lane & 15;
  const uint32_t a0 = lane_bperm(t.ia[0], f), b0 = lane_bperm(t.ib[0], f);
  const uint32_t a1 = lane_bperm(t.ia[1], f), b1 = lane_bperm(t.ib[1], f);
  uint64_t p = (uint64_t)(a0 * t.ma[0]) * (b0 * t.mb[0]);
  p += (uint64_t)(a1 * t.ma[1]) * (b1 * t.mb[1]);
  return carry1<DPP>(rows_sum<false>(p, lane), k);
}

// V2/V3: f holds the limbs in row 0 and 19 x the limbs in row 1
template <bool DPP>
__device__ __forceinline__ uint32_t sq_v23(uint32_t f, const SqTerm2& t, uint32_t lane, uint32_t mrow) {
  const uint32_t k = lane & 15;
  const uint32_t a0 = lane_bperm(t.ia[0], f) << t.sa[0], b0 = lane_bperm(t.ib[0], f);
  const uint32_t a1 = lane_bperm(t.ia[1], f) << t.sa[1], b1 = lane_bperm(t.ib[1], f);
  uint64_t p = (uint64_t)a0 * b0;
  p += (uint64_t)a1 * b1;
  const uint32_t r = carry1<DPP>(rows_sum<true>(p, lane), k) * mrow;
  return k < 10 ? r : 0;
}

template <int V>
__global__ void k_var(const uint32_t* in, uint32_t* out, long long* t, int n) {
  const uint32_t lane = threadIdx.x & 63, k = lane & 15;
  const uint32_t mrow = (lane >> 4) == 1 ? 19u : 1u;
  uint32_t f = k < 10 ? in[16 + k] : 0;
  if (V >= 2) f *= mrow;
  const LaneTerms tm = c_lane_sq.t[lane];
  const SqTerm2 t2 = c_sq2[lane];
  const long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 1
  for (int s = 0; s < n; ++s) {
    if (V == 0) f = sq_v01<false>(f, tm, lane);
    if (V == 1) f = sq_v01<true>(f, tm, lane);
    if (V == 2) f = sq_v23<false>(f, t2, lane, mrow);
    if (V == 3) f = sq_v23<true>(f, t2, lane, mrow);
  }
  const long long t1 = __builtin_amdgcn_s_memtime();
  if (lane < 10) out[lane] = f;
  if (lane == 0) t[0] = t1 - t0;
}

__global__ void k_lane(const uint32_t* in, uint32_t* out, int n) {
  fe f;
  for (int i = 0; i < 10; ++i) f.v[i] = in[16 + i];
  if (threadIdx.x == 0) {
#pragma unroll 1
    for (int s = 0; s < n; ++s) fe_sq_o<2>(f, f);
    for (int i = 0; i < 10; ++i) out[16 + i] = f.v[i];
  }
}

static void sq2_table(SqTerm2 tab[64]) {
  memset(tab, 0, sizeof(SqTerm2) * 64);
  for (int l = 0; l < 64; ++l)  // empty slots: lane 10 (a zero limb: sq_v23 zeroes lanes 10-15)
    for (int s = 0; s < 2; ++s) tab[l].ia[s] = tab[l].ib[s] = 10;
  for (int k = 0; k < 10; ++k) {
    int q = 0;
    for (int i = 0; i < 10; ++i)
      for (int j = i; j < 10; ++j) {
        if ((i + j) % 10 != k) continue;
        const int lane = (q / 2) * 16 + k, s = q % 2;
        const int ma = (i != j ? 2 : 1) * ((i & 1) && (j & 1) ? 2 : 1);
        tab[lane].ia[s] = i;
        tab[lane].sa[s] = ma == 1 ? 0 : ma == 2 ? 1 : 2;
        tab[lane].ib[s] = j + (i + j >= 10 ? 16 : 0);
        ++q;
      }
  }
}

int main() {
  const int n = 252;
  SqTerm2 tab[64];
  sq2_table(tab);
  hipMemcpyToSymbol(HIP_SYMBOL(c_sq2), tab, sizeof tab);
  uint32_t h_in[32] = {0};
  uint64_t x[4] = {0x1234567890abcdefULL, 0x0fedcba987654321ULL, 0x1111222233334444ULL, 0x0555666677778888ULL};
  uint32_t w[8];
  memcpy(w, x, 32);
  fe f0;
  fe_frombytes(f0, w);
  for (int i = 0; i < 10; ++i) h_in[16 + i] = f0.v[i];
  uint32_t *d_in, *d_out;
  long long* d_t;
  hipMalloc(&d_in, sizeof h_in);
  hipMalloc(&d_out, 128);
  hipMalloc(&d_t, 16);
  hipMemcpy(d_in, h_in, sizeof h_in, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k_lane, dim3(1), dim3(64), 0, 0, d_in, d_out, n);
  const char* names[4] = {"V0 bpermute carry, mul scalings", "V1 DPP carry", "V2 no mul scalings",
                          "V3 DPP carry, no mul scalings"};
  for (int rep = 0; rep < 3; ++rep)
    for (int v = 0; v < 4; ++v) {
      if (v == 0) hipLaunchKernelGGL(k_var<0>, dim3(1), dim3(64), 0, 0, d_in, d_out, d_t, n);
      if (v == 1) hipLaunchKernelGGL(k_var<1>, dim3(1), dim3(64), 0, 0, d_in, d_out, d_t, n);
      if (v == 2) hipLaunchKernelGGL(k_var<2>, dim3(1), dim3(64), 0, 0, d_in, d_out, d_t, n);
      if (v == 3) hipLaunchKernelGGL(k_var<3>, dim3(1), dim3(64), 0, 0, d_in, d_out, d_t, n);
      uint32_t o[32];
      long long t[2];
      hipMemcpy(o, d_out, 128, hipMemcpyDeviceToHost);
      hipMemcpy(t, d_t, 16, hipMemcpyDeviceToHost);
      fe a, b;
      for (int i = 0; i < 10; ++i) {
        a.v[i] = o[i];
        b.v[i] = o[16 + i];
      }
      fe_carry(a);
      uint32_t ab[8], bb[8];
      fe_tobytes(ab, a);
      fe_tobytes(bb, b);
      printf("%-34s %7lld ticks (%d squarings, %.0f per square), equal to one lane: %d\n", names[v], t[0], n,
             (double)t[0] / n, memcmp(ab, bb, 32) == 0);
    }
  return 0;
}
