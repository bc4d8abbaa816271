// Microbenchmark: 252 dependent GF(2^255 - 19) squarings on one lane (fe25519.h's carry-serial chain,
// what edv_verify_small_kernel's R decode runs) against the same chain spread over one wave's lanes:
// limb k of the element in lane k; lane 16r + k forms terms 2r and 2r + 1 of column k of the square
// (one MAD each, operands fetched with ds_bpermute, the x2 / x19 factors from a per-lane table), the
// four rows summed with permlane32 / permlane16 swaps, then two carry rounds with the neighbour's
// carry fetched by ds_bpermute or DPP row moves (lane 0 takes 19 x lane 9's).  s_memtime ticks; both results
// compared as canonical bytes on the host.  hipcc -O3 --offload-arch=gfx950 -o ubench_lanesq ubench_lanesq.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
#include "../../indy-plenum_amd/csrc/fe25519.h"
using namespace edv;

struct SqTerm {  // per lane: two (i, j, i-side factor, j-side factor) terms; factor 0 = empty slot
  uint32_t ia[2], ib[2], ma[2], mb[2];
};
__constant__ SqTerm c_sq[64];

__device__ __forceinline__ uint32_t bperm(uint32_t src_lane, uint32_t v) {
  return (uint32_t)__builtin_amdgcn_ds_bpermute((int)(src_lane << 2), (int)v);
}

__device__ __forceinline__ uint32_t dpp_shr1(uint32_t v) {  // lane i <- lane i - 1 (in its row of 16)
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, false);
}
__device__ __forceinline__ uint32_t dpp_ror7(uint32_t v) {  // lane i <- lane (i - 7) mod 16: lane 0 <- lane 9
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x127, 0xf, 0xf, false);
}

// lanes 0..9: limb k in, limb k out (class C plus a few bits on limb 0)
template <bool DPP>
__device__ __forceinline__ uint32_t dist_sq(uint32_t f, const SqTerm& t, uint32_t k) {
  const uint32_t a0 = bperm(t.ia[0], f), b0 = bperm(t.ib[0], f);
  const uint32_t a1 = bperm(t.ia[1], f), b1 = bperm(t.ib[1], f);
  uint64_t p = (uint64_t)(a0 * t.ma[0]) * (b0 * t.mb[0]);
  p += (uint64_t)(a1 * t.ma[1]) * (b1 * t.mb[1]);
  // rows 2, 3 onto rows 0, 1; row 1 onto row 0
  uint32_t lo = (uint32_t)p, hi = (uint32_t)(p >> 32);
  auto rl = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
  auto rh = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
  p += ((uint64_t)rh[1] << 32) | rl[1];
  lo = (uint32_t)p, hi = (uint32_t)(p >> 32);
  auto sl = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
  auto sh = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
  p += ((uint64_t)sh[1] << 32) | sl[1];
  // two carry rounds (lane k <- lane k - 1's carry; lane 0 <- 19 x lane 9's)
  const uint32_t w = (k & 1) ? 25 : 26, mask = (1u << w) - 1, src = k == 0 ? 9 : k - 1, m = k == 0 ? 19 : 1;
  const uint64_t c = p >> w;
  uint32_t cl, ch;
  if (DPP) {  // row_shr:1 for lanes 1..9, row_ror:7 (lane 0 <- lane 9) for lane 0
    cl = k == 0 ? dpp_ror7((uint32_t)c) : dpp_shr1((uint32_t)c);
    ch = k == 0 ? dpp_ror7((uint32_t)(c >> 32)) : dpp_shr1((uint32_t)(c >> 32));
  } else {
    cl = bperm(src, (uint32_t)c), ch = bperm(src, (uint32_t)(c >> 32));
  }
  const uint64_t s = ((uint64_t)ch << 32 | cl) * m + ((uint32_t)p & mask);
  const uint32_t c2s = (uint32_t)(s >> w);
  const uint32_t c2 = DPP ? (k == 0 ? dpp_ror7(c2s) : dpp_shr1(c2s)) : bperm(src, c2s);
  return ((uint32_t)s & mask) + c2 * m;
}

// The same with the second carry round left in place: the element is (l, c) per lane, limb k =
// l_k + m_k c_{k-1} (m_0 = 19, c_{-1} = c_9), and the next square's operand fetch reads both halves
// (8 bpermutes side by side) instead of a dependent third carry fetch.
__device__ __forceinline__ uint32_t op_fetch(uint32_t i, uint32_t l, uint32_t c) {
  const uint32_t lo = bperm(i, l), cc = bperm(i == 0 ? 9 : i - 1, c);
  return lo + cc * (i == 0 ? 19u : 1u);
}
__device__ __forceinline__ void dist_sq_lc(uint32_t& l, uint32_t& c, const SqTerm& t, uint32_t k) {
  const uint32_t a0 = op_fetch(t.ia[0], l, c), b0 = op_fetch(t.ib[0], l, c);
  const uint32_t a1 = op_fetch(t.ia[1], l, c), b1 = op_fetch(t.ib[1], l, c);
  uint64_t p = (uint64_t)(a0 * t.ma[0]) * (b0 * t.mb[0]);
  p += (uint64_t)(a1 * t.ma[1]) * (b1 * t.mb[1]);
  uint32_t lo = (uint32_t)p, hi = (uint32_t)(p >> 32);
  auto rl = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
  auto rh = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
  p += ((uint64_t)rh[1] << 32) | rl[1];
  lo = (uint32_t)p, hi = (uint32_t)(p >> 32);
  auto sl = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
  auto sh = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
  p += ((uint64_t)sh[1] << 32) | sl[1];
  const uint32_t w = (k & 1) ? 25 : 26, mask = (1u << w) - 1, src = k == 0 ? 9 : k - 1, m = k == 0 ? 19 : 1;
  const uint64_t cr = p >> w;
  const uint32_t cl = bperm(src, (uint32_t)cr), ch = bperm(src, (uint32_t)(cr >> 32));
  const uint64_t s = ((uint64_t)ch << 32 | cl) * m + ((uint32_t)p & mask);
  l = (uint32_t)s & mask;
  c = (uint32_t)(s >> w);
}
__global__ void k_dist_lc(const uint32_t* in, uint32_t* out, long long* t, int n) {
  const uint32_t lane = threadIdx.x & 63, k = lane & 15;
  const SqTerm tm = c_sq[lane];
  uint32_t l = lane < 10 ? in[16 + lane] : 0, c = 0;
  const long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 1
  for (int s = 0; s < n; ++s) dist_sq_lc(l, c, tm, k);
  const long long t1 = __builtin_amdgcn_s_memtime();
  const uint32_t cin = bperm(k == 0 ? 9 : k - 1, c);
  const uint32_t f = l + cin * (k == 0 ? 19u : 1u);
  if (lane < 10) out[lane] = f;
  if (lane == 0) t[0] = t1 - t0;
}

template <bool DPP>
__global__ void k_dist(const uint32_t* in, uint32_t* out, long long* t, int n) {
  const uint32_t lane = threadIdx.x & 63, k = lane & 15;
  const SqTerm tm = c_sq[lane];
  uint32_t f = lane < 10 ? in[16 + lane] : 0;
  const long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 1
  for (int s = 0; s < n; ++s) f = dist_sq<DPP>(f, tm, k);
  const long long t1 = __builtin_amdgcn_s_memtime();
  if (lane < 10) out[lane] = f;
  if (lane == 0) t[0] = t1 - t0;
}

__global__ void k_lane(const uint32_t* in, uint32_t* out, long long* t, int n) {
  fe f;
  for (int i = 0; i < 10; ++i) f.v[i] = in[16 + i];
  const long long t0 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) {
#pragma unroll 1
    for (int s = 0; s < n; ++s) fe_sq_o<2>(f, f);
  }
  const long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) {
    t[1] = t1 - t0;
    for (int i = 0; i < 10; ++i) out[16 + i] = f.v[i];
  }
}

static void sq_table(SqTerm tab[64]) {
  memset(tab, 0, sizeof(SqTerm) * 64);
  for (int k = 0; k < 10; ++k) {
    int q = 0;
    for (int i = 0; i < 10; ++i)
      for (int j = i; j < 10; ++j) {
        if ((i + j) % 10 != k) continue;
        const int lane = (q / 2) * 16 + k, s = q % 2;
        tab[lane].ia[s] = i;
        tab[lane].ib[s] = j;
        tab[lane].ma[s] = (i != j ? 2 : 1) * ((i & 1) && (j & 1) ? 2 : 1);
        tab[lane].mb[s] = i + j >= 10 ? 19 : 1;
        ++q;
      }
    if (q > 8) printf("column %d: %d terms\n", k, q);
  }
}

int main() {
  const int n = 252;
  SqTerm tab[64];
  sq_table(tab);
  hipMemcpyToSymbol(HIP_SYMBOL(c_sq), tab, sizeof tab);
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
  for (int rep = 0; rep < 8; ++rep) {
    const bool dpp = rep & 1;  // odd reps: the (l, c) form instead
    if (dpp)
      hipLaunchKernelGGL(k_dist_lc, dim3(1), dim3(64), 0, 0, d_in, d_out, d_t, n);
    else
      hipLaunchKernelGGL(k_dist<false>, dim3(1), dim3(64), 0, 0, d_in, d_out, d_t, n);
    hipLaunchKernelGGL(k_lane, dim3(1), dim3(64), 0, 0, d_in, d_out, d_t, n);
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
    printf("lanes (%s carries) %lld ticks, one lane %lld ticks (%d squarings): %.2fx, equal %d\n", dpp ? "(l, c) form, bpermute" : "bpermute", t[0], t[1], n,
           (double)t[1] / (double)t[0], memcmp(ab, bb, 32) == 0);
  }
  return 0;
}
