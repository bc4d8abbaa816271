// Microbenchmark: a GF(2^255 - 19) product spread over the 16 lanes of a row (radix 2^16, 16 limbs,
// limb k in lane k; column k = sum_t a_t * b_(k-t mod 16), x38 where the index wraps; three carry
// rounds passing carries one lane up with DPP row rotates) against fe25519.h's one-lane product
// chain: 252 dependent squarings each, s_memtime ticks; the row result is checked on the host.
// hipcc -O3 --offload-arch=gfx950 -o ubench_rowfe ubench_rowfe.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
#include "../../indy-plenum_amd/csrc/fe25519.h"
using namespace edv;

template <int CTRL>
__device__ __forceinline__ uint32_t dpp(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, CTRL, 0xf, 0xf, true);
}
// lanes k < T of every row (T = 0..16): the wrapped terms of step T
template <int T>
constexpr uint64_t wrap_mask() {
  return T == 0 ? 0ull : 0x0001000100010001ull * ((1ull << T) - 1);
}
// m ? y : x per lane, m a wave-uniform lane mask (an SGPR pair: no per-step compare)
__device__ __forceinline__ uint32_t sel(uint64_t m, uint32_t x, uint32_t y) {
  uint32_t r;
  asm volatile("v_cndmask_b32 %0, %1, %2, %3" : "=v"(r) : "v"(x), "v"(y), "s"(m));
  return r;
}
// lane k of each row gets lane (k - N) mod 16 (DIR 0) or (k + N) mod 16 (DIR 1) of the same row
template <int DIR, int N>
__device__ __forceinline__ uint32_t rot(uint32_t v) {
  if (N == 0) return v;
  return dpp<0x120 + (DIR ? (16 - N) & 15 : N)>(v);
}
template <int DIR, int T>
__device__ __forceinline__ void step(uint64_t& acc, uint32_t a, uint32_t b, uint32_t b38, int k) {
  const uint32_t at = dpp<0x150 + T>(a);        // a_T in every lane of the row (row_newbcast)
  const uint32_t bt = rot<DIR, T>(b), bt38 = rot<DIR, T>(b38);
  const uint32_t y = sel(wrap_mask<T>(), bt, bt38);  // the wrapped terms carry 2^256 = 38
  acc = (uint64_t)at * y + acc;
}
template <int DIR>
__device__ __forceinline__ uint32_t row_mul(uint32_t a, uint32_t b, int k) {
  const uint32_t b38 = __umul24(b, 38u);
  uint64_t acc = 0;
  step<DIR, 0>(acc, a, b, b38, k); step<DIR, 1>(acc, a, b, b38, k); step<DIR, 2>(acc, a, b, b38, k);
  step<DIR, 3>(acc, a, b, b38, k); step<DIR, 4>(acc, a, b, b38, k); step<DIR, 5>(acc, a, b, b38, k);
  step<DIR, 6>(acc, a, b, b38, k); step<DIR, 7>(acc, a, b, b38, k); step<DIR, 8>(acc, a, b, b38, k);
  step<DIR, 9>(acc, a, b, b38, k); step<DIR, 10>(acc, a, b, b38, k); step<DIR, 11>(acc, a, b, b38, k);
  step<DIR, 12>(acc, a, b, b38, k); step<DIR, 13>(acc, a, b, b38, k); step<DIR, 14>(acc, a, b, b38, k);
  step<DIR, 15>(acc, a, b, b38, k);
  const uint32_t f = sel(0x0001000100010001ull, 1u, 38u);
  // carry round 1: acc < 2^44 -> carry < 2^28
  uint32_t lo = (uint32_t)acc & 0xffffu;
  uint32_t c = (uint32_t)(acc >> 16);
  uint64_t v = (uint64_t)rot<DIR, 1>(c) * f + lo;   // lane k gets carry_(k-1); lane 0 gets 38 carry_15
  lo = (uint32_t)v & 0xffffu;
  c = (uint32_t)(v >> 16);
  v = (uint64_t)rot<DIR, 1>(c) * f + lo;
  lo = (uint32_t)v & 0xffffu;
  c = (uint32_t)(v >> 16);
  return rot<DIR, 1>(c) * f + lo;                    // < 2^16 + 38 * 2^7
}

template <int DIR>
__global__ void k_row(const uint32_t* in, uint32_t* out, long long* t, int n) {
  const int k = threadIdx.x & 15;
  uint32_t a = in[k];
  long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < n; ++i) a = row_mul<DIR>(a, a, k);
  long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x < 16) out[threadIdx.x] = a;
  if (threadIdx.x == 0) t[0] = t1 - t0;
}
__global__ void k_lane(const uint32_t* in, uint32_t* out, long long* t, int n) {
  if (threadIdx.x != 0) return;
  fe a;
  for (int i = 0; i < 10; ++i) a.v[i] = in[16 + i];
  long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < n; ++i) fe_sq_o<2>(a, a);
  long long t1 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < 10; ++i) out[16 + i] = a.v[i];
  t[1] = t1 - t0;
}

// host reference: x^(2^n) mod p with 64-bit limbs via __int128
typedef unsigned __int128 u128;
static void mulmod(uint64_t r[4], const uint64_t a[4], const uint64_t b[4]) {
  uint64_t t[8] = {0};
  for (int i = 0; i < 4; ++i) {
    u128 c = 0;
    for (int j = 0; j < 4; ++j) {
      c += (u128)a[i] * b[j] + t[i + j];
      t[i + j] = (uint64_t)c;
      c >>= 64;
    }
    t[i + 4] = (uint64_t)c;
  }
  u128 c = 0;  // t = lo + 2^256 hi -> lo + 38 hi
  uint64_t s[5];
  for (int i = 0; i < 4; ++i) {
    c += (u128)t[i] + (u128)t[i + 4] * 38;
    s[i] = (uint64_t)c;
    c >>= 64;
  }
  s[4] = (uint64_t)c;
  c = (u128)s[0] + (u128)s[4] * 38;
  r[0] = (uint64_t)c; c >>= 64;
  for (int i = 1; i < 4; ++i) { c += s[i]; r[i] = (uint64_t)c; c >>= 64; }
  if (c) { c = (u128)r[0] + 38; r[0] = (uint64_t)c; c >>= 64; for (int i = 1; i < 4 && c; ++i) { c += r[i]; r[i] = (uint64_t)c; c >>= 64; } }
}
static void canon(uint64_t r[4]) {  // full reduction mod p = 2^255 - 19
  for (int rep = 0; rep < 3; ++rep) {
    uint64_t top = r[3] >> 63;
    r[3] &= 0x7fffffffffffffffULL;
    u128 c = (u128)r[0] + top * 19; r[0] = (uint64_t)c; c >>= 64;
    for (int i = 1; i < 4; ++i) { c += r[i]; r[i] = (uint64_t)c; c >>= 64; }
  }
  // subtract p if >= p
  uint64_t p[4] = {0xffffffffffffffedULL, 0xffffffffffffffffULL, 0xffffffffffffffffULL, 0x7fffffffffffffffULL};
  bool ge = true;
  for (int i = 3; i >= 0; --i) { if (r[i] != p[i]) { ge = r[i] > p[i]; break; } }
  if (ge) { u128 bw = 0; for (int i = 0; i < 4; ++i) { u128 d = (u128)r[i] - p[i] - bw; r[i] = (uint64_t)d; bw = (d >> 64) & 1; } }
}
int main() {
  const int n = 252;
  uint32_t h_in[32] = {0};
  uint64_t x[4] = {0x1234567890abcdefULL, 0x0fedcba987654321ULL, 0x1111222233334444ULL, 0x0555666677778888ULL};
  for (int k = 0; k < 16; ++k) h_in[k] = (uint32_t)(x[k / 4] >> (16 * (k % 4))) & 0xffff;
  // the same value in radix 2^25.5 for the lane form
  {
    uint8_t b[32];
    memcpy(b, x, 32);
    uint32_t w[8];
    memcpy(w, b, 32);
    fe f;
    fe_frombytes(f, w);
    for (int i = 0; i < 10; ++i) h_in[16 + i] = f.v[i];
  }
  uint64_t ref[4] = {x[0], x[1], x[2], x[3]};
  for (int i = 0; i < n; ++i) mulmod(ref, ref, ref);
  canon(ref);
  uint32_t *d_in, *d_out; long long* d_t;
  hipMalloc(&d_in, sizeof h_in); hipMalloc(&d_out, 128); hipMalloc(&d_t, 16);
  hipMemcpy(d_in, h_in, sizeof h_in, hipMemcpyHostToDevice);
  for (int dir = 0; dir < 2; ++dir) {
    for (int rep = 0; rep < 3; ++rep) {
      if (dir == 0) hipLaunchKernelGGL(k_row<0>, dim3(1), dim3(64), 0, 0, d_in, d_out, d_t, n);
      else hipLaunchKernelGGL(k_row<1>, dim3(1), dim3(64), 0, 0, d_in, d_out, d_t, n);
      hipLaunchKernelGGL(k_lane, dim3(1), dim3(64), 0, 0, d_in, d_out, d_t, n);
      uint32_t o[32]; long long t[2];
      hipMemcpy(o, d_out, 128, hipMemcpyDeviceToHost); hipMemcpy(t, d_t, 16, hipMemcpyDeviceToHost);
      uint64_t got[4] = {0, 0, 0, 0};  // sum of limbs * 2^(16k), reduced
      u128 c = 0;
      for (int q = 0; q < 4; ++q) {
        for (int k = 0; k < 4; ++k) c += (u128)o[4 * q + k] << (16 * k);
        got[q] = (uint64_t)c; c >>= 64;
      }
      if (c) { u128 cc = (u128)got[0] + c * 38; got[0] = (uint64_t)cc; cc >>= 64; for (int i = 1; i < 4 && cc; ++i) { cc += got[i]; got[i] = (uint64_t)cc; cc >>= 64; } }
      canon(got);
      fe lf;
      for (int i = 0; i < 10; ++i) lf.v[i] = o[16 + i];
      uint32_t lb[8];
      fe_tobytes(lb, lf);
      printf("dir %d: row %lld ticks, lane %lld ticks (%d squarings); row==ref %d lane==ref %d\n", dir, t[0], t[1], n,
             memcmp(got, ref, 32) == 0, memcmp(lb, ref, 32) == 0);
    }
  }
  return 0;
}
