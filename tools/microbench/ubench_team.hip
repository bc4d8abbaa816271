// Microbenchmark: 252 dependent GF(2^255 - 19) squarings on one lane of one wave (fe25519.h's
// carry-serial chain) against a team of K waves of one workgroup, each computing two of the ten
// 64-bit column sums of every square (zero-started chains), exchanged through LDS (one barrier
// per square, double-buffered) and carried by every wave (fe_carry64).  s_memtime ticks; both
// results checked against each other on the host.  Does spreading a square over waves (each with
// its own issue slot) beat the one-wave chain, which issues a MAD every ~10-13 cycles?
// hipcc -O3 --offload-arch=gfx950 -o ubench_team ubench_team.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
#include "../../indy-plenum_amd/csrc/fe25519.h"
using namespace edv;

// column K of f^2 (radix 2^25.5: x2 for odd x odd, x19 past 2^255), zero-started
template <int K>
__device__ __forceinline__ uint64_t sq_col(const fe& f) {
  uint64_t a = 0;
#pragma unroll
  for (int i = 0; i < 10; ++i) {
#pragma unroll
    for (int j = i; j < 10; ++j) {
      if ((i + j) % 10 != K) continue;
      const bool both_odd = (i & 1) && (j & 1), wrap = i + j >= 10;
      const uint32_t fi = (i != j) ? 2u * f.v[i] : f.v[i];
      const uint32_t fj = wrap ? (both_odd ? 38u * f.v[j] : 19u * f.v[j]) : (both_odd ? 2u * f.v[j] : f.v[j]);
      a += (uint64_t)fi * fj;
    }
  }
  return a;
}

// wave W of a team of K (10 / K columns each) writes its column sums into b[]
template <int K, int W>
__device__ __forceinline__ void cols(const fe& f, uint64_t* b, int lane) {
  constexpr int C = 10 / K;
  uint64_t c[C];
#pragma unroll
  for (int q = 0; q < C; ++q) {
    switch (W * C + q) {
      case 0: c[q] = sq_col<0>(f); break;
      case 1: c[q] = sq_col<1>(f); break;
      case 2: c[q] = sq_col<2>(f); break;
      case 3: c[q] = sq_col<3>(f); break;
      case 4: c[q] = sq_col<4>(f); break;
      case 5: c[q] = sq_col<5>(f); break;
      case 6: c[q] = sq_col<6>(f); break;
      case 7: c[q] = sq_col<7>(f); break;
      case 8: c[q] = sq_col<8>(f); break;
      default: c[q] = sq_col<9>(f); break;
    }
  }
  if (lane == 0)
#pragma unroll
    for (int q = 0; q < C; ++q) b[W * C + q] = c[q];
}

template <int K>
__global__ void k_team(const uint32_t* in, uint32_t* out, long long* t, int n) {
  __shared__ uint64_t buf[2][10];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  fe f;
  for (int i = 0; i < 10; ++i) f.v[i] = in[16 + i];
  __syncthreads();
  const long long t0 = __builtin_amdgcn_s_memtime();
  int par = 0;
#pragma unroll 1
  for (int s = 0; s < n; ++s) {
    switch (wave) {
      case 0: cols<K, 0>(f, buf[par], lane); break;
      case 1: if constexpr (K > 1) cols<K, 1 % K>(f, buf[par], lane); break;
      case 2: if constexpr (K > 2) cols<K, 2 % K>(f, buf[par], lane); break;
      case 3: if constexpr (K > 3) cols<K, 3 % K>(f, buf[par], lane); break;
      case 4: if constexpr (K > 4) cols<K, 4 % K>(f, buf[par], lane); break;
      case 5: if constexpr (K > 5) cols<K, 5 % K>(f, buf[par], lane); break;
      case 6: if constexpr (K > 6) cols<K, 6 % K>(f, buf[par], lane); break;
      case 7: if constexpr (K > 7) cols<K, 7 % K>(f, buf[par], lane); break;
      case 8: if constexpr (K > 8) cols<K, 8 % K>(f, buf[par], lane); break;
      default: if constexpr (K > 9) cols<K, 9 % K>(f, buf[par], lane); break;
    }
    __syncthreads();
    uint64_t h[10];
#pragma unroll
    for (int k = 0; k < 10; ++k) h[k] = buf[par][k];
    fe_carry64(f, h);
    par ^= 1;
  }
  const long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) {
    t[0] = t1 - t0;
    for (int i = 0; i < 10; ++i) out[i] = f.v[i];
  }
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

int main() {
  const int n = 252;
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
  for (int rep = 0; rep < 9; ++rep) {
    const int K = rep % 3 == 0 ? 2 : rep % 3 == 1 ? 5 : 10;
    if (K == 2) hipLaunchKernelGGL(k_team<2>, dim3(1), dim3(64 * 2), 0, 0, d_in, d_out, d_t, n);
    if (K == 5) hipLaunchKernelGGL(k_team<5>, dim3(1), dim3(64 * 5), 0, 0, d_in, d_out, d_t, n);
    if (K == 10) hipLaunchKernelGGL(k_team<10>, dim3(1), dim3(64 * 10), 0, 0, d_in, d_out, d_t, n);
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
    uint32_t ab[8], bb[8];
    fe_tobytes(ab, a);
    fe_tobytes(bb, b);
    printf("team of %d waves %lld ticks, one lane %lld ticks (%d squarings): %.2fx, team==lane %d\n", K, t[0], t[1], n,
           (double)t[1] / (double)t[0], memcmp(ab, bb, 32) == 0);
  }
  return 0;
}
