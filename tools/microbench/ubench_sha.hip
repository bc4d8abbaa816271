// Microbenchmark: SHA-512 compression of 3 blocks on one lane (VALU, sha512.h) against the same
// rounds on wave-uniform values (SALU); s_memtime ticks.  hipcc -O3 --offload-arch=gfx950
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include "../../indy-plenum_amd/csrc/sha512.h"
using namespace edv;

// SALU-friendly SHA-512 compress: plain 64-bit ops on wave-uniform values
__device__ __forceinline__ uint64_t srotr(uint64_t x, int n) { return (x >> n) | (x << (64 - n)); }
#define SROUND(KI, WI) { \
  const uint64_t S1 = srotr(e,14) ^ srotr(e,18) ^ srotr(e,41); \
  const uint64_t ch = (e & f) ^ (~e & g); \
  const uint64_t t1 = h + S1 + ch + (KI) + (WI); \
  const uint64_t S0 = srotr(a,28) ^ srotr(a,34) ^ srotr(a,39); \
  const uint64_t mj = (a & b) | (c & (a | b)); \
  h = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + S0 + mj; }
__device__ void s_compress(uint64_t st[8], uint64_t w[16]) {
  uint64_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], h = st[7];
#pragma unroll
  for (int i = 0; i < 16; ++i) SROUND(SHA512_K[i], w[i])
#pragma unroll 1
  for (int r = 16; r < 80; r += 16) {
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const uint64_t w15 = w[(i + 1) & 15], w2 = w[(i + 14) & 15];
      const uint64_t s0 = srotr(w15, 1) ^ srotr(w15, 8) ^ (w15 >> 7);
      const uint64_t s1 = srotr(w2, 19) ^ srotr(w2, 61) ^ (w2 >> 6);
      w[i] += s0 + w[(i + 9) & 15] + s1;
      SROUND(SHA512_K[r + i], w[i])
    }
  }
  st[0] += a; st[1] += b; st[2] += c; st[3] += d; st[4] += e; st[5] += f; st[6] += g; st[7] += h;
}

__global__ void k_valu(const uint64_t* __restrict__ in, uint64_t* out, long long* t, int blocks) {
  if (threadIdx.x != 0) return;
  uint64_t st[8], w[16];
  for (int j = 0; j < 8; ++j) st[j] = in[j];
  long long t0 = __builtin_amdgcn_s_memtime();
  for (int b = 0; b < blocks; ++b) {
    for (int j = 0; j < 16; ++j) w[j] = in[8 + 16 * b + j];
    sha512_compress(st, w);
  }
  long long t1 = __builtin_amdgcn_s_memtime();
  for (int j = 0; j < 8; ++j) out[j] = st[j];
  t[0] = t1 - t0;
}
__global__ void k_salu(const uint64_t* __restrict__ in, uint64_t* out, long long* t, int blocks) {
  uint64_t st[8], w[16];
  for (int j = 0; j < 8; ++j) st[j] = in[j];
  long long t0 = __builtin_amdgcn_s_memtime();
  for (int b = 0; b < blocks; ++b) {
    for (int j = 0; j < 16; ++j) w[j] = in[8 + 16 * b + j];
    s_compress(st, w);
  }
  long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) {
    for (int j = 0; j < 8; ++j) out[j] = st[j];
    t[0] = t1 - t0;
  }
}
int main() {
  const int blocks = 3;
  uint64_t h_in[8 + 16 * blocks];
  for (int i = 0; i < 8 + 16 * blocks; ++i) h_in[i] = 0x0123456789abcdefULL * (i + 1);
  uint64_t *d_in, *d_out; long long* d_t;
  hipMalloc(&d_in, sizeof h_in); hipMalloc(&d_out, 64 * 2); hipMalloc(&d_t, 16);
  hipMemcpy(d_in, h_in, sizeof h_in, hipMemcpyHostToDevice);
  uint64_t o1[8], o2[8]; long long t1, t2;
  for (int rep = 0; rep < 3; ++rep) {
    hipLaunchKernelGGL(k_valu, dim3(1), dim3(64), 0, 0, d_in, d_out, d_t, blocks);
    hipMemcpy(o1, d_out, 64, hipMemcpyDeviceToHost); hipMemcpy(&t1, d_t, 8, hipMemcpyDeviceToHost);
    hipLaunchKernelGGL(k_salu, dim3(1), dim3(64), 0, 0, d_in, d_out + 8, d_t + 1, blocks);
    hipMemcpy(o2, d_out + 8, 64, hipMemcpyDeviceToHost); hipMemcpy(&t2, d_t + 1, 8, hipMemcpyDeviceToHost);
    printf("valu %lld  salu %lld  (s_memtime ticks, %d blocks) same=%d\n", t1, t2, blocks, memcmp(o1, o2, 64) == 0);
  }
  return 0;
}
