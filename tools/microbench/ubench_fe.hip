// Microbenchmark: throughput of the radix-2^25.5 field multiply / square
// (indy-plenum_amd/csrc/fe25519.h) on gfx950, in field ops per second.
#include <hip/hip_runtime.h>
#include <cstdio>
#include "../../indy-plenum_amd/csrc/fe25519.h"
using namespace edv;

template <int SQ>
__global__ __launch_bounds__(256) void kfe(uint32_t* out, int iters) {
  fe a, b;
  for (int k = 0; k < 10; ++k) { a.v[k] = (threadIdx.x * 7919u + k * 104729u) & 0x1ffffff; b.v[k] = (blockIdx.x * 31u + k * 17u) & 0x1ffffff; }
  fe c = a, d = b;
  for (int it = 0; it < iters; ++it) {
    if (SQ) { fe_sq(a, a); fe_sq(c, c); }
    else { fe_mul(a, a, b); fe_mul(c, c, d); }
  }
  uint32_t r = 0;
  for (int k = 0; k < 10; ++k) r += a.v[k] ^ c.v[k];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

template <int SQ>
static void run(const char* name, uint32_t* d, int blocks) {
  hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
  const int iters = 2000;
  hipLaunchKernelGGL(kfe<SQ>, dim3(blocks), dim3(256), 0, 0, d, iters);
  (void)hipDeviceSynchronize();
  (void)hipEventRecord(e0);
  hipLaunchKernelGGL(kfe<SQ>, dim3(blocks), dim3(256), 0, 0, d, iters);
  (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
  float ms; (void)hipEventElapsedTime(&ms, e0, e1);
  double ops = 2.0 * blocks * 256.0 * iters;
  printf("%-8s blocks=%5d  %9.2f G fe-ops/s  (%.1f instr-slots equiv: %.1f M verifies/s @3050 ops)\n", name, blocks,
         ops / ms / 1e6, 0.0, ops / (ms * 1e-3) / 3050 / 1e6);
}
int main() {
  uint32_t* d; (void)hipMalloc(&d, 256 * 8192 * 4);
  for (int b : {1024, 2048, 4096, 8192}) { run<0>("fe_mul", d, b); run<1>("fe_sq", d, b); }
  return 0;
}
