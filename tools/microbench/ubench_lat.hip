// Microbenchmark: dependent-issue latency of v_mad_u64_u32 chains on gfx950.
// Each lane runs CH interleaved serial chains (acc_c = acc_c + a*b); the
// launch puts WPS waves on every SIMD.  Throughput at CH = 1 and few waves
// shows the latency; CH = 2/4 shows what interleaving independent chains buys.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#define ITERS 8192

template <int CH>
__global__ void kchain(uint32_t* out, uint32_t seed) {
  uint32_t a = seed ^ threadIdx.x, b = seed * 3 + blockIdx.x;
  uint64_t acc[CH];
#pragma unroll
  for (int c = 0; c < CH; ++c) acc[c] = c + threadIdx.x;
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      uint64_t co;
      asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(acc[c]), "=s"(co) : "v"(a), "v"(b));
    }
  }
  uint32_t r = 0;
#pragma unroll
  for (int c = 0; c < CH; ++c) r += (uint32_t)acc[c] + (uint32_t)(acc[c] >> 32);
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

template <int CH>
static void run(uint32_t* d, int wps) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const int threads = 256;  // 4 waves per workgroup (one per SIMD), wps workgroups per CU
  const int blocks = 256 * wps;
  hipLaunchKernelGGL(kchain<CH>, dim3(blocks), dim3(threads), 0, 0, d, 1u);
  (void)hipDeviceSynchronize();
  (void)hipEventRecord(e0);
  for (int r = 0; r < 3; ++r) hipLaunchKernelGGL(kchain<CH>, dim3(blocks), dim3(threads), 0, 0, d, 1u);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms;
  (void)hipEventElapsedTime(&ms, e0, e1);
  const double ops = 3.0 * blocks * threads * (double)ITERS * CH;
  const double per_simd_cycles = ms * 1e-3 * 2.4e9 / (3.0 * ITERS * CH * wps);  // SIMD cycles per wave-MAD
  printf("chains=%d waves/SIMD=%2d  %.3f lane-ops/clk/CU  (%.2f SIMD cycles per wave-MAD @2.4GHz)\n", CH, wps,
         ops / (ms * 1e-3) / 256 / 2.4e9, per_simd_cycles);
}

int main() {
  uint32_t* d;
  (void)hipMalloc(&d, 256 * 1024 * sizeof(uint32_t));
  for (int wps : {1, 2, 3, 4, 5, 8}) {
    run<1>(d, wps);
    run<2>(d, wps);
    run<4>(d, wps);
  }
  (void)hipFree(d);
  return 0;
}
