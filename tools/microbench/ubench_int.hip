// Microbenchmark: VALU throughput of the integer multiply forms usable for
// GF(2^255-19) limb arithmetic on gfx950 (decides the limb representation).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#ifndef NACC
#define NACC 8
#endif
#define ITERS 4096

template <int KIND>
__global__ __launch_bounds__(1024) void kbench(uint32_t* out, uint32_t seed) {
  uint32_t a = seed ^ threadIdx.x, b = seed * 3 + blockIdx.x;
  uint64_t acc[NACC];
  uint32_t acc32[NACC];
  double accd[NACC];
  float accf[NACC];
#pragma unroll
  for (int j = 0; j < NACC; ++j) { acc[j] = j + threadIdx.x; acc32[j] = j * 7 + threadIdx.x; accd[j] = j + 0.5 * threadIdx.x; accf[j] = j; }
  const uint64_t smask = __ballot(threadIdx.x & 1);
  if (KIND == 32) asm volatile("v_cmp_gt_u32 vcc, %0, %1" : : "v"(a), "v"(b) : "vcc");
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int j = 0; j < NACC; ++j) {
      if (KIND == 0) {  // v_mad_u64_u32
        uint64_t c;
        asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(acc[j]), "=s"(c) : "v"(a), "v"(b));
      } else if (KIND == 1) {  // v_mul_lo_u32
        asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(acc32[j]) : "v"(a));
      } else if (KIND == 2) {  // v_mul_hi_u32
        asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(acc32[j]) : "v"(a));
      } else if (KIND == 3) {  // v_mad_u32_u24
        asm volatile("v_mad_u32_u24 %0, %1, %2, %0" : "+v"(acc32[j]) : "v"(a), "v"(b));
      } else if (KIND == 4) {  // v_mul_hi_u32_u24
        asm volatile("v_mul_hi_u32_u24 %0, %0, %1" : "+v"(acc32[j]) : "v"(a));
      } else if (KIND == 5) {  // v_add_co_u32 (32-bit add w/ carry out)
        uint64_t c;
        asm volatile("v_add_co_u32 %0, %1, %0, %2" : "+v"(acc32[j]), "=s"(c) : "v"(a));
      } else if (KIND == 6) {  // v_fma_f64
        asm volatile("v_fma_f64 %0, %1, %2, %0" : "+v"(accd[j]) : "v"((double)a), "v"((double)b));
      } else if (KIND == 7) {  // v_fma_f32
        asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(accf[j]) : "v"((float)a), "v"((float)b));
      } else if (KIND == 8) {  // v_lshrrev_b64
        asm volatile("v_lshrrev_b64 %0, 3, %0" : "+v"(acc[j]));
      } else if (KIND == 9) {  // v_add_u32 (no carry)
        asm volatile("v_add_u32 %0, %0, %1" : "+v"(acc32[j]) : "v"(a));
      } else if (KIND == 10) { // v_lshl_add_u64 (gfx940+)
        asm volatile("v_lshl_add_u64 %0, %0, 1, %1" : "+v"(acc[j]) : "v"((uint64_t)a));
      } else if (KIND == 11) { // v_alignbit_b32
        asm volatile("v_alignbit_b32 %0, %0, %1, 7" : "+v"(acc32[j]) : "v"(a));
      } else if (KIND == 12) { // v_bfe_u32
        asm volatile("v_bfe_u32 %0, %0, 3, 26" : "+v"(acc32[j]));
      } else if (KIND == 13) { // v_mul_u32_u24
        asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(acc32[j]) : "v"(a));
      } else if (KIND == 14) { // v_lshl_add_u32
        asm volatile("v_lshl_add_u32 %0, %0, 4, %1" : "+v"(acc32[j]) : "v"(a));
      } else if (KIND == 15) { // v_and_b32
        asm volatile("v_and_b32 %0, %0, %1" : "+v"(acc32[j]) : "v"(a));
      } else if (KIND == 16) { // v_mov_b32
        asm volatile("v_mov_b32 %0, %1" : "=v"(acc32[j]) : "v"(acc32[(j + 1) % NACC]));
      } else if (KIND == 17) { // v_add_co_u32 + v_addc_co_u32 (64-bit add)
        asm volatile("v_add_co_u32 %0, vcc, %0, %1\n v_addc_co_u32 %2, vcc, %2, 0, vcc" : "+v"(acc32[j]), "+v"(b) : "v"(a) : "vcc");
      } else if (KIND == 18) { // v_mad_u32_u16
        asm volatile("v_mad_u32_u16 %0, %1, %2, %0" : "+v"(acc32[j]) : "v"(a), "v"(b));
      } else if (KIND == 19) { // v_bitop3_b32 (gfx950)
        asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(acc32[j]) : "v"(a), "v"(b));
      } else if (KIND == 20) { // v_cndmask_b32 on a VCC mask
        asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(acc32[j]) : "v"(a));
      } else if (KIND == 21) { // v_lshrrev_b32
        asm volatile("v_lshrrev_b32 %0, 7, %0" : "+v"(acc32[j]));
      } else if (KIND == 22) { // v_cndmask_b32_e64 on an SGPR-pair mask
        asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(acc32[j]) : "v"(a), "s"(smask));
      } else if (KIND == 23) { // v_cmp (vcc) + v_cndmask_b32_e32, as the compiler emits them
        asm volatile("v_cmp_gt_u32 vcc, %1, %2\n\tv_cndmask_b32_e32 %0, %0, %1, vcc" : "+v"(acc32[j]) : "v"(a), "v"(b) : "vcc");
      } else if (KIND == 24) { // v_cmp alone
        asm volatile("v_cmp_gt_u32 vcc, %0, %1" : : "v"(acc32[j]), "v"(b) : "vcc");
      } else if (KIND == 25) { // v_bfi_b32
        asm volatile("v_bfi_b32 %0, %1, %0, %2" : "+v"(acc32[j]) : "v"(a), "v"(b));
      } else if (KIND == 26) { // v_perm_b32
        asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(acc32[j]) : "v"(a), "v"(b));
      } else if (KIND == 27) { // v_sub_u32
        asm volatile("v_sub_u32 %0, %0, %1" : "+v"(acc32[j]) : "v"(a));
      } else if (KIND == 28) { // v_add3_u32
        asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(acc32[j]) : "v"(a), "v"(b));
      } else if (KIND == 29) { // v_lshlrev_b32
        asm volatile("v_lshlrev_b32 %0, 3, %0" : "+v"(acc32[j]));
      } else if (KIND == 30) { // v_ashrrev_i32
        asm volatile("v_ashrrev_i32 %0, 3, %0" : "+v"(acc32[j]));
      } else if (KIND == 31) { // v_bitop3_b32 as a select on a lane mask
        asm volatile("v_bitop3_b32 %0, %1, %0, %2 bitop3:0xca" : "+v"(acc32[j]) : "v"(a), "v"(b));
      } else if (KIND == 32) { // v_cndmask_b32_e32 with vcc set once per kernel by v_cmp
        asm volatile("v_cndmask_b32_e32 %0, %0, %1, vcc" : "+v"(acc32[j]) : "v"(a) : "vcc");
      } else if (KIND == 33) { // v_lshlrev_b64
        asm volatile("v_lshlrev_b64 %0, 3, %0" : "+v"(acc[j]));
      } else if (KIND == 34) { // v_mad_u64_u32 independent of acc chain: 2 accumulators interleaved
        uint64_t c;
        asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(acc[j]), "=s"(c) : "v"(acc32[j]), "v"(b));
      } else if (KIND == 35) { // v_mul_lo_u32 by constant 19 (as the compiler emits 19*g)
        asm volatile("v_mul_lo_u32 %0, %0, 19" : "+v"(acc32[j]));
      } else if (KIND == 36) { // v_sub_co_u32 + v_subb (64-bit sub)
        asm volatile("v_sub_co_u32 %0, vcc, %0, %1\n v_subb_co_u32 %2, vcc, %2, 0, vcc" : "+v"(acc32[j]), "+v"(b) : "v"(a) : "vcc");
      }
    }
  }
  uint32_t r = 0;
#pragma unroll
  for (int j = 0; j < NACC; ++j) r += (uint32_t)acc[j] + (uint32_t)(acc[j] >> 32) + acc32[j] + (uint32_t)accd[j] + (uint32_t)accf[j];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

template <int KIND>
static void run(const char* name, uint32_t* d, int blocks, int waves_per_block) {
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  int threads = 64 * waves_per_block;
  hipLaunchKernelGGL(kbench<KIND>, dim3(blocks), dim3(threads), 0, 0, d, 1u);
  hipDeviceSynchronize();
  hipEventRecord(e0);
  const int reps = 3;
  for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(kbench<KIND>, dim3(blocks), dim3(threads), 0, 0, d, 1u);
  hipEventRecord(e1); hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  double ops = (double)reps * blocks * threads * (double)ITERS * NACC;
  printf("%-20s blocks=%5d thr=%4d  %8.3f Gops/s (lane-ops)  = %.3f lane-ops/clk/CU @2.4GHz\n", name, blocks, threads,
         ops / (ms * 1e6), ops / (ms * 1e-3) / 256 / 2.4e9);
}

int main() {
  uint32_t* d; hipMalloc(&d, 256 * 8 * 1024 * sizeof(uint32_t) * 4);
  hipDeviceProp_t p; hipGetDeviceProperties(&p, 0);
  printf("device %s CUs=%d clock=%d kHz\n", p.gcnArchName, p.multiProcessorCount, p.clockRate);
  int blocks = 256 * 8;
  for (int w : {16}) {
    run<0>("v_mad_u64_u32", d, blocks, w);
    run<1>("v_mul_lo_u32", d, blocks, w);
    run<2>("v_mul_hi_u32", d, blocks, w);
    run<3>("v_mad_u32_u24", d, blocks, w);
    run<4>("v_mul_hi_u32_u24", d, blocks, w);
    run<13>("v_mul_u32_u24", d, blocks, w);
    run<5>("v_add_co_u32", d, blocks, w);
    run<9>("v_add_u32", d, blocks, w);
    run<6>("v_fma_f64", d, blocks, w);
    run<7>("v_fma_f32", d, blocks, w);
    run<8>("v_lshrrev_b64", d, blocks, w);
    run<10>("v_lshl_add_u64", d, blocks, w);
    run<11>("v_alignbit_b32", d, blocks, w);
    run<12>("v_bfe_u32", d, blocks, w);
    run<14>("v_lshl_add_u32", d, blocks, w);
    run<15>("v_and_b32", d, blocks, w);
    run<16>("v_mov_b32", d, blocks, w);
    run<17>("v_add_co+v_addc", d, blocks, w);
    run<19>("v_bitop3_b32", d, blocks, w);
    run<20>("v_cndmask_b32", d, blocks, w);
    run<21>("v_lshrrev_b32", d, blocks, w);
    run<22>("v_cndmask_e64 smask", d, blocks, w);
    run<23>("v_cmp+v_cndmask_e32", d, blocks, w);
    run<24>("v_cmp (vcc)", d, blocks, w);
    run<25>("v_bfi_b32", d, blocks, w);
    run<26>("v_perm_b32", d, blocks, w);
    run<27>("v_sub_u32", d, blocks, w);
    run<28>("v_add3_u32", d, blocks, w);
    run<29>("v_lshlrev_b32", d, blocks, w);
    run<30>("v_ashrrev_i32", d, blocks, w);
    run<31>("v_bitop3 select", d, blocks, w);
    run<32>("v_cndmask_e32 vcc set", d, blocks, w);
    run<33>("v_lshlrev_b64", d, blocks, w);
    run<34>("v_mad_u64_u32 var a", d, blocks, w);
    run<35>("v_mul_lo_u32 x19", d, blocks, w);
    run<36>("v_sub_co+v_subb", d, blocks, w);
  }
  hipFree(d);
  return 0;
}
