// Microbenchmark (development): issue cost of the compare forms the chroma
// kernel's fast path could use on gfx950 -- VOPC e32 into VCC, VOP3 (e64)
// into an SGPR pair, SDWA byte compares -- each paired with an independent
// v_add_u32 (2.7 cycles alone) in 8 chains per lane, 4 waves per SIMD.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define ITERS 4096
#define DEF(NAME, ASM)                                                                            \
  __global__ __launch_bounds__(256) void NAME(uint32_t* out, uint32_t seed) {                     \
    uint32_t v0 = seed + threadIdx.x, v1 = v0 * 3, v2 = v0 * 5, v3 = v0 * 7, v4 = v0 * 11,          \
             v5 = v0 * 13, v6 = v0 * 17, v7 = v0 * 19, k = seed | 1;                               \
    for (int i = 0; i < ITERS; ++i) {                                                             \
      asm volatile(ASM : "+v"(v0) : "v"(k) : "vcc", "s4", "s5"); asm volatile(ASM : "+v"(v1) : "v"(k) : "vcc", "s4", "s5"); \
      asm volatile(ASM : "+v"(v2) : "v"(k) : "vcc", "s4", "s5"); asm volatile(ASM : "+v"(v3) : "v"(k) : "vcc", "s4", "s5"); \
      asm volatile(ASM : "+v"(v4) : "v"(k) : "vcc", "s4", "s5"); asm volatile(ASM : "+v"(v5) : "v"(k) : "vcc", "s4", "s5"); \
      asm volatile(ASM : "+v"(v6) : "v"(k) : "vcc", "s4", "s5"); asm volatile(ASM : "+v"(v7) : "v"(k) : "vcc", "s4", "s5"); \
    }                                                                                             \
    out[blockIdx.x * blockDim.x + threadIdx.x] = v0 ^ v1 ^ v2 ^ v3 ^ v4 ^ v5 ^ v6 ^ v7;           \
  }

DEF(k_add, "v_add_u32 %0, %0, %1")
DEF(k_cmp32, "v_cmp_eq_u32_e32 vcc, %0, %1\n v_add_u32 %0, %0, %1")
DEF(k_cmp64, "v_cmp_eq_u32_e64 s[4:5], %0, %1\n v_add_u32 %0, %0, %1")
DEF(k_cmpsdwa, "v_cmp_gt_u32_sdwa s[4:5], %0, %1 src0_sel:BYTE_0 src1_sel:BYTE_2\n v_add_u32 %0, %0, %1")
DEF(k_cmpsdwa_vcc, "v_cmp_gt_u32_sdwa vcc, %0, %1 src0_sel:BYTE_0 src1_sel:BYTE_2\n v_add_u32 %0, %0, %1")
DEF(k_cnd64, "v_cndmask_b32_e64 %0, %0, %1, s[4:5]\n v_add_u32 %0, %0, %1")
DEF(k_cnd32, "s_mov_b64 vcc, -1\n v_cndmask_b32_e32 %0, %0, %1, vcc\n v_add_u32 %0, %0, %1")
DEF(k_lshr, "v_lshrrev_b32 %0, 7, %0\n v_add_u32 %0, %0, %1")
DEF(k_lshl, "v_lshlrev_b32 %0, 1, %0\n v_add_u32 %0, %0, %1")

template <typename K>
void run(const char* name, K k, int instrs) {
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  uint32_t* out;
  (void)hipMalloc(&out, sizeof(uint32_t) * 256 * cus * 4);
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  hipLaunchKernelGGL(k, dim3(cus * 4), dim3(256), 0, 0, out, 7u);
  float best = 1e9;
  for (int r = 0; r < 5; ++r) {
    (void)hipEventRecord(a);
    hipLaunchKernelGGL(k, dim3(cus * 4), dim3(256), 0, 0, out, 7u);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms;
    (void)hipEventElapsedTime(&ms, a, b);
    if (ms < best) best = ms;
  }
  // 4 waves per SIMD (cus*4 workgroups of 4 waves over cus*4 SIMDs); per SIMD:
  // 4 waves x 8 chains x ITERS x instrs wave-instructions
  const double cycles = best * 1e-3 * 2.4e9, n = 4.0 * 8 * ITERS * instrs;
  printf("%-16s %.2f cycles per wave-instruction (%d per asm)\n", name, cycles / n, instrs);
  (void)hipFree(out);
}

int main() {
  run("v_add_u32", k_add, 1);
  run("cmp_e32+add", k_cmp32, 2);
  run("cmp_e64+add", k_cmp64, 2);
  run("cmp_sdwa+add", k_cmpsdwa, 2);
  run("cmp_sdwa_vcc+add", k_cmpsdwa_vcc, 2);
  run("cnd_e64+add", k_cnd64, 2);
  run("lshr+add", k_lshr, 2);
  run("lshl+add", k_lshl, 2);
  return 0;
}
