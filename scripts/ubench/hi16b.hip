// Probe: a 32-bit VALU read issued right after a 16-bit VOP2 write of the same
// VGPR (whose bits 31:16 held garbage).  Compare with nop-separated variants.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
__global__ void k(uint32_t* out, uint32_t a, uint32_t b) {
  uint32_t r0, r1, r2, r3, r4;
  // back-to-back: 16-bit write then 32-bit add reading it
  asm volatile("v_mov_b32 %0, 0xdead1234\n\tv_max_u16 %0, %1, %2\n\tv_add_u32 %0, 0, %0" : "=&v"(r0) : "v"(a), "v"(b));
  asm volatile("v_mov_b32 %0, 0xdead1234\n\tv_max_u16 %0, %1, %2\n\ts_nop 4\n\tv_add_u32 %0, 0, %0" : "=&v"(r1) : "v"(a), "v"(b));
  asm volatile("v_mov_b32 %0, 0xdead1234\n\tv_max_u16 %0, %1, %2\n\tv_lshrrev_b32 %0, 16, %0" : "=&v"(r2) : "v"(a), "v"(b));
  asm volatile("v_mov_b32 %0, 0xdead1234\n\tv_max_u16 %0, %1, %2\n\ts_nop 4\n\tv_lshrrev_b32 %0, 16, %0" : "=&v"(r3) : "v"(a), "v"(b));
  asm volatile("v_mov_b32 %0, 0xdead1234\n\tv_sub_u16 %0, %1, %2\n\tv_cmp_eq_u32 vcc, %0, %1\n\tv_cndmask_b32 %0, 1, 2, vcc" : "=&v"(r4) : "v"(a), "v"(b) : "vcc");
  out[0] = r0; out[1] = r1; out[2] = r2; out[3] = r3; out[4] = r4;
}
int main() {
  uint32_t* d; hipMalloc(&d, 64 * 4);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, 0x00000005u, 0x00000003u);
  uint32_t h[8]; hipMemcpy(h, d, 5 * 4, hipMemcpyDeviceToHost);
  const char* n[] = {"max16;add32 (b2b)", "max16;nop;add32", "max16;lshr16 (b2b)", "max16;nop;lshr16", "sub16;cmp32==a(5-3=2 vs 5 ->2)"};
  for (int i = 0; i < 5; ++i) printf("%-32s -> 0x%08x\n", n[i], h[i]);
  return 0;
}
