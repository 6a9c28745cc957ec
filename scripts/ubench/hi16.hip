// Probe: what do 16-bit VOP2 ops write to bits 31:16 of the destination on
// gfx950?  dest is preset to 0xDEAD0000 | 0x1234 and must not be an input.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#define PROBE(i, ins) { uint32_t d = 0xDEAD1234u; asm volatile(ins : "+v"(d) : "v"(a), "v"(b)); out[i] = d; }
__global__ void k(uint32_t* out, uint32_t a, uint32_t b) {
  PROBE(0, "v_add_u16 %0, %1, %2")
  PROBE(1, "v_sub_u16 %0, %1, %2")
  PROBE(2, "v_ashrrev_i16 %0, 6, %1")
  PROBE(3, "v_max_i16 %0, %1, %2")
  PROBE(4, "v_min_u16 %0, %1, %2")
  PROBE(5, "v_mul_lo_u16 %0, %1, %2")
  PROBE(6, "v_lshrrev_b16 %0, 1, %1")
  PROBE(7, "v_lshlrev_b16 %0, 7, %1")
  PROBE(8, "v_max_u16 %0, %1, %2")
  PROBE(9, "v_add_u16_e64 %0, %1, %2")
  PROBE(10, "v_mad_u32_u24 %0, %1, %2, 0")
}
int main() {
  uint32_t* d; hipMalloc(&d, 64 * 4);
  hipLaunchKernelGGL(k, dim3(1), dim3(1), 0, 0, d, 0xAAAA0105u, 0x55550203u);
  uint32_t h[16]; hipMemcpy(h, d, 11 * 4, hipMemcpyDeviceToHost);
  const char* n[] = {"add_u16", "sub_u16", "ashrrev_i16", "max_i16", "min_u16", "mul_lo_u16", "lshrrev_b16", "lshlrev_b16", "max_u16", "add_u16_e64", "mad_u32_u24"};
  for (int i = 0; i < 11; ++i) printf("%-12s -> 0x%08x\n", n[i], h[i]);
  return 0;
}
