// Probe: the int16 -> [0,255] clamp sequences over all 65536 low-half inputs.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
__global__ void k(uint32_t* out) {
  const uint32_t x = blockIdx.x * blockDim.x + threadIdx.x;  // 0..65535
  const uint32_t s = x | 0xABCD0000u;                          // garbage high half
  uint32_t a, b, c, d, e;
  asm volatile("v_ashrrev_i16 %0, 6, %1" : "=v"(a) : "v"(s));
  asm volatile("v_max_i16 %0, 0, %1\n\tv_min_i16 %0, 0xff, %0" : "=&v"(b) : "v"(x));
  asm volatile("v_max_i16 %0, 0, %1" : "=v"(c) : "v"(x));
  asm volatile("v_min_i16 %0, 0xff, %1" : "=v"(d) : "v"(x));
  const uint32_t k255 = 255;
  asm volatile("v_min_i16 %0, %2, %1" : "=v"(e) : "v"(x), "v"(k255));
  out[5 * x + 0] = a; out[5 * x + 1] = b; out[5 * x + 2] = c; out[5 * x + 3] = d; out[5 * x + 4] = e;
}
int main() {
  uint32_t* dv; hipMalloc(&dv, 65536 * 5 * 4);
  hipLaunchKernelGGL(k, dim3(256), dim3(256), 0, 0, dv);
  static uint32_t h[65536 * 5]; hipMemcpy(h, dv, sizeof(h), hipMemcpyDeviceToHost);
  int bad[5] = {0}; int first[5] = {-1, -1, -1, -1, -1};
  for (int x = 0; x < 65536; ++x) {
    const int v = (int16_t)x;
    const uint32_t want[5] = {(uint32_t)(uint16_t)(int16_t)(v >> 6), (uint32_t)(v < 0 ? 0 : v > 255 ? 255 : v),
                              (uint32_t)(uint16_t)(int16_t)(v < 0 ? 0 : v), (uint32_t)(uint16_t)(int16_t)(v > 255 ? 255 : v),
                              (uint32_t)(uint16_t)(int16_t)(v > 255 ? 255 : v)};
    for (int i = 0; i < 5; ++i) if (h[5 * x + i] != want[i]) { if (first[i] < 0) first[i] = x; ++bad[i]; }
  }
  const char* n[] = {"ashrrev_i16 6", "max0;min0xff", "max_i16 0", "min_i16 0xff (literal)", "min_i16 vgpr255"};
  for (int i = 0; i < 5; ++i) printf("%-24s bad=%d first=%d got=0x%08x\n", n[i], bad[i], first[i], first[i] >= 0 ? h[5 * first[i] + i] : 0);
  return 0;
}
