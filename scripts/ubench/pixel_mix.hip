// Microbenchmark: VALU throughput of the per-pixel phase-1 math in two
// formulations, no memory traffic: (a) compiler-generated 32-bit ops (v_dot4,
// v_bfe, v_med3, v_max3, v_cmp/v_cndmask), (b) the hand-ordered 16-bit asm
// block of trik_hsv_stripe.hip.  1024-thread blocks, one per CU (4 waves/SIMD),
// as in the hot kernel.  Prints ns per pixel-slot per CU and VALU instr count.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#define ITERS 4096
#include "../../trik-media-sensors-dsp_amd/csrc/trik_hsv_internal.h"
using namespace trik_hsv;
#include "phase1.inc"

__device__ __forceinline__ uint32_t cl8(uint32_t s) { return (uint32_t)min(max(((int)(s << 16)) >> 22, 0), 255); }
__device__ __forceinline__ void phase1_c(uint32_t w, uint32_t lane, Phase1& p0, Phase1& p1) {
  const uint32_t wc = w ^ 0xFF00FF00u;
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const uint32_t kY = j ? (74u << 16) : 74u;
    const uint32_t r = cl8(__builtin_amdgcn_udot4(w, kY | (102u << 24), (uint32_t)-14248, false));
    const uint32_t g = cl8(__builtin_amdgcn_udot4(wc, kY | (25u << 8) | (52u << 24), (uint32_t)-10939, false));
    const uint32_t b = cl8(__builtin_amdgcn_udot4(w, kY | (129u << 8), (uint32_t)-17672, false));
    const uint32_t mx = max(r, max(g, b)), mn = min(r, min(g, b));
    Phase1& p = j ? p1 : p0;
    p.m43_addr = ((mx - mn) << 8) + lane;
    p.sv_addr = __umul24(mx, 260u) + mn;
    uint32_t c = mx == b ? ((r - g) & 0xFFFF) | (43690u << 16) : ((g - b) & 0xFFFF);
    p.c = mx == g ? ((b - r) & 0xFFFF) | (21845u << 16) : c;
  }
}
template <int V>
__global__ __launch_bounds__(1024) void k(uint32_t* out, uint32_t seed) {
  uint32_t w = seed * (threadIdx.x + 1), acc = 0;
  const uint32_t lane = threadIdx.x & 31;
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      Phase1 p0, p1;
      const uint32_t wq = w + q * 0x01010101u;
      if (V == 0) phase1_c(wq, lane, p0, p1); else phase1_word(wq, lane, p0, p1);
      acc += p0.m43_addr ^ p0.sv_addr ^ p0.c ^ p1.m43_addr ^ p1.sv_addr ^ p1.c;
    }
    w += 0x9E3779B9u;
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}
int main() {
  int cus = 0; hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  uint32_t* out; hipMalloc(&out, 1 << 24);
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  for (int v = 0; v < 2; ++v) {
    auto kern = v ? k<1> : k<0>;
    hipLaunchKernelGGL(kern, dim3(cus), dim3(1024), 0, 0, out, 7u);
    hipEventRecord(a);
    for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(kern, dim3(cus), dim3(1024), 0, 0, out, 7u);
    hipEventRecord(b); hipEventSynchronize(b);
    float ms = 0; hipEventElapsedTime(&ms, a, b);
    const double px_per_cu = 5.0 * 1024 * ITERS * 8;  // pixels through one CU
    printf("%s: %.3f ns per 1024 pixels per CU -> %.2f px/clk/CU at 2.4 GHz\n", v ? "asm16" : "c32  ",
           ms * 1e6 / (px_per_cu / 1024), px_per_cu / (ms * 1e-3 * 2.4e9));
  }
  return 0;
}
