// Microbenchmark: VALU issue rate vs waves per SIMD and dependency chains.
// Cycles per wave64 instruction per SIMD, for full-rate (v_add_u32, v_max_u16)
// and half-rate (v_dot4, v_cndmask) ops, and a 1:1 mix, at 1/2/4/8 waves per
// SIMD with 1, 2 or 8 independent chains per wave.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define ITERS 2048
template <int CH>
struct Ch { uint32_t v[CH]; };

#define DEFK(NAME, ASM, NI)                                                        \
  template <int CH>                                                                \
  __global__ __launch_bounds__(256) void NAME(uint32_t* out, uint32_t seed) {      \
    uint32_t v[CH];                                                                \
    _Pragma("unroll") for (int c = 0; c < CH; ++c) v[c] = seed * (c + 3) + threadIdx.x; \
    const uint32_t k = seed | 1;                                                   \
    for (int i = 0; i < ITERS * 8 / CH; ++i) {                                     \
      _Pragma("unroll") for (int c = 0; c < CH; ++c) asm volatile(ASM : "+v"(v[c]) : "v"(k) : "vcc"); \
    }                                                                              \
    uint32_t x = 0;                                                                \
    _Pragma("unroll") for (int c = 0; c < CH; ++c) x ^= v[c];                      \
    out[blockIdx.x * blockDim.x + threadIdx.x] = x;                                \
  }                                                                                \
  constexpr int NAME##_ni = NI;

DEFK(k_add, "v_add_u32 %0, %0, %1", 1)
DEFK(k_max16, "v_max_u16 %0, %0, %1", 1)
DEFK(k_dot4, "v_dot4_u32_u8 %0, %0, %1, %0", 1)
DEFK(k_mix, "v_add_u32 %0, %0, %1\n\tv_max3_u32 %0, %0, %1, %0", 2)
DEFK(k_mix16, "v_max_u16 %0, %0, %1\n\tv_sub_u16 %0, %0, %1\n\tv_mad_u32_u24 %0, %0, %1, %0", 3)
DEFK(k_cmpcnd, "v_cmp_eq_u32 vcc, %0, %1\n\tv_cndmask_b32 %0, %0, %1, vcc", 2)

template <int CH, typename K>
void run(const char* name, K kern, int ni, int cus, int clk, uint32_t* out) {
  hipEvent_t a, b;
  hipEventCreate(&a); hipEventCreate(&b);
  for (int w : {1, 2, 4, 8}) {
    const int blocks = cus * w;  // 256 threads = 4 waves = one per SIMD
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, out, 7u);
    hipEventRecord(a);
    for (int r = 0; r < 3; ++r) hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, out, 7u);
    hipEventRecord(b); hipEventSynchronize(b);
    float ms = 0; hipEventElapsedTime(&ms, a, b);
    const double instr = 3.0 * w * ITERS * 8 * ni;  // per SIMD
    printf("%-10s chains=%d waves/SIMD=%d : %.2f cycles/instr\n", name, CH, w, ms * 1e-3 * clk * 1e3 / instr);
  }
}
#define RUN(K) run<1>(#K, K<1>, K##_ni, cus, clk, out); run<2>(#K, K<2>, K##_ni, cus, clk, out); run<8>(#K, K<8>, K##_ni, cus, clk, out);
int main() {
  int cus = 0, clk = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, 0);
  uint32_t* out; hipMalloc(&out, 1 << 26);
  printf("CUs=%d clock=%d kHz\n", cus, clk);
  RUN(k_add) RUN(k_max16) RUN(k_dot4) RUN(k_mix) RUN(k_mix16) RUN(k_cmpcnd)
  return 0;
}
