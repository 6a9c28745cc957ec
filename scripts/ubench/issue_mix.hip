// Microbenchmark: does SALU issue share the SIMD's issue bandwidth with VALU?
// Cycles per loop iteration per SIMD at 1/2/4 waves per SIMD for
//   valu8      8 independent v_add_u32
//   salu8      8 independent s_add_u32
//   mix8_8     the two interleaved (8 + 8)
//   cmpsel     the chroma kernel's select shape: 5 VOPC to SGPR pairs, 5 SALU
//              combines, 4 v_cndmask_b32_e64
// build: hipcc -O3 --offload-arch=gfx950 -o issue_mix issue_mix.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define ITERS 4096

__global__ __launch_bounds__(256) void valu8(uint32_t* out, uint32_t seed) {
  uint32_t a = seed + threadIdx.x, b = a * 3, c = a * 5, d = a * 7, e = a * 9, f = a * 11, g = a * 13, h = a * 15;
  for (int i = 0; i < ITERS; ++i) {
    asm volatile(
        "v_add_u32 %0, %0, %8\n\tv_add_u32 %1, %1, %8\n\tv_add_u32 %2, %2, %8\n\tv_add_u32 %3, %3, %8\n\t"
        "v_add_u32 %4, %4, %8\n\tv_add_u32 %5, %5, %8\n\tv_add_u32 %6, %6, %8\n\tv_add_u32 %7, %7, %8"
        : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+v"(e), "+v"(f), "+v"(g), "+v"(h)
        : "v"(seed));
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a ^ b ^ c ^ d ^ e ^ f ^ g ^ h;
}

__global__ __launch_bounds__(256) void salu8(uint32_t* out, uint32_t seed) {
  uint32_t a = seed, b = seed * 3, c = seed * 5, d = seed * 7, e = seed * 9, f = seed * 11, g = seed * 13, h = seed * 15;
  for (int i = 0; i < ITERS; ++i) {
    asm volatile(
        "s_add_u32 %0, %0, %8\n\ts_add_u32 %1, %1, %8\n\ts_add_u32 %2, %2, %8\n\ts_add_u32 %3, %3, %8\n\t"
        "s_add_u32 %4, %4, %8\n\ts_add_u32 %5, %5, %8\n\ts_add_u32 %6, %6, %8\n\ts_add_u32 %7, %7, %8"
        : "+s"(a), "+s"(b), "+s"(c), "+s"(d), "+s"(e), "+s"(f), "+s"(g), "+s"(h)
        : "s"(seed)
        : "scc");
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a ^ b ^ c ^ d ^ e ^ f ^ g ^ h;
}

__global__ __launch_bounds__(256) void mix8_8(uint32_t* out, uint32_t seed) {
  uint32_t a = seed + threadIdx.x, b = a * 3, c = a * 5, d = a * 7;
  uint32_t sa = seed, sb = seed * 3, sc = seed * 5, sd = seed * 7;
  for (int i = 0; i < ITERS; ++i) {
    asm volatile(
        "v_add_u32 %0, %0, %8\n\ts_add_u32 %4, %4, %9\n\tv_add_u32 %1, %1, %8\n\ts_add_u32 %5, %5, %9\n\t"
        "v_add_u32 %2, %2, %8\n\ts_add_u32 %6, %6, %9\n\tv_add_u32 %3, %3, %8\n\ts_add_u32 %7, %7, %9\n\t"
        "v_add_u32 %0, %0, %8\n\ts_add_u32 %4, %4, %9\n\tv_add_u32 %1, %1, %8\n\ts_add_u32 %5, %5, %9\n\t"
        "v_add_u32 %2, %2, %8\n\ts_add_u32 %6, %6, %9\n\tv_add_u32 %3, %3, %8\n\ts_add_u32 %7, %7, %9"
        : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+s"(sa), "+s"(sb), "+s"(sc), "+s"(sd)
        : "v"(seed), "s"(seed)
        : "scc");
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a ^ b ^ c ^ d ^ sa ^ sb ^ sc ^ sd;
}

__global__ __launch_bounds__(256) void cmpsel(uint32_t* out, uint32_t seed) {
  uint32_t w = seed * 0x9E3779B9u + threadIdx.x * 0x85EBCA6Bu, dd = w ^ 0x5bd1e995u, m1 = w * 7, m2 = w * 13;
  uint32_t e0 = 0, e1 = 0;
  for (int i = 0; i < ITERS; ++i) {
    uint64_t x, lt0, lt1, le0, le1, k0, k1;
    asm volatile(
        "v_cmp_eq_u32_e64 %[x], %[k], %[d]\n\t"
        "v_cmp_gt_u32_sdwa %[lt0], %[d], %[w] src0_sel:BYTE_0 src1_sel:BYTE_0\n\t"
        "v_cmp_gt_u32_sdwa %[lt1], %[d], %[w] src0_sel:BYTE_0 src1_sel:BYTE_2\n\t"
        "v_cmp_ge_u32_sdwa %[le0], %[d], %[w] src0_sel:BYTE_1 src1_sel:BYTE_0\n\t"
        "v_cmp_ge_u32_sdwa %[le1], %[d], %[w] src0_sel:BYTE_1 src1_sel:BYTE_2\n\t"
        "s_andn2_b64 %[k0], %[le0], %[x]\n\t"
        "s_andn2_b64 %[k1], %[le1], %[x]\n\t"
        "s_andn2_b64 %[le0], %[lt0], %[le0]\n\t"
        "s_andn2_b64 %[le1], %[lt1], %[le1]\n\t"
        "s_or_b64 %[x], %[le0], %[le1]\n\t"
        "v_cndmask_b32_e64 %[e0], %[m2], %[m1], %[lt0]\n\t"
        "v_cndmask_b32_e64 %[e1], %[m2], %[m1], %[lt1]\n\t"
        "v_cndmask_b32_e64 %[e0], 0, %[e0], %[k0]\n\t"
        "v_cndmask_b32_e64 %[e1], 0, %[e1], %[k1]\n\t"
        "v_add_u32 %[w], %[w], %[e0]"
        : [x] "=&s"(x), [lt0] "=&s"(lt0), [lt1] "=&s"(lt1), [le0] "=&s"(le0), [le1] "=&s"(le1), [k0] "=&s"(k0),
          [k1] "=&s"(k1), [e0] "=&v"(e0), [e1] "=&v"(e1), [w] "+v"(w)
        : [d] "v"(dd), [m1] "v"(m1), [m2] "v"(m2), [k] "s"(0xFFu)
        : "scc");
    dd += e1;
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = w ^ dd;
}

template <typename K>
void run(const char* name, K kern, double instr_per_iter, int cus, int clk, uint32_t* out) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int w : {1, 2, 4, 8}) {
    const int blocks = cus * w;  // 256 threads = 4 waves = one per SIMD
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, out, 7u);
    hipEventRecord(a);
    for (int r = 0; r < 3; ++r) hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, out, 7u);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    const double iters = 3.0 * w * ITERS;  // per SIMD
    const double cyc = ms * 1e-3 * clk * 1e3 / iters;
    printf("%-8s waves/SIMD=%d : %.2f cycles/iter per SIMD (%.2f per instruction)\n", name, w, cyc,
           cyc / instr_per_iter);
  }
}

int main() {
  int cus = 0, clk = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, 0);
  uint32_t* out;
  hipMalloc(&out, 1 << 26);
  printf("CUs=%d clock=%d kHz\n", cus, clk);
  run("valu8", valu8, 8, cus, clk, out);
  run("salu8", salu8, 8, cus, clk, out);
  run("mix8_8", mix8_8, 16, cus, clk, out);
  run("cmpsel", cmpsel, 15, cus, clk, out);
  return 0;
}
