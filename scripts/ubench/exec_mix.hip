// Microbenchmark (development only): the per-word select of the chroma-run
// kernel in three shapes, cycles per loop iteration per SIMD at 1/2/4/8 waves
// per SIMD:
//   sel_cnd   4 v_cndmask_b32 + 1.5 v_add3 (the shipped form: e0/e1 selected,
//             then added into the pair counter and the odd counter)
//   sel_exec  the same sums by EXEC-narrowed v_add_u32 (4 EXEC writes, 6 adds)
//   salu16    16 independent s_add_u32 (SALU issue capacity per CU)
//   cmp6      6 SDWA v_cmp into SGPR pairs + 6 SALU combines (the compares)
// build: hipcc -O3 --offload-arch=gfx950 -o exec_mix exec_mix.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define ITERS 4096

__global__ __launch_bounds__(256) void sel_cnd(uint32_t* out, uint32_t seed) {
  const uint32_t m1 = seed * 7 + threadIdx.x, m2 = seed * 13 + threadIdx.x;
  uint32_t p0 = 0, p1 = 0, o = 0, e0 = 0, e1 = 0;
  const uint64_t a = 0x5555aaaa3333ccccull * seed, b = ~a, c = a ^ 0x0f0f0f0f0f0f0f0full, d = a >> 3;
  for (int i = 0; i < ITERS; ++i) {
    asm volatile(
        "v_cndmask_b32_e64 %[e0], %[m2], %[m1], %[a]\n\t"
        "v_cndmask_b32_e64 %[e1], %[m2], %[m1], %[b]\n\t"
        "v_cndmask_b32_e64 %[e0], 0, %[e0], %[c]\n\t"
        "v_cndmask_b32_e64 %[e1], 0, %[e1], %[d]\n\t"
        "v_add3_u32 %[p0], %[p0], %[e0], %[e1]\n\t"
        "v_cndmask_b32_e64 %[e0], %[m2], %[m1], %[c]\n\t"
        "v_cndmask_b32_e64 %[e1], %[m2], %[m1], %[d]\n\t"
        "v_cndmask_b32_e64 %[e0], 0, %[e0], %[a]\n\t"
        "v_cndmask_b32_e64 %[e1], 0, %[e1], %[b]\n\t"
        "v_add3_u32 %[p1], %[p1], %[e0], %[e1]\n\t"
        "v_add3_u32 %[o], %[o], %[e0], %[e1]"
        : [p0] "+v"(p0), [p1] "+v"(p1), [o] "+v"(o), [e0] "=&v"(e0), [e1] "=&v"(e1)
        : [m1] "v"(m1), [m2] "v"(m2), [a] "s"(a), [b] "s"(b), [c] "s"(c), [d] "s"(d));
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = p0 ^ p1 ^ o;
}

__global__ __launch_bounds__(256) void sel_exec(uint32_t* out, uint32_t seed) {
  const uint32_t m1 = seed * 7 + threadIdx.x, m2 = seed * 13 + threadIdx.x;
  uint32_t p0 = 0, p1 = 0, o = 0;
  const uint64_t a = 0x5555aaaa3333ccccull * seed, b = ~a, c = a ^ 0x0f0f0f0f0f0f0f0full, d = a >> 3;
  for (int i = 0; i < ITERS; ++i) {
    uint64_t sv;
    asm volatile(
        "s_mov_b64 %[sv], exec\n\t"
        "s_mov_b64 exec, %[a]\n\t"
        "v_add_u32 %[p0], %[p0], %[m1]\n\t"
        "s_mov_b64 exec, %[b]\n\t"
        "v_add_u32 %[p0], %[p0], %[m2]\n\t"
        "s_mov_b64 exec, %[c]\n\t"
        "v_add_u32 %[p0], %[p0], %[m1]\n\t"
        "v_add_u32 %[o], %[o], %[m1]\n\t"
        "s_mov_b64 exec, %[d]\n\t"
        "v_add_u32 %[p0], %[p0], %[m2]\n\t"
        "v_add_u32 %[o], %[o], %[m2]\n\t"
        "s_mov_b64 exec, %[c]\n\t"
        "v_add_u32 %[p1], %[p1], %[m1]\n\t"
        "s_mov_b64 exec, %[d]\n\t"
        "v_add_u32 %[p1], %[p1], %[m2]\n\t"
        "s_mov_b64 exec, %[a]\n\t"
        "v_add_u32 %[p1], %[p1], %[m1]\n\t"
        "v_add_u32 %[o], %[o], %[m1]\n\t"
        "s_mov_b64 exec, %[b]\n\t"
        "v_add_u32 %[p1], %[p1], %[m2]\n\t"
        "v_add_u32 %[o], %[o], %[m2]\n\t"
        "s_mov_b64 exec, %[sv]"
        : [p0] "+v"(p0), [p1] "+v"(p1), [o] "+v"(o), [sv] "=&s"(sv)
        : [m1] "v"(m1), [m2] "v"(m2), [a] "s"(a), [b] "s"(b), [c] "s"(c), [d] "s"(d));
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = p0 ^ p1 ^ o;
}

__global__ __launch_bounds__(256) void salu16(uint32_t* out, uint32_t seed) {
  uint32_t a = seed, b = seed * 3, c = seed * 5, d = seed * 7, e = seed * 9, f = seed * 11, g = seed * 13,
           h = seed * 15;
  for (int i = 0; i < ITERS; ++i) {
    asm volatile(
        "s_add_u32 %0, %0, %8\n\ts_add_u32 %1, %1, %8\n\ts_add_u32 %2, %2, %8\n\ts_add_u32 %3, %3, %8\n\t"
        "s_add_u32 %4, %4, %8\n\ts_add_u32 %5, %5, %8\n\ts_add_u32 %6, %6, %8\n\ts_add_u32 %7, %7, %8\n\t"
        "s_add_u32 %0, %0, %8\n\ts_add_u32 %1, %1, %8\n\ts_add_u32 %2, %2, %8\n\ts_add_u32 %3, %3, %8\n\t"
        "s_add_u32 %4, %4, %8\n\ts_add_u32 %5, %5, %8\n\ts_add_u32 %6, %6, %8\n\ts_add_u32 %7, %7, %8"
        : "+s"(a), "+s"(b), "+s"(c), "+s"(d), "+s"(e), "+s"(f), "+s"(g), "+s"(h)
        : "s"(seed)
        : "scc");
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a ^ b ^ c ^ d ^ e ^ f ^ g ^ h;
}

__global__ __launch_bounds__(256) void cmp6(uint32_t* out, uint32_t seed) {
  uint32_t w = seed * 0x9E3779B9u + threadIdx.x * 0x85EBCA6Bu, dd = w ^ 0x5bd1e995u;
  uint64_t acc = 0;
  for (int i = 0; i < ITERS; ++i) {
    uint64_t x0, x1, x2, x3, x4, x5;
    asm volatile(
        "v_cmp_gt_u32_sdwa %[x0], %[d], %[w] src0_sel:BYTE_0 src1_sel:BYTE_0\n\t"
        "v_cmp_gt_u32_sdwa %[x1], %[d], %[w] src0_sel:BYTE_0 src1_sel:BYTE_2\n\t"
        "v_cmp_ge_u32_sdwa %[x2], %[d], %[w] src0_sel:BYTE_1 src1_sel:BYTE_0\n\t"
        "v_cmp_ge_u32_sdwa %[x3], %[d], %[w] src0_sel:BYTE_1 src1_sel:BYTE_2\n\t"
        "v_cmp_le_u32_sdwa %[x4], %[d], %[w] src0_sel:BYTE_2 src1_sel:BYTE_0\n\t"
        "v_cmp_le_u32_sdwa %[x5], %[d], %[w] src0_sel:BYTE_2 src1_sel:BYTE_2\n\t"
        "s_andn2_b64 %[x0], %[x0], %[x2]\n\t"
        "s_andn2_b64 %[x1], %[x1], %[x3]\n\t"
        "s_and_b64 %[x2], %[x2], %[x4]\n\t"
        "s_and_b64 %[x3], %[x3], %[x5]\n\t"
        "s_or_b64 %[x0], %[x0], %[x1]\n\t"
        "s_xor_b64 %[acc], %[acc], %[x0]"
        : [x0] "=&s"(x0), [x1] "=&s"(x1), [x2] "=&s"(x2), [x3] "=&s"(x3), [x4] "=&s"(x4), [x5] "=&s"(x5),
          [acc] "+s"(acc)
        : [d] "v"(dd), [w] "v"(w)
        : "scc");
    dd += (uint32_t)acc;
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = w ^ dd;
}

template <typename K>
void run(const char* name, K kern, double instr_per_iter, int cus, int clk, uint32_t* out) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  for (int w : {1, 2, 4, 8}) {
    const int blocks = cus * w;  // 256 threads = 4 waves = one per SIMD
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, out, 7u);
    (void)hipEventRecord(a);
    for (int r = 0; r < 3; ++r) hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, out, 7u);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    const double iters = 3.0 * w * ITERS;  // per SIMD
    const double cyc = ms * 1e-3 * clk * 1e3 / iters;
    printf("%-9s waves/SIMD=%d : %.2f cycles/iter per SIMD (%.2f per instruction)\n", name, w, cyc,
           cyc / instr_per_iter);
  }
}

int main() {
  int cus = 0, clk = 0;
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  (void)hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, 0);
  uint32_t* out;
  (void)hipMalloc(&out, 1 << 26);
  printf("CUs=%d clock=%d kHz\n", cus, clk);
  run("sel_cnd", sel_cnd, 11, cus, clk, out);
  run("sel_exec", sel_exec, 22, cus, clk, out);
  run("salu16", salu16, 16, cus, clk, out);
  run("cmp6", cmp6, 12, cus, clk, out);
  return 0;
}
