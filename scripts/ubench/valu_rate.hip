// Microbenchmark: cycles per wave64 VALU instruction on gfx950, per class.
// 8 independent accumulator chains per lane, inline asm so the exact opcode issues.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define CHAINS 8
#define ITERS 4096

#define DEF(NAME, ASM)                                                              \
  __global__ __launch_bounds__(256) void NAME(uint32_t* out, uint32_t seed) {       \
    uint32_t v0 = seed + threadIdx.x, v1 = v0 * 3, v2 = v0 * 5, v3 = v0 * 7, v4 = v0 * 11, \
             v5 = v0 * 13, v6 = v0 * 17, v7 = v0 * 19, k = seed | 1;                \
    for (int i = 0; i < ITERS; ++i) {                                               \
      asm volatile(ASM : "+v"(v0) : "v"(k)); asm volatile(ASM : "+v"(v1) : "v"(k)); \
      asm volatile(ASM : "+v"(v2) : "v"(k)); asm volatile(ASM : "+v"(v3) : "v"(k)); \
      asm volatile(ASM : "+v"(v4) : "v"(k)); asm volatile(ASM : "+v"(v5) : "v"(k)); \
      asm volatile(ASM : "+v"(v6) : "v"(k)); asm volatile(ASM : "+v"(v7) : "v"(k)); \
    }                                                                               \
    out[blockIdx.x * blockDim.x + threadIdx.x] = v0 ^ v1 ^ v2 ^ v3 ^ v4 ^ v5 ^ v6 ^ v7; \
  }

DEF(k_add, "v_add_u32 %0, %0, %1")
DEF(k_xor, "v_xor_b32 %0, %0, %1")
DEF(k_add3, "v_add3_u32 %0, %0, %1, %0")
DEF(k_bfe, "v_bfe_i32 %0, %0, 6, 10\n v_xor_b32 %0, %0, %1")
DEF(k_med3, "v_med3_i32 %0, %0, 0, %1")
DEF(k_max3, "v_max3_u32 %0, %0, %1, %0")
DEF(k_dot4, "v_dot4_u32_u8 %0, %0, %1, %0")
DEF(k_mad24, "v_mad_u32_u24 %0, %0, %1, %0")
DEF(k_mul24, "v_mul_u32_u24 %0, %0, %1")
DEF(k_mullo, "v_mul_lo_u32 %0, %0, %1")
DEF(k_pkadd, "v_pk_add_u16 %0, %0, %1")
DEF(k_pkmad, "v_pk_mad_u16 %0, %0, %1, %0")
DEF(k_pkmax, "v_pk_max_i16 %0, %0, %1")
DEF(k_perm, "v_perm_b32 %0, %0, %1, %1")
DEF(k_cndmask, "v_cmp_lt_u32 vcc, %0, %1\n v_cndmask_b32 %0, %0, %1, vcc")
DEF(k_fma, "v_fma_f32 %0, %0, %1, %1")
DEF(k_lshladd, "v_lshl_add_u32 %0, %0, 3, %1")
DEF(k_satpk, "v_sat_pk_u8_i16 %0, %0\n v_xor_b32 %0, %0, %1")

DEF(k_sub, "v_sub_u32 %0, %0, %1")
DEF(k_and, "v_and_b32 %0, %0, %1")
DEF(k_or, "v_or_b32 %0, %0, %1")
DEF(k_lshl, "v_lshlrev_b32 %0, 3, %0\n v_xor_b32 %0, %0, %1")
DEF(k_lshr, "v_lshrrev_b32 %0, %1, %0")
DEF(k_ashr, "v_ashrrev_i32 %0, %1, %0")
DEF(k_maxi, "v_max_i32 %0, %0, %1")
DEF(k_minu, "v_min_u32 %0, %0, %1")
DEF(k_cnds, "v_cndmask_b32 %0, %0, %1, s[2:3]")
DEF(k_bfeu, "v_bfe_u32 %0, %0, %1, 8")
DEF(k_lshlor, "v_lshl_or_b32 %0, %0, 3, %1")
DEF(k_andor, "v_and_or_b32 %0, %0, %1, %0")
DEF(k_madi24, "v_mad_i32_i24 %0, %0, %1, %0")
DEF(k_muli24, "v_mul_i32_i24 %0, %0, %1")
DEF(k_maxu16, "v_max_u16 %0, %0, %1")
DEF(k_pksub, "v_pk_sub_u16 %0, %0, %1")
DEF(k_pkshr, "v_pk_lshrrev_b16 %0, %1, %0")
DEF(k_pkashr, "v_pk_ashrrev_i16 %0, %1, %0")
DEF(k_sub16, "v_sub_u16 %0, %0, %1")
DEF(k_bfi, "v_bfi_b32 %0, %0, %1, %0")
DEF(k_alignbit, "v_alignbit_b32 %0, %0, %1, 5")
DEF(k_cvtpk, "v_cvt_pk_u8_f32 %0, %1, 1, %0")
DEF(k_addsdwa, "v_add_u32_sdwa %0, %0, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_1 src1_sel:WORD_0")
DEF(k_max3i16, "v_max3_i16 %0, %0, %1, %0")
DEF(k_mov, "v_mov_b32 %0, %1\n v_xor_b32 %0, %0, %1")
DEF(k_xad, "v_xad_u32 %0, %0, %1, %0")
DEF(k_addlshl, "v_add_lshl_u32 %0, %0, %1, 2")
DEF(k_dot2u16, "v_dot2_u32_u16 %0, %0, %1, %0")
DEF(k_sad, "v_sad_u8 %0, %0, %1, %0")
DEF(k_bcnt, "v_bcnt_u32_b32 %0, %0, %1")
DEF(k_maxu8sdwa, "v_max_u32_sdwa %0, %0, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_1 src1_sel:BYTE_2")
DEF(k_addco, "v_add_co_u32 %0, vcc, %0, %1")
DEF(k_mulhi, "v_mul_hi_u32_u24 %0, %0, %1")
DEF(k_min3i, "v_min3_i32 %0, %0, %1, %0")

DEF(k2_maxi16, "v_max_i16 %0, %0, %1")
DEF(k2_mini16, "v_min_i16 %0, %0, %1")
DEF(k2_minu16, "v_min_u16 %0, %0, %1")
DEF(k2_ashr16, "v_ashrrev_i16 %0, %1, %0")
DEF(k2_lshr16, "v_lshrrev_b16 %0, %1, %0")
DEF(k2_lshl16, "v_lshlrev_b16 %0, %1, %0")
DEF(k2_add16, "v_add_u16 %0, %0, %1")
DEF(k2_mul16, "v_mul_lo_u16 %0, %0, %1")
DEF(k2_mad16, "v_mad_u16 %0, %0, %1, %0")
DEF(k2_cmpeq, "v_cmp_eq_u32 s[4:5], %0, %1\n v_xor_b32 %0, %0, %1")
DEF(k2_cmpeq16, "v_cmp_eq_u16 s[4:5], %0, %1\n v_xor_b32 %0, %0, %1")
DEF(k2_cnde32, "v_cndmask_b32_e32 %0, %0, %1, vcc")
DEF(k2_med3u16, "v_med3_u16 %0, %0, %1, %0")
DEF(k2_med3i16, "v_med3_i16 %0, %0, %1, %0")
DEF(k2_lshlrev, "v_lshlrev_b32 %0, %1, %0")
DEF(k2_max3u, "v_max3_u32 %0, %0, %1, %0")
DEF(k2_subrev, "v_subrev_u32 %0, %0, %1")
DEF(k2_andimm, "v_and_b32 %0, 0xff00, %0\n v_xor_b32 %0, %0, %1")
DEF(k2_addimm, "v_add_u32 %0, 0x1234, %0\n v_xor_b32 %0, %0, %1")
DEF(k2_not, "v_not_b32 %0, %0\n v_xor_b32 %0, %0, %1")

DEF(k3_pkmad, "v_pk_mad_u16 %0, %0, %1, %0")
DEF(k3_subclamp, "v_sub_u16 %0, %0, %1 clamp")
DEF(k3_or3, "v_or3_b32 %0, %0, %1, %0")
DEF(k3_lshlor, "v_lshl_or_b32 %0, %0, 3, %1")
DEF(k3_addu24, "v_mad_u32_u24 %0, %0, %1, %0")
DEF(k3_mulhi16, "v_mul_hi_u32_u24 %0, %0, %1")
DEF(k3_addc, "v_add_u32 %0, 0xff00ff, %0\n v_xor_b32 %0, %0, %1")
DEF(k3_subb16, "v_subrev_u16 %0, %0, %1")
DEF(k3_cvtu16, "v_cvt_f32_ubyte0 %0, %0\n v_xor_b32 %0, %0, %1")

typedef void (*K)(uint32_t*, uint32_t);
struct T { const char* name; K k; int instrs_per_step; };

int main() {
  T tests[] = {{"v_add_u32", k_add, 1}, {"v_dot4_u32_u8", k_dot4, 1}, {"v_cndmask sgpr", k_cnds, 1}, {"v_cmp+cndmask", k_cndmask, 2},
               {"v_pk_mad_u16", k3_pkmad, 1},
               {"v_sub_u16 clamp", k3_subclamp, 1},
               {"v_or3_b32", k3_or3, 1},
               {"v_lshl_or_b32", k3_lshlor, 1},
               {"v_mad_u32_u24", k3_addu24, 1},
               {"v_mul_hi_u32_u24", k3_mulhi16, 1},
               {"v_add_u32+xor", k3_addc, 2},
               {"v_subrev_u16", k3_subb16, 1},
               {"v_cvt_f32_ubyte0+xor", k3_cvtu16, 2}};
  int dev = 0, cus = 0, clk = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, dev);
  uint32_t* out;
  hipMalloc(&out, 1 << 26);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  printf("CUs=%d clock=%d kHz\n", cus, clk);
  for (int waves_per_simd : {8}) {
    const int blocks = cus * waves_per_simd;  // 256 threads = 4 waves = 1 per SIMD
    for (auto& t : tests) {
      hipLaunchKernelGGL(t.k, dim3(blocks), dim3(256), 0, 0, out, 7u);
      hipEventRecord(a);
      for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(t.k, dim3(blocks), dim3(256), 0, 0, out, 7u);
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms = 0;
      hipEventElapsedTime(&ms, a, b);
      const double instr_per_simd = 5.0 * (double)waves_per_simd * ITERS * CHAINS * t.instrs_per_step;
      const double cycles = ms * 1e-3 * clk * 1e3;
      printf("waves/SIMD=%d %-22s %.2f cycles per wave-instruction (at %d MHz nominal)\n",
             waves_per_simd, t.name, cycles / instr_per_simd, clk / 1000);
    }
  }
  return 0;
}
