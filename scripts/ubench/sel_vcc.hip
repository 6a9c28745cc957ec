// Microbenchmark (development only): the chroma-run kernel's per-word select
// (scripts/../csrc/trik_hsv_chroma.hip select2_impl) in two encodings, cycles
// per loop iteration per SIMD at 1/2/4/8 waves per SIMD:
//   word_e64  7 compares into SGPR pairs, 8 SALU combines, 4 v_cndmask_b32_e64
//             and the v_add3 into the pair counter (the shipped form)
//   word_e32  the same with the selects as v_cndmask_b32_e32 (32-bit VOP2
//             encoding) on VCC, VCC written by SALU (s_mov_b64 / the k0, k1
//             s_and_b64 straight into VCC): +2 SALU per word
//   word_pipe word_e64's two words interleaved: both words' compares, then
//             their SALU combines, then their selects
//   form_cmp  the shipped word form (compares into SGPR masks, selects) with the
//             pair counter, the odd-pixel counter and the flag mask; the
//             "per VALU instruction" column is per WORD here
//   form_swar the same outputs by a SWAR form (swar_word: VERDICT r5 lever a)
//   cnd_e64   4 v_cndmask_b32_e64 + v_add3 alone (masks in SGPRs)
//   cnd_e32   the same as v_cndmask_b32_e32, VCC from s_mov_b64 before each
// Two independent words per iteration.
// build: hipcc -O3 --offload-arch=gfx950 -o sel_vcc sel_vcc.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define ITERS 4096

#define CMPS(X, LT0, LT1, LE0, LE1, GE0, GE1, D, A, W)                                        \
  "v_cmp_eq_u32_e64 " X ", %[k], " D "\n\t"                                                  \
  "v_cmp_gt_u32_sdwa " LT0 ", " D ", " W " src0_sel:BYTE_0 src1_sel:BYTE_0\n\t"              \
  "v_cmp_gt_u32_sdwa " LT1 ", " D ", " W " src0_sel:BYTE_0 src1_sel:BYTE_2\n\t"              \
  "v_cmp_ge_u32_sdwa " LE0 ", " D ", " W " src0_sel:BYTE_1 src1_sel:BYTE_0\n\t"              \
  "v_cmp_ge_u32_sdwa " LE1 ", " D ", " W " src0_sel:BYTE_1 src1_sel:BYTE_2\n\t"              \
  "v_cmp_le_u32_sdwa " GE0 ", " A ", " W " src0_sel:BYTE_1 src1_sel:BYTE_0\n\t"              \
  "v_cmp_le_u32_sdwa " GE1 ", " A ", " W " src0_sel:BYTE_1 src1_sel:BYTE_2\n\t"

__global__ __launch_bounds__(256) void word_e64(uint32_t* out, uint32_t seed) {
  uint32_t w = seed * 0x9E3779B9u + threadIdx.x * 0x85EBCA6Bu, w2 = w ^ 0x1234567u;
  uint32_t d = w ^ 0x5bd1e995u, bw = w * 3u, m1 = w * 7, m2 = w * 13, P = 0, P2 = 0;
  uint64_t acc = 0;
  for (int i = 0; i < ITERS; ++i) {
    uint64_t x, lt0, lt1, le0, le1, ge0, ge1, t, q;
    uint32_t e0, e1;
    asm volatile(
        CMPS("%[x]", "%[lt0]", "%[lt1]", "%[le0]", "%[le1]", "%[ge0]", "%[ge1]", "%[d]", "%[a]", "%[w]")
        "s_andn2_b64 %[t], %[lt0], %[le0]\n\t"
        "s_andn2_b64 %[q], %[lt1], %[le1]\n\t"
        "s_or_b64 %[q], %[q], %[t]\n\t"
        "s_or_b64 %[q], %[q], %[x]\n\t"
        "s_andn2_b64 %[le0], %[le0], %[x]\n\t"
        "s_andn2_b64 %[le1], %[le1], %[x]\n\t"
        "s_and_b64 %[ge0], %[le0], %[ge0]\n\t"
        "s_and_b64 %[ge1], %[le1], %[ge1]\n\t"
        "v_cndmask_b32_e64 %[e0], %[m2], %[m1], %[lt0]\n\t"
        "v_cndmask_b32_e64 %[e1], %[m2], %[m1], %[lt1]\n\t"
        "v_cndmask_b32_e64 %[e0], 0, %[e0], %[ge0]\n\t"
        "v_cndmask_b32_e64 %[e1], 0, %[e1], %[ge1]\n\t"
        "v_add3_u32 %[P], %[P], %[e0], %[e1]\n\t"
        "s_xor_b64 %[acc], %[acc], %[q]"
        : [x] "=&s"(x), [lt0] "=&s"(lt0), [lt1] "=&s"(lt1), [le0] "=&s"(le0), [le1] "=&s"(le1), [ge0] "=&s"(ge0),
          [ge1] "=&s"(ge1), [t] "=&s"(t), [q] "=&s"(q), [e0] "=&v"(e0), [e1] "=&v"(e1), [P] "+v"(P), [acc] "+s"(acc)
        : [w] "v"(w), [d] "v"(d), [a] "v"(bw), [m1] "v"(m1), [m2] "v"(m2), [k] "s"(0xFFu)
        : "scc");
    asm volatile(
        CMPS("%[x]", "%[lt0]", "%[lt1]", "%[le0]", "%[le1]", "%[ge0]", "%[ge1]", "%[d]", "%[a]", "%[w]")
        "s_andn2_b64 %[t], %[lt0], %[le0]\n\t"
        "s_andn2_b64 %[q], %[lt1], %[le1]\n\t"
        "s_or_b64 %[q], %[q], %[t]\n\t"
        "s_or_b64 %[q], %[q], %[x]\n\t"
        "s_andn2_b64 %[le0], %[le0], %[x]\n\t"
        "s_andn2_b64 %[le1], %[le1], %[x]\n\t"
        "s_and_b64 %[ge0], %[le0], %[ge0]\n\t"
        "s_and_b64 %[ge1], %[le1], %[ge1]\n\t"
        "v_cndmask_b32_e64 %[e0], %[m2], %[m1], %[lt0]\n\t"
        "v_cndmask_b32_e64 %[e1], %[m2], %[m1], %[lt1]\n\t"
        "v_cndmask_b32_e64 %[e0], 0, %[e0], %[ge0]\n\t"
        "v_cndmask_b32_e64 %[e1], 0, %[e1], %[ge1]\n\t"
        "v_add3_u32 %[P], %[P], %[e0], %[e1]\n\t"
        "s_xor_b64 %[acc], %[acc], %[q]"
        : [x] "=&s"(x), [lt0] "=&s"(lt0), [lt1] "=&s"(lt1), [le0] "=&s"(le0), [le1] "=&s"(le1), [ge0] "=&s"(ge0),
          [ge1] "=&s"(ge1), [t] "=&s"(t), [q] "=&s"(q), [e0] "=&v"(e0), [e1] "=&v"(e1), [P] "+v"(P2), [acc] "+s"(acc)
        : [w] "v"(w2), [d] "v"(d), [a] "v"(bw), [m1] "v"(m1), [m2] "v"(m2), [k] "s"(0xFFu)
        : "scc");
    d += (uint32_t)acc;
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = P ^ P2 ^ d;
}

__global__ __launch_bounds__(256) void word_e32(uint32_t* out, uint32_t seed) {
  uint32_t w = seed * 0x9E3779B9u + threadIdx.x * 0x85EBCA6Bu, w2 = w ^ 0x1234567u;
  uint32_t d = w ^ 0x5bd1e995u, bw = w * 3u, m1 = w * 7, m2 = w * 13, P = 0, P2 = 0;
  uint64_t acc = 0;
  for (int i = 0; i < ITERS; ++i) {
    uint64_t x, lt0, lt1, le0, le1, ge0, ge1, t, q;
    uint32_t e0, e1;
    asm volatile(
        CMPS("%[x]", "%[lt0]", "%[lt1]", "%[le0]", "%[le1]", "%[ge0]", "%[ge1]", "%[d]", "%[a]", "%[w]")
        "s_andn2_b64 %[t], %[lt0], %[le0]\n\t"
        "s_andn2_b64 %[q], %[lt1], %[le1]\n\t"
        "s_or_b64 %[q], %[q], %[t]\n\t"
        "s_or_b64 %[q], %[q], %[x]\n\t"
        "s_andn2_b64 %[le0], %[le0], %[x]\n\t"
        "s_andn2_b64 %[le1], %[le1], %[x]\n\t"
        "s_mov_b64 vcc, %[lt0]\n\t"
        "v_cndmask_b32_e32 %[e0], %[m2], %[m1], vcc\n\t"
        "s_mov_b64 vcc, %[lt1]\n\t"
        "v_cndmask_b32_e32 %[e1], %[m2], %[m1], vcc\n\t"
        "s_and_b64 vcc, %[le0], %[ge0]\n\t"
        "v_cndmask_b32_e32 %[e0], 0, %[e0], vcc\n\t"
        "s_and_b64 vcc, %[le1], %[ge1]\n\t"
        "v_cndmask_b32_e32 %[e1], 0, %[e1], vcc\n\t"
        "v_add3_u32 %[P], %[P], %[e0], %[e1]\n\t"
        "s_xor_b64 %[acc], %[acc], %[q]"
        : [x] "=&s"(x), [lt0] "=&s"(lt0), [lt1] "=&s"(lt1), [le0] "=&s"(le0), [le1] "=&s"(le1), [ge0] "=&s"(ge0),
          [ge1] "=&s"(ge1), [t] "=&s"(t), [q] "=&s"(q), [e0] "=&v"(e0), [e1] "=&v"(e1), [P] "+v"(P), [acc] "+s"(acc)
        : [w] "v"(w), [d] "v"(d), [a] "v"(bw), [m1] "v"(m1), [m2] "v"(m2), [k] "s"(0xFFu)
        : "scc", "vcc");
    asm volatile(
        CMPS("%[x]", "%[lt0]", "%[lt1]", "%[le0]", "%[le1]", "%[ge0]", "%[ge1]", "%[d]", "%[a]", "%[w]")
        "s_andn2_b64 %[t], %[lt0], %[le0]\n\t"
        "s_andn2_b64 %[q], %[lt1], %[le1]\n\t"
        "s_or_b64 %[q], %[q], %[t]\n\t"
        "s_or_b64 %[q], %[q], %[x]\n\t"
        "s_andn2_b64 %[le0], %[le0], %[x]\n\t"
        "s_andn2_b64 %[le1], %[le1], %[x]\n\t"
        "s_mov_b64 vcc, %[lt0]\n\t"
        "v_cndmask_b32_e32 %[e0], %[m2], %[m1], vcc\n\t"
        "s_mov_b64 vcc, %[lt1]\n\t"
        "v_cndmask_b32_e32 %[e1], %[m2], %[m1], vcc\n\t"
        "s_and_b64 vcc, %[le0], %[ge0]\n\t"
        "v_cndmask_b32_e32 %[e0], 0, %[e0], vcc\n\t"
        "s_and_b64 vcc, %[le1], %[ge1]\n\t"
        "v_cndmask_b32_e32 %[e1], 0, %[e1], vcc\n\t"
        "v_add3_u32 %[P], %[P], %[e0], %[e1]\n\t"
        "s_xor_b64 %[acc], %[acc], %[q]"
        : [x] "=&s"(x), [lt0] "=&s"(lt0), [lt1] "=&s"(lt1), [le0] "=&s"(le0), [le1] "=&s"(le1), [ge0] "=&s"(ge0),
          [ge1] "=&s"(ge1), [t] "=&s"(t), [q] "=&s"(q), [e0] "=&v"(e0), [e1] "=&v"(e1), [P] "+v"(P2), [acc] "+s"(acc)
        : [w] "v"(w2), [d] "v"(d), [a] "v"(bw), [m1] "v"(m1), [m2] "v"(m2), [k] "s"(0xFFu)
        : "scc", "vcc");
    d += (uint32_t)acc;
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = P ^ P2 ^ d;
}

__global__ __launch_bounds__(256) void cnd_e64(uint32_t* out, uint32_t seed) {
  const uint32_t m1 = seed * 7 + threadIdx.x, m2 = seed * 13 + threadIdx.x;
  uint32_t p0 = 0, p1 = 0, e0, e1, e2, e3;
  const uint64_t a = 0x5555aaaa3333ccccull * seed, b = ~a, c = a ^ 0x0f0f0f0f0f0f0f0full, d = a >> 3;
  for (int i = 0; i < ITERS; ++i) {
    asm volatile(
        "v_cndmask_b32_e64 %[e0], %[m2], %[m1], %[a]\n\t"
        "v_cndmask_b32_e64 %[e1], %[m2], %[m1], %[b]\n\t"
        "v_cndmask_b32_e64 %[e2], %[m1], %[m2], %[a]\n\t"
        "v_cndmask_b32_e64 %[e3], %[m1], %[m2], %[b]\n\t"
        "v_cndmask_b32_e64 %[e0], 0, %[e0], %[c]\n\t"
        "v_cndmask_b32_e64 %[e1], 0, %[e1], %[d]\n\t"
        "v_cndmask_b32_e64 %[e2], 0, %[e2], %[d]\n\t"
        "v_cndmask_b32_e64 %[e3], 0, %[e3], %[c]\n\t"
        "v_add3_u32 %[p0], %[p0], %[e0], %[e1]\n\t"
        "v_add3_u32 %[p1], %[p1], %[e2], %[e3]"
        : [p0] "+v"(p0), [p1] "+v"(p1), [e0] "=&v"(e0), [e1] "=&v"(e1), [e2] "=&v"(e2), [e3] "=&v"(e3)
        : [m1] "v"(m1), [m2] "v"(m2), [a] "s"(a), [b] "s"(b), [c] "s"(c), [d] "s"(d));
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = p0 ^ p1;
}

__global__ __launch_bounds__(256) void cnd_e32(uint32_t* out, uint32_t seed) {
  const uint32_t m1 = seed * 7 + threadIdx.x, m2 = seed * 13 + threadIdx.x;
  uint32_t p0 = 0, p1 = 0, e0, e1, e2, e3;
  const uint64_t a = 0x5555aaaa3333ccccull * seed, b = ~a, c = a ^ 0x0f0f0f0f0f0f0f0full, d = a >> 3;
  for (int i = 0; i < ITERS; ++i) {
    asm volatile(
        "s_mov_b64 vcc, %[a]\n\t"
        "v_cndmask_b32_e32 %[e0], %[m2], %[m1], vcc\n\t"
        "s_mov_b64 vcc, %[b]\n\t"
        "v_cndmask_b32_e32 %[e1], %[m2], %[m1], vcc\n\t"
        "s_mov_b64 vcc, %[a]\n\t"
        "v_cndmask_b32_e32 %[e2], %[m1], %[m2], vcc\n\t"
        "s_mov_b64 vcc, %[b]\n\t"
        "v_cndmask_b32_e32 %[e3], %[m1], %[m2], vcc\n\t"
        "s_mov_b64 vcc, %[c]\n\t"
        "v_cndmask_b32_e32 %[e0], 0, %[e0], vcc\n\t"
        "s_mov_b64 vcc, %[d]\n\t"
        "v_cndmask_b32_e32 %[e1], 0, %[e1], vcc\n\t"
        "v_cndmask_b32_e32 %[e2], 0, %[e2], vcc\n\t"
        "s_mov_b64 vcc, %[c]\n\t"
        "v_cndmask_b32_e32 %[e3], 0, %[e3], vcc\n\t"
        "v_add3_u32 %[p0], %[p0], %[e0], %[e1]\n\t"
        "v_add3_u32 %[p1], %[p1], %[e2], %[e3]"
        : [p0] "+v"(p0), [p1] "+v"(p1), [e0] "=&v"(e0), [e1] "=&v"(e1), [e2] "=&v"(e2), [e3] "=&v"(e3)
        : [m1] "v"(m1), [m2] "v"(m2), [a] "s"(a), [b] "s"(b), [c] "s"(c), [d] "s"(d)
        : "vcc");
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = p0 ^ p1;
}


// the two words' compares first, then both SALU combines, then both selects:
// independent work between each VALU -> SALU -> VALU dependency
__global__ __launch_bounds__(256) void word_pipe(uint32_t* out, uint32_t seed) {
  uint32_t w = seed * 0x9E3779B9u + threadIdx.x * 0x85EBCA6Bu, w2 = w ^ 0x1234567u;
  uint32_t d = w ^ 0x5bd1e995u, bw = w * 3u, m1 = w * 7, m2 = w * 13, P = 0, P2 = 0;
  uint64_t acc = 0;
  for (int i = 0; i < ITERS; ++i) {
    uint64_t x, lt0, lt1, le0, le1, ge0, ge1, t, q;
    uint64_t y, mt0, mt1, me0, me1, mg0, mg1, u, r;
    uint32_t e0, e1, f0, f1;
    asm volatile(
        CMPS("%[x]", "%[lt0]", "%[lt1]", "%[le0]", "%[le1]", "%[ge0]", "%[ge1]", "%[d]", "%[a]", "%[w]")
        CMPS("%[y]", "%[mt0]", "%[mt1]", "%[me0]", "%[me1]", "%[mg0]", "%[mg1]", "%[d]", "%[a]", "%[w2]")
        "s_andn2_b64 %[t], %[lt0], %[le0]\n\t"
        "s_andn2_b64 %[q], %[lt1], %[le1]\n\t"
        "s_or_b64 %[q], %[q], %[t]\n\t"
        "s_or_b64 %[q], %[q], %[x]\n\t"
        "s_andn2_b64 %[le0], %[le0], %[x]\n\t"
        "s_andn2_b64 %[le1], %[le1], %[x]\n\t"
        "s_and_b64 %[ge0], %[le0], %[ge0]\n\t"
        "s_and_b64 %[ge1], %[le1], %[ge1]\n\t"
        "v_cndmask_b32_e64 %[e0], %[m2], %[m1], %[lt0]\n\t"
        "v_cndmask_b32_e64 %[e1], %[m2], %[m1], %[lt1]\n\t"
        "s_andn2_b64 %[u], %[mt0], %[me0]\n\t"
        "s_andn2_b64 %[r], %[mt1], %[me1]\n\t"
        "s_or_b64 %[r], %[r], %[u]\n\t"
        "s_or_b64 %[r], %[r], %[y]\n\t"
        "s_andn2_b64 %[me0], %[me0], %[y]\n\t"
        "s_andn2_b64 %[me1], %[me1], %[y]\n\t"
        "s_and_b64 %[mg0], %[me0], %[mg0]\n\t"
        "s_and_b64 %[mg1], %[me1], %[mg1]\n\t"
        "v_cndmask_b32_e64 %[e0], 0, %[e0], %[ge0]\n\t"
        "v_cndmask_b32_e64 %[e1], 0, %[e1], %[ge1]\n\t"
        "v_cndmask_b32_e64 %[f0], %[m2], %[m1], %[mt0]\n\t"
        "v_cndmask_b32_e64 %[f1], %[m2], %[m1], %[mt1]\n\t"
        "v_add3_u32 %[P], %[P], %[e0], %[e1]\n\t"
        "v_cndmask_b32_e64 %[f0], 0, %[f0], %[mg0]\n\t"
        "v_cndmask_b32_e64 %[f1], 0, %[f1], %[mg1]\n\t"
        "v_add3_u32 %[P2], %[P2], %[f0], %[f1]\n\t"
        "s_xor_b64 %[acc], %[acc], %[q]\n\t"
        "s_xor_b64 %[acc], %[acc], %[r]"
        : [x] "=&s"(x), [lt0] "=&s"(lt0), [lt1] "=&s"(lt1), [le0] "=&s"(le0), [le1] "=&s"(le1), [ge0] "=&s"(ge0),
          [ge1] "=&s"(ge1), [t] "=&s"(t), [q] "=&s"(q), [y] "=&s"(y), [mt0] "=&s"(mt0), [mt1] "=&s"(mt1),
          [me0] "=&s"(me0), [me1] "=&s"(me1), [mg0] "=&s"(mg0), [mg1] "=&s"(mg1), [u] "=&s"(u), [r] "=&s"(r),
          [e0] "=&v"(e0), [e1] "=&v"(e1), [f0] "=&v"(f0), [f1] "=&v"(f1), [P] "+v"(P), [P2] "+v"(P2), [acc] "+s"(acc)
        : [w] "v"(w), [w2] "v"(w2), [d] "v"(d), [a] "v"(bw), [m1] "v"(m1), [m2] "v"(m2), [k] "s"(0xFFu)
        : "scc");
    d += (uint32_t)acc;
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = P ^ P2 ^ d;
}


// The VERDICT r5 lever (a): a SWAR fast path for one YUYV word -- both
// pixels' Y against broadcast thresholds in 16-bit lanes with a guard bit
// (Y + 256 - t: bit 8 of a lane set iff Y >= t), the classes by bit logic,
// the byte-spread masks weighted by the classes' pixel counts
// (v_mad_u32_u24), the word's flag by one compare.  Same outputs as the
// shipped select (the pair counter P, the odd-pixel counter O, the flag mask).
__device__ __forceinline__ void swar_word(uint32_t w, uint32_t d, uint32_t bw, uint32_t m1, uint32_t m2,
                                          uint32_t& P, uint32_t& O, uint64_t& q) {
  const uint32_t Z = (w & 0x00FF00FFu) | 0x01000100u;             // [Y0 + 256, Y1 + 256]
  const uint32_t T1 = __builtin_amdgcn_perm(0u, d, 0x0C000C00u);   // [b1, b1]
  const uint32_t T2 = __builtin_amdgcn_perm(0u, d, 0x0C010C01u);   // [b2, b2]
  const uint32_t TA = __builtin_amdgcn_perm(0u, bw, 0x0C010C01u);  // [A, A]
  const uint32_t ge1 = Z - T1, gt2 = Z - 0x00010001u - T2, geA = Z - TA;
  const uint32_t c1 = geA & ~(ge1 | gt2) & 0x01000100u;  // A <= Y < b1, Y <= b2: M1
  const uint32_t c2 = geA & ge1 & ~gt2 & 0x01000100u;    // A <= Y, b1 <= Y <= b2: M2
  const uint32_t fl = ~ge1 & gt2 & 0x01000100u;          // b2 < Y < b1: the exact path
  const bool x = d == 0x00FFu;
  uint32_t es = __umul24((uint32_t)__builtin_popcount(c1), m1) + __umul24((uint32_t)__builtin_popcount(c2), m2);
  uint32_t e1 = __umul24(c1 >> 24, m1) + __umul24(c2 >> 24, m2);
  P += x ? 0u : es;
  O += x ? 0u : e1;
  q |= __builtin_amdgcn_ballot_w64(fl != 0u || x);
}

// the shipped select in C form (select2w's compares and selects) with the
// same outputs, for a like-for-like count
__device__ __forceinline__ void cmp_word(uint32_t w, uint32_t d, uint32_t bw, uint32_t m1, uint32_t m2,
                                         uint32_t& P, uint32_t& O, uint64_t& q) {
  uint64_t x, lt0, lt1, le0, le1, ge0, ge1;
  asm volatile(CMPS("%[x]", "%[lt0]", "%[lt1]", "%[le0]", "%[le1]", "%[ge0]", "%[ge1]", "%[d]", "%[a]", "%[w]")
               "s_nop 0"
               : [x] "=&s"(x), [lt0] "=&s"(lt0), [lt1] "=&s"(lt1), [le0] "=&s"(le0), [le1] "=&s"(le1),
                 [ge0] "=&s"(ge0), [ge1] "=&s"(ge1)
               : [w] "v"(w), [d] "v"(d), [a] "v"(bw), [k] "s"(0xFFu));
  q |= x | (lt0 & ~le0) | (lt1 & ~le1);
  const uint64_t k0 = le0 & ge0 & ~x, k1 = le1 & ge1 & ~x;
  uint32_t e0, e1;
  asm volatile(
      "v_cndmask_b32_e64 %[e0], %[m2], %[m1], %[lt0]\n\t"
      "v_cndmask_b32_e64 %[e1], %[m2], %[m1], %[lt1]\n\t"
      "v_cndmask_b32_e64 %[e0], 0, %[e0], %[k0]\n\t"
      "v_cndmask_b32_e64 %[e1], 0, %[e1], %[k1]"
      : [e0] "=&v"(e0), [e1] "=&v"(e1)
      : [m1] "v"(m1), [m2] "v"(m2), [lt0] "s"(lt0), [lt1] "s"(lt1), [k0] "s"(k0), [k1] "s"(k1));
  P = P + e0 + e1;
  O += e1;
}

template <bool SWAR>
__global__ __launch_bounds__(256) void word_form(uint32_t* out, uint32_t seed) {
  uint32_t w = seed * 0x9E3779B9u + threadIdx.x * 0x85EBCA6Bu, w2 = w ^ 0x1234567u;
  uint32_t d = (w ^ 0x5bd1e995u) & 0xFFFFu, bw = (w * 3u) & 0xFFFFu, m1 = (w * 7) & 0x01010101u, m2 = (w * 13) & 0x01010101u;
  uint32_t P = 0, P2 = 0, O = 0;
  uint64_t q = 0;
  for (int i = 0; i < ITERS; ++i) {
    if (SWAR) {
      swar_word(w, d, bw, m1, m2, P, O, q);
      swar_word(w2, d, bw, m1, m2, P2, O, q);
    } else {
      cmp_word(w, d, bw, m1, m2, P, O, q);
      cmp_word(w2, d, bw, m1, m2, P2, O, q);
    }
    w += 0x01000101u;
    w2 += 0x00010001u;
    d ^= (uint32_t)q & 0xFFu;
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = P ^ P2 ^ O ^ (uint32_t)q;
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
    printf("%-9s waves/SIMD=%d : %.2f cycles/iter per SIMD (%.2f per VALU instruction)\n", name, w, cyc,
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
  run("word_e64", word_e64, 24, cus, clk, out);  // 2 words x (7 cmp + 4 cndmask + 1 add3)
  run("word_e32", word_e32, 24, cus, clk, out);
  run("word_pipe", word_pipe, 24, cus, clk, out);
  run("form_cmp", word_form<false>, 2, cus, clk, out);  // per word (2 words per iteration)
  run("form_swar", word_form<true>, 2, cus, clk, out);
  run("cnd_e64", cnd_e64, 10, cus, clk, out);
  run("cnd_e32", cnd_e32, 10, cus, clk, out);
  return 0;
}
