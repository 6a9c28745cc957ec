// trik_hsv_chroma.hip -- the chroma-run hot kernel for gfx950.
//
// Same result as the stripe kernel (the reference's WSEQ:251-284 convert +
// WSEQ:316-354 threshold/centroid for up to 4 ranges, bit-exact), by a
// different route that trades per-pixel arithmetic for one table lookup per
// YUYV word:
//
//  * Every pixel's detection mask depends only on its (Y, U, V), and the two
//    pixels of a YUYV word share (U, V).  For a fixed chroma c = (U, V) the
//    mask as a function of Y ("the chroma's profile") is, for most c,
//        Y <= b2 ? (Y < b1 ? M1 : M2) : 0
//    because all three channels rise together with Y (74/64 per step) and
//    saturate, so V rises, S falls and H stays put between saturation events.
//    The builder (chroma_summary_kernel + chroma_block_kernel, once per range
//    set) evaluates all 2^24 (Y,U,V) with the exact per-pixel arithmetic and
//    stores per chroma the descriptor b1 | b2 << 8 (16 bits; 128 KB for all
//    chromas: it lives in LDS) and per 16-chroma block the mask pair
//    M1 | M2 << 4 (stored as its offset in a palette of <= 32 pairs).  A descriptor with b1 > b2 + 1 is a "window": the same
//    select gives M1 below it and 0 above it, and the pixels inside it
//    (b2 < Y < b1) are flagged for the exact path -- so a chroma of another
//    shape costs only the pixels in its window.  The exception code
//    kChromaExc flags both pixels of the word.
//  * The hot loop per YUYV word: one v_perm for c, three LDS reads (run
//    descriptor, block word, the byte-spread mask pair), seven compares
//    (exception code; Y0/Y1 < b1, <= b2, >= the block's cut) and four
//    selects; the flags are SALU operations on the compare masks.
//    Accumulation is the stripe kernel's (byte-packed per-lane counters,
//    lanes own chunk columns and walk rows).
//  * Flagged words are compacted into a per-wave LDS queue (ballot + mbcnt);
//    every 64 queued words one "drain" round computes their flagged pixels
//    exactly (the stripe kernel's per-pixel arithmetic, with small LDS
//    tables: LUT43, LUT255 and the per-range H, S and V masks) and
//    accumulates them with explicit (x, y) weights.  (Looking them up in a
//    global per-(Y, c) table instead was slower: the gather's latency is
//    exposed in the drain.)
#include <hip/hip_runtime.h>

#include <type_traits>

// gfx950 only: the fused step's completion protocol relies on GFX9 memory
// counters (vmcnt counts atomics without return; no separate store counter)
#if defined(__HIP_DEVICE_COMPILE__) && !defined(__gfx950__)
#error "trik_hsv_chroma.hip targets gfx950 only"
#endif

#include "trik_hsv_internal.h"
#include "trik_hsv_pixel.h"
#include "trik_hsv_stripe_px.h"

namespace trik_hsv {

namespace {

constexpr int kMaxBlock = 1024;
constexpr int kChunkWords = 8;  // YUYV words per lane and step (two 4-word pieces, 16 pixels)
// steps per tile: byte counters P_i <= 2 * steps, O <= kChunkWords * steps
constexpr int kMaxSteps = 31;
static_assert(4 * 2 * kMaxSteps <= 255, "flush group sums fit a byte");
constexpr int kQueueCap = 128;  // blob kernel, entries per wave: < 64 waiting + <= 64 added by one word slot
// Hot kernel: at most 15 waves (960 lanes) per workgroup.  A lane's step is
// two pieces of 4 words; a piece with a flagged word becomes one record of
// the wave's queue (its 4 words + a meta word), so a step costs two
// compactions, not one per word slot.  kRecCap records per wave is what the
// LDS image leaves; a step starts with < 64 records queued.
constexpr int kHotLanes = 960;
// the hot kernel's workgroup: 16 waves (4 per SIMD) whatever the tile's
// lane count (<= kHotLanes: 10 wave-sized units at VGA); the waves pull the
// units, so one more wave than units per tile costs nothing and fills the
// fourth SIMD
constexpr int kHotWaves = 16;
constexpr int kRecCap = 70;

// LDS image of the chroma kernel (dynamic LDS from address 0).  The block
// masks and the mask-pair table sit below 64 KiB so their reads take an
// immediate DS offset; the run descriptors follow.
constexpr uint32_t kLdsBlocks = 0;                    // u16 [4096]  the 16-chroma block's pair offset | cut << 8
constexpr uint32_t kLdsPairs = 8192;                  // u32 [kChromaPalette][2] byte-spread (M1, M2) of the palette
constexpr uint32_t kLdsLut43 = kLdsPairs + 8 * kChromaPalette;  // u16 [256]   s_mult43_div (WSEQ:389-407)
constexpr uint32_t kLdsLut255 = kLdsLut43 + 512;      // u16 [256]   s_mult255_div
constexpr uint32_t kLdsHue = kLdsLut255 + 512;        // u8  [256]   hue test per H (bit t = range t)
constexpr uint32_t kLdsSat = kLdsHue + 256;           // u8  [256]   saturation test per S
constexpr uint32_t kLdsVal = kLdsSat + 256;           // u8  [256]   value test per V
constexpr uint32_t kLdsRuns = kLdsVal + 256;          // u16 [65536] b1 | b2 << 8 per chroma
constexpr uint32_t kLdsQueues = kLdsRuns + 131072;    // blob kernel: per wave kQueueCap x {word, pos}
static_assert(kLdsBlocks + 8192 <= kLdsPairs, "LDS layout");
// hot kernel records: per wave kRecCap x 16 B of words, then all waves' meta
// words (kRecCap x 4 B per wave): f (bits 0-3: the piece's flagged words,
// bit 3 - j = word j) | x / 8 (bits 4-15) | row in the tile (bits 16-31)
constexpr uint32_t kLdsRecWords = kLdsQueues;
constexpr uint32_t kLdsRecMeta = kLdsRecWords + kHotWaves * kRecCap * 16;
// fused step: the workgroup's 12 u64 totals (3 per range)
constexpr uint32_t kLdsTotals = (kLdsRecMeta + kHotWaves * kRecCap * 4 + 7u) & ~7u;
// + the last-workgroup flag; then the workgroup's exact-path word count and
// its waves-done count
constexpr uint32_t kLdsWords = kLdsTotals + 12 * 8 + 8;
// + the workgroup's unit counter (hot kernel: units handed out to waves)
constexpr uint32_t kLdsUnits = kLdsWords + 8;
constexpr uint32_t kLdsBytes = kLdsUnits + 4;
static_assert(kLdsBytes <= 160 * 1024, "chroma kernel LDS image");
static_assert((kRecCap * 16) % 16 == 0 && kRecCap >= 64 + 4, "record queue");

typedef __attribute__((address_space(3))) uint8_t* lds8_t;
typedef __attribute__((address_space(3))) uint16_t* lds16_t;
typedef __attribute__((address_space(3))) uint32_t* lds32_t;
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) u32x2* lds64_t;
typedef __attribute__((address_space(3))) u32x4* lds128_t;
__device__ __forceinline__ uint32_t ld8(uint32_t a) { return *(lds8_t)(uintptr_t)a; }
__device__ __forceinline__ uint32_t ld16(uint32_t a) { return *(lds16_t)(uintptr_t)a; }
__device__ __forceinline__ u32x2 ld64(uint32_t a) { return *(lds64_t)(uintptr_t)a; }
__device__ __forceinline__ unsigned long long ld_u64(uint32_t a) {
  return *(__attribute__((address_space(3))) unsigned long long*)(uintptr_t)a;
}
__device__ __forceinline__ void st_u64(uint32_t a, unsigned long long v) {
  *(__attribute__((address_space(3))) unsigned long long*)(uintptr_t)a = v;
}
__device__ __forceinline__ void lds_add_u64(uint32_t a, unsigned long long v) {
  __hip_atomic_fetch_add((__attribute__((address_space(3))) unsigned long long*)(uintptr_t)a, v, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_WORKGROUP);
}
// the workgroup's done counts: acq_rel, so a wave's adds come before it
// counts itself and the last wave reads them after
__device__ __forceinline__ uint32_t lds_add_rtn_u32(uint32_t a, uint32_t v) {
  return __hip_atomic_fetch_add((__attribute__((address_space(3))) uint32_t*)(uintptr_t)a, v, __ATOMIC_ACQ_REL,
                                __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void st64(uint32_t a, uint32_t x, uint32_t y) {
  u32x2 v;
  v.x = x;
  v.y = y;
  *(lds64_t)(uintptr_t)a = v;
}

#define TRIK_SELECT2_CMPS                                                                       \
  "v_cmp_eq_u32_e64 %[x], %[k], %[d]\n\t"                                                       \
  "v_cmp_gt_u32_sdwa %[lt0], %[d], %[w] src0_sel:BYTE_0 src1_sel:BYTE_0\n\t"                    \
  "v_cmp_gt_u32_sdwa %[lt1], %[d], %[w] src0_sel:BYTE_0 src1_sel:BYTE_2\n\t"                    \
  "v_cmp_ge_u32_sdwa %[le0], %[d], %[w] src0_sel:BYTE_1 src1_sel:BYTE_0\n\t"                    \
  "v_cmp_ge_u32_sdwa %[le1], %[d], %[w] src0_sel:BYTE_1 src1_sel:BYTE_2\n\t"                    \
  "v_cmp_le_u32_sdwa %[ge0], %[a], %[w] src0_sel:BYTE_1 src1_sel:BYTE_0\n\t"                    \
  "v_cmp_le_u32_sdwa %[ge1], %[a], %[w] src0_sel:BYTE_1 src1_sel:BYTE_2"
// The selects; q0 / q1 per pixel (MASKS) or only their union (the word is
// flagged: one SALU op fewer per word).
template <bool PER_PIXEL>
__device__ __forceinline__ void select2_impl(uint32_t w, uint32_t d, uint32_t bw, uint32_t m1, uint32_t m2, uint64_t vm,
                                             uint32_t& e0, uint32_t& e1, uint64_t& q0, uint64_t& q1) {
  uint64_t x, lt0, lt1, le0, le1, ge0, ge1;
  asm volatile(TRIK_SELECT2_CMPS
               : [x] "=&s"(x), [lt0] "=&s"(lt0), [lt1] "=&s"(lt1), [le0] "=&s"(le0), [le1] "=&s"(le1),
                 [ge0] "=&s"(ge0), [ge1] "=&s"(ge1)
               : [w] "v"(w), [d] "v"(d), [a] "v"(bw), [k] "s"(kChromaExc));
  if (PER_PIXEL) {
    q0 = (x | (lt0 & ~le0)) & vm;
    q1 = (x | (lt1 & ~le1)) & vm;
  } else {
    q0 = (x | (lt0 & ~le0) | (lt1 & ~le1)) & vm;
    q1 = 0;
  }
  const uint64_t k0 = le0 & ge0 & ~x & vm, k1 = le1 & ge1 & ~x & vm;
  asm volatile(
      "v_cndmask_b32_e64 %[e0], %[m2], %[m1], %[lt0]\n\t"
      "v_cndmask_b32_e64 %[e1], %[m2], %[m1], %[lt1]\n\t"
      "v_cndmask_b32_e64 %[e0], 0, %[e0], %[k0]\n\t"
      "v_cndmask_b32_e64 %[e1], 0, %[e1], %[k1]"
      : [e0] "=&v"(e0), [e1] "=&v"(e1)
      : [m1] "v"(m1), [m2] "v"(m2), [lt0] "s"(lt0), [lt1] "s"(lt1), [k0] "s"(k0), [k1] "s"(k1));
}
// The fast-path masks of the two pixels of YUYV word w under run descriptor
// d = b1 | b2 << 8, block word bw (cut A in its byte 1) and mask pair (m1,
// m2): with lt = Y < b1, le = Y <= b2, ge = Y >= A, e = le && ge ? (lt ? m1 :
// m2) : 0.  Byte operands straight from w, d and bw by SDWA compares; the
// selects follow all compares (the VALU-writes-SGPR -> v_cndmask distance
// needs no nops).  q0 / q1 (wave masks, SALU) flag the pixels the exact path
// resolves: a window pixel (lt and not le, where the select gives 0; windows
// lie above the cut) or any pixel of an exception-code word (le is cleared,
// so the select gives 0 as well).  vm masks lanes without a valid row.
__device__ __forceinline__ void select2(uint32_t w, uint32_t d, uint32_t bw, uint32_t m1, uint32_t m2, uint64_t vm,
                                        uint32_t& e0, uint32_t& e1, uint64_t& q0, uint64_t& q1) {
  select2_impl<true>(w, d, bw, m1, m2, vm, e0, e1, q0, q1);
}
// The same, with only the word's flag (q0 | q1).
__device__ __forceinline__ uint64_t select2w(uint32_t w, uint32_t d, uint32_t bw, uint32_t m1, uint32_t m2,
                                             uint64_t vm, uint32_t& e0, uint32_t& e1) {
  uint64_t q, unused;
  select2_impl<false>(w, d, bw, m1, m2, vm, e0, e1, q, unused);
  return q;
}

// Record store (a piece's 4 words at wa, its meta word at ma) by the lanes of
// wave mask m only: EXEC narrowed and restored inside one asm block (no
// branch).  The compiler's own LDS counters stay conservative: LDS operations
// of a wave complete in order.
__device__ __forceinline__ void store_record(uint64_t m, uint32_t wa, u32x4 w, uint32_t ma, uint32_t meta) {
  uint64_t saved;
  asm volatile(
      "s_and_saveexec_b64 %[sv], %[m]\n\t"
      "ds_write_b128 %[wa], %[w]\n\t"
      "ds_write_b32 %[ma], %[mt]\n\t"
      "s_mov_b64 exec, %[sv]"
      : [sv] "=&s"(saved)
      : [m] "s"(m), [wa] "v"(wa), [w] "v"(w), [ma] "v"(ma), [mt] "v"(meta)
      : "memory", "scc");
}

// one 16-byte streaming (nontemporal) load
__device__ __forceinline__ uint4 ld_nt16(const uint8_t* p) {
  const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
  return make_uint4(v.x, v.y, v.z, v.w);
}

// 2 v + (this lane's bit of wave mask m): one v_addc_co_u32 with the mask as
// its carry-in (a record's flag bits, shifted in word by word; the carry-in
// is written by SALU, no wait state)
__device__ __forceinline__ uint32_t shift_in(uint32_t v, uint64_t m) {
  uint32_t r;
  uint64_t co;
  asm volatile("v_addc_co_u32_e64 %0, %1, %2, %2, %3" : "=v"(r), "=&s"(co) : "v"(v), "s"(m));
  return r;
}
// 4-bit mask (range t -> bit t) -> byte-spread (range t -> bit 8t)
__device__ __forceinline__ uint32_t spread4(uint32_t m) { return (m * 0x00204081u) & 0x01010101u; }

// chroma index U | V << 8 of a YUYV word (b0=Y0, b1=U, b2=Y1, b3=V)
__device__ __forceinline__ uint32_t chroma_of(uint32_t w) { return __builtin_amdgcn_perm(w, w, 0x0C0C0301u); }
// the same shifted left by 8 (U << 8 | V << 16): the hot loop's run-descriptor
// address 2c is then one right shift (v_lshrrev: half the issue cost of the
// v_lshlrev that 2c needs; C4 -1 %, scripts/ab/r05j.py)
__device__ __forceinline__ uint32_t chroma_of8(uint32_t w) { return __builtin_amdgcn_perm(w, w, 0x0C03010Cu); }

// The exact mask (bit t = range t) of pixel PIX of YUYV word w: the stripe
// kernel's arithmetic (trik_hsv_stripe_px.h: WSEQ:181-249 via v_dot4, the
// 16-bit wrap in v_bfe) with LUT43/LUT255 and the H, S, V tests from LDS.
template <int PIX>
__device__ __forceinline__ uint32_t exact_mask(uint32_t w) {
  constexpr uint32_t kY = PIX == 0 ? 74u : (74u << 16);
  const uint32_t wc = w ^ 0xFF00FF00u;
  const int r = stripe_px::clamp8_shift6(__builtin_amdgcn_udot4(w, kY | (102u << 24), (uint32_t)-14248, false));
  const int g = stripe_px::clamp8_shift6(
      __builtin_amdgcn_udot4(wc, kY | (25u << 8) | (52u << 24), (uint32_t)-10939, false));
  const int b = stripe_px::clamp8_shift6(__builtin_amdgcn_udot4(w, kY | (129u << 8), (uint32_t)-17672, false));
  const int mx = max(r, max(g, b)), mn = min(r, min(g, b));
  const uint32_t d = (uint32_t)(mx - mn);
  const int m = (int)ld16(kLdsLut43 + 2u * d);
  const uint32_t S = (ld16(kLdsLut255 + 2u * (uint32_t)mx) * d) >> 8;
  // hue case select as in stripe_px::phase1 (G > B > R on ties), branch-free
  const bool eqG = mx == g, eqB = mx == b;
  const int dR = g - b, dG = b - r, dB = r - g;
  const int diff = eqG ? dG : (eqB ? dB : dR);
  const int base = eqG ? 21845 : (eqB ? 43690 : 0);
  const uint32_t H = ((uint32_t)(base + m * diff) >> 8) & 0xFFu;
  return ld8(kLdsHue + H) & ld8(kLdsSat + S) & ld8(kLdsVal + (uint32_t)mx);
}

// ---------------------------------------------------------------------------
// Builder
// ---------------------------------------------------------------------------
// The exact-path tables (LUT43, LUT255, per-value H, S, V range masks) at
// their LDS image addresses (exact_mask reads them there).
__device__ __forceinline__ void stage_exact_tables(const RangeTables* t, int tid, int n) {
  for (int i = tid; i < 256; i += n) {
    *(lds16_t)(uintptr_t)(kLdsLut43 + 2 * i) = t->lut43[i];
    *(lds16_t)(uintptr_t)(kLdsLut255 + 2 * i) = t->lut255[i];
    *(lds8_t)(uintptr_t)(kLdsHue + i) = t->hue[i];
    *(lds8_t)(uintptr_t)(kLdsSat + i) = t->smask[i];
    *(lds8_t)(uintptr_t)(kLdsVal + i) = t->vmask[i];
  }
}

// The hot kernels' LDS image (block words, mask-pair palette, run
// descriptors, exact-path tables) staged by a 1024-lane workgroup: every
// lane issues all its global loads (8 run chunks, a block chunk, a palette
// entry, the exact tables' entries) before its first LDS store, so the
// workgroup pays one load latency instead of one per chunk (a load-store
// loop waited ~8 times).
__device__ __forceinline__ void stage_chroma_image(const ChromaTables* ct, const RangeTables* rt, int t) {
  constexpr int kRunChunks = 131072 / 16, kBlockChunks = 8192 / 16;
  static_assert(kRunChunks % 1024 == 0 && kBlockChunks <= 1024 && kChromaPalette <= 1024, "1024-lane staging");
  const u32x4* runs = reinterpret_cast<const u32x4*>(ct->runs);
  u32x4 r[kRunChunks / 1024];
#pragma unroll
  for (int k = 0; k < kRunChunks / 1024; ++k) r[k] = runs[t + 1024 * k];
  u32x4 blk = {0u, 0u, 0u, 0u};
  if (t < kBlockChunks) blk = reinterpret_cast<const u32x4*>(ct->blocks)[t];
  uint32_t p0 = 0, p1 = 0;
  if (t < kChromaPalette) {
    p0 = ct->palette[2 * t];
    p1 = ct->palette[2 * t + 1];
  }
  uint32_t l43 = 0, l255 = 0, hu = 0, sm = 0, vm = 0;
  if (t < 256) {
    l43 = rt->lut43[t];
    l255 = rt->lut255[t];
    hu = rt->hue[t];
    sm = rt->smask[t];
    vm = rt->vmask[t];
  }
#pragma unroll
  for (int k = 0; k < kRunChunks / 1024; ++k) *(lds128_t)(uintptr_t)(kLdsRuns + 16u * (uint32_t)(t + 1024 * k)) = r[k];
  if (t < kBlockChunks) *(lds128_t)(uintptr_t)(kLdsBlocks + 16u * (uint32_t)t) = blk;
  if (t < kChromaPalette) st64(kLdsPairs + 8u * (uint32_t)t, p0, p1);
  if (t < 256) {
    *(lds16_t)(uintptr_t)(kLdsLut43 + 2 * t) = (uint16_t)l43;
    *(lds16_t)(uintptr_t)(kLdsLut255 + 2 * t) = (uint16_t)l255;
    *(lds8_t)(uintptr_t)(kLdsHue + t) = (uint8_t)hu;
    *(lds8_t)(uintptr_t)(kLdsSat + t) = (uint8_t)sm;
    *(lds8_t)(uintptr_t)(kLdsVal + t) = (uint8_t)vm;
  }
}

// One workgroup of 1024 per V: the exact T-bit mask of every (Y, U) -- the
// 256 chromas' profiles, two Y per YUYV word through exact_mask (the stripe
// kernel's arithmetic on LDS tables, held to the oracle on all 2^24 triples)
// into LDS -- then each chroma's profile summarised as its runs with the
// trailing zero run removed:
//   bits 0-1 number of runs (3 = more than two), 4-7 v1, 8-11 v2,
//   12-20 end of run 1, 21-29 end of run 2 (two runs) or of the last nonzero
//   run (more than two).
// The walk is split in four 64-Y segments per chroma (one thread each: its
// first and last mask, its value changes -- the first three with their Y --
// and its last nonzero Y), which one thread per chroma then joins.
constexpr uint32_t kSumStride = 260;  // profile rows, padded against bank conflicts
constexpr uint32_t kSumProf = 16384;  // [256][kSumStride] u8, after the exact tables
constexpr uint32_t kSumSeg = kSumProf + 256 * kSumStride;  // [4][256] segment records of 8 u32
constexpr uint32_t kSumLds = kSumSeg + 4 * 256 * 32;
static_assert(kLdsVal + 256 <= kSumProf && kSumLds <= 160 * 1024, "summary LDS image");
__global__ __launch_bounds__(1024) void chroma_summary_kernel(const RangeTables* t, ChromaTables* ct) {
  const uint32_t V = blockIdx.x, tid = threadIdx.x;
  stage_exact_tables(t, (int)tid, (int)blockDim.x);
  if (V == 0 && tid == 0) {  // summed by the block kernel's palette pass; the hot kernel's count
    ct->flagged_cost = 0ull;
    ct->flagged_words = 0ull;
  }
  __syncthreads();
  const uint32_t U = tid & 255u, seg = tid >> 8;  // a wave: 64 chromas, one segment
  const uint32_t row = kSumProf + U * kSumStride;
  for (uint32_t j = seg * 32u; j < seg * 32u + 32u; ++j) {
    const uint32_t w = (2u * j) | (U << 8) | ((2u * j + 1u) << 16) | (V << 24);
    *(lds16_t)(uintptr_t)(row + 2u * j) = (uint16_t)(exact_mask<0>(w) | (exact_mask<1>(w) << 8));
  }
  __syncthreads();
  {  // this segment: Y in [64 seg, 64 seg + 64)
    const uint32_t y0 = 64u * seg;
    uint32_t q = *(lds32_t)(uintptr_t)(row + y0);
    const uint32_t first = q & 0xFFu;
    // (the first three changes in three registers by selects: an array
    // indexed by a per-lane count would live in scratch memory)
    uint32_t prev = first, c = 0, cz = 0, ev0 = 0, ev1 = 0, ev2 = 0;  // ev: Y | value << 16
    int lnz = first ? (int)y0 : -1;
    for (uint32_t k = 1; k < 64; ++k) {
      if ((k & 3u) == 0) q = *(lds32_t)(uintptr_t)(row + y0 + k);
      const uint32_t m = (q >> (8u * (k & 3u))) & 0xFFu;
      const uint32_t e = (y0 + k) | (m << 16);
      const bool chg = m != prev;
      ev0 = chg && c == 0 ? e : ev0;
      ev1 = chg && c == 1 ? e : ev1;
      ev2 = chg && c == 2 ? e : ev2;
      c += chg ? 1u : 0u;
      prev = m;
      lnz = m ? (int)(y0 + k) : lnz;
      cz = m ? c : cz;
    }
    const uint32_t ne = c < 3 ? c : 3u;
    const uint32_t ev[3] = {ev0, ev1, ev2};
    const uint32_t rec = kSumSeg + (seg * 256u + U) * 32u;
    *(lds32_t)(uintptr_t)(rec + 0) = first | (prev << 8) | (ne << 16);
    *(lds32_t)(uintptr_t)(rec + 4) = c;
    *(lds32_t)(uintptr_t)(rec + 8) = cz;
    *(lds32_t)(uintptr_t)(rec + 12) = (uint32_t)lnz;
    *(lds32_t)(uintptr_t)(rec + 16) = ev[0];
    *(lds32_t)(uintptr_t)(rec + 20) = ev[1];
    *(lds32_t)(uintptr_t)(rec + 24) = ev[2];
  }
  __syncthreads();
  if (tid >= 256u) return;
  // the join: the run sequence is the segments' changes in order, plus a
  // change at a segment's first Y when its first mask differs from the last
  // mask before it
  const uint32_t c = U | (V << 8);
  uint32_t v0 = 0, v1 = 0, v2 = 0;   // run values (selects, not a dynamically indexed array)
  int e0 = 256, e1 = 256, e2 = 256;  // exclusive end of runs 0..2 (the next run's first Y)
  int n_ev = 0;                      // changes so far (run k starts at the k-th change)
  int last_nz_run = -1, last_nz_end = 0;
  uint32_t cur = 0;
  for (uint32_t sg = 0; sg < 4; ++sg) {
    const uint32_t rec = kSumSeg + (sg * 256u + U) * 32u;
    const uint32_t h = *(lds32_t)(uintptr_t)(rec + 0);
    const uint32_t first = h & 0xFFu, last = (h >> 8) & 0xFFu, ne = h >> 16;
    const int cnt = (int)*(lds32_t)(uintptr_t)(rec + 4), cz = (int)*(lds32_t)(uintptr_t)(rec + 8);
    const int lnz = (int)*(lds32_t)(uintptr_t)(rec + 12);
    auto change = [&](int y, uint32_t v) {
      e0 = n_ev == 0 ? y : e0;
      e1 = n_ev == 1 ? y : e1;
      e2 = n_ev == 2 ? y : e2;
      v1 = n_ev == 0 ? v : v1;
      v2 = n_ev == 1 ? v : v2;
      ++n_ev;
    };
    if (sg == 0) {
      v0 = first;
    } else if (first != cur) {
      change((int)(64u * sg), first);
    }
    const int before = n_ev;  // changes before this segment's own
    for (uint32_t i = 0; i < 3; ++i) {
      const uint32_t e = *(lds32_t)(uintptr_t)(rec + 16 + 4 * i);
      if (i < ne && n_ev < 3) change((int)(e & 0xFFFFu), e >> 16);
    }
    n_ev = before + cnt;
    if (lnz >= 0) {
      last_nz_run = before + cz;
      last_nz_end = lnz + 1;
    }
    cur = last;
  }
  // runs up to and including the last nonzero one
  const int n = last_nz_run + 1;  // 0: all zero
  // a: end of the first run (its value v1 = the mask at Y = 0, maybe 0);
  // ab: end of run 2 (n == 2) or of the last nonzero run (n > 2)
  auto pack = [&](int nn, uint32_t v1, uint32_t v2, int a) -> uint32_t {
    if (nn == 0) return 0u;
    const int ab = nn == 1 ? a : last_nz_end;
    return (uint32_t)(nn > 2 ? 3 : nn) | (v1 << 4) | ((nn == 2 ? v2 : 0u) << 8) | ((uint32_t)a << 12) |
           ((uint32_t)ab << 21);
  };
  const uint32_t sf = pack(n, v0, v1, e0);
  ct->summary[c] = sf;
  // the profile from its first nonzero Y on: without a leading zero run the
  // same; with one, the runs after it (runs 1 and 2 become runs 0 and 1)
  const bool lead0 = v0 == 0u && n > 0;
  ct->summary_drop[c] = lead0 ? pack(n - 1, v1, v2, e1) : sf;
  ct->first_nz[c] = (uint16_t)(n == 0 ? 256 : (lead0 ? e0 : 0));
  (void)e2;
}

// The run descriptor of one chroma under block masks (M1, M2).  With
// lt = Y < b1 and le = Y <= b2 the hot kernel's mask is le ? (lt ? M1 : M2) : 0:
//  * b1 <= b2 + 1 ("runs"): M1 on [0, b1), M2 on [b1, b2], 0 above b2;
//  * b1 >  b2 + 1 ("window"): M1 on [0, b2], 0 on [b1, 255], and the pixels
//    with b2 < Y < b1 (lt and not le: the select gives 0) are computed exactly;
//  * kChromaExc: both pixels of the word are computed exactly (le is masked).
__device__ __forceinline__ uint32_t chroma_desc(uint32_t s, uint32_t M1, uint32_t M2) {
  const uint32_t n = s & 3u;
  if (n == 0) {  // all zero
    if (M1 == 0) return 255u | (254u << 8);
    if (M2 == 0) return 0u | (255u << 8);
    return kChromaExc;
  }
  const uint32_t v1 = (s >> 4) & 15u, v2 = (s >> 8) & 15u;
  const uint32_t a = (s >> 12) & 511u, ab = (s >> 21) & 511u;
  if (n == 1) {
    if (v1 == M2) return 0u | ((a - 1u) << 8);
    if (v1 == M1 && a <= 255u) return a | ((a - 1u) << 8);
  }
  if (n == 2 && v1 == M1 && v2 == M2) return a | ((ab - 1u) << 8);
  // window: the profile must be M1 at Y = 0 and 0 at Y = 255
  if (v1 != M1 || ab > 255u) return kChromaExc;
  const uint32_t b2 = a - 1u, b1 = ab;
  if (b2 == 0u && b1 == 255u) return kChromaExc;  // that window is the exception code
  return b1 | (b2 << 8);
}

// Expected exact-path words per 65536 words of a chroma (uniform Y): a window
// of L values flags a word with probability 1 - (1 - L/256)^2.
__device__ __forceinline__ uint32_t chroma_cost(uint32_t d) {
  if (d == kChromaExc) return 65536u;
  const uint32_t b1 = d & 255u, b2 = d >> 8;
  if (b1 <= b2 + 1u) return 0u;
  const uint32_t L = b1 - b2 - 1u;
  return L * (512u - L);
}

// The descriptor of chroma i of a block under mask pair k and cut A: its
// profile is zero below first_nz = f, so with f > A the cut changes nothing
// (the full summary), with f == A the profile from A on is described (the
// summary without the leading zero run), and with f < A the cut would clear
// nonzero pixels: the exception code.
__device__ __forceinline__ uint32_t chroma_desc_cut(uint32_t sf, uint32_t sd, uint32_t f, uint32_t k, uint32_t A) {
  if (f < A) return kChromaExc;
  return chroma_desc(f == A ? sd : sf, k & 15u, k >> 4);
}

// One wave per 16-chroma block b = (V << 4) | (U >> 4), 16 blocks per
// workgroup: the candidate mask pairs k = M1 | M2 << 4 and cuts A (0, or the
// first nonzero Y of one of the block's chromas) are listed in the wave's LDS
// and their combinations spread over its 64 lanes; the wave keeps the
// (cost, k, A) with the fewest expected exact-path words over the block
// (ties: smaller k, then smaller A).
// PALETTE = false: all pairs whose masks occur in the block (best[b]).
// PALETTE = true: every workgroup first ranks the pairs the first pass chose
// (from best[], in LDS; workgroup 0 stores the result): the palette is the
// (up to) kChromaPalette most used pairs (ties: the smaller k), palette_of[k]
// = 8 * slot or 0xFF, with the byte-spread pair of each slot.  Then the
// palette's pairs only (the same choice when the unrestricted pair made the
// palette, which is nearly always), the block word (the pair's palette offset
// | the cut << 8), the run descriptors, and the blocks' expected exact-path
// words added into flagged_cost (one atomic per workgroup).
constexpr int kBlocksPerGroup = 16;
template <bool PALETTE>
__global__ __launch_bounds__(1024) void chroma_block_kernel(ChromaTables* ct) {
  __shared__ uint32_t sf[kBlocksPerGroup][16], sd[kBlocksPerGroup][16], fz[kBlocksPerGroup][16];
  __shared__ uint32_t pairs[kBlocksPerGroup][256], cuts[kBlocksPerGroup][17];
  __shared__ uint32_t hist[256];
  __shared__ uint8_t pal_of[256];
  __shared__ unsigned long long part[kBlocksPerGroup];
  const uint32_t tid = threadIdx.x, lane = tid & 63u, wv = tid >> 6;
  const int b = (int)(blockIdx.x * kBlocksPerGroup + wv);
  const uint32_t c0 = ((uint32_t)(b >> 4) << 8) | ((uint32_t)(b & 15) << 4);
  if (lane < 16) {
    sf[wv][lane] = ct->summary[c0 + lane];
    sd[wv][lane] = ct->summary_drop[c0 + lane];
    fz[wv][lane] = ct->first_nz[c0 + lane];
  }
  if (PALETTE) {  // the palette, from the first pass's choices
    if (tid < 256u) hist[tid] = 0u;
    __syncthreads();
    for (uint32_t i = tid; i < 4096u; i += blockDim.x) atomicAdd(&hist[(uint32_t)(ct->best[i] >> 9) & 255u], 1u);
    __syncthreads();
    if (tid < 256u) {
      const uint32_t k = tid, n = hist[k];
      uint32_t rank = 0;
      for (uint32_t j = 0; j < 256; ++j) {
        const uint32_t m = hist[j];
        rank += (m > n) | ((m == n) & (j < k));
      }
      const bool in = n > 0 && rank < (uint32_t)kChromaPalette;
      pal_of[k] = in ? (uint8_t)(8u * rank) : (uint8_t)0xFFu;
      if (blockIdx.x == 0) {
        ct->pair_hist[k] = n;
        ct->palette_of[k] = pal_of[k];
        if (in) {
          ct->palette[2 * rank] = spread4(k & 15u);
          ct->palette[2 * rank + 1] = spread4(k >> 4);
        }
      }
    }
    __syncthreads();
  } else {
    __builtin_amdgcn_wave_barrier();
  }
  unsigned long long best = ~0ull;
  // the palette pass: when this block's unrestricted choice (pass 1) made the
  // palette, it is also the cheapest palette choice (the same keys over a
  // subset that contains it) -- no second search
  if (PALETTE) {
    const unsigned long long b1 = ct->best[b];
    if (pal_of[(uint32_t)(b1 >> 9) & 255u] != 0xFFu) best = b1;
  }
  if (best == ~0ull) {  // (wave-uniform)
    // the cuts: 0, then each chroma's first nonzero Y in (0, 255]
    const uint32_t f = lane < 16 ? fz[wv][lane] : 0u;
    const uint64_t cm = __builtin_amdgcn_ballot_w64(lane < 16 && f != 0u && f <= 255u);
    if (lane == 0) cuts[wv][0] = 0u;
    if ((cm >> lane) & 1u) cuts[wv][1 + __builtin_amdgcn_mbcnt_lo((uint32_t)cm, 0u)] = f;
    const uint32_t nc = 1u + (uint32_t)__builtin_popcountll(cm);
    // the pairs: lane l stands for pairs l, l + 64, l + 128, l + 192
    uint32_t present = 1u;  // mask values appearing (value 0 always a candidate)
    if (!PALETTE) {
      for (int i = 0; i < 16; ++i) {
        const uint32_t a = sf[wv][i], d = sd[wv][i];
        if (a & 3u) present |= 1u << ((a >> 4) & 15u);
        if ((a & 3u) == 2u) present |= 1u << ((a >> 8) & 15u);
        if (d & 3u) present |= 1u << ((d >> 4) & 15u);
        if ((d & 3u) == 2u) present |= 1u << ((d >> 8) & 15u);
      }
    }
    uint32_t np = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const uint32_t k = lane + 64u * (uint32_t)q;
      const bool take = PALETTE ? pal_of[k] != 0xFFu
                                : (((present >> (k & 15u)) & 1u) && ((present >> (k >> 4)) & 1u));
      const uint64_t pm = __builtin_amdgcn_ballot_w64(take);
      if (take)
        pairs[wv][np + __builtin_amdgcn_mbcnt_hi((uint32_t)(pm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)pm, 0u))] = k;
      np += (uint32_t)__builtin_popcountll(pm);
    }
    __builtin_amdgcn_wave_barrier();
    unsigned long long mine = ~0ull;
    for (uint32_t combo = lane; combo < np * nc; combo += 64u) {
      const uint32_t k = pairs[wv][combo / nc], A = cuts[wv][combo % nc];
      uint32_t cost = 0;
      for (int i = 0; i < 16; ++i) cost += chroma_cost(chroma_desc_cut(sf[wv][i], sd[wv][i], fz[wv][i], k, A));
      const unsigned long long key = ((unsigned long long)cost << 17) | ((unsigned long long)k << 9) | A;
      if (key < mine) mine = key;
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      const unsigned long long o = __shfl_xor(mine, off, 64);
      if (o < mine) mine = o;
    }
    best = mine;
  }
  if (!PALETTE) {
    if (lane == 0) ct->best[b] = best;  // the palette pass histograms the pairs
    return;
  }
  const uint32_t bk = (uint32_t)(best >> 9) & 255u, bA = (uint32_t)best & 511u;
  if (lane < 16) ct->runs[c0 + lane] = (uint16_t)chroma_desc_cut(sf[wv][lane], sd[wv][lane], fz[wv][lane], bk, bA);
  if (lane == 0) {
    ct->blocks[b] = (uint16_t)(pal_of[bk] | (bA << 8));
    ct->block_cost[b] = (uint32_t)(best >> 17);
    part[wv] = best >> 17;
  }
  __syncthreads();
  if (tid == 0) {
    unsigned long long sum = 0;
    for (int i = 0; i < kBlocksPerGroup; ++i) sum += part[i];
    atomicAdd(&ct->flagged_cost, sum);
  }
}


// ---------------------------------------------------------------------------
// Hot kernel
// ---------------------------------------------------------------------------
// cpr chunk columns per row, k lanes' rows per step (a lane's first piece),
// rstep rows per step, steps per tile.  YUYV: a lane's chunk is two 16-byte
// pieces, the second dy rows below and dx pixels right of the first (dy = k,
// dx = 0, rstep = 2k; rows wider than kHotLanes pieces: dy = 0, dx = W/2,
// rstep = k); ov7670: one 16-pixel piece (dy = dx = 0, rstep = k).
struct ChromaGeom {
  int32_t cpr, k, rstep, dy, dx, steps, tiles_per_frame;
  int32_t steps_last;  // steps of a frame's last tile
  int64_t n_tiles;
  int32_t flush_rounds;  // drain rounds between unpacks of the 16-bit exception sums
  // divisions of the per-unit setup by multiplication: units per tile (the
  // workgroup's waves) and tiles per frame (wave-uniform: SALU), and a lane's
  // index in its tile by cpr: ro = lt * cpr_inv >> 20 with cpr_inv =
  // ceil(2^20 / cpr), exact for lt < 1024 and cpr < 1024
  FastDiv fd_units, fd_tiles;
  uint32_t cpr_inv;
  int32_t tail_ok;  // the past-the-end loads read the handle's sink (KernelArgs::tail)
  int64_t tail_span;  // bytes from a tile's base those loads span (chroma_tail_span)
  int32_t units;  // wave-sized units per tile: ceil(k * cpr / 64) <= kHotWaves
};

// The 12 per-lane values (3 per range, 4 ranges) summed over the wave: two
// lane-half swaps (permlane32 / permlane16) leave three values per lane, each
// the partial sum of one value over lanes 16 apart, then four DPP row steps.
// Value i + 3 * r ends in lane 16 r + 15 (r = 0..3) of v[i], i = 0..2.
__device__ __forceinline__ void wave_sums12(uint32_t (&v)[12]) {
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    const auto s = __builtin_amdgcn_permlane32_swap(v[i], v[i + 6], false, false);
    v[i] = s[0] + s[1];
  }
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const auto s = __builtin_amdgcn_permlane16_swap(v[i], v[i + 3], false, false);
    v[i] = s[0] + s[1];
  }
#pragma unroll
  for (int i = 0; i < 3; ++i) v[i] += __builtin_amdgcn_update_dpp(0u, v[i], 0x111, 0xF, 0xF, true);
#pragma unroll
  for (int i = 0; i < 3; ++i) v[i] += __builtin_amdgcn_update_dpp(0u, v[i], 0x112, 0xF, 0xF, true);
#pragma unroll
  for (int i = 0; i < 3; ++i) v[i] += __builtin_amdgcn_update_dpp(0u, v[i], 0x114, 0xF, 0xF, true);
#pragma unroll
  for (int i = 0; i < 3; ++i) v[i] += __builtin_amdgcn_update_dpp(0u, v[i], 0x118, 0xF, 0xF, true);
}

// One chunk = 8 YUYV words (16 pixels) in two 4-word pieces: YUYV, two
// 16-byte pieces (8 pixels each) at p and pb -- the same columns of two rows,
// so that one load instruction of a wave reads 1 KiB contiguous; ov7670, 16
// luma + 16 chroma bytes of one row of the two planes (pb unused).
template <int LAYOUT>
__device__ __forceinline__ void load_chunk(const uint8_t* p, const uint8_t* pb, int64_t plane, uint32_t (&w)[8]) {
  if (LAYOUT == TRIK_HSV_LAYOUT_YUYV) {
    const u32x4 va = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
    const u32x4 vb = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(pb));
    w[0] = va.x; w[1] = va.y; w[2] = va.z; w[3] = va.w;
    w[4] = vb.x; w[5] = vb.y; w[6] = vb.z; w[7] = vb.w;
  } else {
    const uint4 vy = ld_nt16(p);  // (nontemporal: 1 % faster, scripts/ab/r05l_c7.py)
    const uint4 vc = ld_nt16(p + plane);
    const uint32_t yy[4] = {vy.x, vy.y, vy.z, vy.w}, cc[4] = {vc.x, vc.y, vc.z, vc.w};
    // OSEQ:369-373: U = odd chroma byte, V = even chroma byte
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      w[2 * j] = __builtin_amdgcn_perm(cc[j], yy[j], 0x04010500u);
      w[2 * j + 1] = __builtin_amdgcn_perm(cc[j], yy[j], 0x06030702u);
    }
  }
}

__device__ __forceinline__ uint32_t pack_bits(uint32_t e) { return ((e * 0x01020408u) >> 24) & 0xFu; }

// Per-lane sums of the exception pixels a lane drained: EN byte-packed counts
// (range t in byte t), SX/SY 16-bit fields (ranges 0,2 | 1,3) of x and of the
// row relative to the tile's first row; unpacked into 32-bit per-range sums
// every flush_rounds rounds and at the tile end.
struct ExcSums {
  uint32_t EN = 0, SX02 = 0, SX13 = 0, SY02 = 0, SY13 = 0;
  int rounds = 0;
};

template <int LAYOUT, int NR, bool MASKS>
__global__ __launch_bounds__(kMaxBlock) void chroma_kernel(KernelArgs a, ChromaGeom g, const ChromaTables* ct) {
  if (gated_out(a.gate, a.gate_max, a.gate_le)) return;
  constexpr int CW = kChunkWords;
  const int t = threadIdx.x;
  static_assert(64 * kHotWaves == 1024, "the hot kernel's workgroup stages the image");
  stage_chroma_image(ct, a.tables, t);  // the block words, palette, run descriptors, exact-path tables
  // This workgroup's units: an even share of the batch's wave-sized units
  // (unit u: tile u / U, lanes 64 (u % U) ..), whatever the frame boundaries
  // (a frame's units may lie in several workgroups: the fused step counts
  // them done per frame)
  const uint32_t U = (uint32_t)g.units;                    // wave-sized units per tile
  const uint32_t n_units_all = (uint32_t)(g.n_tiles * U);  // (< 2^32: chroma_geometry)
  const uint32_t u_begin = (uint32_t)((uint64_t)n_units_all * blockIdx.x / gridDim.x);
  const uint32_t u_end = (uint32_t)((uint64_t)n_units_all * (blockIdx.x + 1) / gridDim.x);
  const uint32_t upf = U * (uint32_t)g.tiles_per_frame;   // units per frame
  if (a.fused && t < 12) st_u64(kLdsTotals + 8 * t, 0ull);
  if (t < 3) *(lds32_t)(uintptr_t)(kLdsWords + 4 * t) = 0u;
  __syncthreads();

  const int lane = t & 63;
  const uint32_t wave = (uint32_t)(t >> 6);
  const uint32_t rw_s = __builtin_amdgcn_readfirstlane(kLdsRecWords + wave * (kRecCap * 16u));
  const uint32_t rm_s = __builtin_amdgcn_readfirstlane(kLdsRecMeta + wave * (kRecCap * 4u));
  // YUYV: a lane's 8 words are 4 from row y (piece a) and 4 from row y + dy,
  // dx pixels right (piece b; word i at x0 + 2 (i & 3)); ov7670: 8 words of
  // row y (piece b 8 pixels right; word i at x0 + 2i)
  constexpr bool SPLIT = LAYOUT == TRIK_HSV_LAYOUT_YUYV;
  const int64_t plane = (int64_t)a.height * a.line_length;
  const int64_t rowstep = (int64_t)g.rstep * a.line_length;
  const int half = SPLIT ? g.dy : 0;  // rows between a chunk's two pieces
  const uint32_t dx = SPLIT ? (uint32_t)g.dx : 0u;  // and pixels
  const int64_t hb = (int64_t)half * a.line_length + 2 * (int64_t)dx;
  constexpr int kQBlock = 5;  // Q block: CW * n * (n + 1) <= 255
  auto xoff = [=](int i) { return SPLIT ? (i < 4 ? 0u : dx) + 2u * (uint32_t)(i & 3) : 2u * (uint32_t)i; };
  const uint32_t meta_b = ((SPLIT ? dx >> 3 : 1u) << 4) + ((uint32_t)half << 16);

  uint32_t resolved = 0;  // words this wave's exact path resolved (wave-uniform)
  // The fused step's per-frame completion (wave-uniform): a unit's sums go
  // to its frame's accumulator by device atomics, which execute at the memory
  // side; once they are performed (this wave's vmcnt wait at its NEXT unit's
  // end, when they long have been) the unit counts itself done on the
  // frame's counter, and the count that counter returned is examined at the
  // unit end after that (its latency hides behind a unit's loads).  The wave
  // that counts a frame's last unit finalizes it.
  int32_t pend_f = -1;  // frame of this wave's last emitted unit, not counted yet
  int32_t chk_f = -1;   // frame whose count was issued, not examined yet
  uint32_t chk_r = 0;   // lane 0: that count's value before this wave's add
  // the frame's sums (exchanged for zero: the accumulator is clean for the
  // next launch), its targets (WSEQ:486-505), its share of the totals
  auto finalize = [&](int32_t F) {
    unsigned long long* acc = a.frame_acc + 16 * (int64_t)F;
    if (lane < NR) {
      const uint64_t n = atomicExch(acc + 3 * lane, 0ull);
      const uint64_t sx = atomicExch(acc + 3 * lane + 1, 0ull);
      const uint64_t sy = atomicExch(acc + 3 * lane + 2, 0ull);
      const int64_t o = (int64_t)F * a.sums_ranges + a.range_offset + lane;
      a.sums[o] = TrikHsvTargetSums{(int64_t)n, (int64_t)sx, (int64_t)sy};
      if (a.targets) a.targets[o] = target_of(n, sx, sy, a.width, a.height);
      if (a.totals) {
        lds_add_u64(kLdsTotals + 24u * (uint32_t)lane, n);
        lds_add_u64(kLdsTotals + 24u * (uint32_t)lane + 8u, sx);
        lds_add_u64(kLdsTotals + 24u * (uint32_t)lane + 16u, sy);
      }
    }
    if (lane == 0)  // the unit count (word 24 of the frame's line)
      __hip_atomic_store(reinterpret_cast<uint32_t*>(acc + 12), 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  };
  auto examine = [&]() {  // the count issued at the previous unit end
    if (chk_f < 0) return;
    if (__builtin_amdgcn_readfirstlane(chk_r) + 1u == upf) finalize(chk_f);
    chk_f = -1;
  };
  auto count_done = [&]() {  // the last emitted unit, once its atomics are performed
    if (pend_f < 0) return;
    // The release between this wave's relaxed accumulator adds and its
    // relaxed count add: on gfx950 (GFX9 counters) vmcnt also counts atomics
    // without return, and device-scope atomics execute at the memory side, so
    // once vmcnt is 0 the adds are performed for every later atomic (the
    // finalizing wave's atomicExch included).  A release fence would also
    // write back this CU's L2 lines (buffer_wbl2) at every unit end.  The
    // file is gfx950-only (see the guard at the top).
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    uint32_t r = 0;
    if (lane == 0) r = atomicAdd(reinterpret_cast<uint32_t*>(a.frame_acc + 16 * (int64_t)pend_f + 12), 1u);
    chk_r = r;
    chk_f = pend_f;
    pend_f = -1;
  };
  // Units handed to the workgroup's waves in order as they finish (a wave's
  // first unit is its own index): the waves of a SIMD with fewer waves run
  // faster and take more units, so the SIMDs end together.
  for (uint32_t u = u_begin + __builtin_amdgcn_readfirstlane(wave); u < u_end;) {  // (wave-uniform: SGPRs)
    uint32_t next = 0;
    if (lane == 0) next = __hip_atomic_fetch_add((__attribute__((address_space(3))) uint32_t*)(uintptr_t)kLdsUnits,
                                                 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    // (wave-uniform divisions by multiplication; the results are moved to
    // SGPRs, else everything derived from them stays in VGPRs)
    // (tile indices fit 32 bits: chroma_geometry)
    const uint32_t tile = __builtin_amdgcn_readfirstlane(fdiv(u, g.fd_units));
    const int f = (int)__builtin_amdgcn_readfirstlane(fdiv(tile, g.fd_tiles));
    const int trem = (int)(tile - (uint32_t)f * (uint32_t)g.tiles_per_frame);
    const int lt = (int)((u - tile * U) * 64u) + lane;  // the lane's index in the tile (< 1024)
    const bool active = lt < g.k * g.cpr;
    const uint32_t q = __umul24((uint32_t)lt, g.cpr_inv) >> 20;  // lt / cpr
    const int col = active ? lt - (int)__umul24(q, (uint32_t)g.cpr) : 0;
    const int ro = active ? (int)q : 0;
    const int col_bytes = LAYOUT == TRIK_HSV_LAYOUT_YUYV ? col * 16 : col * 2 * CW;
    const uint32_t x0 = (uint32_t)col * (SPLIT ? 8u : 2u * CW);
    const uint32_t voff = (uint32_t)ro * (uint32_t)a.line_length + (uint32_t)col_bytes;
    // a record's meta word without its flag bits: x / 8 of the piece's first
    // pixel and its row in the tile (piece b: xb8 * 8 pixels right, half rows down)
    const uint32_t meta_x = (x0 >> 3) << 4;
    const int r0 = trem * g.rstep * g.steps;
    const int y0 = r0 + ro;
    const int steps = trem == g.tiles_per_frame - 1 ? g.steps_last : g.steps;
    const uint8_t* p = a.frames + (int64_t)f * a.frame_stride + (int64_t)y0 * a.line_length + col_bytes;

    uint32_t P[CW], O = 0, Q = 0, CumS = 0, CumA = 0, CumB = 0;
#pragma unroll
    for (int i = 0; i < CW; ++i) P[i] = 0;
    uint32_t Qa = 0, Qb = 0, Ba = 0, Bb = 0;
    int nb = 0;
    // record queue (wave-uniform count) and this lane's exact-path sums
    int qn = 0;
    ExcSums ex;
    // the exact-path sums unpacked into 12 per-lane values (then zeroed)
    auto unpack_exc = [&](uint32_t (&v)[12]) {
#pragma unroll
      for (int rr = 0; rr < NR; ++rr) {
        const uint32_t sx = (rr & 1) ? ex.SX13 : ex.SX02, sy = (rr & 1) ? ex.SY13 : ex.SY02;
        const int sh = (rr >> 1) * 16;
        const uint32_t n = (ex.EN >> (8 * rr)) & 0xFFu;
        v[3 * rr + 0] += n;
        v[3 * rr + 1] += (sx >> sh) & 0xFFFFu;
        v[3 * rr + 2] += ((sy >> sh) & 0xFFFFu) + __umul24((uint32_t)r0, n);  // (24-bit: full-rate multiply)
      }
      ex.EN = ex.SX02 = ex.SX13 = ex.SY02 = ex.SY13 = 0;
      ex.rounds = 0;
    };
    // 12 per-lane values summed over the wave into the frame's sums (fused
    // step: its accumulator): device atomics (fire and forget: no wave waits
    // for another)
    auto emit = [&](uint32_t (&v)[12]) {
      wave_sums12(v);
      // lane 16 r + 15 holds values 3 r .. 3 r + 2: range r's N, sum x, sum y
      const int rr = lane >> 4;
      if ((lane & 15) == 15 && rr < NR) {
        unsigned long long* dst =
            a.fused ? a.frame_acc + 16 * (int64_t)f + 3 * rr
                    : reinterpret_cast<unsigned long long*>(
                          &a.sums[(int64_t)f * a.sums_ranges + a.range_offset + rr].points);
#pragma unroll
        for (int j = 0; j < 3; ++j)
          if (v[j]) atomicAdd(dst + j, (unsigned long long)v[j]);
      }
    };
    // One drain round: lanes 0..take-1 take the last take records, resolve
    // the first flagged word of each exactly (which of its pixels the fast
    // path left to this path: select2; the exact masks: exact_mask) and
    // accumulate them with explicit (x, y); a record with more flagged words
    // goes back to the queue with its remaining bits.  Verification mode
    // writes the exact masks.
    auto drain = [&](int take) {
      resolved += (uint32_t)take;
      const uint32_t base = (uint32_t)(qn - take);
      const bool act = lane < take;
      const uint32_t rec = rw_s + 16u * (base + (uint32_t)lane);
      const uint32_t meta = act ? *(lds32_t)(uintptr_t)(rm_s + 4u * (base + (uint32_t)lane)) : 0u;
      const uint32_t fl = meta & 15u;
      if (act) {
        const uint32_t i = 3u - (uint32_t)__builtin_ctz(fl);
        const uint32_t w = *(lds32_t)(uintptr_t)(rec + 4u * i);  // the record's first flagged word
        const uint32_t x = ((meta >> 4) & 0xFFFu) * 8u + 2u * i, yr = meta >> 16;
        const uint32_t d = ld16(kLdsRuns + 2u * chroma_of(w));
        const uint32_t lo = d & 0xFFu, hi = d >> 8, Y0 = w & 0xFFu, Y1 = (w >> 16) & 0xFFu;
        const bool xw = d == kChromaExc;
        const bool f0 = xw | ((Y0 < lo) & (Y0 > hi)), f1 = xw | ((Y1 < lo) & (Y1 > hi));
        const uint32_t m0 = f0 ? exact_mask<0>(w) : 0u;
        const uint32_t m1 = f1 ? exact_mask<1>(w) : 0u;
        if (MASKS) {
          uint8_t* mp = a.masks + ((int64_t)f * a.height + r0 + yr) * a.width + x;
          if (f0) mp[0] = a.mask_shift ? (uint8_t)(mp[0] | (m0 << a.mask_shift)) : (uint8_t)m0;
          if (f1) mp[1] = a.mask_shift ? (uint8_t)(mp[1] | (m1 << a.mask_shift)) : (uint8_t)m1;
        }
        const uint32_t e0 = spread4(m0), e1 = spread4(m1);
        ex.EN += e0 + e1;
        const uint32_t a0 = e0 & 0x00FF00FFu, a1 = e1 & 0x00FF00FFu;
        const uint32_t b0 = (e0 >> 8) & 0x00FF00FFu, b1 = (e1 >> 8) & 0x00FF00FFu;
        ex.SX02 += (a0 + a1) * x + a1;
        ex.SX13 += (b0 + b1) * x + b1;
        ex.SY02 += (a0 + a1) * yr;
        ex.SY13 += (b0 + b1) * yr;
      }
      if (++ex.rounds == g.flush_rounds) {  // (rare: the 16-bit sums would overflow)
        uint32_t v[12] = {};
        unpack_exc(v);
        emit(v);
      }
      // records with flagged words left go back, compacted, where the
      // drained ones were (their reads above come first: LDS is in order)
      const uint32_t rest = fl & (fl - 1u);
      const uint64_t left = __builtin_amdgcn_ballot_w64(rest != 0u);
      if (left) {  // (rare on camera-like and uniform input: a piece with two flagged words)
        u32x4 w4 = {0u, 0u, 0u, 0u};
        if (rest) w4 = *(lds128_t)(uintptr_t)rec;
        const uint32_t idx =
            __builtin_amdgcn_mbcnt_hi((uint32_t)(left >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)left, base));
        store_record(left, rw_s + 16u * idx, w4, rm_s + 4u * idx, (meta & ~15u) | rest);
      }
      __builtin_amdgcn_wave_barrier();
      qn = (int)base + (int)__builtin_popcountll(left);
    };
    // Append the records of one piece slot (wave mask m: the lanes whose
    // piece has a flagged word; meta with their flag bits), draining first
    // when the queue cannot take them.
    auto append = [&](uint64_t m, u32x4 w4, uint32_t meta) {
      if (m == 0) return;
      const int cnt = (int)__builtin_popcountll(m);
      while (qn + cnt > kRecCap) drain(qn < 64 ? qn : 64);
      const uint32_t idx =
          __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, (uint32_t)qn));
      store_record(m, rw_s + 16u * idx, w4, rm_s + 4u * idx, meta);
      qn += cnt;
    };

    // a row inside the frame for lanes whose rows run past it (re-read, masked)
    const uint8_t* pf = active && y0 < a.height ? p : a.frames + (int64_t)f * a.frame_stride + col_bytes;
    // steps whose first (second) piece row lies inside the frame
    const bool full = (r0 + steps * g.rstep <= a.height) && (g.k * g.cpr) % 64 == 0;
    // (only partial tiles need them: the divisions run on the VALU)
    int vsteps = steps, vstepsb = steps;
    if (!full) {
      vsteps = active ? max(0, min(steps, (a.height - y0 + g.rstep - 1) / g.rstep)) : 0;
      vstepsb = active ? max(0, min(steps, (a.height - y0 - half + g.rstep - 1) / g.rstep)) : 0;
    }
    const uint8_t* tbase = a.frames + (int64_t)f * a.frame_stride + (int64_t)r0 * a.line_length;
    auto run = [&](auto full_c) {
      constexpr bool FULL = decltype(full_c)::value;
      // One step: the chunk's 8 words.  All LDS lookups are issued before
      // any record write (the queue shares LDS, so the compiler keeps the
      // order), then the selects, then the two pieces' records.
      auto step = [&](const uint32_t (&cw)[CW], int s) {
        const bool valid = FULL || s < vsteps, validb = SPLIT ? (FULL || s < vstepsb) : valid;
        // lanes with a valid row (rows past the frame re-read a valid row:
        // their pixels are masked out of the sums and the queue)
        const uint64_t vma = FULL ? ~0ull : __builtin_amdgcn_ballot_w64(valid);
        const uint64_t vmb = FULL ? ~0ull : (SPLIT ? __builtin_amdgcn_ballot_w64(validb) : vma);
        uint32_t c[CW], d[CW], cut[CW], pr[CW], e[2 * CW];
        u32x2 mm[CW];
#pragma unroll
        for (int i = 0; i < CW; ++i) c[i] = chroma_of8(cw[i]);
#pragma unroll
        for (int i = 0; i < CW; ++i) {
          d[i] = ld16(kLdsRuns + (c[i] >> 7));
          // the block word: the pair's palette offset | the cut << 8
          cut[i] = ld16(kLdsBlocks + ((c[i] >> 11) & 0x1FFEu));
          pr[i] = cut[i] & 0xFFu;
        }
#pragma unroll
        for (int i = 0; i < CW; ++i) mm[i] = ld64(kLdsPairs + pr[i]);
        // pin the descriptors as 32-bit values here (ds_read_u16 zero-extends):
        // otherwise the zero extension is sunk past the drain branches and
        // costs a v_and per word
#pragma unroll
        for (int i = 0; i < CW; ++i) asm volatile("" : "+v"(d[i]), "+v"(cut[i]));
        // per piece: the lanes with a flagged word (SALU) and the record's
        // meta word with the flag bits (bit 3 - j = word j of the piece),
        // shifted in word by word (one v_addc each, round 6: C3 -0.3 %, C4
        // -0.8 %, scripts/ab/r06c_flags.py) so that each word's flag mask dies
        // at once (held for the appends, the eight masks pushed the unit's
        // SGPRs into spills)
        uint64_t ma = 0, mb = 0;
        const uint32_t meta_a = meta_x | ((uint32_t)(ro + s * g.rstep) << 16);
        uint32_t fa = meta_a >> 4, fb = (meta_a + meta_b) >> 4;  // (flag bits 0-3 of the meta words are 0)
#pragma unroll
        for (int i = 0; i < CW; ++i) {
          uint64_t q0 = 0, q1 = 0, bal;
          if (MASKS) {
            select2(cw[i], d[i], cut[i], mm[i].x, mm[i].y, i < 4 ? vma : vmb, e[2 * i], e[2 * i + 1], q0, q1);
            bal = q0 | q1;
          } else {
            bal = select2w(cw[i], d[i], cut[i], mm[i].x, mm[i].y, i < 4 ? vma : vmb, e[2 * i], e[2 * i + 1]);
          }
          // formed here, so the word's compare masks die here (sunk into the
          // append branches they would all stay live in SGPRs)
          asm volatile("" : "+s"(bal));
          if (i < 4) {
            ma |= bal;
            fa = shift_in(fa, bal);
          } else {
            mb |= bal;
            fb = shift_in(fb, bal);
          }
          if (MASKS && (i < 4 ? valid : validb)) {  // verification mode: the exact path writes the flagged pixels
            const int y = y0 + s * g.rstep + (i < 4 ? 0 : half);
            uint8_t* mp = a.masks + ((int64_t)f * a.height + y) * a.width + x0 + xoff(i);
            const uint8_t m0 = (uint8_t)(pack_bits(e[2 * i]) << a.mask_shift);
            const uint8_t m1 = (uint8_t)(pack_bits(e[2 * i + 1]) << a.mask_shift);
            if (!__builtin_amdgcn_inverse_ballot_w64(q0)) mp[0] = a.mask_shift ? (uint8_t)(mp[0] | m0) : m0;
            if (!__builtin_amdgcn_inverse_ballot_w64(q1)) mp[1] = a.mask_shift ? (uint8_t)(mp[1] | m1) : m1;
          }
        }
        u32x4 wa, wb;
        wa.x = cw[0]; wa.y = cw[1]; wa.z = cw[2]; wa.w = cw[3];
        wb.x = cw[4]; wb.y = cw[5]; wb.z = cw[6]; wb.w = cw[7];
        append(ma, wa, fa);
        append(mb, wb, fb);
        while (qn >= 64) drain(64);
#pragma unroll
        for (int i = 0; i < CW; ++i) P[i] = P[i] + e[2 * i] + e[2 * i + 1];
#pragma unroll
        for (int i = 0; i < CW; i += 2) O = O + e[2 * i + 1] + e[2 * i + 3];
#pragma unroll
        for (int i = 0; i < CW; i += 2) Q = Q + P[i] + P[i + 1];
        ++nb;
        if (nb == kQBlock || s + 1 == steps) {
          // n * x for the block length n: a shift-add for full blocks (n is
          // wave-uniform), a multiply only for a tile's last, partial block
          auto flush = [&](auto times) {
            const uint32_t T = Q - times(CumS);
            Qa += T & 0x00FF00FFu;
            Qb += (T >> 8) & 0x00FF00FFu;
            Ba += times(CumA);
            Bb += times(CumB);
            // group sums of the pair counters stay below 256 per byte
            // (4 * 2 * kMaxSteps <= 255), so one split per group
            CumS = CumA = CumB = 0;
#pragma unroll
            for (int g0 = 0; g0 < CW; g0 += 4) {
              const uint32_t G = P[g0] + P[g0 + 1] + P[g0 + 2] + P[g0 + 3];
              CumS += G;
              CumA += G & 0x00FF00FFu;
              CumB += (G >> 8) & 0x00FF00FFu;
            }
          };
          if (nb == kQBlock) flush([](uint32_t x) { return x * (uint32_t)kQBlock; });
          else flush([&](uint32_t x) { return x * (uint32_t)nb; });
          Q = 0;
          nb = 0;
        }
      };
      // rows of step s + 1 loaded while step s is processed (a third buffer,
      // two steps ahead, measured no faster: the kernel is VALU-bound)
      // (the load past the tile's last step is unconditional: that keeps the
      // step's wait at "this step's data", where a branch around it makes the
      // compiler wait for every load in flight.  Its data is never used.  It
      // reads the handle's L2-resident sink when the lanes' offsets fit inside
      // it (tail_ok: chroma_tail_span <= KernelArgs::tail_bytes, checked on
      // the host) -- re-reading the tile's last rows instead cost 2.2 % extra
      // HBM reads, scripts/ab/r05s_tail.py -- and otherwise those rows)
      const uint8_t* rb = tbase;
      const uint8_t* const tail = a.tail;
      auto ld = [&](int s, uint32_t (&w)[CW]) {
        if (FULL) load_chunk<LAYOUT>(rb + voff, rb + hb + voff, plane, w);
        else
          load_chunk<LAYOUT>(s < vsteps ? pf + (int64_t)s * rowstep : pf,
                             s < vstepsb ? pf + hb + (int64_t)s * rowstep : pf, plane, w);
      };
      uint32_t wa[CW], wb[CW];
      ld(0, wa);
      for (int s = 0; s < steps; s += 2) {
        if (FULL) rb = s + 1 < steps ? rb + rowstep : (g.tail_ok ? tail : rb);
        ld(s + 1, wb);
        step(wa, s);
        if (s + 1 >= steps) break;
        if (FULL) rb = s + 2 < steps ? rb + rowstep : (g.tail_ok ? tail : rb);
        ld(s + 2, wa);
        step(wb, s + 1);
      }
    };
    if (full) run(std::true_type{});
    else run(std::false_type{});
    while (qn > 0) drain(qn < 64 ? qn : 64);
    Qa += Ba;
    Qb += Bb;

    uint32_t acc[12] = {};
    // x offsets within the chunk: 2 (i & 3) (+ dx for the second piece) or
    // 2 i; nb2: pixels of the second pieces (rows + half, columns + dx).  The
    // weighted sums are formed on the byte-packed counters with ranges 0, 2
    // (A) and 1, 3 (B) spread into 16-bit halves (one v_perm each), two
    // ranges per operation: halves stay below 2^16 (P bytes <= 2 * kMaxSteps,
    // O bytes <= 8 * kMaxSteps).
    auto half_a = [](uint32_t v) { return __builtin_amdgcn_perm(0u, v, 0x0C020C00u); };  // bytes 0, 2
    auto half_b = [](uint32_t v) { return __builtin_amdgcn_perm(0u, v, 0x0C030C01u); };  // bytes 1, 3
    uint32_t XA = half_a(O), XB = half_b(O), NA = 0, NB = 0;
    if (SPLIT) {
      const uint32_t S1 = P[1] + P[5], S2 = P[2] + P[6], S3 = P[3] + P[7];  // bytes <= 4 * kMaxSteps
      XA += 2u * half_a(S1) + 4u * half_a(S2) + 6u * half_a(S3);
      XB += 2u * half_b(S1) + 4u * half_b(S2) + 6u * half_b(S3);
      const uint32_t N = P[4] + P[5] + P[6] + P[7];  // bytes <= 8 * kMaxSteps
      NA = half_a(N);
      NB = half_b(N);
    } else {
#pragma unroll
      for (int i = 1; i < CW; ++i) {
        XA += (uint32_t)(2 * i) * half_a(P[i]);
        XB += (uint32_t)(2 * i) * half_b(P[i]);
      }
    }
    static_assert(8 * kMaxSteps + 2 * kChunkWords * kChunkWords * 2 * kMaxSteps < 65536, "16-bit halves");
#pragma unroll
    for (int rr = 0; rr < NR; ++rr) {
      const int hs = (rr >> 1) * 16;
      const uint32_t c = ((rr & 1) ? (CumB >> hs) : (CumA >> hs)) & 0xFFFFu;
      uint32_t wx = (((rr & 1) ? XB : XA) >> hs) & 0xFFFFu, nb2 = 0;
      if (SPLIT) {
        nb2 = (((rr & 1) ? NB : NA) >> hs) & 0xFFFFu;
        wx += __umul24(dx, nb2);
      }
      const uint32_t qq = ((rr & 1) ? (Qb >> ((rr >> 1) * 16)) : (Qa >> ((rr >> 1) * 16))) & 0xFFFFu;
      acc[3 * rr + 0] = c;
      acc[3 * rr + 1] = __umul24(x0, c) + wx;
      acc[3 * rr + 2] = __umul24((uint32_t)y0, c) + __umul24((uint32_t)g.rstep, __umul24((uint32_t)steps, c) - qq) +
                        __umul24((uint32_t)half, nb2);
    }
    unpack_exc(acc);
    if (a.fused) {
      examine();
      count_done();
    }
    emit(acc);
    if (a.fused) pend_f = f;
    u = u_begin + __builtin_amdgcn_readfirstlane(next) + (blockDim.x >> 6);  // after the waves' first units
  }
  if (a.fused) {  // this wave's last counts
    examine();
    count_done();
    examine();
  }
  // the exact-path word count: per workgroup in LDS, one device atomic by its
  // last wave (AUTO's measured share, ChromaTables::flagged_words)
  if (lane == 0) {
    if (resolved) lds_add_rtn_u32(kLdsWords, resolved);
    const uint32_t done = lds_add_rtn_u32(kLdsWords + 4, 1u);
    if (done + 1 == (blockDim.x >> 6)) {
      const uint32_t n = *(lds32_t)(uintptr_t)kLdsWords;
      if (n) atomicAdd(const_cast<unsigned long long*>(&ct->flagged_words), (unsigned long long)n);
    }
  }
  if (!a.fused) return;
  // fused step: the per-target totals (the workgroup's finalized frames'
  // sums, in LDS once every wave is here).  Every workgroup stores its totals; the
  // last one to finish (a device-scope counter, reset by it for the next
  // launch) sums them into a.totals.
  if (!a.totals) return;
  __syncthreads();
  // wave 0 alone publishes (its 12 stores, one device-scope fence: an L2
  // write-back per workgroup, not per wave) and counts the workgroup done
  if (t < 64) {
    unsigned long long* part = a.wg_part + 12 * (int64_t)blockIdx.x;
    if (t < 12) {
      part[t] = ld_u64(kLdsTotals + 8u * (uint32_t)t);
      st_u64(kLdsTotals + 8u * (uint32_t)t, 0ull);
    }
    __threadfence();
    if (t == 0) {
      const uint32_t done = atomicAdd(a.wg_cnt, 1u);
      *(lds32_t)(uintptr_t)(kLdsTotals + 96) = done + 1 == gridDim.x ? 1u : 0u;
      if (done + 1 == gridDim.x) __threadfence();  // the last one: acquire the others' totals
    }
  }
  __syncthreads();
  if (*(lds32_t)(uintptr_t)(kLdsTotals + 96) == 0u) return;
  for (uint32_t j = (uint32_t)t; j < 12u * gridDim.x; j += blockDim.x)
    lds_add_u64(kLdsTotals + 8u * (j % 12u),
                __hip_atomic_load(a.wg_part + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
  __syncthreads();
  if (t < 3 * NR)
    reinterpret_cast<unsigned long long*>(&a.totals[a.range_offset + t / 3].points)[t % 3] =
        ld_u64(kLdsTotals + 8u * (uint32_t)t);
  if (t == 0) *a.wg_cnt = 0u;
}




// ---------------------------------------------------------------------------
// The ov7670 multi-blob sensor's metapixel bitmap on the chroma-run tables
// ---------------------------------------------------------------------------
// BMB:171-190 / CLU:185-186: a metapixel (4x4 pixels) is set when more than 2
// of its pixels are in the sticky range.  Same per-word fast path and exact
// path as chroma_kernel, for one range: a lane takes an item = (frame,
// metapixel row, 16-pixel column chunk) -- four rows of 8 words, four
// metapixels -- and counts per metapixel; flagged words are queued per wave
// with their owner lane and metapixel, and the drain adds their exact bits to
// the owner's byte-packed counter word in LDS, which the owner adds before it
// writes the four flags.
constexpr uint32_t kLdsBlobCounts = kLdsQueues + 16 * kQueueCap * 8;  // u32 [1024]: 4 byte counts per lane
constexpr uint32_t kLdsBlobBytes = kLdsBlobCounts + 4 * kMaxBlock;
static_assert(kLdsBlobBytes <= 160 * 1024, "blob meta LDS image");

struct BlobChromaGeom {
  FastDiv per_frame;  // bh * cpr items per frame
  FastDiv per_row;    // cpr items per metapixel row
  uint32_t total;     // n_frames * bh * cpr
  int32_t bw, bh;
};

__global__ __launch_bounds__(kMaxBlock) void blob_chroma_meta_kernel(BlobArgs a, BlobChromaGeom g,
                                                                      const ChromaTables* ct,
                                                                      const RangeTables* rt) {
  if (gated_out(a.gate, a.gate_max, a.gate_le)) return;
  const int t = threadIdx.x;
  // the chroma kernel's tables (one range), zeroed count words
  stage_chroma_image(ct, rt, t);
  *(lds32_t)(uintptr_t)(kLdsBlobCounts + 4u * (uint32_t)t) = 0u;
  __syncthreads();
  const int lane = t & 63;
  const uint32_t qbase_s = __builtin_amdgcn_readfirstlane(kLdsQueues + (uint32_t)(t >> 6) * (kQueueCap * 8));
  const uint32_t wave0 = (uint32_t)(t & ~63);
  const uint32_t my_counts = kLdsBlobCounts + 4u * (uint32_t)t;
  const int64_t ll = a.line_length, plane = (int64_t)a.height * a.line_length;
  int qn = 0;
  // One drain round: lanes 0..take-1 resolve queue entries 0..take-1 exactly
  // and add their bits to the owner's counter word; the rest moves up.
  auto drain = [&](int take) {
    if (lane < take) {
      const u32x2 ent = ld64(qbase_s + 8u * (uint32_t)lane);
      const uint32_t w = ent.x;
      const uint32_t d = ld16(kLdsRuns + 2u * chroma_of(w));
      const uint32_t lo = d & 0xFFu, hi = d >> 8, Y0 = w & 0xFFu, Y1 = (w >> 16) & 0xFFu;
      const bool xw = d == kChromaExc;
      const bool f0 = xw | ((Y0 < lo) & (Y0 > hi)), f1 = xw | ((Y1 < lo) & (Y1 > hi));
      const uint32_t n = (f0 ? exact_mask<0>(w) & 1u : 0u) + (f1 ? exact_mask<1>(w) & 1u : 0u);
      if (n) {
        const uint32_t owner = wave0 + (ent.y & 63u), j = ent.y >> 6;
        __hip_atomic_fetch_add((__attribute__((address_space(3))) uint32_t*)(uintptr_t)(kLdsBlobCounts + 4u * owner),
                               n << (8u * j), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
    }
    const int rest = qn - take;
    if (rest > 0) {
      u32x2 mv = {0u, 0u};
      if (lane < rest) mv = ld64(qbase_s + 8u * (uint32_t)(take + lane));
      __builtin_amdgcn_wave_barrier();
      if (lane < rest) st64(qbase_s + 8u * (uint32_t)lane, mv.x, mv.y);
    }
    qn = rest;
  };
  // Items in grid-stride order; a lane's item is four pixel rows of its 16
  // columns.  The rows are software-pipelined across items: the next row
  // (the next item's first at an item's last) is loaded while this one is
  // processed, two 32-byte buffers per lane (the loads past the batch re-read
  // the lane's last item: unconditional, so waits stay "this row's data").
  const uint32_t stride = gridDim.x * (uint32_t)kMaxBlock;
  uint32_t base = blockIdx.x * (uint32_t)kMaxBlock;
  if (base >= g.total) return;
  struct Item {
    const uint8_t* p;
    uint32_t f, mr, ch;
    bool valid;
  };
  auto item_at = [&](uint32_t b, const Item& fallback) {
    Item r;
    const uint32_t item = b + (uint32_t)t;
    r.valid = item < g.total;
    if (!r.valid && b != blockIdx.x * (uint32_t)kMaxBlock) return Item{fallback.p, fallback.f, fallback.mr, fallback.ch, false};
    const uint32_t it = r.valid ? item : 0u;
    r.f = fdiv(it, g.per_frame);
    const uint32_t rem = it - r.f * g.per_frame.d;
    r.mr = fdiv(rem, g.per_row);
    r.ch = rem - r.mr * g.per_row.d;
    r.p = a.frames + (int64_t)r.f * a.frame_stride + (int64_t)(4 * r.mr) * ll + 16 * (int64_t)r.ch;
    return r;
  };
  Item cur = item_at(base, Item{a.frames, 0u, 0u, 0u, false});
  uint4 by[2], bc[2];
  by[0] = ld_nt16(cur.p);
  bc[0] = ld_nt16(cur.p + plane);
  for (;;) {
    const uint64_t vm = __builtin_amdgcn_ballot_w64(cur.valid);
    const uint32_t nb = base + stride;
    const Item nxt = item_at(nb < g.total ? nb : base, cur);
    uint32_t cnt[4] = {0u, 0u, 0u, 0u};
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      // the next row: this item's r + 1, or the next item's row 0
      const uint8_t* np = r < 3 ? cur.p + (r + 1) * ll : nxt.p;
      // streaming loads (nontemporal: 9 % faster on scenes than plain loads,
      // scripts/ab/r05k_blob.py)
      by[(r + 1) & 1] = ld_nt16(np);
      bc[(r + 1) & 1] = ld_nt16(np + plane);
      const uint4 vy = by[r & 1], vc = bc[r & 1];
      const uint32_t yy[4] = {vy.x, vy.y, vy.z, vy.w}, cc[4] = {vc.x, vc.y, vc.z, vc.w};
      // the row's 8 words in two halves of 4 (registers: the next row's
      // buffer stays live)
#pragma unroll
      for (int hf = 0; hf < 2; ++hf) {
        uint32_t w[4], d[4], cut[4];
        u32x2 mm[4];
#pragma unroll
        for (int k = 0; k < 2; ++k) stripe_px::ov7670_words(yy[2 * hf + k], cc[2 * hf + k], w[2 * k], w[2 * k + 1]);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const uint32_t c = chroma_of8(w[i]);
          d[i] = ld16(kLdsRuns + (c >> 7));
          cut[i] = ld16(kLdsBlocks + ((c >> 11) & 0x1FFEu));
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) mm[i] = ld64(kLdsPairs + (cut[i] & 0xFFu));
#pragma unroll
        for (int i = 0; i < 4; ++i) asm volatile("" : "+v"(d[i]), "+v"(cut[i]));
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int wi = 4 * hf + i;  // the word's index in the row: metapixel wi >> 1
          uint32_t e0, e1;
          uint64_t q0, q1;
          select2(w[i], d[i], cut[i], mm[i].x, mm[i].y, vm, e0, e1, q0, q1);
          cnt[wi >> 1] += e0 + e1;  // one range: the spread masks are 0 or 1
          const uint64_t bal = q0 | q1;
          if (bal == 0) continue;  // no lane of the wave flagged this word slot (the common case)
          const uint32_t idx =
              __builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u));
          if (__builtin_amdgcn_inverse_ballot_w64(bal)) {
            const uint32_t qa = __builtin_amdgcn_readfirstlane(qbase_s + 8u * (uint32_t)qn) + 8u * idx;
            *(lds32_t)(uintptr_t)qa = w[i];
            *(lds32_t)(uintptr_t)(qa + 4u) = (uint32_t)lane | ((uint32_t)(wi >> 1) << 6);
          }
          qn += __builtin_popcountll(bal);
          if (qn >= 64) drain(64);
        }
      }
    }
    while (qn > 0) drain(qn < 64 ? qn : 64);
    __builtin_amdgcn_wave_barrier();
    const uint32_t extra = *(lds32_t)(uintptr_t)my_counts;
    *(lds32_t)(uintptr_t)my_counts = 0u;
    if (cur.valid) {
      uint32_t flags = 0;
#pragma unroll
      for (int j = 0; j < 4; ++j) flags |= (cnt[j] + ((extra >> (8 * j)) & 0xFFu) > 2u ? 1u : 0u) << (8 * j);
      *reinterpret_cast<uint32_t*>(a.meta + ((int64_t)cur.f * g.bh + cur.mr) * g.bw + 4 * (int64_t)cur.ch) = flags;
    }
    if (nb >= g.total) break;
    base = nb;
    cur = nxt;
  }
}

template <int LAYOUT, int NR, bool MASKS>
int launch_t(const KernelArgs& a, const ChromaGeom& g, const ChromaTables* ct, hipStream_t s) {
  auto kern = chroma_kernel<LAYOUT, NR, MASKS>;
  hipError_t e = set_dynamic_lds(reinterpret_cast<const void*>(kern), (int)kLdsBytes);
  if (e != hipSuccess) return e;
  // one workgroup per CU the stream may use (a CU-masked stream: its mask),
  // less the CUs left free for kernels on other streams
  const int cus_all = stream_cus(s);
  const int cus = cus_all - a.reserved_cus >= 1 ? cus_all - a.reserved_cus : 1;
  const int block = 64 * kHotWaves;
  const int64_t grid = g.n_tiles < cus ? g.n_tiles : cus;  // one workgroup per CU (LDS image)
  hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(block), kLdsBytes, s, a, g, ct);
  return hipGetLastError();
}

template <int LAYOUT, bool MASKS>
int launch_nr(const KernelArgs& a, const ChromaGeom& g, const ChromaTables* ct, hipStream_t s) {
  switch (a.n_ranges) {
    case 1: return launch_t<LAYOUT, 1, MASKS>(a, g, ct, s);
    case 2: return launch_t<LAYOUT, 2, MASKS>(a, g, ct, s);
    case 3: return launch_t<LAYOUT, 3, MASKS>(a, g, ct, s);
    case 4: return launch_t<LAYOUT, 4, MASKS>(a, g, ct, s);
  }
  return hipErrorInvalidValue;
}

}  // namespace

int build_chroma_tables(const RangeTables* t, ChromaTables* ct, hipStream_t s) {
  hipError_t e = set_dynamic_lds(reinterpret_cast<const void*>(chroma_summary_kernel), (int)kSumLds);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(chroma_summary_kernel, dim3(256), dim3(1024), kSumLds, s, t, ct);
  e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(chroma_block_kernel<false>, dim3(4096 / kBlocksPerGroup), dim3(64 * kBlocksPerGroup), 0, s, ct);
  hipLaunchKernelGGL(chroma_block_kernel<true>, dim3(4096 / kBlocksPerGroup), dim3(64 * kBlocksPerGroup), 0, s, ct);
  return hipGetLastError();
}

// Chunk columns of 8 (YUYV: one 16-byte piece of each of two rows) or
// 2*kChunkWords (ov7670) pixels; k rows per half step, as many as fit a
// kHotLanes-lane workgroup, rounded down to whole waves when that keeps >= 7/8
// of the lanes (the kernel's uniform fast path needs whole waves).
bool chroma_geometry(const KernelArgs& a, ChromaGeom& g) {
  const bool split = a.layout == TRIK_HSV_LAYOUT_YUYV;
  // rows of more than kHotLanes pieces: the two pieces from the two halves of one row
  const bool wide = split && a.width / 8 > kHotLanes;
  const int px = split ? (wide ? 16 : 8) : 2 * kChunkWords;
  if (a.width <= 0 || a.width % px || a.height <= 0) return false;
  const int cpr = a.width / px;
  if (cpr > kHotLanes) return false;
  const int64_t need = 16;  // vector loads
  if ((reinterpret_cast<uintptr_t>(a.frames) % need) || (a.frame_stride % need) || (a.line_length % need))
    return false;
  // 640 lanes when that makes whole waves: fewer, longer units per frame (the
  // per-unit epilogue over more steps; VGA: 10 units of 30 steps instead of
  // 15 of 20 -- C3 -0.3 %, scenes -1 %, scripts/ab/r05n_k.py)
  int k = 640 / cpr;
  if (k == 0 || (k * cpr) % 64 != 0) {
    k = kHotLanes / cpr;
    for (int kk = k; kk * 8 >= k * 7; --kk)
      if ((kk * cpr) % 64 == 0) { k = kk; break; }
  }
  g.cpr = cpr;
  g.k = k;
  g.dy = split && !wide ? k : 0;
  g.dx = wide ? a.width / 2 : 0;
  g.rstep = k + g.dy;
  const int steps_total = (a.height + g.rstep - 1) / g.rstep;
  g.tiles_per_frame = (steps_total + kMaxSteps - 1) / kMaxSteps;
  g.steps = (steps_total + g.tiles_per_frame - 1) / g.tiles_per_frame;
  g.tiles_per_frame = (steps_total + g.steps - 1) / g.steps;  // every tile has >= 1 step
  g.steps_last = steps_total - (g.tiles_per_frame - 1) * g.steps;
  g.n_tiles = (int64_t)g.tiles_per_frame * a.n_frames;
  if (g.n_tiles * ((g.k * g.cpr + 63) / 64) > 0xFFFFFFFFll) return false;  // 32-bit tile and unit indices
  // per drain round a lane adds <= 2 pixels: byte counts <= 2r, x sums <= 2r*W,
  // row sums <= 2r*rows; the 16-bit sums must take at least one round
  const int rows = g.steps * g.rstep;
  const int span = a.width > rows ? a.width : rows;
  if (2LL * span > 65535) return false;
  int r = 65535 / (2 * span);
  g.flush_rounds = r > 127 ? 127 : r;
  g.units = (g.k * g.cpr + 63) / 64;
  // the past-the-end loads read the handle's sink when the lanes' offsets fit
  // (YUYV: a lane's two loads lie within (k + dy) rows + 2 dx bytes of the
  // tile base; ov7670: within k rows of it and of the chroma plane H rows on)
  g.tail_span = split ? (int64_t)(g.k + g.dy) * a.line_length + 2LL * g.dx + 16
                      : (int64_t)a.height * a.line_length + (int64_t)g.k * a.line_length + 16;
  g.tail_ok = a.tail != nullptr && g.tail_span <= a.tail_bytes;
  g.fd_units = make_div((uint32_t)g.units);
  g.fd_tiles = make_div((uint32_t)g.tiles_per_frame);
  g.cpr_inv = (uint32_t)(((1u << 20) + (uint32_t)cpr - 1) / (uint32_t)cpr);
  return true;
}

bool chroma_geometry_ok(const KernelArgs& a) {
  ChromaGeom g;
  return chroma_geometry(a, g);
}

int64_t chroma_tail_span(const KernelArgs& a) {
  ChromaGeom g;
  return chroma_geometry(a, g) ? g.tail_span : -1;
}

// The fused step splits the units evenly over the workgroups and completes
// frames by their unit counts: any batch the kernel takes (not the
// verification mode, which writes masks instead).
bool chroma_fused_ok(const KernelArgs& a) {
  ChromaGeom g;
  return !a.masks && chroma_geometry(a, g);
}

int launch_chroma(const KernelArgs& a, const ChromaTables* ct, bool write_masks, hipStream_t s) {
  ChromaGeom g;
  if (!chroma_geometry(a, g)) return hipErrorNotSupported;
  if (g.n_tiles == 0) return hipSuccess;
  if (a.fused && (write_masks || !chroma_fused_ok(a) || !a.wg_part || !a.wg_cnt || !a.frame_acc))
    return hipErrorInvalidValue;
  // every lane's past-the-end load stays inside the sink (or is not redirected)
  if (g.tail_ok && (g.tail_span > a.tail_bytes || g.tail_span <= 0)) return hipErrorInvalidValue;
  if (a.layout == TRIK_HSV_LAYOUT_YUYV)
    return write_masks ? launch_nr<TRIK_HSV_LAYOUT_YUYV, true>(a, g, ct, s)
                       : launch_nr<TRIK_HSV_LAYOUT_YUYV, false>(a, g, ct, s);
  return write_masks ? launch_nr<TRIK_HSV_LAYOUT_OV7670, true>(a, g, ct, s)
                     : launch_nr<TRIK_HSV_LAYOUT_OV7670, false>(a, g, ct, s);
}


bool blob_chroma_ok(const BlobArgs& a) {
  return a.width > 0 && a.width % 16 == 0 && a.height % 4 == 0 && a.line_length % 16 == 0 &&
         (reinterpret_cast<uintptr_t>(a.frames) % 16) == 0 && (a.n_frames <= 1 || a.frame_stride % 16 == 0);
}

int launch_blob_meta_chroma(const BlobArgs& a, const ChromaTables* ct, const RangeTables* rt, hipStream_t s) {
  if (!blob_chroma_ok(a)) return hipErrorNotSupported;
  const int bw = a.width >> 2, bh = a.height >> 2, cpr = a.width >> 4;
  const int64_t total = (int64_t)a.n_frames * bh * cpr;
  if (total <= 0) return hipSuccess;
  if (total >= (1ll << 31)) return hipErrorInvalidValue;
  hipError_t e = set_dynamic_lds(reinterpret_cast<const void*>(blob_chroma_meta_kernel), (int)kLdsBlobBytes);
  if (e != hipSuccess) return e;
  const int cus = device_cus();
  BlobChromaGeom g;
  g.per_frame = make_div((uint32_t)(bh * cpr));
  g.per_row = make_div((uint32_t)cpr);
  g.total = (uint32_t)total;
  g.bw = bw;
  g.bh = bh;
  const int64_t blocks = (total + kMaxBlock - 1) / kMaxBlock;
  hipLaunchKernelGGL(blob_chroma_meta_kernel, dim3((unsigned)(blocks < cus ? blocks : cus)), dim3(kMaxBlock),
                     kLdsBlobBytes, s, a, g, ct, rt);
  return hipGetLastError();
}

}  // namespace trik_hsv
