// trik_hsv_stripe_px.h -- the hot kernel's per-pixel arithmetic (YUYV word ->
// detection mask via the StripeTables LDS image), shared by stripe_kernel
// (trik_hsv_stripe.hip) and the multi-blob bitmap kernel (trik_hsv_blob.hip).
// Both stage the StripeTables image at LDS address 0 (no static LDS).
#pragma once

#include <hip/hip_runtime.h>

#include "trik_hsv_internal.h"

namespace trik_hsv {
namespace stripe_px {

// LDS by absolute byte address.  The kernel has no static LDS, so its dynamic
// LDS (the StripeTables image) starts at address 0; addressing it through
// integer-derived address-space-3 pointers lets every table address be one
// VALU op (no symbol base to add).
typedef __attribute__((address_space(3))) const uint8_t* lds_u8_ptr;
typedef __attribute__((address_space(3))) const uint32_t* lds_u32_ptr;
__device__ __forceinline__ uint32_t lds_u32(uint32_t addr) { return *(lds_u32_ptr)(uintptr_t)addr; }
__device__ __forceinline__ uint32_t lds_u8(uint32_t addr) { return *(lds_u8_ptr)(uintptr_t)addr; }

// Phase 1 for both pixels of a YUYV word w (b0=Y0, b1=U, b2=Y1, b3=V):
//  * presums of WSEQ:183-201 with v_dot4_u32_u8; wc =
//    w ^ 0xFF00FF00 carries complemented chroma for the negative G weights
//    (WSEQ:188-190);
//  * x = (int16)presum >> 6 clamped to [0, 255] (WSEQ:203-205): the
//    reference's _add2 keeps 16-bit lanes, so only bits 15:0 of the presum
//    matter (B wraps for 27,136 triples) -- one v_bfe_i32 + one v_med3_i32;
//  * max, min (WSEQ:207-216) and the hue case select of WSEQ:226-246
//    (priority G > B > R on ties): diff and base;
//  * LDS byte addresses of this pixel's LUT43[max - min] copy (per-bank
//    replicated row, StripeTables::rows) and of its sat&val mask
//    sv[max * 260 + min].
// Plain 32-bit code: on gfx950 this kernel's time follows its VALU
// instruction count (the 16-bit full-rate forms measured no faster in
// context, scripts/ubench/pixel_mix.hip), and the compiler schedules it and
// enforces the v_dot4 / VCC wait states itself.
struct Phase1 {
  uint32_t m43_addr, sv_addr, diff, base;
  uint32_t rgb888;  // the clamped pixel (the preview's colour); dead code where unused
  int r, g, b;      // its clamped channels (the 2:1 preview packs RGB565X from them)
};
constexpr int log2i(int v) { return v <= 1 ? 0 : 1 + log2i(v / 2); }
constexpr int kM43Shift = log2i(4 * kM43Copies);  // byte stride of one m43 entry's copies
constexpr int kHueShift = log2i(4 * kHueCopies);
static_assert((1 << kM43Shift) == 4 * kM43Copies && (1 << kHueShift) == 4 * kHueCopies, "pow2 copies");
__device__ __forceinline__ int clamp8_shift6(uint32_t s) {
  const int x = ((int)(s << 16)) >> 22;  // bits 15:6, sign from 15 (v_bfe_i32)
  const int lo = x < 0 ? 0 : x;
  return lo > 255 ? 255 : lo;            // v_med3_i32
}
template <int PIX>
__device__ __forceinline__ Phase1 phase1(uint32_t w, uint32_t wc, uint32_t m43_lane) {
  constexpr uint32_t kY = PIX == 0 ? 74u : (74u << 16);
  const int r = clamp8_shift6(__builtin_amdgcn_udot4(w, kY | (102u << 24), (uint32_t)-14248, false));
  const int g = clamp8_shift6(__builtin_amdgcn_udot4(wc, kY | (25u << 8) | (52u << 24), (uint32_t)-10939, false));
  const int b = clamp8_shift6(__builtin_amdgcn_udot4(w, kY | (129u << 8), (uint32_t)-17672, false));
  const int mx = max(r, max(g, b));
  const int mn = min(r, min(g, b));
  Phase1 p;
  p.rgb888 = ((uint32_t)r << 16) | ((uint32_t)g << 8) | (uint32_t)b;
  p.r = r;
  p.g = g;
  p.b = b;
  p.m43_addr = ((uint32_t)(mx - mn) << kM43Shift) + m43_lane;
  p.sv_addr = __umul24((uint32_t)mx, (uint32_t)kSvStride) + (uint32_t)mn;
  const bool eqG = mx == g, eqB = mx == b;
  const int dR = g - b, dG = b - r, dB = r - g;
  int diff = eqB ? dB : dR;
  p.diff = (uint32_t)(eqG ? dG : diff);
  uint32_t base = eqB ? 43690u : 0u;
  p.base = eqG ? 21845u : base;
  return p;
}

// The sat&val table address alone (ranges that accept every hue): clamp8 is
// monotone, so max and min of the clamped channels are the clamped max and min
// of the unclamped ones (two clamps per pixel instead of three).
template <int PIX>
__device__ __forceinline__ uint32_t sv_addr_only(uint32_t w, uint32_t wc) {
  constexpr uint32_t kY = PIX == 0 ? 74u : (74u << 16);
  auto shift6 = [](uint32_t s) { return ((int)(s << 16)) >> 22; };  // v_bfe_i32 s, 6, 10
  const int r = shift6(__builtin_amdgcn_udot4(w, kY | (102u << 24), (uint32_t)-14248, false));
  const int g = shift6(__builtin_amdgcn_udot4(wc, kY | (25u << 8) | (52u << 24), (uint32_t)-10939, false));
  const int b = shift6(__builtin_amdgcn_udot4(w, kY | (129u << 8), (uint32_t)-17672, false));
  const int mx = min(max(max(r, max(g, b)), 0), 255);
  const int mn = min(max(min(r, min(g, b)), 0), 255);
  return __umul24((uint32_t)mx, (uint32_t)kSvStride) + (uint32_t)mn;
}

// The value-only table address (ranges that accept every hue and every
// saturation): m = max(R', G', sext16(B')) of the unclamped presums,
// 4 * ((m >> 6) + 512) into a table of 1024 byte-spread value masks whose
// entries below 512 / above 767 hold V = 0 / V = 255 (the clamp).
template <int PIX>
__device__ __forceinline__ uint32_t v_addr(uint32_t w, uint32_t wc) {
  constexpr uint32_t kY = PIX == 0 ? 74u : (74u << 16);
  const int r = (int)__builtin_amdgcn_udot4(w, kY | (102u << 24), (uint32_t)-14248, false);  // int16 range
  const int g = (int)__builtin_amdgcn_udot4(wc, kY | (25u << 8) | (52u << 24), (uint32_t)-10939, false);
  const int b = ((int)(__builtin_amdgcn_udot4(w, kY | (129u << 8), (uint32_t)-17672, false) << 16)) >> 16;
  const int m = max(r, max(g, b));
  return (uint32_t)(((m >> 6) + 512) << 2);
}

// Phase 2: h = base + m * diff (WSEQ:226-246; m < 2^14, |diff| < 2^8, so one
// v_mad_i32_i24), whose bits 15:8 (H) select the byte-spread hue mask (range t
// -> bit 8t); returns the LDS byte address of this lane's copy.
// (LLVM would fuse the multiply-add into a quarter-rate v_mad_u64_u32.)
__device__ __forceinline__ uint32_t phase2_addr(uint32_t m, const Phase1& p, uint32_t hue_lane) {
  uint32_t h;
  asm("v_mad_i32_i24 %0, %1, %2, %3" : "=v"(h) : "v"(m), "v"(p.diff), "v"(p.base));
  return (((h >> 8) & 0xFFu) << kHueShift) + hue_lane;
}

// Combine: spread sv's bit t to bit 8t (terms at t + 7s are disjoint for
// t, s < 4) and AND with the hue mask.
__device__ __forceinline__ uint32_t combine(uint32_t hue, uint32_t sv) {
  return hue & __umul24(sv, 0x00204081u);
}

// ov7670 planes -> the two YUYV words of 4 pixels (OSEQ:360-373: U = odd
// chroma byte, V = even chroma byte): yy = Y0..Y3, cc = V0 U0 V1 U1.
__device__ __forceinline__ void ov7670_words(uint32_t yy, uint32_t cc, uint32_t& w0, uint32_t& w1) {
  w0 = __builtin_amdgcn_perm(cc, yy, 0x04010500u);
  w1 = __builtin_amdgcn_perm(cc, yy, 0x06030702u);
}

}  // namespace stripe_px
}  // namespace trik_hsv
