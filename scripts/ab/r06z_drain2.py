# round-6 A/B, hot kernel: the drain resolves a record's word with one packed
# HSV computation for both pixels (the pixels of a word share U and V: R, G, B,
# max, min and the hue differences in 16-bit halves, as autoDetectHsv's
# hsv_pair), branch-free, instead of one exact_mask per flagged pixel under
# two EXEC branches (both taken in nearly every 64-record round).
#  drain2
FILE = "trik_hsv_chroma.hip"
_FN = r'''
// Both pixels' exact masks of YUYV word w in one packed 16-bit HSV pass (see
// exact_mask; the reference's 16-bit wrap as mod-2^16 arithmetic).
typedef unsigned short u16x2_t __attribute__((ext_vector_type(2)));
typedef short i16x2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ i16x2_t pk_chan(u16x2_t Y, uint32_t c) {
  const u16x2_t cc = {(unsigned short)c, (unsigned short)c};
  const u16x2_t x = Y * (u16x2_t){74, 74} + cc;
  const i16x2_t s = __builtin_bit_cast(i16x2_t, x) >> (i16x2_t){6, 6};
  return __builtin_elementwise_min(__builtin_elementwise_max(s, (i16x2_t){0, 0}), (i16x2_t){255, 255});
}
__device__ __forceinline__ void exact_mask2(uint32_t w, uint32_t& e0, uint32_t& e1) {
  const uint32_t wc = w ^ 0xFF00FF00u;
  const uint32_t cr = __builtin_amdgcn_udot4(w, 102u << 24, (uint32_t)-14248, false);
  const uint32_t cg = __builtin_amdgcn_udot4(wc, (25u << 8) | (52u << 24), (uint32_t)-10939, false);
  const uint32_t cb = __builtin_amdgcn_udot4(w, 129u << 8, (uint32_t)-17672, false);
  const u16x2_t Y = __builtin_bit_cast(u16x2_t, w & 0x00FF00FFu);
  const i16x2_t R = pk_chan(Y, cr), G = pk_chan(Y, cg), B = pk_chan(Y, cb);
  const i16x2_t MX = __builtin_elementwise_max(__builtin_elementwise_max(R, G), B);
  const i16x2_t MN = __builtin_elementwise_min(__builtin_elementwise_min(R, G), B);
  const i16x2_t D = MX - MN, dBR = B - R, dRG = R - G, dGB = G - B;
  const bool eg0 = MX.x == G.x, eb0 = MX.x == B.x, eg1 = MX.y == G.y, eb1 = MX.y == B.y;
  const i16x2_t df0 = eg0 ? dBR : (eb0 ? dRG : dGB), df1 = eg1 ? dBR : (eb1 ? dRG : dGB);
  const int b0 = eg0 ? 21845 : (eb0 ? 43690 : 0), b1 = eg1 ? 21845 : (eb1 ? 43690 : 0);
  const uint32_t d0 = (uint16_t)D.x, d1 = (uint16_t)D.y, m0 = (uint16_t)MX.x, m1 = (uint16_t)MX.y;
  const uint32_t H0 = ((uint32_t)(b0 + (int)ld16(kLdsLut43 + 2u * d0) * (int)df0.x) >> 8) & 0xFFu;
  const uint32_t H1 = ((uint32_t)(b1 + (int)ld16(kLdsLut43 + 2u * d1) * (int)df1.y) >> 8) & 0xFFu;
  const uint32_t S0 = (ld16(kLdsLut255 + 2u * m0) * d0) >> 8, S1 = (ld16(kLdsLut255 + 2u * m1) * d1) >> 8;
  e0 = ld8(kLdsHue + H0) & ld8(kLdsSat + S0) & ld8(kLdsVal + m0);
  e1 = ld8(kLdsHue + H1) & ld8(kLdsSat + S1) & ld8(kLdsVal + m1);
}
'''
_ANCHOR = "// ---------------------------------------------------------------------------\n// Builder\n"
VARIANTS = {
    "r6z_base": [("kMaxBlock = 1024;", "kMaxBlock = 1024;")],
    "drain2": [(_ANCHOR, _FN + _ANCHOR),
               ("        const uint32_t m0 = f0 ? exact_mask<0>(w) : 0u;\n        const uint32_t m1 = f1 ? exact_mask<1>(w) : 0u;\n",
                "        uint32_t m0, m1;\n        exact_mask2(w, m0, m1);\n        if (!f0) m0 = 0u;\n        if (!f1) m1 = 0u;\n")],
}
