// trik_hsv_pixel.h -- per-pixel arithmetic of the reference path, as plain
// device functions, for the kernels that visit pixels individually (the
// generic reduce kernel, the preview and the HSV histogram).  The hot stripe
// kernel has its own instruction-tuned form of the same arithmetic
// (trik_hsv_stripe.hip); the exhaustive parity tests hold both to the oracle.
//
// SURVEY Appendix A; equal to WSEQ:181-249 (WSEQ as in include/trik_hsv.h) on
// all 2^24 (Y, U, V) inputs.
#pragma once

#include "trik_hsv_internal.h"

namespace trik_hsv {

__device__ __forceinline__ int clamp8(int v) { return min(max(v, 0), 255); }

struct PixelRgb {
  int r, g, b;
  __device__ __forceinline__ uint32_t rgb888() const {
    return ((uint32_t)r << 16) | ((uint32_t)g << 8) | (uint32_t)b;
  }
};

// convert2xYuyvToRgb888, WSEQ:181-205
__device__ __forceinline__ PixelRgb pixel_rgb(int Y, int U, int V) {
  const int y74 = 74 * Y;
  PixelRgb p;
  p.r = clamp8((102 * V + y74 - 14248) >> 6);
  p.g = clamp8((-52 * V - 25 * U + y74 + 8696) >> 6);
  p.b = clamp8(((int)(int16_t)(129 * U + y74 - 17672)) >> 6);  // _add2 wraps at 16 bits
  return p;
}

// convertRgb888ToHsv hue byte, WSEQ:207-249 (G > B > R on ties)
__device__ __forceinline__ uint32_t pixel_hue(const PixelRgb& p, int mx, int mn, const RangeTables& t) {
  const int m = t.lut43[mx - mn];
  int h;
  if (mx == p.g)
    h = 21845 + m * (p.b - p.r);
  else if (mx == p.b)
    h = 43690 + m * (p.r - p.g);
  else
    h = m * (p.g - p.b);
  return ((uint32_t)h >> 8) & 0xFFu;
}

// (Y,U,V) -> T-bit mask of the ranges whose H, S and V tests all pass.
__device__ __forceinline__ uint32_t detect_pixel(int Y, int U, int V, const RangeTables& t) {
  const PixelRgb p = pixel_rgb(Y, U, V);
  const int mx = max(p.r, max(p.g, p.b));
  const int mn = min(p.r, min(p.g, p.b));
  return (uint32_t)t.hue[pixel_hue(p, mx, mn, t)] & (uint32_t)t.sv[(mx << 8) | mn];
}

// Full HSV word V<<16 | S<<8 | H (WSEQ:207-249), S = (LUT255[max]*delta)>>8.
__device__ __forceinline__ uint32_t pixel_hsv(const PixelRgb& p, const RangeTables& t) {
  const int mx = max(p.r, max(p.g, p.b));
  const int mn = min(p.r, min(p.g, p.b));
  const uint32_t s = ((uint32_t)t.lut255[mx] * (uint32_t)(mx - mn)) >> 8;
  return ((uint32_t)mx << 16) | (s << 8) | pixel_hue(p, mx, mn, t);
}

// detectHsvPixel (WSEQ:171-179) for one packed range: per-byte "outside the
// bounds" bits compared with the expected pattern (1 for a wrapped hue).
__device__ __forceinline__ bool detect_packed(uint32_t H, uint32_t S, uint32_t V, const PackedRange& r) {
  const uint32_t out = ((H < (r.from & 0xFFu)) | (H > (r.to & 0xFFu))) |
                       (((S < ((r.from >> 8) & 0xFFu)) | (S > ((r.to >> 8) & 0xFFu))) << 1) |
                       (((V < ((r.from >> 16) & 0xFFu)) | (V > ((r.to >> 16) & 0xFFu))) << 2);
  return out == r.expect;
}

// H, S, V bytes (WSEQ:207-249) with LUT43 / LUT255 from any address space.
template <typename L>
__device__ __forceinline__ void pixel_hsv_bytes(const PixelRgb& p, const L* l43, const L* l255, uint32_t& H,
                                                uint32_t& S, uint32_t& V) {
  const int mx = max(p.r, max(p.g, p.b)), mn = min(p.r, min(p.g, p.b));
  const int m = l43[mx - mn];
  int h;
  if (mx == p.g) h = 21845 + m * (p.b - p.r);
  else if (mx == p.b) h = 43690 + m * (p.r - p.g);
  else h = m * (p.g - p.b);
  H = ((uint32_t)h >> 8) & 0xFFu;
  S = ((uint32_t)l255[mx] * (uint32_t)(mx - mn)) >> 8;
  V = (uint32_t)mx;
}

// writeOutputPixel, WSEQ:66-70: 0x00RRGGBB -> B5 G6 R5 (R in the low bits),
// little-endian bytes (the output line length need not be even).
__device__ __forceinline__ void write_px565(uint8_t* dst, uint32_t rgb888) {
  const uint32_t v = ((rgb888 >> 19) & 0x001fu) | ((rgb888 >> 5) & 0x07e0u) | ((rgb888 << 8) & 0xf800u);
  dst[0] = (uint8_t)v;
  dst[1] = (uint8_t)(v >> 8);
}

// drawOutputPixelBound (WSEQ:72-89, OSEQ:77-90): the source point clamped to
// the image, then through the scale maps.
struct Canvas {
  uint8_t* out;
  int out_ll, width, height;
  const uint32_t* wi2wo;
  const uint32_t* hi2ho;
  __device__ void px(int32_t col, int32_t row, uint32_t rgb) const {
    const int32_t sc = col < 0 ? 0 : (col > width - 1 ? width - 1 : col);
    const int32_t sr = row < 0 ? 0 : (row > height - 1 ? height - 1 : row);
    write_px565(out + (int64_t)(int32_t)hi2ho[sr] * out_ll + (int64_t)(int32_t)wi2wo[sc] * 2, rgb);
  }
};

// The preview scale maps (wi2wo then hi2ho, W + H contiguous words) staged
// in LDS by one wave when they fit kMapLdsBytes: every drawn point looks up
// both maps, and from LDS that lookup no longer waits on a global load.
constexpr size_t kMapLdsBytes = 32 * 1024;
template <bool LDSMAP>
__device__ inline Canvas stage_canvas(uint32_t* smaps, uint8_t* out, int out_ll, int width, int height,
                                      const uint32_t* wi2wo, const uint32_t* hi2ho, int lane) {
  if (LDSMAP) {
    for (int i = lane; i < width + height; i += 64) smaps[i] = wi2wo[i];
    __syncthreads();
    return Canvas{out, out_ll, width, height, smaps, smaps + width};
  }
  return Canvas{out, out_ll, width, height, wi2wo, hi2ho};
}

// The 8 magenta guide lines of the object sensors (WSEQ:136-166,471-485;
// OSEQ:227-255,548-561): 4 vertical and 4 horizontal lines of 2 x 100 points
// around the centre, step = H/6; one colour, so any lane order.
__device__ __forceinline__ void draw_guides(const Canvas& cv, int lane, int nlanes) {
  const int step = cv.height / 6, hh = cv.height / 2, hw = cv.width / 2;
  for (int k = lane; k < 8 * 100; k += nlanes) {
    const int line = k / 100, adj = k % 100, off = (line & 3) < 2 ? ((line & 3) - 2) : ((line & 3) - 1);
    if (line < 4) {
      const int32_t col = hw + off * step;
      cv.px(col, hh - adj, 0xff00ff);
      cv.px(col, hh + adj, 0xff00ff);
    } else {
      const int32_t row = hh + off * step;
      cv.px(hw - adj, row, 0xff00ff);
      cv.px(hw + adj, row, 0xff00ff);
    }
  }
}

// x / d for 32-bit x via a host-computed multiplier (round-up method):
// q = (umulhi(x, magic) + x) >> shift, exact for every 32-bit x.
struct FastDiv {
  uint32_t magic, shift, d;
};
inline FastDiv make_div(uint32_t d) {
  uint32_t s = 0;
  while ((1ull << s) < d) ++s;
  const uint64_t m = ((1ull << 32) * ((1ull << s) - d)) / d + 1;
  return FastDiv{(uint32_t)m, s, d};
}
__device__ __forceinline__ uint32_t fdiv(uint32_t x, const FastDiv& f) {
  return (uint32_t)(((uint64_t)__umulhi(x, f.magic) + x) >> f.shift);
}

// (Y, U, V) of pixel `col` of row `row`: packed YUYV (WSEQ:262-270) or the
// ov7670 planes (OSEQ:360-373: U = odd chroma byte, V = even chroma byte).
__device__ __forceinline__ void fetch_yuv(const uint8_t* frame, int height, int line_length, int layout,
                                          int row, int col, int& Y, int& U, int& V) {
  if (layout == TRIK_HSV_LAYOUT_YUYV) {
    const uint8_t* p = frame + (int64_t)row * line_length + 4 * (col >> 1);
    Y = p[2 * (col & 1)];
    U = p[1];
    V = p[3];
  } else {
    const uint8_t* yrow = frame + (int64_t)row * line_length;
    const uint8_t* crow = frame + (int64_t)line_length * height + (int64_t)row * line_length;
    Y = yrow[col];
    V = crow[col & ~1];
    U = crow[col | 1];
  }
}

}  // namespace trik_hsv
