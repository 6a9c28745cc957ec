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
