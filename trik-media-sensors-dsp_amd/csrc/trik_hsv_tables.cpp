// trik_hsv_tables.cpp -- host-side "range compiler": turns a group of InArgs
// HSV ranges into the LDS lookup tables the hot kernel uses.
//
// The reference tests a packed HSV word against packed bounds per pixel
// (detectHsvPixel, WSEQ:171-179): mask = cmpltu4(hsv, from) | cmpgtu4(hsv, to),
// det = (mask == expect).  The H, S and V lanes of that mask are independent,
// so det = hue_ok(H) && sat_ok(S) && val_ok(V) with
//   hue_ok(H) = ((H < from.H) || (H > to.H)) == expect.bit0
//   sat_ok(S) = !((S < from.S) || (S > to.S)),   val_ok likewise,
// which is exactly what the tables below enumerate.
#include <string.h>

#include "trik_hsv_internal.h"

namespace trik_hsv {

static inline int32_t clamp_range(int32_t lo, int32_t v, int32_t hi) {  // stdcpp.hpp:38-44
  return v < lo ? lo : (v > hi ? hi : v);
}

PackedRange pack_range(const TRIK_VIDTRANSCODE_CV_InArgsAlg& r) {  // WSEQ:425-445
  const uint32_t hf = (uint32_t)clamp_range(0, ((int32_t)r.detectHueFrom * 255) / 359, 255);
  const uint32_t ht = (uint32_t)clamp_range(0, ((int32_t)r.detectHueTo * 255) / 359, 255);
  const uint32_t sf = (uint32_t)clamp_range(0, ((int32_t)r.detectSatFrom * 255) / 100, 255);
  const uint32_t st = (uint32_t)clamp_range(0, ((int32_t)r.detectSatTo * 255) / 100, 255);
  const uint32_t vf = (uint32_t)clamp_range(0, ((int32_t)r.detectValFrom * 255) / 100, 255);
  const uint32_t vt = (uint32_t)clamp_range(0, ((int32_t)r.detectValTo * 255) / 100, 255);
  PackedRange p;
  if (hf <= ht) {
    p.from = (vf << 16) | (sf << 8) | hf;
    p.to = (vt << 16) | (st << 8) | ht;
    p.expect = 0;
  } else {  // hue wrap through 0
    p.from = (vf << 16) | (sf << 8) | ((ht + 1) & 0xFF);
    p.to = (vt << 16) | (st << 8) | ((hf - 1) & 0xFF);
    p.expect = 1;
  }
  return p;
}

static inline bool outside(uint32_t x, uint32_t lo, uint32_t hi) { return x < lo || x > hi; }

// Everything but the sat/val table: the LUTs and the per-value H, S, V tests
// (what the chroma-run builder and kernel read).
void compile_tables_head(const TRIK_VIDTRANSCODE_CV_InArgsAlg* ranges, int n, RangeTables* out) {
  memset(out->hue, 0, sizeof(out->hue));
  memset(out->smask, 0, sizeof(out->smask));
  memset(out->vmask, 0, sizeof(out->vmask));
  out->lut43[0] = 0;
  out->lut255[0] = 0;
  for (uint32_t i = 1; i < 256; ++i) {  // WSEQ:400-406
    out->lut43[i] = (uint16_t)((43u * 256u) / i);
    out->lut255[i] = (uint16_t)((255u * 256u) / i);
  }
  for (int t = 0; t < n; ++t) {
    const PackedRange p = pack_range(ranges[t]);
    const uint8_t bit = (uint8_t)(1u << t);
    const uint32_t fh = p.from & 0xFF, th = p.to & 0xFF;
    const uint32_t fs = (p.from >> 8) & 0xFF, ts = (p.to >> 8) & 0xFF;
    const uint32_t fv = (p.from >> 16) & 0xFF, tv = (p.to >> 16) & 0xFF;
    for (uint32_t h = 0; h < 256; ++h)
      if ((outside(h, fh, th) ? 1u : 0u) == (p.expect & 1u)) out->hue[h] |= bit;
    for (uint32_t x = 0; x < 256; ++x) {
      if (!outside(x, fs, ts)) out->smask[x] |= bit;
      if (!outside(x, fv, tv)) out->vmask[x] |= bit;
    }
  }
}

// The sat/val table sv[mx * 256 + mn] (compile_tables_head first: it reads
// lut255).  S = (LUT255[mx] * d) >> 8 with d = mx - mn does not fall as d
// grows, so the d with fs <= S <= ts form one interval [d_lo, d_hi]: solved
// per mx instead of testing every (mx, mn).
void compile_tables_sv(const TRIK_VIDTRANSCODE_CV_InArgsAlg* ranges, int n, RangeTables* out) {
  memset(out->sv, 0, sizeof(out->sv));
  const uint16_t* lut255 = out->lut255;
  for (int t = 0; t < n; ++t) {
    const PackedRange p = pack_range(ranges[t]);
    const uint8_t bit = (uint8_t)(1u << t);
    const uint32_t fs = (p.from >> 8) & 0xFF, ts = (p.to >> 8) & 0xFF;
    const uint32_t fv = (p.from >> 16) & 0xFF, tv = (p.to >> 16) & 0xFF;
    for (uint32_t mx = fv; mx <= tv && mx < 256; ++mx) {
      const uint32_t L = lut255[mx];
      uint32_t d_lo, d_hi;
      if (L == 0) {  // mx = 0: S = 0
        if (fs > 0) continue;
        d_lo = 0;
        d_hi = mx;
      } else {
        d_lo = (256u * fs + L - 1) / L;          // the least d with L d >= 256 fs
        d_hi = (256u * (ts + 1) - 1) / L;        // the largest d with L d < 256 (ts + 1)
        if (d_hi > mx) d_hi = mx;
      }
      uint8_t* row = out->sv + mx * 256;
      for (uint32_t d = d_lo; d <= d_hi; ++d) row[mx - d] |= bit;
    }
  }
}

void compile_tables(const TRIK_VIDTRANSCODE_CV_InArgsAlg* ranges, int n, RangeTables* out) {
  compile_tables_head(ranges, n, out);
  compile_tables_sv(ranges, n, out);
}

void compile_stripe_tables(const RangeTables& base, int n, StripeTables* out) {
  memset(out, 0, sizeof(*out));
  const uint8_t keep = (uint8_t)((1u << (n < 4 ? n : 4)) - 1u);
  for (int mx = 0; mx < 256; ++mx)
    for (int mn = 0; mn < 256; ++mn) out->sv[mx * kSvStride + mn] = base.sv[mx * 256 + mn] & keep;
  for (int i = 0; i < 256; ++i) {
    uint32_t spread = 0;
    for (int t = 0; t < n && t < 4; ++t) spread |= ((uint32_t)(base.hue[i] >> t) & 1u) << (8 * t);
    for (int c = 0; c < kHueCopies; ++c) out->hue[i * kHueCopies + c] = spread;
    for (int c = 0; c < kM43Copies; ++c) out->m43[i * kM43Copies + c] = base.lut43[i];
  }
}

int detect_mode(const RangeTables& t, int n) {
  const uint8_t all = (uint8_t)((1u << (n < 4 ? n : 4)) - 1u);
  if (n <= 0) return kDetectFull;
  for (int h = 0; h < 256; ++h)
    if ((t.hue[h] & all) != all) return kDetectFull;
  for (int x = 0; x < 256; ++x)
    if ((t.smask[x] & all) != all) return kDetectSV;
  return kDetectV;
}

void preview_maps(int width, int height, int out_w, int out_h, uint32_t* maps, int col_lo, int col_hi) {
  // WSEQ:371-387: shift = min(out/in) in double, maps truncate i * shift
  const double sw = width > 0 ? (double)out_w / width : 0.0;
  const double sh = height > 0 ? (double)out_h / height : 0.0;
  const double shift = sw < sh ? sw : sh;
  uint32_t* wi2wo = maps;
  uint32_t* hi2ho = wi2wo + width;
  int32_t* last_row = reinterpret_cast<int32_t*>(hi2ho + height);
  int32_t* last_col = last_row + out_h;
  for (int i = 0; i < width; ++i) wi2wo[i] = (uint32_t)(i * shift);
  for (int i = 0; i < height; ++i) hi2ho[i] = (uint32_t)(i * shift);
  for (int i = 0; i < out_h; ++i) last_row[i] = -1;
  for (int i = 0; i < out_w; ++i) last_col[i] = -1;
  // scan order: a later source row/column overwrites (proceedImageHsv)
  for (int i = 0; i < height; ++i)
    if (hi2ho[i] < (uint32_t)out_h) last_row[hi2ho[i]] = i;
  for (int i = 0; i < width; ++i)
    if (i >= col_lo && i <= col_hi && wi2wo[i] < (uint32_t)out_w) last_col[wi2wo[i]] = i;
}

void auto_range_zone(int width, int height, int32_t& c_lo, int32_t& c_hi, int32_t& r_lo, int32_t& r_hi) {
  // HsvRangeDetector::initImg (cv_hsv_range_detector.hpp:88-108), zone scale 6
  // (WSEQ:32): uint16_t fields, so differences wrap modulo 2^16.
  const uint16_t h_height = (uint16_t)((uint32_t)height / 2);
  const uint16_t h_width = (uint16_t)((uint32_t)width / 2);
  const uint16_t step = (uint16_t)((uint32_t)height / 6);
  c_lo = (uint16_t)(h_width - step);
  c_hi = (uint16_t)(h_width + step);
  r_lo = (uint16_t)(h_height - step);
  r_hi = (uint16_t)(h_height + step);
}

}  // namespace trik_hsv
