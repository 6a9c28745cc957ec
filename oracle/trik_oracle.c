/*
 * trik_oracle.c -- CPU restatement of the TRIK HSV-threshold + centroid path.
 *
 * TEST INFRASTRUCTURE ONLY (see trik_oracle.h).  Never linked into, or called
 * by, the product library.  File:line citations are relative to the
 * reference checkout; WSEQ / OSEQ are defined in trik_oracle.h.
 */
#define _GNU_SOURCE
#include "trik_oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------------ */
/* C64x+ intrinsic emulation.  Lane conventions: halfword "hi" = bits 31..16,
 * "lo" = bits 15..0; byte bN = bits 8N+7..8N.                               */
/* ------------------------------------------------------------------------ */

static inline uint32_t lo16(uint32_t a) { return a & 0xFFFFu; }
static inline uint32_t hi16(uint32_t a) { return a >> 16; }
static inline int32_t s16(uint32_t h) { return (int32_t)(int16_t)(uint16_t)h; }
static inline uint32_t byte_of(uint32_t a, int n) { return (a >> (8 * n)) & 0xFFu; }

/* four u8 x u8 -> u16 products, packed lo->hi into 64 bits */
uint64_t trik_c64x_mpyu4ll(uint32_t a, uint32_t b) {
  uint64_t r = 0;
  for (int n = 0; n < 4; ++n)
    r |= (uint64_t)(byte_of(a, n) * byte_of(b, n)) << (16 * n);
  return r;
}

/* sum of unsigned a bytes times signed b bytes */
int32_t trik_c64x_dotpus4(uint32_t a, uint32_t b) {
  int32_t s = 0;
  for (int n = 0; n < 4; ++n)
    s += (int32_t)byte_of(a, n) * (int32_t)(int8_t)byte_of(b, n);
  return s;
}

/* two independent 16-bit adds, wrapping */
uint32_t trik_c64x_add2(uint32_t a, uint32_t b) {
  return (((hi16(a) + hi16(b)) & 0xFFFFu) << 16) | ((lo16(a) + lo16(b)) & 0xFFFFu);
}

uint32_t trik_c64x_packh2(uint32_t a, uint32_t b) { return (hi16(a) << 16) | hi16(b); }
uint32_t trik_c64x_packlh2(uint32_t a, uint32_t b) { return (lo16(a) << 16) | hi16(b); }
uint32_t trik_c64x_pack2(uint32_t a, uint32_t b) { return (lo16(a) << 16) | lo16(b); }
uint32_t trik_c64x_packhl2(uint32_t a, uint32_t b) { return (hi16(a) << 16) | lo16(b); }

/* arithmetic shift right of each signed halfword */
uint32_t trik_c64x_shr2(uint32_t a, uint32_t n) {
  uint32_t h = (uint32_t)(s16(hi16(a)) >> n) & 0xFFFFu;
  uint32_t l = (uint32_t)(s16(lo16(a)) >> n) & 0xFFFFu;
  return (h << 16) | l;
}

/* clear bits lo..hi inclusive */
uint32_t trik_c64x_clr(uint32_t a, uint32_t lo, uint32_t hi) {
  uint32_t width = hi - lo + 1;
  uint32_t mask = (width >= 32) ? 0xFFFFFFFFu : (((1u << width) - 1u) << lo);
  return a & ~mask;
}

static inline uint32_t sat_u8(int32_t v) { return v < 0 ? 0u : (v > 255 ? 255u : (uint32_t)v); }

/* saturate the four signed halfwords of (a,b) to u8: a.hi->b3, a.lo->b2, b.hi->b1, b.lo->b0 */
uint32_t trik_c64x_spacku4(uint32_t a, uint32_t b) {
  return (sat_u8(s16(hi16(a))) << 24) | (sat_u8(s16(lo16(a))) << 16) |
         (sat_u8(s16(hi16(b))) << 8) | sat_u8(s16(lo16(b)));
}

uint32_t trik_c64x_unpkhu4(uint32_t a) { return (byte_of(a, 3) << 16) | byte_of(a, 2); }
uint32_t trik_c64x_unpklu4(uint32_t a) { return (byte_of(a, 1) << 16) | byte_of(a, 0); }

uint32_t trik_c64x_maxu4(uint32_t a, uint32_t b) {
  uint32_t r = 0;
  for (int n = 0; n < 4; ++n) {
    uint32_t x = byte_of(a, n), y = byte_of(b, n);
    r |= (x > y ? x : y) << (8 * n);
  }
  return r;
}

uint32_t trik_c64x_minu4(uint32_t a, uint32_t b) {
  uint32_t r = 0;
  for (int n = 0; n < 4; ++n) {
    uint32_t x = byte_of(a, n), y = byte_of(b, n);
    r |= (x < y ? x : y) << (8 * n);
  }
  return r;
}

/* bit1 = (a.hi == b.hi), bit0 = (a.lo == b.lo) */
uint32_t trik_c64x_cmpeq2(uint32_t a, uint32_t b) {
  return ((hi16(a) == hi16(b)) ? 2u : 0u) | ((lo16(a) == lo16(b)) ? 1u : 0u);
}

/* a.hi*b.hi - a.lo*b.lo, signed 16x16 */
int32_t trik_c64x_dotpn2(uint32_t a, uint32_t b) {
  return s16(hi16(a)) * s16(hi16(b)) - s16(lo16(a)) * s16(lo16(b));
}

/* bytes (a.b3, a.b1, b.b3, b.b1) */
uint32_t trik_c64x_packh4(uint32_t a, uint32_t b) {
  return (byte_of(a, 3) << 24) | (byte_of(a, 1) << 16) | (byte_of(b, 3) << 8) | byte_of(b, 1);
}

uint32_t trik_c64x_cmpltu4(uint32_t a, uint32_t b) {
  uint32_t r = 0;
  for (int n = 0; n < 4; ++n) r |= (byte_of(a, n) < byte_of(b, n) ? 1u : 0u) << n;
  return r;
}

uint32_t trik_c64x_cmpgtu4(uint32_t a, uint32_t b) {
  uint32_t r = 0;
  for (int n = 0; n < 4; ++n) r |= (byte_of(a, n) > byte_of(b, n) ? 1u : 0u) << n;
  return r;
}

/* swap the two bytes of each halfword */
uint32_t trik_c64x_swap4(uint32_t a) {
  return ((a & 0x00FF00FFu) << 8) | ((a & 0xFF00FF00u) >> 8);
}

static inline uint32_t itoll_hi(uint64_t x) { return (uint32_t)(x >> 32); }
static inline uint32_t itoll_lo(uint64_t x) { return (uint32_t)x; }

/* ------------------------------------------------------------------------ */
/* Division LUTs, WSEQ:389-407 (s_mult43_div / s_mult255_div).               */
/* ------------------------------------------------------------------------ */

static uint16_t g_lut43[256], g_lut255[256];
static pthread_once_t g_lut_once = PTHREAD_ONCE_INIT;

static void lut_init(void) {
  g_lut43[0] = 0;
  g_lut255[0] = 0;
  for (uint32_t i = 1; i < 256; ++i) {
    g_lut43[i] = (uint16_t)((43u * 256u) / i);
    g_lut255[i] = (uint16_t)((255u * 256u) / i);
  }
}

void trik_oracle_luts(uint16_t lut43[256], uint16_t lut255[256]) {
  pthread_once(&g_lut_once, lut_init);
  memcpy(lut43, g_lut43, sizeof g_lut43);
  memcpy(lut255, g_lut255, sizeof g_lut255);
}

/* ------------------------------------------------------------------------ */
/* Derivation 1: intrinsic-level restatement.                                */
/* ------------------------------------------------------------------------ */

/* WSEQ:181-205.  Constants: 409/4=102 (V->R), 298/4=74 (Y), 516/4=129 (U->B),
 * -208/4=-52 (V->G), -100/4=-25 (U->G); additive terms WSEQ:192-195. */
void trik_oracle_pair_rgb_c64x(uint32_t yuyv, uint32_t rgb_out[2]) {
  const uint32_t k_mul = (102u << 24) | (74u << 16) | (129u << 8) | 74u;
  const uint32_t k_dot = ((uint32_t)(uint8_t)(int8_t)-52 << 24) | ((uint32_t)(uint8_t)(int8_t)-25 << 8);
  const uint32_t c_r = (uint16_t)(128 / 4 + (-128 * 409 - 16 * 298) / 4);
  const uint32_t c_g = (uint16_t)(128 / 4 + (+128 * 100 + 128 * 208 - 16 * 298) / 4);
  const uint32_t c_b = (uint16_t)(128 / 4 + (-128 * 516 - 16 * 298) / 4);

  const uint64_t prod = trik_c64x_mpyu4ll(yuyv, k_mul);         /* (102V,74Y1 | 129U,74Y0) */
  const uint32_t dot = (uint32_t)trik_c64x_dotpus4(yuyv, k_dot); /* -52V - 25U */
  const uint32_t rgb_h = trik_c64x_add2(trik_c64x_packh2(0, itoll_hi(prod)), c_r);
  const uint32_t rgb_l = trik_c64x_add2(trik_c64x_packlh2(dot, itoll_lo(prod)), (c_g << 16) | c_b);
  const uint32_t y1 = trik_c64x_pack2(itoll_lo(prod), itoll_lo(prod));
  const uint32_t y2 = trik_c64x_pack2(itoll_hi(prod), itoll_hi(prod));
  const uint32_t p1h = trik_c64x_clr(trik_c64x_shr2(trik_c64x_add2(rgb_h, y1), 6), 16, 31);
  const uint32_t p1l = trik_c64x_shr2(trik_c64x_add2(rgb_l, y1), 6);
  const uint32_t p2h = trik_c64x_clr(trik_c64x_shr2(trik_c64x_add2(rgb_h, y2), 6), 16, 31);
  const uint32_t p2l = trik_c64x_shr2(trik_c64x_add2(rgb_l, y2), 6);
  rgb_out[0] = trik_c64x_spacku4(p1h, p1l);
  rgb_out[1] = trik_c64x_spacku4(p2h, p2l);
}

/* WSEQ:207-249. */
uint32_t trik_oracle_hsv_c64x(uint32_t rgb) {
  pthread_once(&g_lut_once, lut_init);
  const uint32_t or16 = trik_c64x_unpkhu4(rgb);  /* (0, R) */
  const uint32_t gb16 = trik_c64x_unpklu4(rgb);  /* (G, B) */
  const uint32_t max2 = trik_c64x_maxu4(rgb, rgb >> 8);
  const uint32_t mx = trik_c64x_clr(trik_c64x_maxu4(max2, max2 >> 8), 8, 31);
  const uint32_t mx_mx = trik_c64x_pack2(mx, mx);
  const uint32_t val_x256 = mx << 8;
  const uint32_t min2 = trik_c64x_minu4(rgb, rgb >> 8);
  const uint32_t mn = trik_c64x_minu4(min2, min2 >> 8);
  const uint32_t delta = mx - mn;
  const uint32_t sat_x256 = (uint32_t)g_lut255[mx] * delta;
  const uint32_t m43 = trik_c64x_pack2(g_lut43[delta], g_lut43[delta]);
  const uint32_t cmp = trik_c64x_cmpeq2(mx_mx, gb16);
  int32_t hue_x256;
  if (cmp == 0)
    hue_x256 = 0 + trik_c64x_dotpn2(m43, trik_c64x_packhl2(gb16, gb16));
  else if (cmp == 1)
    hue_x256 = (0x10000 * 2) / 3 + trik_c64x_dotpn2(m43, trik_c64x_packlh2(or16, gb16));
  else
    hue_x256 = (0x10000 * 1) / 3 + trik_c64x_dotpn2(m43, trik_c64x_pack2(gb16, or16));
  const uint32_t sat_hue = trik_c64x_pack2(sat_x256, (uint32_t)hue_x256);
  return trik_c64x_packh4(val_x256, sat_hue);
}

/* ------------------------------------------------------------------------ */
/* Derivation 2: closed form.                            */
/* ------------------------------------------------------------------------ */

static inline int32_t sext16(int32_t v) { return (int32_t)(int16_t)(uint16_t)(v & 0xFFFF); }
static inline uint32_t clamp8_shift6(int32_t v) { return sat_u8(v >> 6); }

uint32_t trik_oracle_rgb_closed(uint32_t y, uint32_t u, uint32_t v) {
  const int32_t Y = (int32_t)y, U = (int32_t)u, V = (int32_t)v;
  const uint32_t r = clamp8_shift6(102 * V + 74 * Y - 14248);
  const uint32_t g = clamp8_shift6(-52 * V - 25 * U + 74 * Y + 8696);
  const uint32_t b = clamp8_shift6(sext16(129 * U + 74 * Y - 17672));
  return (r << 16) | (g << 8) | b;
}

uint32_t trik_oracle_hsv_closed(uint32_t rgb) {
  pthread_once(&g_lut_once, lut_init);
  const int32_t r = (int32_t)byte_of(rgb, 2), g = (int32_t)byte_of(rgb, 1), b = (int32_t)byte_of(rgb, 0);
  const int32_t mx = r > g ? (r > b ? r : b) : (g > b ? g : b);
  const int32_t mn = r < g ? (r < b ? r : b) : (g < b ? g : b);
  const int32_t d = mx - mn;
  const uint32_t s = ((uint32_t)g_lut255[mx] * (uint32_t)d) >> 8;
  const int32_t m = g_lut43[d];
  int32_t h;
  if (mx == g)
    h = 21845 + m * (b - r);
  else if (mx == b)
    h = 43690 + m * (r - g);
  else
    h = m * (g - b);
  const uint32_t H = ((uint32_t)h >> 8) & 0xFFu;
  return ((uint32_t)mx << 16) | (s << 8) | H;
}

/* ------------------------------------------------------------------------ */
/* Range packing and detection: WSEQ:425-445, WSEQ:171-179, stdcpp range(). */
/* ------------------------------------------------------------------------ */

static inline int32_t clamp_range(int32_t lo, int32_t v, int32_t hi) {
  return v < lo ? lo : (v > hi ? hi : v); /* stdcpp.hpp:38-44 */
}

void trik_oracle_pack_range(const trik_oracle_range* r, uint32_t* from, uint32_t* to,
                            uint32_t* expect) {
  const uint32_t hf = (uint32_t)clamp_range(0, ((int32_t)r->hue_from * 255) / 359, 255);
  const uint32_t ht = (uint32_t)clamp_range(0, ((int32_t)r->hue_to * 255) / 359, 255);
  const uint32_t sf = (uint32_t)clamp_range(0, ((int32_t)r->sat_from * 255) / 100, 255);
  const uint32_t st = (uint32_t)clamp_range(0, ((int32_t)r->sat_to * 255) / 100, 255);
  const uint32_t vf = (uint32_t)clamp_range(0, ((int32_t)r->val_from * 255) / 100, 255);
  const uint32_t vt = (uint32_t)clamp_range(0, ((int32_t)r->val_to * 255) / 100, 255);
  if (hf <= ht) {
    *from = (vf << 16) | (sf << 8) | hf;
    *to = (vt << 16) | (st << 8) | ht;
    *expect = 0;
  } else {
    /* hue wrap; the reference's assert at WSEQ:441 is compiled out (NDEBUG) */
    *from = (vf << 16) | (sf << 8) | ((ht + 1) & 0xFFu);
    *to = (vt << 16) | (st << 8) | ((hf - 1) & 0xFFu);
    *expect = 1;
  }
}

int trik_oracle_detect(uint32_t hsv, uint32_t from, uint32_t to, uint32_t expect) {
  const uint32_t m = trik_c64x_cmpltu4(hsv, from) | trik_c64x_cmpgtu4(hsv, to);
  return m == expect;
}

void trik_oracle_yuv_table(uint64_t* out, int closed) {
  for (uint32_t v = 0; v < 256; ++v)
    for (uint32_t u = 0; u < 256; ++u)
      for (uint32_t y = 0; y < 256; ++y) {
        uint32_t rgb;
        if (closed) {
          rgb = trik_oracle_rgb_closed(y, u, v);
        } else {
          uint32_t pair[2];
          trik_oracle_pair_rgb_c64x(y | (u << 8) | (y << 16) | (v << 24), pair);
          rgb = pair[0];
        }
        const uint32_t hsv = closed ? trik_oracle_hsv_closed(rgb) : trik_oracle_hsv_c64x(rgb);
        out[y | (u << 8) | (v << 16)] = ((uint64_t)rgb << 32) | hsv;
      }
}

/* ------------------------------------------------------------------------ */
/* Frame: WSEQ:412-508 (run) with WSEQ:251-284 / OSEQ:343-387 and            */
/* WSEQ:316-354 (proceedImageHsv), T ranges evaluated side by side.          */
/* ------------------------------------------------------------------------ */

#define TRIK_ORACLE_MAX_RANGES 64

/* The YUYV word (Y0 U Y1 V) of pixels 2q, 2q+1 of a row: WSEQ:262-270 for
 * packed YUYV; OSEQ:360-373 for the ov7670 planes (U = odd chroma byte,
 * V = even chroma byte). */
static uint32_t pair_word(const uint8_t* frame, int height, int line_length, int layout, int row,
                          int q) {
  if (layout == TRIK_ORACLE_LAYOUT_OV7670) {
    const uint8_t* yrow = frame + (int64_t)row * line_length;
    const uint8_t* crow = frame + (int64_t)line_length * height + (int64_t)row * line_length;
    const uint32_t c = trik_c64x_swap4((uint32_t)crow[2 * q] | ((uint32_t)crow[2 * q + 1] << 8));
    const uint32_t yy = (uint32_t)yrow[2 * q] | ((uint32_t)yrow[2 * q + 1] << 8);
    return trik_c64x_unpklu4(yy) | (trik_c64x_unpklu4(c) << 8);
  }
  const uint8_t* p = frame + (int64_t)row * line_length + 4 * q;
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

int trik_oracle_frame(const uint8_t* frame, int64_t frame_size, int width, int height,
                      int line_length, int layout, const trik_oracle_range* ranges,
                      int n_ranges, int64_t* sums, uint8_t* mask) {
  if (width < 0 || height < 0 || width % 32 != 0 || height % 4 != 0) return -1;
  if (n_ranges < 0 || n_ranges > TRIK_ORACLE_MAX_RANGES) return -1;
  const int64_t need = (int64_t)height * line_length * (layout == TRIK_ORACLE_LAYOUT_OV7670 ? 2 : 1);
  /* WSEQ:415 checks H*lineLength against the buffer; the ov7670 chroma plane
   * follows the luma plane (OSEQ:347), so both planes must be present. */
  if ((int64_t)height * line_length > frame_size || need > frame_size) return -1;

  uint32_t from[TRIK_ORACLE_MAX_RANGES], to[TRIK_ORACLE_MAX_RANGES], expect[TRIK_ORACLE_MAX_RANGES];
  int32_t tx[TRIK_ORACLE_MAX_RANGES], ty[TRIK_ORACLE_MAX_RANGES];
  uint32_t tn[TRIK_ORACLE_MAX_RANGES];
  for (int t = 0; t < n_ranges; ++t) {
    trik_oracle_pack_range(&ranges[t], &from[t], &to[t], &expect[t]);
    tx[t] = 0; ty[t] = 0; tn[t] = 0; /* WSEQ:421-423 */
  }

  for (int row = 0; row < height && width > 0; ++row) {
    uint32_t row_n[TRIK_ORACLE_MAX_RANGES], row_x[TRIK_ORACLE_MAX_RANGES];
    for (int t = 0; t < n_ranges; ++t) { row_n[t] = 0; row_x[t] = 0; }
    for (int q = 0; q < width / 2; ++q) { /* one YUYV word = pixels 2q, 2q+1 */
      const uint32_t yuyv = pair_word(frame, height, line_length, layout, row, q);
      uint32_t rgb[2];
      trik_oracle_pair_rgb_c64x(yuyv, rgb);
      for (int k = 0; k < 2; ++k) {
        const uint32_t col = (uint32_t)(2 * q + k);
        const uint32_t hsv = trik_oracle_hsv_c64x(rgb[k]);
        uint8_t bits = 0;
        for (int t = 0; t < n_ranges; ++t) {
          const int det = trik_oracle_detect(hsv, from[t], to[t], expect[t]);
          row_n[t] += (uint32_t)det;
          row_x[t] += det ? col : 0;
          if (det && t < 8) bits |= (uint8_t)(1u << t);
        }
        if (mask) mask[(int64_t)row * width + col] = bits;
      }
    }
    for (int t = 0; t < n_ranges; ++t) { /* WSEQ:350-352 */
      tx[t] += (int32_t)row_x[t];
      ty[t] += (int32_t)((uint32_t)row * row_n[t]);
      tn[t] += row_n[t];
    }
  }
  for (int t = 0; t < n_ranges; ++t) {
    sums[3 * t + 0] = (int64_t)tn[t];
    sums[3 * t + 1] = (int64_t)tx[t];
    sums[3 * t + 2] = (int64_t)ty[t];
  }
  return 0;
}

void trik_oracle_targets(const int64_t sums[3], int width, int height, int8_t* target_x,
                         int8_t* target_y, uint8_t* target_size) {
  const uint32_t points = (uint32_t)sums[0];
  if (points > 0) { /* WSEQ:486-499 */
    const int32_t cx = (int32_t)((uint32_t)(int32_t)sums[1] / points);
    const int32_t cy = (int32_t)((uint32_t)(int32_t)sums[2] / points);
    const uint32_t radius = (uint32_t)ceilf(sqrtf((float)points / 3.1415927f));
    *target_x = (int8_t)(((cx - width / 2) * 100 * 2) / width);
    *target_y = (int8_t)(((cy - height / 2) * 100 * 2) / height);
    *target_size = (uint8_t)((uint32_t)(radius * 100 * 4) / (uint32_t)(width + height));
  } else { /* WSEQ:500-505 */
    *target_x = 0;
    *target_y = 0;
    *target_size = 0;
  }
}

/* ------------------------------------------------------------------------ */
/* Batch over POSIX threads (CPU baseline).                                  */
/* ------------------------------------------------------------------------ */

typedef struct batch_job {
  const uint8_t* frames;
  int64_t stride;
  int first, count, width, height, line_length, layout, n_ranges;
  const trik_oracle_range* ranges;
  int64_t* sums;
  int8_t* targets;
  int rc;
} batch_job;

static void* batch_worker(void* arg) {
  batch_job* j = (batch_job*)arg;
  j->rc = 0;
  for (int f = j->first; f < j->first + j->count; ++f) {
    int64_t* s = j->sums + (int64_t)f * j->n_ranges * 3;
    if (trik_oracle_frame(j->frames + (int64_t)f * j->stride, j->stride, j->width, j->height,
                          j->line_length, j->layout, j->ranges, j->n_ranges, s, NULL) != 0) {
      j->rc = -1;
      return NULL;
    }
    if (j->targets)
      for (int t = 0; t < j->n_ranges; ++t) {
        int8_t* o = j->targets + ((int64_t)f * j->n_ranges + t) * 3;
        trik_oracle_targets(s + 3 * t, j->width, j->height, &o[0], &o[1], (uint8_t*)&o[2]);
      }
  }
  return NULL;
}

int trik_oracle_batch(const uint8_t* frames, int64_t frame_stride, int n_frames, int width,
                      int height, int line_length, int layout, const trik_oracle_range* ranges,
                      int n_ranges, int64_t* sums, int8_t* targets, int n_threads) {
  if (n_threads < 1) n_threads = 1;
  if (n_threads > n_frames) n_threads = n_frames > 0 ? n_frames : 1;
  pthread_t tid[256];
  batch_job jobs[256];
  if (n_threads > 256) n_threads = 256;
  int per = n_frames / n_threads, extra = n_frames % n_threads, at = 0;
  for (int i = 0; i < n_threads; ++i) {
    const int cnt = per + (i < extra ? 1 : 0);
    jobs[i] = (batch_job){frames, frame_stride, at, cnt, width, height, line_length,
                          layout, n_ranges, ranges, sums, targets, 0};
    at += cnt;
  }
  for (int i = 1; i < n_threads; ++i) pthread_create(&tid[i], NULL, batch_worker, &jobs[i]);
  batch_worker(&jobs[0]);
  int rc = jobs[0].rc;
  for (int i = 1; i < n_threads; ++i) {
    pthread_join(tid[i], NULL);
    if (jobs[i].rc) rc = jobs[i].rc;
  }
  return rc;
}

/* ------------------------------------------------------------------------ */
/* Synthetic frames (bit-identical to the device generator).                 */
/* ------------------------------------------------------------------------ */

static inline uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

/* scene palette in (Y,U,V): red, green, blue, yellow, cyan, magenta */
static const uint8_t k_palette[6][3] = {
    {81, 90, 240}, {145, 54, 34}, {41, 240, 110}, {210, 16, 146}, {170, 166, 16}, {106, 202, 222}};

static void scene_pixel(uint64_t smix, int f, int x, int y, int w, int h, uint32_t* Y,
                        uint32_t* U, uint32_t* V) {
  *Y = (uint32_t)(x * 3 + y * 2 + f * 7) & 0xFFu;
  *U = (uint32_t)(128 + ((x - w / 2) * 64) / (w > 0 ? w : 1));
  *V = (uint32_t)(128 + ((y - h / 2) * 64) / (h > 0 ? h : 1));
  for (int k = 0; k < 6; ++k) {
    const uint64_t r = splitmix64(smix ^ ((uint64_t)(uint32_t)f << 8) ^ (uint64_t)k);
    const int cx = (int)(r % (uint64_t)(w > 0 ? w : 1));
    const int cy = (int)((r >> 20) % (uint64_t)(h > 0 ? h : 1));
    const int rad = 8 + (int)((r >> 40) % (uint64_t)(h / 6 + 1));
    const int dx = x - cx, dy = y - cy;
    if (dx * dx + dy * dy <= rad * rad) {
      *Y = k_palette[k][0];
      *U = k_palette[k][1];
      *V = k_palette[k][2];
    }
  }
}

void trik_oracle_synth(uint8_t* frames, int64_t frame_stride, int first_frame, int n_frames,
                       int width, int height, int line_length, int layout, int kind,
                       uint64_t seed) {
  const uint64_t smix = splitmix64(seed);
  const int64_t plane = (int64_t)height * line_length;
  const int64_t frame_bytes = plane * (layout == TRIK_ORACLE_LAYOUT_OV7670 ? 2 : 1);
  for (int i = 0; i < n_frames; ++i) {
    const int f = first_frame + i;
    uint8_t* fr = frames + (int64_t)i * frame_stride;
    if (kind == 0) {
      /* byte b = byte (b & 7) of splitmix64(smix ^ f<<32 ^ (b >> 3)) */
      for (int64_t w = 0; w * 8 < frame_bytes; ++w) {
        const uint64_t wv = splitmix64(smix ^ ((uint64_t)(uint32_t)f << 32) ^ (uint64_t)w);
        for (int k = 0; k < 8 && w * 8 + k < frame_bytes; ++k) fr[w * 8 + k] = (uint8_t)(wv >> (8 * k));
      }
      continue;
    }
    memset(fr, 0, (size_t)frame_bytes);
    for (int y = 0; y < height; ++y)
      for (int x = 0; x < width; x += 2) {
        uint32_t Y0, U, V, Y1, U1, V1;
        scene_pixel(smix, f, x, y, width, height, &Y0, &U, &V);
        scene_pixel(smix, f, x + 1, y, width, height, &Y1, &U1, &V1);
        if (layout == TRIK_ORACLE_LAYOUT_OV7670) {
          fr[(int64_t)y * line_length + x] = (uint8_t)Y0;
          fr[(int64_t)y * line_length + x + 1] = (uint8_t)Y1;
          fr[plane + (int64_t)y * line_length + x] = (uint8_t)V;     /* even = V */
          fr[plane + (int64_t)y * line_length + x + 1] = (uint8_t)U; /* odd = U */
        } else {
          uint8_t* p = fr + (int64_t)y * line_length + 2 * x;
          p[0] = (uint8_t)Y0; p[1] = (uint8_t)U; p[2] = (uint8_t)Y1; p[3] = (uint8_t)V;
        }
      }
  }
}

/* ------------------------------------------------------------------------ */
/* Whole run: preview, overlays, auto HSV range (WSEQ:358-508).              */
/* ------------------------------------------------------------------------ */

static int32_t clamp_i32(int32_t lo, int32_t v, int32_t hi) { /* range<T>, stdcpp.hpp:38-44 */
  if (v < lo) return lo;
  if (v > hi) return hi;
  return v;
}

typedef struct run_ctx {
  int width, height, out_line_length;
  const uint32_t* wi2wo;
  const uint32_t* hi2ho;
  uint8_t* out;
} run_ctx;

/* writeOutputPixel, WSEQ:66-70: 0x00RRGGBB -> B5 G6 R5 with R in the low bits */
static void write_px(uint8_t* dst, uint32_t rgb888) {
  const uint16_t v = (uint16_t)(((rgb888 >> 19) & 0x001f) | ((rgb888 >> 5) & 0x07e0) |
                                ((rgb888 << 8) & 0xf800));
  dst[0] = (uint8_t)v;
  dst[1] = (uint8_t)(v >> 8);
}

/* drawOutputPixelBound, WSEQ:72-89 (the source point is clamped to the image) */
static void draw_bound(const run_ctx* c, int32_t col, int32_t row, uint32_t rgb888) {
  const int32_t sc = clamp_i32(0, col, c->width - 1);
  const int32_t sr = clamp_i32(0, row, c->height - 1);
  const int64_t ofs = (int64_t)(int32_t)c->hi2ho[sr] * c->out_line_length +
                      (int64_t)(int32_t)c->wi2wo[sc] * 2;
  write_px(c->out + ofs, rgb888);
}

/* drawOutputCircle, WSEQ:91-134 (midpoint circle) */
static void draw_circle(const run_ctx* c, int32_t col, int32_t row, int32_t radius, uint32_t rgb) {
  int32_t err = 1 - radius, err_y = 1, err_x = -2 * radius, x = radius, y = 0;
  draw_bound(c, col, row + radius, rgb);
  draw_bound(c, col, row - radius, rgb);
  draw_bound(c, col + radius, row, rgb);
  draw_bound(c, col - radius, row, rgb);
  while (y < x) {
    if (err >= 0) {
      x -= 1;
      err_x += 2;
      err += err_x;
    }
    y += 1;
    err_y += 2;
    err += err_y;
    draw_bound(c, col + x, row + y, rgb);
    draw_bound(c, col + x, row - y, rgb);
    draw_bound(c, col - x, row + y, rgb);
    draw_bound(c, col - x, row - y, rgb);
    draw_bound(c, col + y, row + x, rgb);
    draw_bound(c, col + y, row - x, rgb);
    draw_bound(c, col - y, row + x, rgb);
    draw_bound(c, col - y, row - x, rgb);
  }
}

/* drawRgbTargetCenterLine / ...HorizontalCenterLine, WSEQ:136-166 */
static void draw_vline(const run_ctx* c, int32_t col, int32_t row, uint32_t rgb) {
  for (int adj = 0; adj < 100; ++adj) {
    draw_bound(c, col, row - adj, rgb);
    draw_bound(c, col, row + adj, rgb);
  }
}
static void draw_hline(const run_ctx* c, int32_t col, int32_t row, uint32_t rgb) {
  for (int adj = 0; adj < 100; ++adj) {
    draw_bound(c, col - adj, row, rgb);
    draw_bound(c, col + adj, row, rgb);
  }
}

/* HsvRangeDetector (cv_hsv_range_detector.hpp:79-198): H/S/V histograms of
 * the central zone; the value whose count first exceeds the running maximum
 * (scan order, strict >) wins; scaled by float constants in double. */
static void auto_range(const uint64_t* img, int width, int height, int zone_scale,
                       trik_oracle_outargs* oa) {
  const uint16_t h_height = (uint16_t)(height / 2), h_width = (uint16_t)(width / 2);
  const uint16_t step = (uint16_t)(height / zone_scale);
  const uint16_t left_p = (uint16_t)(h_width - step), right_p = (uint16_t)(h_width + step);
  const uint16_t top_p = (uint16_t)(h_height - step), bot_p = (uint16_t)(h_height + step);
  uint32_t hh[256], hs[256], hv[256];
  memset(hh, 0, sizeof hh);
  memset(hs, 0, sizeof hs);
  memset(hv, 0, sizeof hv);
  uint32_t max_h = 0, max_s = 0, max_v = 0;
  int32_t max_hc = 0, max_sc = 0, max_vc = 0;
  for (int row = 0; row < height; ++row)
    for (int col = 0; col < width; ++col) {
      const uint32_t p = (uint32_t)img[(int64_t)row * width + col];
      const uint8_t h = (uint8_t)p, s = (uint8_t)(p >> 8), v = (uint8_t)(p >> 16);
      if (left_p < col && right_p > col && top_p < row && bot_p > row) {
        hh[h]++;
        hs[s]++;
        hv[v]++;
        if (hh[h] > (uint32_t)max_hc) { max_h = h; max_hc = (int32_t)hh[h]; }
        if (hs[s] > (uint32_t)max_sc) { max_s = s; max_sc = (int32_t)hs[s]; }
        if (hv[v] > (uint32_t)max_vc) { max_v = v; max_vc = (int32_t)hv[v]; }
      }
    }
  oa->detect_hue = (uint16_t)((double)max_h * 1.4f);
  oa->detect_hue_tol = 15;
  oa->detect_sat = (uint16_t)((double)max_s * 0.39f);
  oa->detect_sat_tol = 30;
  oa->detect_val = (uint16_t)((double)max_v * 0.39f);
  oa->detect_val_tol = 30;
  oa->detect_written = 1;
}

int trik_oracle_run(const uint8_t* frame, int64_t frame_size, int width, int height,
                    int line_length, int layout, const trik_oracle_range* range, int auto_detect,
                    int out_width, int out_height, int out_line_length, uint8_t* out,
                    int64_t out_size, trik_oracle_outargs* oa) {
  enum { kZoneScale = 6 }; /* WSEQ:32 */
  memset(oa, 0, sizeof *oa);
  if (width < 0 || height < 0 || width % 32 != 0 || height % 4 != 0) return -1; /* WSEQ:365-369 */
  const int64_t need = (int64_t)height * line_length * (layout == TRIK_ORACLE_LAYOUT_OV7670 ? 2 : 1);
  if ((int64_t)height * line_length > frame_size || need > frame_size) return -1; /* WSEQ:415 */
  if (out && (int64_t)out_height * out_line_length > out_size) return -1;          /* WSEQ:417 */

  /* WSEQ:371-387: scale maps, truncated double products */
  const double sw = (double)out_width / width, sh = (double)out_height / height;
  const double shift = sw < sh ? sw : sh;
  uint32_t* wi2wo = (uint32_t*)malloc(sizeof(uint32_t) * (size_t)(width > 0 ? width : 1));
  uint32_t* hi2ho = (uint32_t*)malloc(sizeof(uint32_t) * (size_t)(height > 0 ? height : 1));
  uint64_t* img = (uint64_t*)malloc(sizeof(uint64_t) * (size_t)((int64_t)width * height > 0 ? (int64_t)width * height : 1));
  if (!wi2wo || !hi2ho || !img) {
    free(wi2wo); free(hi2ho); free(img);
    return -1;
  }
  for (int i = 0; i < width; ++i) wi2wo[i] = (uint32_t)(i * shift);
  for (int i = 0; i < height; ++i) hi2ho[i] = (uint32_t)(i * shift);

  uint32_t from, to, expect;
  trik_oracle_pack_range(range, &from, &to, &expect);
  int32_t tx = 0, ty = 0;
  uint32_t tn = 0;
  const run_ctx ctx = {width, height, out_line_length, wi2wo, hi2ho, out};
  if (height > 0 && width > 0) {
    for (int row = 0; row < height; ++row) /* convertImageYuyvToHsv */
      for (int q = 0; q < width / 2; ++q) {
        uint32_t rgb[2];
        trik_oracle_pair_rgb_c64x(pair_word(frame, height, line_length, layout, row, q), rgb);
        for (int k = 0; k < 2; ++k)
          img[(int64_t)row * width + 2 * q + k] =
              ((uint64_t)rgb[k] << 32) | trik_oracle_hsv_c64x(rgb[k]);
      }
    if (auto_detect) auto_range(img, width, height, kZoneScale, oa);
    for (int row = 0; row < height; ++row) { /* proceedImageHsv */
      uint32_t row_n = 0, row_x = 0;
      for (int col = 0; col < width; ++col) {
        const uint64_t e = img[(int64_t)row * width + col];
        const int det = trik_oracle_detect((uint32_t)e, from, to, expect);
        row_n += (uint32_t)det;
        row_x += det ? (uint32_t)col : 0;
        if (out)
          write_px(out + (int64_t)hi2ho[row] * out_line_length + (int64_t)wi2wo[col] * 2,
                   det ? 0x00ffffu : (uint32_t)(e >> 32));
      }
      tx += (int32_t)row_x;
      ty += (int32_t)((uint32_t)row * row_n);
      tn += row_n;
    }
  }
  if (out && width > 0 && height > 0) { /* WSEQ:471-485 (degenerate sizes would index s_hi2ho[-1]) */
    const int step = height / kZoneScale, h_height = height / 2, h_width = width / 2;
    draw_vline(&ctx, h_width - 2 * step, h_height, 0xff00ff);
    draw_vline(&ctx, h_width - step, h_height, 0xff00ff);
    draw_vline(&ctx, h_width + step, h_height, 0xff00ff);
    draw_vline(&ctx, h_width + 2 * step, h_height, 0xff00ff);
    draw_hline(&ctx, h_width, h_height - 2 * step, 0xff00ff);
    draw_hline(&ctx, h_width, h_height - step, 0xff00ff);
    draw_hline(&ctx, h_width, h_height + step, 0xff00ff);
    draw_hline(&ctx, h_width, h_height + 2 * step, 0xff00ff);
  }
  const int64_t sums[3] = {(int64_t)tn, (int64_t)tx, (int64_t)ty};
  trik_oracle_targets(sums, width, height, &oa->target_x, &oa->target_y, &oa->target_size);
  if (out && tn > 0) { /* WSEQ:486-494 */
    const int32_t cx = (int32_t)((uint32_t)tx / tn), cy = (int32_t)((uint32_t)ty / tn);
    const uint32_t radius = (uint32_t)ceilf(sqrtf((float)tn / 3.1415927f));
    draw_circle(&ctx, cx, cy, (int32_t)radius, 0xffff00);
  }
  free(wi2wo);
  free(hi2ho);
  free(img);
  return 0;
}

/* ------------------------------------------------------------------------ */
/* ov7670 line sensor (LSEQ = trik/ov7670/line_sensor/include/internal/      */
/* cv_line_detector_seqpass.hpp).                                            */
/* ------------------------------------------------------------------------ */

int trik_oracle_line_run(const uint8_t* frame, int64_t frame_size, int width, int height,
                         int line_length, int val_from, int val_to, int32_t band[2],
                         int out_width, int out_height, int out_line_length, uint8_t* out,
                         int64_t out_size, trik_oracle_outargs* oa, int64_t sums[3]) {
  enum { kStep = 40 }; /* LSEQ:422 */
  memset(oa, 0, sizeof *oa);
  if (width < 0 || height < 0 || width % 32 != 0 || height % 4 != 0) return -1; /* LSEQ:328-332 */
  if (2LL * height * line_length > frame_size) return -1; /* both planes (LSEQ:378, :211-214) */
  if (out && (int64_t)out_height * out_line_length > out_size) return -1;        /* LSEQ:380 */

  const double sw = (double)out_width / width, sh = (double)out_height / height;
  const double shift = sw < sh ? sw : sh; /* LSEQ:334-348 */
  uint32_t* wi2wo = (uint32_t*)malloc(sizeof(uint32_t) * (size_t)(width > 0 ? width : 1));
  uint32_t* hi2ho = (uint32_t*)malloc(sizeof(uint32_t) * (size_t)(height > 0 ? height : 1));
  if (!wi2wo || !hi2ho) {
    free(wi2wo); free(hi2ho);
    return -1;
  }
  for (int i = 0; i < width; ++i) wi2wo[i] = (uint32_t)(i * shift);
  for (int i = 0; i < height; ++i) hi2ho[i] = (uint32_t)(i * shift);

  /* LSEQ:391-414: H and S bounds 0..255 unscaled, V scaled as the object sensor */
  trik_oracle_range r = {0, 359, 0, 100, (uint8_t)val_from, (uint8_t)val_to};
  uint32_t from, to, expect;
  trik_oracle_pack_range(&r, &from, &to, &expect);
  from = (from & 0x00FF0000u); /* H from 0, S from 0 */
  to = (to & 0x00FF0000u) | 0x0000FFFFu;
  expect = 0;

  int32_t tx = 0;
  uint32_t tn = 0, cross = 0;
  const run_ctx ctx = {width, height, out_line_length, wi2wo, hi2ho, out};
  if (height > 0 && width > 0) {
    for (int row = 0; row < height; ++row) { /* convertImageYuyvToHsv + proceedImageHsv */
      uint32_t row_n = 0, row_x = 0;
      for (int q = 0; q < width / 2; ++q) {
        uint32_t rgb[2];
        trik_oracle_pair_rgb_c64x(pair_word(frame, height, line_length, TRIK_ORACLE_LAYOUT_OV7670, row, q), rgb);
        for (int k = 0; k < 2; ++k) {
          const int col = 2 * q + k;
          if (col >= 5 && col <= width - 5) { /* LSEQ:288 */
            const int det = trik_oracle_detect(trik_oracle_hsv_c64x(rgb[k]), from, to, expect);
            row_n += (uint32_t)det;
            row_x += det ? (uint32_t)col : 0;
            if (out)
              write_px(out + (int64_t)hi2ho[row] * out_line_length + (int64_t)wi2wo[col] * 2,
                       det ? 0x00ffffu : rgb[k]);
          }
        }
      }
      tx += (int32_t)row_x;
      tn += row_n;
      if ((uint32_t)row >= (uint32_t)band[0] && (uint32_t)row <= (uint32_t)band[1]) cross += row_n;
    }
  }
  const int h_width = width / 2, h_height = height / 2;
  const int32_t draw_y = 0; /* m_inImageFirstRow - H/2 + H/2 with scale coefficient 1 */
  if (out && width > 0 && height > 0) {
    const int32_t cols[4] = {h_width - kStep, h_width + kStep, h_width - 2 * kStep, h_width + 2 * kStep};
    for (int k = 0; k < 4; ++k) /* drawRgbThinLine, LSEQ:104-116 */
      for (int adj = 0; adj < height; ++adj) draw_bound(&ctx, cols[k], draw_y + adj, 0xff00ff);
  }
  band[0] = h_height; /* LSEQ:449-450 */
  band[1] = h_height + 2 * kStep;
  const int cross_size = width > 0 ? (int)((uint32_t)(cross * 100u) / (uint32_t)(width * 2 * kStep)) : 0;
  if (out && width > 0 && height > 0)
    for (int k = 0; k < 2; ++k) /* drawRgbHorizontalLine, LSEQ:118-130 */
      for (int adj = 0; adj < width; ++adj) draw_bound(&ctx, adj, band[k], 0xff0000);
  if (tn > 10) { /* LSEQ:462-474 */
    const int32_t cx = (int32_t)((uint32_t)tx / tn);
    if (out)
      for (int adj = 0; adj < height; ++adj) /* drawRgbTargetCenterLine, LSEQ:88-102 */
        for (int d = -1; d <= 1; ++d) draw_bound(&ctx, cx + d, draw_y + adj, 0xff0000);
    oa->target_x = (int8_t)(((cx - width / 2) * 100 * 2) / width);
    oa->target_y = (int8_t)cross_size;
    oa->target_size = (uint8_t)((uint32_t)(tn * 100u) / (uint32_t)(height * width));
  }
  if (sums) {
    sums[0] = (int64_t)tn;
    sums[1] = (int64_t)tx;
    sums[2] = (int64_t)cross;
  }
  free(wi2wo);
  free(hi2ho);
  return 0;
}

/* ------------------------------------------------------------------------ */
/* webcam line sensor (LSEQW = trik/webcam/line_sensor/include/internal/     */
/* cv_line_detector_seqpass.hpp).                                            */
/* ------------------------------------------------------------------------ */

int trik_oracle_wline_run(const uint8_t* frame, int64_t frame_size, int width, int height,
                          int line_length, int val_from, int val_to, int out_width, int out_height,
                          int out_line_length, uint8_t* out, int64_t out_size, trik_oracle_outargs* oa,
                          int64_t sums[3]) {
  memset(oa, 0, sizeof *oa);
  if (width < 0 || height < 0 || width % 32 != 0 || height % 4 != 0) return -1; /* LSEQW:297-301 */
  if ((int64_t)height * line_length > frame_size) return -1;                    /* LSEQW:333 */
  if (out && (int64_t)out_height * out_line_length > out_size) return -1;       /* LSEQW:335 */

  /* LSEQW:304-305: the smaller of the two output/input ratios, in double */
  const double rw = (double)out_width / width, rh = (double)out_height / height;
  const double shift = rh < rw ? rh : rw;
  uint32_t* col_map = (uint32_t*)malloc(sizeof(uint32_t) * (size_t)(width > 0 ? width : 1));
  uint32_t* row_map = (uint32_t*)malloc(sizeof(uint32_t) * (size_t)(height > 0 ? height : 1));
  if (!col_map || !row_map) {
    free(col_map); free(row_map);
    return -1;
  }
  for (int c = 0; c < width; ++c) col_map[c] = (uint32_t)(c * shift);
  for (int r = 0; r < height; ++r) row_map[r] = (uint32_t)(r * shift);

  /* LSEQW:345-364: H 0..255 and S 0..255 (unscaled constants), V scaled and
   * clamped as the object sensor does; never the wrapped-hue form */
  const trik_oracle_range vr = {0, 0, 0, 0, (uint8_t)val_from, (uint8_t)val_to};
  uint32_t lo, hi, expect;
  trik_oracle_pack_range(&vr, &lo, &hi, &expect);
  lo &= 0x00FF0000u;
  hi = (hi & 0x00FF0000u) | 0x0000FFFFu;

  /* LSEQW:197-269 with m_imageScaleCoeff = 1: every row, first row 0 */
  int32_t acc_x = 0, acc_y = 0;
  uint32_t acc_n = 0;
  for (int row = 0; row < height; ++row) {
    uint32_t n_row = 0, x_row = 0;
    for (int q = 0; q < width / 2; ++q) {
      uint32_t rgb[2];
      trik_oracle_pair_rgb_c64x(pair_word(frame, height, line_length, TRIK_ORACLE_LAYOUT_YUYV, row, q), rgb);
      for (int k = 0; k < 2; ++k) {
        const int col = 2 * q + k;
        const int hit = trik_oracle_detect(trik_oracle_hsv_c64x(rgb[k]), lo, hi, 0);
        n_row += (uint32_t)hit;
        x_row += hit ? (uint32_t)col : 0u;
        if (out)
          write_px(out + (int64_t)row_map[row] * out_line_length + (int64_t)col_map[col] * 2,
                   hit ? 0x00ffffu : rgb[k]);
      }
    }
    acc_x += (int32_t)x_row;
    acc_y += (int32_t)((uint32_t)row * n_row);
    acc_n += n_row;
  }

  const run_ctx ctx = {width, height, out_line_length, col_map, row_map, out};
  const int mid = width / 2;
  if (out && width > 0 && height > 0) { /* drawRgbThinLine x4 from row 0 (LSEQW:396-399) */
    const int32_t at[4] = {mid - 40, mid + 40, mid - 80, mid + 80};
    for (int k = 0; k < 4; ++k)
      for (int r = 0; r < height; ++r) draw_bound(&ctx, at[k], r, 0xff00ff);
  }
  if (acc_n > 10) { /* LSEQW:405-417 */
    const int32_t tx = (int32_t)((uint32_t)acc_x / acc_n);
    if (out)
      for (int r = 0; r < height; ++r) /* drawRgbTargetCenterLine */
        for (int c = tx - 1; c <= tx + 1; ++c) draw_bound(&ctx, c, r, 0xff0000);
    oa->target_x = (int8_t)(((tx - width / 2) * 200) / width);
    oa->target_size = (uint8_t)((acc_n * 100u) / (uint32_t)(width * height));
  }
  if (sums) {
    sums[0] = (int64_t)acc_n;
    sums[1] = (int64_t)acc_x;
    sums[2] = (int64_t)acc_y;
  }
  free(col_map);
  free(row_map);
  return 0;
}

/* ------------------------------------------------------------------------ */
/* ov7670 object sensor: metapixel bitmap + clusterer (OSEQ:516-602).        */
/* ------------------------------------------------------------------------ */

static int value_range(int v, int adj, int lo, int hi) { /* makeValueRange, stdcpp.hpp:70-79 */
  v += adj;
  return v > hi ? hi : (v < lo ? lo : v);
}
static int value_wrap(int v, int adj, int lo, int hi) { /* makeValueWrap, stdcpp.hpp:81-90 */
  v += adj;
  while (v > hi) v -= hi - lo + 1;
  while (v < lo) v += hi - lo + 1;
  return v;
}

void trik_oracle_blob_range(const trik_oracle_blob_args* a, trik_oracle_blob_state* st) {
  /* BMB:110-130: from/to around the centre, scaled as the webcam's (int16 range) */
  const int hf = value_wrap(a->hue, -(int)a->hue_tol, 0, 359);
  const int ht = value_wrap(a->hue, +(int)a->hue_tol, 0, 359);
  const int sf = value_range(a->sat, -(int)a->sat_tol, 0, 100);
  const int st_ = value_range(a->sat, +(int)a->sat_tol, 0, 100);
  const int vf = value_range(a->val, -(int)a->val_tol, 0, 100);
  const int vt = value_range(a->val, +(int)a->val_tol, 0, 100);
  const uint32_t h0 = (uint32_t)clamp_range(0, (hf * 255) / 359, 255);
  const uint32_t h1 = (uint32_t)clamp_range(0, (ht * 255) / 359, 255);
  const uint32_t s0 = (uint32_t)clamp_range(0, (sf * 255) / 100, 255);
  const uint32_t s1 = (uint32_t)clamp_range(0, (st_ * 255) / 100, 255);
  const uint32_t v0 = (uint32_t)clamp_range(0, (vf * 255) / 100, 255);
  const uint32_t v1 = (uint32_t)clamp_range(0, (vt * 255) / 100, 255);
  if (h0 <= h1) { /* resetHsvRange, BMB:62-77 */
    st->from = (v0 << 16) | (s0 << 8) | h0;
    st->to = (v1 << 16) | (s1 << 8) | h1;
    st->expect = 0;
  } else {
    st->from = (v0 << 16) | (s0 << 8) | ((h1 + 1) & 0xFFu);
    st->to = (v1 << 16) | (s1 << 8) | ((h0 - 1) & 0xFFu);
    st->expect = 1;
  }
}

static int blob_pop16(uint16_t x) { /* pop(), stdcpp.hpp:58-68 */
  int n = 0;
  for (; x; x &= (uint16_t)(x - 1)) ++n;
  return n;
}

/* CLU:44-52: the smallest non-zero of the four, 0 when all are 0 */
static uint16_t blob_min4(const uint16_t a[4]) {
  uint16_t v = a[0];
  for (int n = 1; n < 4; ++n)
    if ((a[n] < v && a[n] != 0) || v == 0) v = a[n];
  return v;
}

typedef struct blob_cluster { int32_t x, y, size, label; } blob_cluster;

/* size descending, ties by ascending label: an insertion-stable merge sort */
static void blob_sort(blob_cluster* c, blob_cluster* tmp, int n) {
  for (int w = 1; w < n; w *= 2)
    for (int lo = 0; lo < n; lo += 2 * w) {
      const int mid = lo + w < n ? lo + w : n, hi = lo + 2 * w < n ? lo + 2 * w : n;
      int i = lo, j = mid, k = lo;
      while (i < mid && j < hi) tmp[k++] = (c[j].size > c[i].size) ? c[j++] : c[i++];
      while (i < mid) tmp[k++] = c[i++];
      while (j < hi) tmp[k++] = c[j++];
      for (k = lo; k < hi; ++k) c[k] = tmp[k];
    }
}

int trik_oracle_blob_run(const uint8_t* frame, int64_t frame_size, int width, int height,
                         int line_length, const trik_oracle_blob_args* args,
                         trik_oracle_blob_state* state, int out_width, int out_height,
                         int out_line_length, uint8_t* out, int64_t out_size, int8_t targets[24],
                         uint8_t* meta, uint16_t* labels_out, int32_t top[24], int32_t* n_labels) {
  memset(targets, 0, 24);
  if (top) memset(top, 0, 24 * sizeof(int32_t));
  if (n_labels) *n_labels = 0;
  if (width < 0 || height < 0 || width % 32 != 0 || height % 4 != 0) return -1; /* OSEQ:462-466 */
  if (2LL * height * line_length > frame_size) return -1; /* both planes (OSEQ:517, :347) */
  if (out && (int64_t)out_height * out_line_length > out_size) return -1;
  const int bw = width / 4, bh = height / 4; /* OSEQ:441-444 */
  if ((int64_t)((bw + 1) / 2) * ((bh + 1) / 2) + 1 > 65535) return -1; /* uint16 labels */
  if (args->set_hsv_range) trik_oracle_blob_range(args, state);

  const double sw = (double)out_width / width, sh = (double)out_height / height;
  const double shift = sw < sh ? sw : sh; /* OSEQ:468-470 */
  const size_t npx = (size_t)((int64_t)width * height > 0 ? (int64_t)width * height : 1);
  const size_t nmp = (size_t)(bw * bh > 0 ? bw * bh : 1);
  uint32_t* wi2wo = (uint32_t*)malloc(sizeof(uint32_t) * (size_t)(width > 0 ? width : 1));
  uint32_t* hi2ho = (uint32_t*)malloc(sizeof(uint32_t) * (size_t)(height > 0 ? height : 1));
  uint32_t* rgb = (uint32_t*)malloc(sizeof(uint32_t) * npx);
  uint16_t* bitmap = (uint16_t*)calloc(nmp, sizeof(uint16_t));
  uint16_t* lab = (uint16_t*)calloc(nmp, sizeof(uint16_t));
  uint16_t* eq = (uint16_t*)malloc(sizeof(uint16_t) * (nmp + 2));
  blob_cluster* cl = (blob_cluster*)malloc(sizeof(blob_cluster) * (nmp + 2));
  blob_cluster* tmp = (blob_cluster*)malloc(sizeof(blob_cluster) * (nmp + 2));
  if (!wi2wo || !hi2ho || !rgb || !bitmap || !lab || !eq || !cl || !tmp) {
    free(wi2wo); free(hi2ho); free(rgb); free(bitmap); free(lab); free(eq); free(cl); free(tmp);
    return -1;
  }
  for (int i = 0; i < width; ++i) wi2wo[i] = (uint32_t)(i * shift);
  for (int i = 0; i < height; ++i) hi2ho[i] = (uint32_t)(i * shift);

  int n = 1; /* CLU:180-183: label 0 is the background */
  eq[0] = 0;
  memset(&cl[0], 0, sizeof cl[0]);
  if (height > 0 && width > 0) {
    for (int row = 0; row < height; ++row) /* convertImageYuyvToHsv + BitmapBuilder::run */
      for (int q = 0; q < width / 2; ++q) {
        uint32_t px[2];
        trik_oracle_pair_rgb_c64x(pair_word(frame, height, line_length, TRIK_ORACLE_LAYOUT_OV7670, row, q), px);
        for (int k = 0; k < 2; ++k) {
          const int col = 2 * q + k;
          rgb[(int64_t)row * width + col] = px[k];
          const int det = trik_oracle_detect(trik_oracle_hsv_c64x(px[k]), state->from, state->to, state->expect);
          bitmap[(row / 4) * bw + col / 4] |= (uint16_t)(det << ((row % 4) * 4 + col % 4));
        }
      }
    for (int r = 0; r < bh; ++r) /* Clusterizer::run, CLU:185-190 */
      for (int c = 0; c < bw; ++c) {
        if (blob_pop16(bitmap[r * bw + c]) <= 2) continue;
        uint16_t a[4] = {0, 0, 0, 0}; /* left, up-left, up, up-right (CLU:70-84) */
        if (r != 0) {
          a[2] = lab[(r - 1) * bw + c];
          if (c != 0) a[1] = lab[(r - 1) * bw + c - 1];
          if (c != bw - 1) a[3] = lab[(r - 1) * bw + c + 1];
        }
        if (c != 0) a[0] = lab[r * bw + c - 1];
        const uint16_t m = blob_min4(a);
        if (m) { /* CLU:91-97 */
          lab[r * bw + c] = m;
          cl[m].x += c;
          cl[m].y += r;
          cl[m].size++;
          for (int i = 0; i < 4; ++i)
            if (a[i] && !(a[i] == m || eq[a[i]] == eq[m])) eq[a[i]] = eq[m];
        } else { /* CLU:98-112: new label, its first metapixel not counted */
          lab[r * bw + c] = (uint16_t)n;
          eq[n] = (uint16_t)n;
          memset(&cl[n], 0, sizeof cl[n]);
          ++n;
        }
      }
  }
  for (int i = 0; i < n; ++i) { /* postProcessing, CLU:115-127 */
    cl[i].label = i;
    if (i != eq[i]) {
      cl[eq[i]].x += cl[i].x;
      cl[eq[i]].y += cl[i].y;
      cl[eq[i]].size += cl[i].size;
      cl[i].size = 0;
    }
  }
  blob_sort(cl, tmp, n);
  if (n_labels) *n_labels = n;
  if (meta)
    for (int i = 0; i < bw * bh; ++i) meta[i] = blob_pop16(bitmap[i]) > 2;
  if (labels_out) memcpy(labels_out, lab, sizeof(uint16_t) * (size_t)(bw * bh));

  const run_ctx ctx = {width, height, out_line_length, wi2wo, hi2ho, out};
  if (out && width > 0 && height > 0) {
    for (int row = 0; row < height; ++row) /* proceedImageHsv, OSEQ:387-420 */
      for (int col = 0; col < width; ++col) {
        const int det = lab[(row / 4) * bw + col / 4] != 0; /* getMinEqCluster(label) != 0 */
        write_px(out + (int64_t)hi2ho[row] * out_line_length + (int64_t)wi2wo[col] * 2,
                 det ? 0x00ffffu : rgb[(int64_t)row * width + col]);
      }
    const int step = height / 6, h_height = height / 2, h_width = width / 2; /* OSEQ:548-561 */
    draw_vline(&ctx, h_width - step, h_height, 0xff00ff);
    draw_vline(&ctx, h_width + step, h_height, 0xff00ff);
    draw_vline(&ctx, h_width - 2 * step, h_height, 0xff00ff);
    draw_vline(&ctx, h_width + 2 * step, h_height, 0xff00ff);
    draw_hline(&ctx, h_width, h_height - step, 0xff00ff);
    draw_hline(&ctx, h_width, h_height + step, 0xff00ff);
    draw_hline(&ctx, h_width, h_height - 2 * step, 0xff00ff);
    draw_hline(&ctx, h_width, h_height + 2 * step, 0xff00ff);
  }
  for (int i = 0; i < 8; ++i) { /* OSEQ:563-590 */
    const int32_t csize = i < n ? cl[i].size : 0;
    if (top && i < n) {
      top[3 * i] = cl[i].size;
      top[3 * i + 1] = cl[i].x;
      top[3 * i + 2] = cl[i].y;
    }
    const int root = (int)sqrtf((float)(uint16_t)csize); /* getSize() is uint16_t */
    const uint32_t radius = (uint32_t)ceilf((float)root / 3.1415927f);
    const int size = (int)((radius * 100u * 4u) / (uint32_t)(bw + bh));
    if (size > 4) {
      const int32_t x = (cl[i].x / (csize + 1)) * 4, y = (cl[i].y / (csize + 1)) * 4; /* CLU:139-147 */
      if (out && width > 0 && height > 0)
        for (int dc = -1; dc <= 1; ++dc) /* drawFatPixel, OSEQ:92-108 */
          for (int dr = -1; dr <= 1; ++dr) draw_bound(&ctx, x + dc, y + dr, 0xff0000);
      targets[3 * i + 2] = (int8_t)(uint8_t)size;
      targets[3 * i] = (int8_t)(((x - width / 2) * 100 * 2) / width);
      targets[3 * i + 1] = (int8_t)(((y - height / 2) * 100 * 2) / height);
    }
  }
  free(wi2wo); free(hi2ho); free(rgb); free(bitmap); free(lab); free(eq); free(cl); free(tmp);
  return 0;
}
