/*
 * trik_oracle_wsgl.c -- a second reference text, restated: the webcam object
 * sensor's single-pass BallDetector,
 *   trik/webcam/object_sensor/include/internal/cv_ball_detector_singlepass.hpp
 * (alias WSGL; cv_ball_detector.hpp:54-55 selects the sequential-pass file,
 * WSEQ, and keeps this one commented out).
 *
 * TEST INFRASTRUCTURE ONLY (see trik_oracle.h).  It exists to tie the oracle
 * to a second text of the reference: WSGL computes the same detection and
 * centroid in one pass per YUYV word (YUV -> RGB -> HSV -> range test ->
 * sums), where WSEQ converts the frame to an HSV buffer first.  The
 * restatement follows WSGL's statements in its own order over the C64x+
 * intrinsic emulation of trik_oracle.c; it shares no code with the WSEQ
 * restatement beyond those intrinsics and the LUT definition (WSGL:229-236,
 * identical to WSEQ:389-407).  tests/test_oracle_wsgl.py requires the two to
 * agree on every (Y, U, V) triple and on whole frames.  This does not pin
 * parity (the reference still cannot be run here); it checks the oracle
 * against a second reading of the reference's algorithm.
 */
#include <math.h>
#include <pthread.h>
#include <stdint.h>

#include "trik_oracle.h"

typedef struct wsgl_state {
  uint64_t detect_range; /* m_detectRange: hi word = From, lo word = To */
  uint32_t detect_expected;
  uint16_t mult43_div[256], mult255_div[256];
  int32_t target_x, target_y; /* m_targetX / m_targetY (int32, WSGL:21-23) */
  uint32_t target_points;
} wsgl_state;

static int32_t wsgl_range(int32_t lo, int32_t v, int32_t hi) { /* stdcpp.hpp range<T> */
  return v < lo ? lo : (v > hi ? hi : v);
}

static uint64_t wsgl_itoll(uint32_t hi, uint32_t lo) { return ((uint64_t)hi << 32) | lo; }
static uint32_t wsgl_hill(uint64_t x) { return (uint32_t)(x >> 32); }
static uint32_t wsgl_loll(uint64_t x) { return (uint32_t)x; }

/* WSGL:229-236 (setup: the division tables) */
static void wsgl_setup(wsgl_state* s) {
  s->mult43_div[0] = 0;
  s->mult255_div[0] = 0;
  for (uint32_t idx = 1; idx < 256u; ++idx) {
    s->mult43_div[idx] = (uint16_t)((43u * 256u) / idx);
    s->mult255_div[idx] = (uint16_t)((255u * 256u) / idx);
  }
}

/* WSGL:258-277 (run: the InArgs range scaled and packed) */
static void wsgl_set_range(wsgl_state* s, const trik_oracle_range* r) {
  const uint32_t hue_from = (uint32_t)wsgl_range(0, ((int32_t)r->hue_from * 255) / 359, 255);
  const uint32_t hue_to = (uint32_t)wsgl_range(0, ((int32_t)r->hue_to * 255) / 359, 255);
  const uint32_t sat_from = (uint32_t)wsgl_range(0, ((int32_t)r->sat_from * 255) / 100, 255);
  const uint32_t sat_to = (uint32_t)wsgl_range(0, ((int32_t)r->sat_to * 255) / 100, 255);
  const uint32_t val_from = (uint32_t)wsgl_range(0, ((int32_t)r->val_from * 255) / 100, 255);
  const uint32_t val_to = (uint32_t)wsgl_range(0, ((int32_t)r->val_to * 255) / 100, 255);
  if (hue_from <= hue_to) {
    s->detect_range = wsgl_itoll((val_from << 16) | (sat_from << 8) | hue_from,
                                 (val_to << 16) | (sat_to << 8) | hue_to);
    s->detect_expected = 0x0;
  } else {
    /* (the assert hue_from > 0 && hue_to < 255 is compiled out; the packed
     * bytes wrap as the uint32 arithmetic does) */
    s->detect_range = wsgl_itoll((val_from << 16) | (sat_from << 8) | ((hue_to + 1) & 0xFFu),
                                 (val_to << 16) | (sat_to << 8) | ((hue_from - 1) & 0xFFu));
    s->detect_expected = 0x1;
  }
}

/* WSGL:111-161 (testifyRgbPixel): is the 0x00RRGGBB pixel in the range? */
static int wsgl_testify(const wsgl_state* s, uint32_t rgb888) {
  const uint32_t rgb_or16 = trik_c64x_unpkhu4(rgb888);
  const uint32_t rgb_gb16 = trik_c64x_unpklu4(rgb888);
  const uint32_t rgb_max2 = trik_c64x_maxu4(rgb888, rgb888 >> 8);
  const uint32_t rgb_max = trik_c64x_clr(trik_c64x_maxu4(rgb_max2, rgb_max2 >> 8), 8, 31);
  const uint32_t rgb_max_max = trik_c64x_pack2(rgb_max, rgb_max);
  const uint32_t hsv_ooo_val_x256 = rgb_max << 8;
  const uint32_t rgb_min2 = trik_c64x_minu4(rgb888, rgb888 >> 8);
  const uint32_t rgb_min = trik_c64x_minu4(rgb_min2, rgb_min2 >> 8);
  const uint32_t rgb_delta = rgb_max - rgb_min;
  const uint32_t hsv_sat_x256 = (uint32_t)s->mult255_div[rgb_max] * rgb_delta;
  const uint32_t hsv_hue_mult43_div = trik_c64x_pack2(s->mult43_div[rgb_delta], s->mult43_div[rgb_delta]);
  int32_t hsv_hue_x256;
  const uint32_t rgb_cmp = trik_c64x_cmpeq2(rgb_max_max, rgb_gb16);
  if (rgb_cmp == 0)
    hsv_hue_x256 = (int32_t)((0x10000 * 0) / 3) +
                   trik_c64x_dotpn2(hsv_hue_mult43_div, trik_c64x_packhl2(rgb_gb16, rgb_gb16));
  else if (rgb_cmp == 1)
    hsv_hue_x256 = (int32_t)((0x10000 * 2) / 3) +
                   trik_c64x_dotpn2(hsv_hue_mult43_div, trik_c64x_packlh2(rgb_or16, rgb_gb16));
  else
    hsv_hue_x256 = (int32_t)((0x10000 * 1) / 3) +
                   trik_c64x_dotpn2(hsv_hue_mult43_div, trik_c64x_pack2(rgb_gb16, rgb_or16));
  const uint32_t hsv_sat_hue_x256 = trik_c64x_pack2(hsv_sat_x256, (uint32_t)hsv_hue_x256);
  const uint32_t hsv = trik_c64x_packh4(hsv_ooo_val_x256, hsv_sat_hue_x256);
  const uint32_t hsv_det = trik_c64x_cmpltu4(hsv, wsgl_hill(s->detect_range)) |
                           trik_c64x_cmpgtu4(hsv, wsgl_loll(s->detect_range));
  return hsv_det == s->detect_expected;
}

/* WSGL:164-178 (proceedRgbPixel), sums only (the preview is not restated) */
static void wsgl_proceed_rgb(wsgl_state* s, uint32_t src_row, uint32_t src_col, uint32_t rgb888) {
  if (wsgl_testify(s, rgb888)) {
    s->target_x += (int32_t)src_col;
    s->target_y += (int32_t)src_row;
    ++s->target_points;
  }
}

/* WSGL:181-213 (proceedTwoYuyvPixels): the word's two RGB pixels */
static void wsgl_two_pixels(uint32_t yuyv, uint32_t* p1, uint32_t* p2) {
  const uint64_t s64_yuyv1 = trik_c64x_mpyu4ll(
      yuyv, ((uint32_t)(uint8_t)(409 / 4) << 24) | ((uint32_t)(uint8_t)(298 / 4) << 16) |
                ((uint32_t)(uint8_t)(516 / 4) << 8) | ((uint32_t)(uint8_t)(298 / 4)));
  const uint32_t u32_yuyv2 = (uint32_t)trik_c64x_dotpus4(
      yuyv, ((uint32_t)(uint8_t)(-208 / 4) << 24) | ((uint32_t)(uint8_t)(-100 / 4) << 8));
  const uint32_t rgb_h = trik_c64x_add2(trik_c64x_packh2(0, wsgl_hill(s64_yuyv1)),
                                        (uint32_t)(uint16_t)(128 / 4 + (-128 * 409 - 16 * 298) / 4));
  const uint32_t rgb_l = trik_c64x_add2(
      trik_c64x_packlh2(u32_yuyv2, wsgl_loll(s64_yuyv1)),
      ((uint32_t)(uint16_t)(128 / 4 + (+128 * 100 + 128 * 208 - 16 * 298) / 4) << 16) |
          (uint32_t)(uint16_t)(128 / 4 + (-128 * 516 - 16 * 298) / 4));
  const uint32_t y1y1 = trik_c64x_pack2(wsgl_loll(s64_yuyv1), wsgl_loll(s64_yuyv1));
  const uint32_t y2y2 = trik_c64x_pack2(wsgl_hill(s64_yuyv1), wsgl_hill(s64_yuyv1));
  const uint32_t p1h = trik_c64x_clr(trik_c64x_shr2(trik_c64x_add2(rgb_h, y1y1), 6), 16, 31);
  const uint32_t p1l = trik_c64x_shr2(trik_c64x_add2(rgb_l, y1y1), 6);
  const uint32_t p2h = trik_c64x_clr(trik_c64x_shr2(trik_c64x_add2(rgb_h, y2y2), 6), 16, 31);
  const uint32_t p2l = trik_c64x_shr2(trik_c64x_add2(rgb_l, y2y2), 6);
  *p1 = trik_c64x_spacku4(p1h, p1l);
  *p2 = trik_c64x_spacku4(p2h, p2l);
}

/* Every (Y, U, V) triple through WSGL: out[y | u << 8 | v << 16] bit 0 =
 * detection of the word's first pixel (Y0 = y), bit 1 = of its second pixel
 * (Y1 = y), for the word whose other luma is 255 - y.  V planes over 8
 * threads. */
typedef struct wsgl_job {
  const wsgl_state* s;
  uint8_t* out;
  uint32_t v0, v1;
} wsgl_job;

static void* wsgl_table_worker(void* arg) {
  const wsgl_job* j = (const wsgl_job*)arg;
  for (uint32_t v = j->v0; v < j->v1; ++v)
    for (uint32_t u = 0; u < 256u; ++u)
      for (uint32_t y = 0; y < 256u; ++y) {
        uint32_t a1, a2, b1, b2;
        wsgl_two_pixels(y | (u << 8) | ((255u - y) << 16) | (v << 24), &a1, &a2);
        wsgl_two_pixels((255u - y) | (u << 8) | (y << 16) | (v << 24), &b1, &b2);
        j->out[y | (u << 8) | (v << 16)] = (uint8_t)(wsgl_testify(j->s, a1) | (wsgl_testify(j->s, b2) << 1));
      }
  return NULL;
}

void trik_oracle_wsgl_table(const trik_oracle_range* range, uint8_t* out) {
  wsgl_state s;
  wsgl_setup(&s);
  wsgl_set_range(&s, range);
  enum { kThreads = 8 };
  pthread_t th[kThreads];
  wsgl_job jobs[kThreads];
  for (int i = 0; i < kThreads; ++i) {
    jobs[i] = (wsgl_job){&s, out, 256u * (uint32_t)i / kThreads, 256u * (uint32_t)(i + 1) / kThreads};
    if (pthread_create(&th[i], NULL, wsgl_table_worker, &jobs[i]) != 0) {
      wsgl_table_worker(&jobs[i]);
      th[i] = 0;
    }
  }
  for (int i = 0; i < kThreads; ++i)
    if (th[i]) pthread_join(th[i], NULL);
}

/* WSGL:245-346 (run) on one packed-YUYV frame, one range: the sums
 * (points, sum x, sum y) and OutArgs targetX / targetY / targetSize.
 * Returns 0 when run() returns false (buffer too small), else 1. */
int trik_oracle_wsgl_run(const uint8_t* frame, int64_t frame_size, int width, int height, int line_length,
                         const trik_oracle_range* range, int64_t sums[3], int32_t target[3]) {
  wsgl_state s;
  wsgl_setup(&s);
  if ((int64_t)height * line_length > frame_size) return 0;
  s.target_x = 0;
  s.target_y = 0;
  s.target_points = 0;
  wsgl_set_range(&s, range);
  if (height > 0 && width > 0) {
    for (uint32_t src_row = 0; src_row < (uint32_t)height; ++src_row) {
      const uint8_t* src = frame + (int64_t)src_row * line_length;
      for (uint32_t src_col = 0; src_col < (uint32_t)width; src_col += 2) {
        const uint32_t yuyv = (uint32_t)src[0] | ((uint32_t)src[1] << 8) | ((uint32_t)src[2] << 16) |
                              ((uint32_t)src[3] << 24);  /* *srcImage++ (little-endian C674x) */
        src += 4;
        uint32_t p1, p2;
        wsgl_two_pixels(yuyv, &p1, &p2);
        wsgl_proceed_rgb(&s, src_row, src_col + 0, p1);
        wsgl_proceed_rgb(&s, src_row, src_col + 1, p2);
      }
    }
  }
  sums[0] = s.target_points;
  sums[1] = s.target_x;
  sums[2] = s.target_y;
  /* WSGL:321-345 */
  if (s.target_points > 0) {
    /* int32 / uint32: the usual conversions make it an unsigned division */
    const int32_t target_x = (int32_t)((uint32_t)s.target_x / s.target_points);
    const int32_t target_y = (int32_t)((uint32_t)s.target_y / s.target_points);
    const uint32_t target_radius = (uint32_t)ceilf(sqrtf((float)s.target_points / 3.1415927f));
    target[0] = ((target_x - width / 2) * 100 * 2) / width;
    target[1] = ((target_y - height / 2) * 100 * 2) / height;
    target[2] = (int32_t)((target_radius * 100u * 4u) / (uint32_t)(width + height));
  } else {
    target[0] = target[1] = target[2] = 0;
  }
  return 1;
}
