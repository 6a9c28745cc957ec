/*
 * trik_oracle.h -- CPU restatement of the TRIK HSV-threshold + centroid path.
 *
 * TEST INFRASTRUCTURE ONLY.  This is the parity checker for the MI355X HIP
 * path in trik-media-sensors-dsp_amd/.  Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load it.  The product library
 * (libtrik_hsv.so) never links or calls it.
 *
 * What it restates (paths relative to the reference checkout):
 *   trik/webcam/object_sensor/include/internal/cv_ball_detector_seqpass.hpp
 *     (alias WSEQ)  -- the active webcam object-sensor implementation
 *   trik/ov7670/object_sensor/include/internal/cv_ball_detector_seqpass.hpp
 *     (alias OSEQ)  -- the ov7670 semi-planar input layout (OSEQ:343-387)
 *
 * Two independent derivations of the per-pixel arithmetic live here:
 *   1. an intrinsic-level restatement that follows WSEQ:181-249 step by step
 *      over a C emulation of the TI C64x+ intrinsics it uses (semantics from
 *      TI's published C64x+ intrinsic definitions);
 *   2. a closed-form restatement.
 * tests/test_oracle.py requires them to agree on all 2^24 inputs.
 *
 * PARITY STATUS: the reference ships no tests, fixtures or golden vectors,
 * and its hot path cannot be compiled here (it needs TI's <c6x.h> and the
 * XDAIS headers, which are absent; building it with stand-in headers is not
 * allowed).  Parity is therefore "unpinned" by reference artefacts.  It is
 * pinned instead by the two derivations above, per-intrinsic unit tests and
 * the SURVEY Appendix A known-answer table.  See DESIGN.md section 3.
 */
#ifndef TRIK_ORACLE_H_
#define TRIK_ORACLE_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum {
  TRIK_ORACLE_LAYOUT_YUYV   = 0, /* packed Y0 U Y1 V (webcam, WSEQ:251-284) */
  TRIK_ORACLE_LAYOUT_OV7670 = 1  /* Y plane + chroma plane (OSEQ:343-387) */
};

/* Mirrors TRIK_VIDTRANSCODE_CV_InArgsAlg (webcam trik_vidtranscode_cv.h:48-56). */
typedef struct trik_oracle_range {
  uint16_t hue_from, hue_to; /* 0..359 */
  uint8_t sat_from, sat_to;  /* 0..100 */
  uint8_t val_from, val_to;  /* 0..100 */
} trik_oracle_range;

/* --- C64x+ intrinsic emulation (exported for the per-intrinsic unit tests) --- */
uint64_t trik_c64x_mpyu4ll(uint32_t a, uint32_t b);
int32_t  trik_c64x_dotpus4(uint32_t a, uint32_t b);
uint32_t trik_c64x_add2(uint32_t a, uint32_t b);
uint32_t trik_c64x_packh2(uint32_t a, uint32_t b);
uint32_t trik_c64x_packlh2(uint32_t a, uint32_t b);
uint32_t trik_c64x_pack2(uint32_t a, uint32_t b);
uint32_t trik_c64x_packhl2(uint32_t a, uint32_t b);
uint32_t trik_c64x_shr2(uint32_t a, uint32_t n);
uint32_t trik_c64x_clr(uint32_t a, uint32_t lo, uint32_t hi);
uint32_t trik_c64x_spacku4(uint32_t a, uint32_t b);
uint32_t trik_c64x_unpkhu4(uint32_t a);
uint32_t trik_c64x_unpklu4(uint32_t a);
uint32_t trik_c64x_maxu4(uint32_t a, uint32_t b);
uint32_t trik_c64x_minu4(uint32_t a, uint32_t b);
uint32_t trik_c64x_cmpeq2(uint32_t a, uint32_t b);
int32_t  trik_c64x_dotpn2(uint32_t a, uint32_t b);
uint32_t trik_c64x_packh4(uint32_t a, uint32_t b);
uint32_t trik_c64x_cmpltu4(uint32_t a, uint32_t b);
uint32_t trik_c64x_cmpgtu4(uint32_t a, uint32_t b);
uint32_t trik_c64x_swap4(uint32_t a);

/* --- per-pixel arithmetic --- */
/* s_mult43_div / s_mult255_div, WSEQ:389-407. */
void     trik_oracle_luts(uint16_t lut43[256], uint16_t lut255[256]);
/* WSEQ:181-205: one YUYV word (b0=Y0,b1=U,b2=Y1,b3=V) -> two 0x00RRGGBB words. */
void     trik_oracle_pair_rgb_c64x(uint32_t yuyv, uint32_t rgb_out[2]);
/* WSEQ:207-249: 0x00RRGGBB -> 0x00VVSSHH. */
uint32_t trik_oracle_hsv_c64x(uint32_t rgb888);
/* SURVEY Appendix A closed forms of the same two stages. */
uint32_t trik_oracle_rgb_closed(uint32_t y, uint32_t u, uint32_t v);
uint32_t trik_oracle_hsv_closed(uint32_t rgb888);

/* WSEQ:425-445: InArgs -> packed (from, to, expect) words. */
void     trik_oracle_pack_range(const trik_oracle_range* r, uint32_t* from,
                                uint32_t* to, uint32_t* expect);
/* WSEQ:171-179. */
int      trik_oracle_detect(uint32_t hsv, uint32_t from, uint32_t to, uint32_t expect);

/* Table of (rgb<<32 | hsv) for every (Y,U,V): index = Y | U<<8 | V<<16.
 * closed != 0 selects the closed-form derivation. out has 2^24 entries. */
void     trik_oracle_yuv_table(uint64_t* out, int closed);

/* One frame through WSEQ:412-508 (or the OSEQ layout) for T ranges.
 * sums[3*t + {0,1,2}] = {targetPoints, targetX sum, targetY sum} as the
 * reference accumulates them (WSEQ:316-354).  mask (optional, W*H bytes)
 * receives the per-pixel T-bit detection mask (bit t = range t).
 * Returns 0, or -1 where the reference's setup/run would fail
 * (W%32, H%4, negative dims: WSEQ:365-369; H*lineLength > size: WSEQ:415). */
int      trik_oracle_frame(const uint8_t* frame, int64_t frame_size, int width,
                           int height, int line_length, int layout,
                           const trik_oracle_range* ranges, int n_ranges,
                           int64_t* sums, uint8_t* mask);

/* WSEQ:486-505 epilogue: sums {N, sumX, sumY} -> targetX/Y/Size. */
void     trik_oracle_targets(const int64_t sums[3], int width, int height,
                             int8_t* target_x, int8_t* target_y, uint8_t* target_size);

/* Batch of frames split over n_threads POSIX threads (the CPU baseline).
 * sums is [n_frames][n_ranges][3]; targets is [n_frames][n_ranges][3] bytes
 * (x, y, size) and may be NULL. */
int      trik_oracle_batch(const uint8_t* frames, int64_t frame_stride, int n_frames,
                           int width, int height, int line_length, int layout,
                           const trik_oracle_range* ranges, int n_ranges,
                           int64_t* sums, int8_t* targets, int n_threads);

/* The clean-room scalar CPU baseline (trik_cpu_baseline.c): the same sums as
 * trik_oracle_batch (n_ranges <= 32), computed the way a plain CPU port would
 * (closed-form arithmetic, no intrinsic emulation), frames split over
 * n_threads POSIX threads.  Used by bench.py's cpu_baseline only. */
int      trik_cpu_batch(const uint8_t* frames, int64_t frame_stride, int n_frames,
                        int width, int height, int line_length, int layout,
                        const trik_oracle_range* ranges, int n_ranges, int64_t* sums,
                        int n_threads);

/* The single-pass webcam detector (WSGL, trik_oracle_wsgl.c): a second
 * reference text restated for cross-checking the WSEQ restatement above.
 * table: out[Y | U << 8 | V << 16] bit 0 / bit 1 = detection of the first /
 * second pixel of a YUYV word with that luma (2^24 bytes).  run: one packed
 * YUYV frame, one range: sums {N, sum x, sum y} and target {x, y, size};
 * returns 0 when WSGL's run() would return false, else 1. */
void     trik_oracle_wsgl_table(const trik_oracle_range* range, uint8_t* out);
int      trik_oracle_wsgl_run(const uint8_t* frame, int64_t frame_size, int width, int height,
                              int line_length, const trik_oracle_range* range, int64_t sums[3],
                              int32_t target[3]);

/* Synthetic frame generators shared bit-for-bit with the device generator
 * (synth kernels in trik-media-sensors-dsp_amd/csrc/trik_hsv_kernels.hip).
 * kind 0 = uniform random bytes, kind 1 = scene (gradients + 6 discs). */
void     trik_oracle_synth(uint8_t* frames, int64_t frame_stride, int first_frame,
                           int n_frames, int width, int height, int line_length,
                           int layout, int kind, uint64_t seed);

/* OutArgsAlg fields written by one run (WPUB:64-74). */
typedef struct trik_oracle_outargs {
  int8_t target_x, target_y;
  uint8_t target_size;
  uint8_t detect_written; /* 1 when autoDetectHsv filled the detect* fields */
  uint16_t detect_hue, detect_hue_tol, detect_sat, detect_sat_tol, detect_val, detect_val_tol;
} trik_oracle_outargs;

/* The whole of BallDetector::setup + run (WSEQ:358-508) for one frame and one
 * range, as the codec's process() drives it:
 *   - per-pixel RGB/HSV image (WSEQ:251-284, or the OSEQ:343-387 layout);
 *   - autoDetectHsv: HsvRangeDetector::detect (cv_hsv_range_detector.hpp:
 *     88-201, zone scale 6, WSEQ:32,455-462) into the detect* fields;
 *   - proceedImageHsv (WSEQ:316-354): sums, and the RGB565X preview written
 *     through the truncated double scale maps (WSEQ:371-387), detected pixels
 *     as 0x00ffff, last writer wins;
 *   - guide lines and target circle (WSEQ:66-166, 471-485), then OutArgs
 *     (WSEQ:486-505).
 * out may be NULL (no preview stream).  Returns 0, or -1 where setup/run
 * would fail (geometry WSEQ:365-369, buffer sizes WSEQ:415-418). */
int      trik_oracle_run(const uint8_t* frame, int64_t frame_size, int width, int height,
                         int line_length, int layout, const trik_oracle_range* range,
                         int auto_detect, int out_width, int out_height, int out_line_length,
                         uint8_t* out, int64_t out_size, trik_oracle_outargs* oa);

/* The ov7670 line sensor, LineDetector::setup + run (trik/ov7670/line_sensor/
 * include/internal/cv_line_detector_seqpass.hpp:258-301, 376-476; LSEQ):
 *   - the object sensor's per-pixel HSV on the ov7670 planes;
 *   - detection by V only (hue and saturation bounds fixed at 0..255,
 *     LSEQ:391-396), in columns 5 <= col <= W-5 only (LSEQ:288);
 *   - cross points: detected pixels of rows hStart..hStop, where hStart and
 *     hStop are the values the PREVIOUS run left (LSEQ:298 reads them before
 *     LSEQ:449-450 sets them to H/2 and H/2+80); *band is that state, in and
 *     out (the reference leaves it uninitialised before the first run);
 *   - preview writes for the window columns only, thin guide lines, the two
 *     band lines and the 3-pixel target line (LSEQ:433-463);
 *   - OutArgs: targetX as the object sensor, targetY = cross points * 100 /
 *     (W * 80), targetSize = N * 100 / (W * H), all 0 unless N > 10.
 * autoDetectHsv is not restated: the line sensor's detector is a simulated
 * annealing seeded by srand(time(NULL)) (cv_hsv_range_detector.hpp there),
 * so its output is not reproducible; detect* are left untouched.
 * sums (optional) receives {N, sumX, crossPoints}. */
int      trik_oracle_line_run(const uint8_t* frame, int64_t frame_size, int width, int height,
                              int line_length, int val_from, int val_to, int32_t band[2],
                              int out_width, int out_height, int out_line_length, uint8_t* out,
                              int64_t out_size, trik_oracle_outargs* oa, int64_t sums[3]);

/* The webcam line sensor, LineDetector<YUV422, RGB565X>::setup + run
 * (trik/webcam/line_sensor/include/internal/cv_line_detector_seqpass.hpp:
 * 290-420; LSEQW): packed YUYV, the object sensor's per-pixel HSV, detection
 * by V only (H and S bounds 0..255), every pixel of every row
 * (m_imageScaleCoeff = 1); the preview written for every pixel through the
 * object sensor's maps, four thin magenta lines at columns W/2 +- 40 and
 * W/2 +- 80, and, when N > 10, the 3-column red target line; OutArgs
 * targetX as the object sensor, targetY 0, targetSize = N * 100 / (W * H),
 * all 0 unless N > 10.  autoDetectHsv is not restated (simulated annealing
 * seeded by srand(time(NULL))).  sums (optional) receives {N, sumX, sumY}. */
int      trik_oracle_wline_run(const uint8_t* frame, int64_t frame_size, int width, int height,
                               int line_length, int val_from, int val_to, int out_width,
                               int out_height, int out_line_length, uint8_t* out, int64_t out_size,
                               trik_oracle_outargs* oa, int64_t sums[3]);

/* ---- ov7670 object sensor: metapixel bitmap + clusterer -> 8 targets ------
 * BLOB = BallDetector<YUV422P, RGB565X> of trik/ov7670/object_sensor/include/
 * internal/cv_ball_detector_seqpass.hpp:516-602 (OSEQ), with BitmapBuilder
 * (cv_bitmap_builder_reference.hpp:107-217, BMB) and Clusterizer
 * (cv_clusterizer_reference.hpp:85-202, CLU). */

/* TRIK_VIDTRANSCODE_CV_InArgsAlg of trik/ov7670/object_sensor/
 * trik_vidtranscode_cv.h:51-60 (XDAS_Bool restated as int32). */
typedef struct trik_oracle_blob_args {
  int32_t set_hsv_range;
  uint16_t hue, hue_tol;    /* 0..359 */
  uint8_t sat, sat_tol;     /* 0..100 */
  uint8_t val, val_tol;     /* 0..100 */
  int32_t auto_detect;      /* not restated (srand(time) annealing) */
} trik_oracle_blob_args;

/* BitmapBuilder's sticky packed range (BMB:45-46, 62-77): set only when
 * set_hsv_range; uninitialised in the reference before that, zero here. */
typedef struct trik_oracle_blob_state {
  uint32_t from, to, expect;
} trik_oracle_blob_state;

/* BMB:110-130 + resetHsvRange: centre/tolerance -> packed range */
void     trik_oracle_blob_range(const trik_oracle_blob_args* a, trik_oracle_blob_state* st);

/* One run:
 *   - per-pixel HSV (the object sensor's, ov7670 planes) and detection with the
 *     sticky range (updated first when set_hsv_range);
 *   - bitmap: 4x4 metapixels of bw = W/4 x bh = H/4, bit (row%4)*4 + col%4
 *     (BMB:171-190); a metapixel is "set" when more than 2 of its 16 pixels
 *     are detected (CLU:185-186);
 *   - clusterer, literally: raster scan over set metapixels, label = the
 *     smallest non-zero label among left, up-left, up, up-right (CLU:70-84,
 *     44-52), else a new label whose first metapixel is not counted
 *     (CLU:98-112); equivalences one level deep (CLU:92-96); postProcessing
 *     folds each label into its equivalence target in label order, zeroing
 *     only the size (CLU:115-127);
 *   - sort by size, descending; ties by ascending label (the reference's
 *     std::sort leaves their order unspecified);
 *   - targets i < 8 (OSEQ:572-598): r = ceil(floor(sqrt(size)) / pi),
 *     size% = r*400/(bw+bh), kept when > 4, x/y = (sum / (size+1)) * 4 in
 *     percent of the half-frame; entries past the label count have size 0
 *     (the reference reads past the end of its vector);
 *   - preview: every pixel through the truncated double scale maps, set
 *     metapixels as 0x00ffff (OSEQ:387-420), the 8 guide lines, then a 3x3
 *     red "fat pixel" per kept target (OSEQ:556-580).
 * targets: 8 x {x, y, size}; meta (optional, bw*bh): 1 for set metapixels;
 * labels (optional, bw*bh): the label map; top (optional, 8 x {size, sum_x,
 * sum_y} after postProcessing and sorting); *n_labels: labels including 0.
 * Returns -1 where setup/run would fail, or when the label count could
 * exceed the reference's uint16 labels. */
int      trik_oracle_blob_run(const uint8_t* frame, int64_t frame_size, int width, int height,
                              int line_length, const trik_oracle_blob_args* args,
                              trik_oracle_blob_state* state, int out_width, int out_height,
                              int out_line_length, uint8_t* out, int64_t out_size,
                              int8_t targets[24], uint8_t* meta, uint16_t* labels,
                              int32_t top[24], int32_t* n_labels);

#ifdef __cplusplus
}
#endif

#endif /* TRIK_ORACLE_H_ */
