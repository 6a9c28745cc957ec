// trik_hsv_internal.h -- shared between the host C++ (ABI, table compiler)
// and the HIP kernels.  Not part of the public ABI (include/trik_hsv.h).
#pragma once

#include <hip/hip_runtime.h>

#include <string>
#include <stdint.h>

#include "../../include/trik_hsv.h"

namespace trik_hsv {

// Ranges handled by one launch of the hot kernel (per-pixel masks are
// byte-spread: range t -> bits 8t..8t+7 of a 32-bit word).
constexpr int kRangesPerLaunch = 4;

// Device-side lookup tables compiled from one group of <= 4 ranges
// (trik_hsv_tables.cpp).  Staged into LDS by every workgroup.
//   sv[mx * 256 + mn] : bit t = range t's saturation AND value tests pass for a
//                       pixel with max channel mx and min channel mn (mn <= mx).
//                       S = (LUT255[mx] * (mx - mn)) >> 8 (WSEQ:223-224), V = mx.
//   hue[H]            : bit t = range t's hue test passes (incl. wrap, WSEQ:433-445).
//   lut43[d], lut255[m] : s_mult43_div, s_mult255_div (WSEQ:389-407).
//   smask[S], vmask[V] : bit t = range t's saturation / value test passes
//                       (the two factors of sv, for the chroma kernel's exact path).
struct alignas(16) RangeTables {
  uint8_t sv[256 * 256];
  uint8_t hue[256];
  uint16_t lut43[256];
  uint16_t lut255[256];
  uint8_t smask[256];
  uint8_t vmask[256];
};
static_assert(sizeof(RangeTables) == 65536 + 256 + 512 + 512 + 512, "table layout");

// Packed form of one InArgs range (WSEQ:425-445).
struct PackedRange {
  uint32_t from, to, expect;
};

// Tables of the stripe kernel (trik_hsv_stripe.hip), staged in LDS.  Sized so
// that two 1024-thread workgroups fit one CU (2 x 78,848 B of 160 KiB), i.e.
// 8 waves per SIMD:
//   sv[mx * 260 + mn] : T-bit (sat AND val) mask for max mx, min mn (offset 0,
//                       so its address is one v_mad_u32_u24); rows padded to
//                       260 bytes so the bank rotates with mx
//   hue[H][kHueCopies] : byte-spread hue mask (range t -> bit 8t)
//   m43[d][kM43Copies] : s_mult43_div (WSEQ:389-407)
// The two small tables are replicated and interleaved so that lane L reads
// copy L % copies: a wave's random lookups spread over the LDS banks.
constexpr int kSvStride = 260;
constexpr int kHueCopies = 8;
constexpr int kM43Copies = 4;
struct alignas(16) StripeTables {
  uint8_t sv[256 * kSvStride];
  uint32_t hue[256 * kHueCopies];
  uint32_t m43[256 * kM43Copies];
};
static_assert(sizeof(StripeTables) == 66560 + 256 * 4 * (kHueCopies + kM43Copies), "table layout");
static_assert(2 * sizeof(StripeTables) <= 160 * 1024, "two workgroups per CU");

// Tables of the chroma-run kernel (trik_hsv_chroma.hip), one set per group of
// <= 4 ranges, built on the device from RangeTables:
//   runs[c]     : descriptor b1 | b2 << 8 of chroma c = U | V << 8: the
//                 fast path's mask is Y >= A && Y <= b2 ? (Y < b1 ? M1 : M2) : 0
//                 (A: the block's cut); with b1 > b2 + 1 the pixels
//                 b2 < Y < b1 go to the exact path (a "window", always above
//                 A), and kChromaExc sends both pixels there
//   summary[c]  : builder scratch (run summary of the chroma's profile)
constexpr uint32_t kChromaExc = 0x00FFu;  // b1 = 255, b2 = 0: the builder never makes this window
//   blocks[b]   : low byte: 8 x the palette slot of block b's mask pair (the
//                 hot kernel's LDS offset of the pair); high byte: the block's
//                 leading-zero cut A: pixels with Y < A are 0 (the
//                 fast path masks them), so a chroma whose profile is zero
//                 below A describes only its profile from A on -- the
//                 0 | M1 | M2 | 0 profiles of overlapping ranges become runs
//   palette     : the byte-spread (M1, M2) of each palette slot; palette_of[k]
//                 is 8 x the slot of pair k, or 0xFF; pair_hist: blocks per pair
//   summary / summary_drop / first_nz : builder scratch, per chroma: the run
//                 summary of the profile from Y = 0 and from its first nonzero
//                 Y on, and that Y (256: all zero); best[b]: the block's
//                 packed (cost, pair, cut) choice; block_cost[b]: its cost
//                 after the palette pass
constexpr int kChromaPalette = 32;  // 8 x slot fits the block byte
struct alignas(16) ChromaTables {
  uint16_t runs[65536];
  uint16_t blocks[4096];
  uint32_t summary[65536];
  uint32_t summary_drop[65536];
  uint16_t first_nz[65536];
  unsigned long long best[4096];
  uint32_t block_cost[4096];  // the palette pass's cost per block (summed by its last workgroup)
  uint32_t pair_hist[256];
  uint32_t palette[2 * kChromaPalette];
  uint8_t palette_of[256];
  // sum over all chromas of the expected exact-path words per 65536 words
  // (chroma_cost): / 2^32 = the expected share of words the exact path takes
  // on uniform input; the host's AUTO selector reads it
  unsigned long long flagged_cost;
  // words the hot kernel's exact path resolved, summed over its launches on
  // these tables (zeroed by the build): the host's AUTO selector reads it back
  // now and then to compare the input's actual share with flagged_cost's
  unsigned long long flagged_words;
};

PackedRange pack_range(const TRIK_VIDTRANSCODE_CV_InArgsAlg& r);
void compile_tables(const TRIK_VIDTRANSCODE_CV_InArgsAlg* ranges, int n, RangeTables* out);
// compile_tables in two parts: the head (LUTs, per-value H/S/V tests) first,
// then the sat/val table (which reads the head's lut255)
void compile_tables_head(const TRIK_VIDTRANSCODE_CV_InArgsAlg* ranges, int n, RangeTables* out);
void compile_tables_sv(const TRIK_VIDTRANSCODE_CV_InArgsAlg* ranges, int n, RangeTables* out);
void compile_stripe_tables(const RangeTables& base, int n, StripeTables* out);
// Which tests of detectHsvPixel (WSEQ:171-179) a group of n compiled ranges
// needs: kDetectFull; kDetectSV when each accepts every hue value; kDetectV
// when each also accepts every saturation value.
enum DetectMode { kDetectFull = 0, kDetectSV = 1, kDetectV = 2 };
int detect_mode(const RangeTables& t, int n);

struct KernelArgs {
  const uint8_t* frames;
  int64_t frame_stride;
  int32_t n_frames;
  int32_t width, height, line_length;
  int32_t layout;
  int32_t n_ranges;      // ranges in this launch (1..4)
  int32_t range_offset;  // index of this launch's first range in the sums array
  int32_t sums_ranges;   // ranges per frame in the sums array (row pitch)
  const RangeTables* tables;
  const StripeTables* stripe_tables;
  TrikHsvTargetSums* sums;
  uint8_t* masks;        // verification mode only
  int32_t mask_shift;    // bit position of this launch's range 0 in the mask byte
  // the detection the stripe kernel needs for this group (detect_mode()):
  // kDetectSV when every range accepts every hue, kDetectV when every range
  // also accepts every saturation
  int32_t detect_mode = 0;
  // Device-side kernel choice while the host does not know a new range set's
  // exact-path share yet: with gate set the kernel runs only if
  // (*gate <= gate_max) == gate_le (one uniform load per workgroup).
  const unsigned long long* gate = nullptr;
  unsigned long long gate_max = 0;
  int32_t gate_le = 0;
  // The fused step (chroma-run kernel; chroma_fused_ok): the workgroups split
  // the batch's wave-sized units evenly, whatever the frame boundaries; a
  // frame's units add into its accumulator (frame_acc: one 128-B line per
  // frame, 12 sums and the unit count) and count themselves done; the wave
  // that counts a frame's last
  // unit reads and clears the accumulator, stores the frame's sums and
  // targets and adds them to its workgroup's totals; the last workgroup sums
  // the workgroups' partial totals.  One launch, no memset.  DESIGN.md 4.5.
  int32_t fused = 0;
  TrikHsvTarget* targets = nullptr;       // [n_frames][sums_ranges], or NULL
  TrikHsvTargetSums* totals = nullptr;    // [sums_ranges], or NULL
  unsigned long long* wg_part = nullptr;  // scratch: [workgroups][12]
  uint32_t* wg_cnt = nullptr;             // scratch: 0 between launches
  unsigned long long* frame_acc = nullptr;  // scratch: [n_frames][16], 0 between launches
  // The chroma-run kernel's past-the-end loads (one per lane and tile, never
  // consumed) read this per-handle sink instead of the frames when the
  // lane's offsets fit (chroma_tail_span() <= tail_bytes); otherwise they
  // re-read the tile's last rows.  No load depends on another allocation.
  const uint8_t* tail = nullptr;
  int64_t tail_bytes = 0;
  // CUs the chroma-run kernel leaves free (trik_hsv_set_reserved_cus)
  int32_t reserved_cus = 0;
};

// The target of one (frame, range) from its sums: WSEQ:486-505 (unsigned
// centroid division, fp32 sqrtf / ceil radius).  The reference's int32 /
// uint32 arithmetic: the sums are non-negative, so 64-bit division agrees
// wherever the reference's 32-bit accumulators do not overflow, and stays
// exact beyond.
__device__ __forceinline__ TrikHsvTarget target_of(uint64_t points, uint64_t sum_x, uint64_t sum_y, int width,
                                                   int height) {
  TrikHsvTarget r = {0, 0, 0, 0};
  if (points > 0) {
    // 32-bit divisions whenever the sums fit (every frame of the reference's
    // sizes), 64-bit ones beyond
    const bool narrow = ((sum_x | sum_y | points) >> 32) == 0;
    const int32_t cx = (int32_t)(narrow ? (uint32_t)sum_x / (uint32_t)points : sum_x / points);
    const int32_t cy = (int32_t)(narrow ? (uint32_t)sum_y / (uint32_t)points : sum_y / points);
    const float q = __fdiv_rn((float)(uint32_t)points, 3.1415927f);
    const uint32_t radius = (uint32_t)ceilf(__fsqrt_rn(q));  // WSEQ:492
    r.x = (int8_t)(((cx - width / 2) * 100 * 2) / width);   // WSEQ:496-498
    r.y = (int8_t)(((cy - height / 2) * 100 * 2) / height);
    r.size = (uint8_t)((uint32_t)(radius * 100 * 4) / (uint32_t)(width + height));
  }
  return r;
}

__device__ __forceinline__ bool gated_out(const unsigned long long* gate, unsigned long long gate_max, int gate_le) {
  return gate && ((*gate <= gate_max) != (gate_le != 0));
}

// The AUTO rule: the chroma-run kernel while a range group's expected
// exact-path cost (ChromaTables::flagged_cost, share * 2^32) is at most this.
constexpr unsigned long long kChromaMaxCost = (unsigned long long)(TRIK_HSV_CHROMA_MAX_SHARE * 4294967296.0);

// RGB565X preview of N frames for one range (trik_hsv_operator.hip).
struct PreviewArgs {
  const uint8_t* frames;
  int64_t frame_stride;
  int32_t n_frames, width, height, line_length, layout;
  PackedRange range;          // the preview's range (WSEQ:425-445)
  const StripeTables* tables = nullptr;  // that range compiled as range 0 (device)
  int32_t aligned4;           // frames, strides, line lengths and previews 4-byte aligned
  int32_t out_w, out_h, out_ll;
  uint8_t* previews;
  int64_t preview_stride;
  const int32_t* last_row;  // [out_h]: last source row mapped to each output row, or -1
  const int32_t* last_col;  // [out_w]
  const uint32_t* wi2wo;    // [width]  WSEQ:375-379
  const uint32_t* hi2ho;    // [height] WSEQ:381-385
  // ov7670 multi-blob preview: when set, a pixel is "detected" iff its 4x4
  // metapixel is set ([n][H/4][W/4], OSEQ:411-413) instead of by `range`
  const uint8_t* meta = nullptr;
  // >= 0 when the maps are the 2:1 ones: last_row[r] = rows2_first + 2 r for
  // every output row and last_col[c] = 2 c + 1 for the output columns in
  // [rows2_c0, rows2_c1), -1 (not written) outside (preview_rows2_kernel)
  int32_t rows2_first = -1, rows2_c0 = 0, rows2_c1 = 0;
  // the object sensors' guide lines as output bits ([out_h][out_w / 8], bit
  // c % 8 of byte c / 8; 2:1 maps only, else NULL): the 2:1 kernel draws them
  // as it writes the preview, and the overlay then draws only the circle
  const uint8_t* guide_bits = nullptr;
  int32_t guides_drawn = 0;  // set by launch_preview for the overlay
  // range 0 accepts every hue (its detect_mode() is not kDetectFull): the 2:1
  // kernel tests the sat&val mask alone
  int32_t hue_free = 0;
  // The line sensors' overlays drawn by preview_rows2_kernel in the same pass
  // (launch_line_preview; LSEQ:419-474, LSEQW:396-417 through
  // drawOutputPixelBound), set when ovl_ok (the column map is monotone with
  // steps of 0 or 1, so the output columns a source interval hits are one
  // interval): magenta on output columns ovl_mag[] of every row, red on rows
  // ovl_band[] (-1: none) over columns [ovl_c_lo, ovl_c_hi], and red on frame
  // f's target columns wi2wo[clamp(cx - 1 .. cx + 1)] (ovl_sums[f].points > 10)
  const TrikHsvTargetSums* ovl_sums = nullptr;
  int32_t ovl_ok = 0, ovl_half = 0;  // ovl_half: wi2wo[c] = c / 2 for every c
  int32_t ovl_mag[4] = {-1, -1, -1, -1}, ovl_band[2] = {-1, -1}, ovl_c_lo = 0, ovl_c_hi = -1;
};

// Auto HSV range of N frames (trik_hsv_operator.hip); out[f][6] = detectHue,
// detectHueTolerance, detectSat, detectSatTolerance, detectVal, detectValTolerance.
struct AutoRangeArgs {
  const uint8_t* frames;
  int64_t frame_stride;
  int32_t n_frames, width, height, line_length, layout;
  int32_t c_lo, c_hi, r_lo, r_hi;  // exclusive zone bounds (uint16 values, hpp:88-108)
  int32_t aligned4;                // frames, stride and line length 4-byte aligned
  uint16_t* out;
};

// ov7670 line sensor of N frames (trik_hsv_line.hip).  sums[f] = {N, sumX,
// crossPoints} (crossPoints in the sum_y slot), zeroed by the caller.
struct LineArgs {
  const uint8_t* frames;
  int64_t frame_stride;
  int32_t n_frames, width, height, line_length;
  uint32_t val_lo, val_hi;           // scaled V bounds (LSEQ:397-398)
  int32_t band_start, band_stop;     // cross-point rows (LSEQ:298)
  TrikHsvTargetSums* sums;
  TrikHsvTarget* targets;            // may be NULL
};

// Per-device facts, cached thread-safely per device (trik_hsv_device.cpp):
// the current device's CU count, and a kernel's dynamic-LDS attribute set once
// per (device, kernel).
int device_cus();
// the CUs stream s may use: its CU mask's (hipExtStreamCreateWithCUMask), else
// the device's
int stream_cus(hipStream_t s);
hipError_t set_dynamic_lds(const void* kern, int bytes);

// Launchers (trik_hsv_kernels.hip, trik_hsv_operator.hip, trik_hsv_line.hip).
// Return hipError_t as int.
int launch_reduce(const KernelArgs& a, bool write_masks, hipStream_t s);
// The optimised hot kernel (trik_hsv_stripe.hip); returns hipErrorNotSupported
// when the geometry needs the generic kernel (misaligned input, width > 8192).
int launch_stripe(const KernelArgs& a, bool write_masks, hipStream_t s);
// The chroma-run hot kernel (trik_hsv_chroma.hip): tables built once per
// range set; launch returns hipErrorNotSupported when the geometry needs
// another kernel.
int build_chroma_tables(const RangeTables* t, ChromaTables* ct, hipStream_t s);
bool chroma_geometry_ok(const KernelArgs& a);
// the fused step applies (frames whole per workgroup, >= 4 frames each; no
// verification masks)
bool chroma_fused_ok(const KernelArgs& a);
int launch_chroma(const KernelArgs& a, const ChromaTables* ct, bool write_masks, hipStream_t s);
// Bytes from a tile's base that the chroma-run kernel's past-the-end loads
// span for this geometry (YUYV: (k + dy) rows + 2 dx; ov7670: a luma plane
// and k rows), or -1 when the kernel does not take the geometry.
int64_t chroma_tail_span(const KernelArgs& a);
// The per-handle sink's size: spans up to this read the sink (ov7670 frames
// up to ~2 Mpixel), larger ones re-read the tile's last rows.
constexpr int64_t kChromaTailSink = 4 << 20;
// Sets the calling thread's trik_hsv_last_error() message; returns code.
int32_t set_error(int32_t code, const std::string& msg);
// The packed ranges of up to kTableGroups groups of <= 4 (kernel argument).
constexpr int kTableGroups = 16;
struct TableBuildArgs {
  uint32_t from[kTableGroups * 4], to[kTableGroups * 4], expect[kTableGroups * 4];
  int32_t n_ranges;  // over all groups
};
// compile_tables + compile_stripe_tables on the device from the packed ranges
// alone (groups <= kTableGroups): no host-built table crosses PCIe.
int launch_compile_tables(const TableBuildArgs& args, int groups, RangeTables* d_tables, StripeTables* d_stripe,
                          hipStream_t s);
int launch_totals(int n_frames, int n_ranges, const TrikHsvTargetSums* sums, TrikHsvTargetSums* totals,
                  hipStream_t s);
int launch_targets(const TrikHsvFrameBatch& b, int n_ranges, const TrikHsvTargetSums* sums,
                   TrikHsvTarget* targets, hipStream_t s);
int launch_synth(const TrikHsvFrameBatch& b, uint8_t* frames, int first_frame, int kind,
                 uint64_t seed, hipStream_t s);
// preview_kernel then overlay_kernel (circle from sums[f * sums_pitch])
int launch_preview(const PreviewArgs& a, const TrikHsvTargetSums* sums, int sums_pitch, hipStream_t s);
int launch_auto_range(const AutoRangeArgs& a, hipStream_t s);
int launch_line(const LineArgs& a, hipStream_t s);
// preview body as launch_preview's first kernel, then the line sensor's overlay
int launch_preview_body(const PreviewArgs& a, hipStream_t s);
int launch_line_overlay(const PreviewArgs& a, const TrikHsvTargetSums* sums, hipStream_t s);
// the webcam line sensor (trik/webcam/line_sensor): OutArgs from the sums of
// the V-only range (targetY 0), and its overlay (thin lines, target line)
int launch_wline_targets(int n_frames, int width, int height, const TrikHsvTargetSums* sums, TrikHsvTarget* targets,
                         hipStream_t s);
int launch_wline_overlay(const PreviewArgs& a, const TrikHsvTargetSums* sums, hipStream_t s);
// preview_rows2_kernel alone (hipErrorNotSupported where it does not apply)
int launch_preview_rows2(const PreviewArgs& a, hipStream_t s);
// a line sensor's whole preview: body and overlay (band = 1: the ov7670 line
// sensor's band lines), fused into one pass where the 2:1 kernel applies
int launch_line_preview(PreviewArgs a, const TrikHsvTargetSums* sums, int band, hipStream_t s);

// ov7670 multi-blob sensor of N frames (trik_hsv_blob.hip).
struct BlobArgs {
  const uint8_t* frames;
  int64_t frame_stride;
  int32_t n_frames, width, height, line_length;
  PackedRange range;         // the sticky BitmapBuilder range (BMB:62-77)
  const StripeTables* tables;  // that range compiled as range 0 (device)
  int32_t aligned4;          // frames, stride and line length 4-byte aligned
  uint8_t* meta;             // [n][H/4][W/4]: 1 for set metapixels
  uint16_t* labels;          // optional [n][H/4][W/4]: the clusterer's label map
  int32_t* stats;            // scratch [n][max_labels][3] int32: the own {x, y, size}, folded in place
  int32_t max_labels;        // blob_max_labels(W/4, H/4)
  TrikHsvTarget* targets;    // [n][8]
  int32_t* top;              // [n][8][3]: size, sum_x, sum_y of the 8 largest clusters
  int32_t* n_labels;         // optional [n]
  int32_t meta_lds = 0;      // set by launch_blob: the bitmap staged in LDS
  int32_t meta_ready = 0;    // the bitmap is already written (launch_blob_meta_chroma)
  // set by launch_blob: the own statistics as one packed u64 per label,
  // size | sum_x << pack_sx | sum_y << pack_sy (0: three int32 per label)
  int32_t pack_sx = 0, pack_sy = 0;
  // gate of the bitmap kernel (as KernelArgs::gate): the chroma-run bitmap and
  // the stripe-arithmetic bitmap are both launched, one of them runs
  const unsigned long long* gate = nullptr;
  unsigned long long gate_max = 0;
  int32_t gate_le = 0;
};
// Labels a frame can need: seeds are pairwise non-adjacent in the 8-neighbourhood
// (a metapixel next to an earlier set one is never a seed), so at most
// ceil(bw/2) * ceil(bh/2) of them, plus the background label 0.
inline int64_t blob_max_labels(int bw, int bh) { return (int64_t)((bw + 1) / 2) * ((bh + 1) / 2) + 1; }
int launch_blob(const BlobArgs& a, hipStream_t s);
// The metapixel bitmap on the chroma-run tables of the sticky range (ct, rt:
// its ChromaTables and RangeTables); hipErrorNotSupported when the geometry
// needs the generic kernel (width % 16, 16-byte aligned frames and lines).
// launch_blob with a.meta_from_chroma set then runs only the clusterer.
bool blob_chroma_ok(const BlobArgs& a);
int launch_blob_meta_chroma(const BlobArgs& a, const ChromaTables* ct, const RangeTables* rt, hipStream_t s);
// guide lines + a 3x3 mark per kept target (OSEQ:548-580), from BlobArgs.top
int launch_blob_overlay(const PreviewArgs& a, const int32_t* top, hipStream_t s);

// Host side of the preview geometry (trik_hsv_tables.cpp): the reference's
// scale maps and their inverses, packed as
//   wi2wo[width], hi2ho[height], last_row[out_h], last_col[out_w]  (32-bit each).
// Only source columns col_lo..col_hi write (the line sensor's window).
void preview_maps(int width, int height, int out_w, int out_h, uint32_t* maps, int col_lo = 0,
                  int col_hi = 0x7FFFFFFF);
// Zone bounds of HsvRangeDetector::initImg (hpp:88-108) for zone scale 6.
void auto_range_zone(int width, int height, int32_t& c_lo, int32_t& c_hi, int32_t& r_lo,
                     int32_t& r_hi);

}  // namespace trik_hsv
