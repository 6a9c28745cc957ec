// trik_hsv_operator.hip -- the operator's outputs besides the target sums
// (SURVEY 8(f) rows 1 and 2), paths relative to the reference checkout, WSEQ
// as in include/trik_hsv.h:
//
//  preview_gather_kernel  the RGB565X preview stream written by proceedImageHsv
//                     (WSEQ:316-354): every source pixel is written through the
//                     truncated scale maps (WSEQ:371-387), last writer wins, a
//                     detected pixel as 0x00ffff.  Computed as a gather: output
//                     pixel (r', c') takes the last source row / column that
//                     maps onto it (host-built inverse maps); never-written
//                     output pixels and the line padding are written as zero
//                     (the zero fill of WFXNS:234).
//  overlay_kernel     the guide lines and target circle of WSEQ:66-166,471-494,
//                     one wave per frame, lines before circle as the reference.
//  auto_range_kernel  HsvRangeDetector::detect (trik/webcam/object_sensor/
//                     include/internal/cv_hsv_range_detector.hpp:88-198; zone
//                     scale 6, WSEQ:32,455-462): H, S and V histograms of the
//                     central zone; the reference keeps the value whose count
//                     first exceeds the running maximum in scan order.  A value
//                     with the final maximum count M occurs exactly M times, so
//                     its M-th occurrence is its last one: the winner is the
//                     max-count value with the earliest last occurrence -- one
//                     pass of LDS histograms plus atomicMax of scan positions.
#include <hip/hip_runtime.h>

#include "trik_hsv_internal.h"
#include "trik_hsv_pixel.h"
#include "trik_hsv_stripe_px.h"

namespace trik_hsv {

namespace {

struct Luts {
  uint16_t l43[256], l255[256];
};
constexpr Luts make_luts() {  // WSEQ:400-406
  Luts l{};
  for (uint32_t i = 1; i < 256; ++i) {
    l.l43[i] = (uint16_t)((43u * 256u) / i);
    l.l255[i] = (uint16_t)((255u * 256u) / i);
  }
  return l;
}
__constant__ Luts c_luts = make_luts();


// The preview as a grid-stride gather over 4-byte output groups (two output
// pixels each) of the whole batch: 1024-lane workgroups, two per CU, the
// single range's StripeTables image at LDS address 0 and the hot kernel's
// per-pixel arithmetic (phase1 also yields the clamped colour); with
// a.meta set (the multi-blob preview) detection is the metapixel flag and no
// tables are staged.  Every byte of the out_h x out_ll preview is written.
constexpr int kPreviewQ = 2;  // output groups per lane of the gather
struct PreviewGeom {
  FastDiv per_frame;  // out_h * quads per row
  FastDiv per_row;    // quads per row
  uint32_t total;
  uint32_t map_off;  // LDS byte offset of the row and column maps as u16 (0xFFFF = -1), or 0: read from memory
};
__global__ __launch_bounds__(1024) __attribute__((amdgpu_waves_per_eu(8)))
void preview_gather_kernel(PreviewArgs a, PreviewGeom g) {
  using namespace stripe_px;
  if (!a.meta) {
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
    const u32x4* src = reinterpret_cast<const u32x4*>(a.tables);
    typedef __attribute__((address_space(3))) u32x4* lds_u128_wptr;
    lds_u128_wptr dst = (lds_u128_wptr)(uintptr_t)0;
    for (int i = threadIdx.x; i < (int)(sizeof(StripeTables) / 16); i += blockDim.x) dst[i] = src[i];
  }
  typedef __attribute__((address_space(3))) uint16_t* lds_u16_ptr;
  const lds_u16_ptr maps = (lds_u16_ptr)(uintptr_t)g.map_off;  // [out_h] rows, then [out_w] columns
  if (g.map_off) {
    for (int i = threadIdx.x; i < a.out_h; i += blockDim.x) maps[i] = (uint16_t)a.last_row[i];
    for (int i = threadIdx.x; i < a.out_w; i += blockDim.x) maps[a.out_h + i] = (uint16_t)a.last_col[i];
  }
  __syncthreads();
  auto map_at = [&](const int32_t* mem, int off, int i) -> int {
    if (!g.map_off) return mem[i];
    const uint32_t v = maps[off + i];
    return v == 0xFFFFu ? -1 : (int)v;
  };
  const int t = threadIdx.x;
  const uint32_t hue_lane = (uint32_t)offsetof(StripeTables, hue) + ((t % kHueCopies) << 2);
  const uint32_t m43_lane = (uint32_t)offsetof(StripeTables, m43) + ((t % kM43Copies) << 2);
  const uint32_t qpr = g.per_row.d;
  const int64_t ll = a.line_length;
  // kQ output groups per thread, 64 apart (each load and store instruction of
  // a wave stays on consecutive groups), in phases (positions, map loads, frame
  // loads, arithmetic, stores) so that a thread's loads are in flight together:
  // the loop is bound by the map -> frame -> LDS chain, not by bytes
  constexpr int kQ = kPreviewQ;
  const uint32_t lane = t & 63u, wave_step = (gridDim.x * blockDim.x) >> 6;
  const uint32_t n_chunks = (g.total + 64u * kQ - 1) / (64u * kQ);
  for (uint32_t ch = (blockIdx.x * blockDim.x + t) >> 6; ch < n_chunks; ch += wave_step) {
    uint32_t ff[kQ], rr[kQ], qq[kQ];
    bool ok[kQ];
#pragma unroll
    for (int u = 0; u < kQ; ++u) {
      const uint32_t i = ch * 64u * kQ + 64u * u + lane;
      ok[u] = i < g.total;
      ff[u] = fdiv(i, g.per_frame);
      const uint32_t rem = i - ff[u] * g.per_frame.d;
      rr[u] = fdiv(rem, g.per_row);
      qq[u] = rem - rr[u] * qpr;
    }
    int sr[kQ], sc[kQ][2];
#pragma unroll
    for (int u = 0; u < kQ; ++u) {
      sr[u] = ok[u] ? map_at(a.last_row, 0, (int)rr[u]) : -1;
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        const int c = 2 * (int)qq[u] + k;
        sc[u][k] = ok[u] && c < a.out_w ? map_at(a.last_col, a.out_h, c) : -1;
      }
    }
    uint32_t w[kQ][2];  // each pixel as a YUYV word with its Y in byte 0
#pragma unroll
    for (int u = 0; u < kQ; ++u) {
      const uint8_t* fr = a.frames + (int64_t)ff[u] * a.frame_stride;
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        w[u][k] = 0u;
        if (sr[u] < 0 || sc[u][k] < 0) continue;
        if (a.layout == TRIK_HSV_LAYOUT_YUYV && a.aligned4) {
          w[u][k] = *reinterpret_cast<const uint32_t*>(fr + (int64_t)sr[u] * ll + 4 * (sc[u][k] >> 1));
        } else if (a.layout == TRIK_HSV_LAYOUT_OV7670 && a.aligned4) {
          // Y from the luma plane, the V, U byte pair as one u16 (OSEQ:343-387)
          const int64_t off = (int64_t)sr[u] * ll + sc[u][k];
          const uint32_t Y = fr[off];
          const uint32_t vu = *reinterpret_cast<const uint16_t*>(fr + ll * a.height + (off & ~(int64_t)1));
          w[u][k] = Y | ((vu >> 8) << 8) | ((vu & 0xFFu) << 24);
        } else {
          int Y, U, V;
          fetch_yuv(fr, a.height, a.line_length, a.layout, sr[u], sc[u][k], Y, U, V);
          w[u][k] = (uint32_t)Y | ((uint32_t)U << 8) | ((uint32_t)V << 24);
        }
      }
    }
    uint32_t out[kQ];
#pragma unroll
    for (int u = 0; u < kQ; ++u) {
      uint32_t v[2] = {0u, 0u};
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        if (sr[u] < 0 || sc[u][k] < 0) continue;
        uint32_t x = w[u][k];
        if (a.layout == TRIK_HSV_LAYOUT_YUYV && a.aligned4 && (sc[u][k] & 1))
          x = __builtin_amdgcn_perm(x, x, 0x03020102u);
        const Phase1 p = phase1<0>(x, x ^ 0xFF00FF00u, m43_lane);
        uint32_t det;
        if (a.meta) {
          det = a.meta[((int64_t)ff[u] * (a.height >> 2) + (sr[u] >> 2)) * (a.width >> 2) + (sc[u][k] >> 2)];
        } else {
          const uint32_t m = lds_u32(p.m43_addr), sv = lds_u8(p.sv_addr);
          det = combine(lds_u32(phase2_addr(m, p, hue_lane)), sv) & 1u;
        }
        const uint32_t rgb = det ? 0x00ffffu : p.rgb888;
        v[k] = ((rgb >> 19) & 0x001fu) | ((rgb >> 5) & 0x07e0u) | ((rgb << 8) & 0xf800u);
      }
      out[u] = v[0] | (v[1] << 16);
    }
#pragma unroll
    for (int u = 0; u < kQ; ++u) {
      if (!ok[u]) continue;
      uint8_t* row = a.previews + (int64_t)ff[u] * a.preview_stride + (int64_t)rr[u] * a.out_ll;
      const int b0 = 4 * (int)qq[u];
      if (a.aligned4 && b0 + 4 <= a.out_ll) {
        __builtin_nontemporal_store(out[u], reinterpret_cast<uint32_t*>(row + b0));  // (as the 2:1 kernel's)
      } else {
        for (int k = 0; k < 4 && b0 + k < a.out_ll; ++k) row[b0 + k] = (uint8_t)(out[u] >> (8 * k));
      }
    }
  }
}

// The same preview when the scale maps are the 2:1 ones (output row r' is
// written last by source row r0 + 2 r', output column c' by source column
// 2 c' + 1 -- the reference's defaults, 640x480 -> 320x240), with the written
// output columns one contiguous window [rows2_c0, rows2_c1) (the line
// sensor's 5 <= col <= W - 5; zero outside).  Output pixel c' is the odd
// pixel of source pixel pair c'.  A unit reads 16 bytes per plane and writes
// its output pixels as 8-byte stores: packed YUYV, 2 x 4 words -> 8 pixels (a
// wave reads 2 KiB of one row); ov7670, 16 luma + 16 chroma bytes -> 8 pixels
// (U = odd chroma byte, OSEQ:369-373).  No maps, no gather.  (A YUYV
// unit is two 16-byte pieces, 8 output pixels: the per-unit address and
// index work is shared by 8 pixels, as in the ov7670 form.)  Lane t of the
// grid takes units t, t + T, t + 2T, ... (T = the grid's lanes), kRowsQ of
// them per round with their loads issued together; the (frame, row, group) of
// the next unit follows from the current one by adding T's decomposition with
// carries (one division per lane, not per unit).  The RGB565X value is packed
// from the clamped channels directly; detection is range 0 (bit 0 of the hue
// and sat&val masks; HUEFREE, a range that accepts every hue -- the line
// sensors' V ranges: the sat&val mask alone) or the metapixel flag
// (multi-blob).  WIN: some output columns are outside the written window.
struct PreviewRowsGeom {
  FastDiv per_frame;  // out_h * groups per row
  FastDiv per_row;    // groups per row (out_w / pixels per unit)
  uint32_t total;
  uint32_t step_f, step_r, step_q;  // the grid's lane count T as (frames, rows, groups)
};
constexpr int kRowsQ = 1;  // units per lane and round (8 output pixels: 2 spill at 64 VGPRs)
// (m & a) | (~m & b): one v_bfi_b32 (in asm: LLVM turns the expression back
// into two ANDs and an OR)
__device__ __forceinline__ uint32_t bfi32(uint32_t m, uint32_t a, uint32_t b) {
  uint32_t r;
  asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(r) : "s"(m), "v"(a), "v"(b));
  return r;
}
constexpr uint32_t rgb565x(uint32_t rgb) {  // write_px565's value
  return ((rgb >> 19) & 0x001fu) | ((rgb >> 5) & 0x07e0u) | ((rgb << 8) & 0xf800u);
}
template <int LAYOUT, bool WIN, bool HUEFREE, bool OVL = false, bool GUIDES = false, bool META = false>
__global__ __launch_bounds__(1024) __attribute__((amdgpu_waves_per_eu(8)))
void preview_rows2_kernel(PreviewArgs a, PreviewRowsGeom g) {
  using namespace stripe_px;
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
  constexpr bool YUYV = LAYOUT == TRIK_HSV_LAYOUT_YUYV;
  constexpr int PX = 8;  // output pixels per unit
  // (META: the multi-blob preview's metapixel flags as the detection, a
  // template argument so that no other form computes their addresses)
  if (!META) {
    const u32x4* src = reinterpret_cast<const u32x4*>(a.tables);
    typedef __attribute__((address_space(3))) u32x4* lds_u128_wptr;
    lds_u128_wptr dst = (lds_u128_wptr)(uintptr_t)0;
    for (int i = threadIdx.x; i < (int)(sizeof(StripeTables) / 16); i += blockDim.x) dst[i] = src[i];
    __syncthreads();
  }
  const int t = threadIdx.x;
  const uint32_t hue_lane = (uint32_t)offsetof(StripeTables, hue) + ((t % kHueCopies) << 2);
  const uint32_t m43_lane = (uint32_t)offsetof(StripeTables, m43) + ((t % kM43Copies) << 2);
  const uint32_t gpr = g.per_row.d, out_h = (uint32_t)a.out_h, nf = (uint32_t)a.n_frames;
  const int64_t plane = (int64_t)a.height * a.line_length;
  // this lane's first unit
  const uint32_t i0 = blockIdx.x * blockDim.x + (uint32_t)t;
  uint32_t f = fdiv(i0, g.per_frame);
  const uint32_t rem = i0 - f * g.per_frame.d;
  uint32_t r = fdiv(rem, g.per_row);
  uint32_t q = rem - r * gpr;
  auto advance = [&]() {  // (f, r, q) += (step_f, step_r, step_q) with carries
    q += g.step_q;
    const bool cq = q >= gpr;
    q = cq ? q - gpr : q;
    r += g.step_r + (cq ? 1u : 0u);
    const bool cr = r >= out_h;
    r = cr ? r - out_h : r;
    f += g.step_f + (cr ? 1u : 0u);
  };
  while (f < nf) {
    uint32_t ff[kRowsQ], rr[kRowsQ], qq[kRowsQ], tpts[kRowsQ], tsx[kRowsQ], gbits[kRowsQ];
    u32x4 w[kRowsQ], wc[kRowsQ];
#pragma unroll
    for (int u = 0; u < kRowsQ; ++u) {
      ff[u] = f;
      rr[u] = r;
      qq[u] = q;
      const uint32_t fl = f < nf ? f : 0u;  // past the end: re-read frame 0, not stored
      if (OVL) {  // the low words of points and sumX, loaded with the frame's
        const uint32_t* ts = reinterpret_cast<const uint32_t*>(a.ovl_sums + fl);
        tpts[u] = ts[0];
        tsx[u] = ts[2];
      }
      // (32-bit offsets and one 64-bit multiply-add per address: launch_rows2
      // checks that strides and in-frame offsets fit 32 bits, rows 24)
      const uint8_t* src = a.frames + (uint64_t)fl * (uint32_t)a.frame_stride +
                           (__umul24((uint32_t)a.rows2_first + 2u * r, (uint32_t)a.line_length) + (YUYV ? 32u : 16u) * q);
      if (GUIDES) gbits[u] = a.guide_bits[r * gpr + q];  // (the same bytes for every frame: cached)
      w[u] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(src));
      // YUYV: the unit's second piece; ov7670: its chroma bytes
      wc[u] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(YUYV ? src + 16 : src + plane));
      advance();
    }
#pragma unroll
    for (int u = 0; u < kRowsQ; ++u) {
      uint32_t ws[PX];
      if (YUYV) {
        ws[0] = w[u].x; ws[1] = w[u].y; ws[2] = w[u].z; ws[3] = w[u].w;
        ws[4] = wc[u].x; ws[5] = wc[u].y; ws[6] = wc[u].z; ws[7] = wc[u].w;
      } else {  // the word (-, U, Y1, V) of output pixel 2d + j: luma byte 2j + 1, chroma bytes 2j, 2j + 1
        const uint32_t yy[4] = {w[u].x, w[u].y, w[u].z, w[u].w}, cc[4] = {wc[u].x, wc[u].y, wc[u].z, wc[u].w};
#pragma unroll
        for (int d = 0; d < 4; ++d) {
          ws[(2 * d) % PX] = __builtin_amdgcn_perm(cc[d], yy[d], 0x0401050Cu);
          ws[(2 * d + 1) % PX] = __builtin_amdgcn_perm(cc[d], yy[d], 0x0603070Cu);
        }
      }
      // OVL: red columns [t_lo, t_hi] of this frame's target line (empty
      // unless points > 10), red over [ovl_c_lo, ovl_c_hi] on a band row
      uint32_t t_lo = 1u, t_hi = 0u;
      bool band_row = false;
      if (OVL) {
        const uint32_t n = tpts[u];
        if (n > 10) {  // LSEQ:464-474: drawRgbTargetCenterLine(targetX), columns cx - 1 .. cx + 1
          const int32_t cx = (int32_t)(tsx[u] / n), wm = a.width - 1;
          const int32_t c0 = cx - 1 < 0 ? 0 : (cx - 1 > wm ? wm : cx - 1);
          const int32_t c1 = cx + 1 < 0 ? 0 : (cx + 1 > wm ? wm : cx + 1);
          // ovl_half: wi2wo[c] = c / 2 (the 2:1 maps), no dependent map loads
          t_lo = a.ovl_half ? (uint32_t)c0 >> 1 : a.wi2wo[c0];
          t_hi = a.ovl_half ? (uint32_t)c1 >> 1 : a.wi2wo[c1];
        }
        band_row = (int32_t)rr[u] == a.ovl_band[0] || (int32_t)rr[u] == a.ovl_band[1];
      }
      uint32_t v[PX];
#pragma unroll
      for (int k = 0; k < PX; ++k) {
        const Phase1 p = phase1<1>(ws[k], ws[k] ^ 0xFF00FF00u, m43_lane);  // the odd pixel: Y in byte 2
        const uint32_t c = PX * qq[u] + (uint32_t)k;                        // its output column
        uint32_t det;
        if (META) {
          const int64_t sr = (int64_t)a.rows2_first + 2 * (int64_t)rr[u];
          const int64_t sc = 2 * (int64_t)c + 1;
          det = a.meta[((int64_t)(ff[u] < nf ? ff[u] : 0u) * (a.height >> 2) + (sr >> 2)) * (a.width >> 2) +
                       (sc >> 2)];
        } else if (HUEFREE) {
          det = lds_u8(p.sv_addr) & 1u;
        } else {
          const uint32_t m = lds_u32(p.m43_addr), sv = lds_u8(p.sv_addr);
          det = lds_u32(phase2_addr(m, p, hue_lane)) & sv & 1u;  // range 0 (combine keeps bit 0 in place)
        }
        // RGB565X of det ? 0x00ffff : rgb888 (WSEQ:316-354): R >> 3 | (G >> 2) << 5 | (B >> 3) << 11
        // (as two bitfield inserts: g << 3 keeps g's bits 2-7 in bits 5-10, b << 8
        // its bits 3-7 in bits 11-15; r >> 3 has nothing above bit 4)
        const uint32_t c565 = bfi32(0xF800u, (uint32_t)p.b << 8, bfi32(0x07E0u, (uint32_t)p.g << 3, (uint32_t)p.r >> 3));
        v[k] = det ? 0xFFE0u : c565;
        if (WIN) v[k] = c >= (uint32_t)a.rows2_c0 && c < (uint32_t)a.rows2_c1 ? v[k] : 0u;
        if (OVL) {  // thin lines (magenta) first, then the band and target lines (red) over them
          const bool mag = (int32_t)c == a.ovl_mag[0] || (int32_t)c == a.ovl_mag[1] ||
                           (int32_t)c == a.ovl_mag[2] || (int32_t)c == a.ovl_mag[3];
          const bool red = (band_row && (int32_t)c >= a.ovl_c_lo && (int32_t)c <= a.ovl_c_hi) ||
                           (c >= t_lo && c <= t_hi);
          v[k] = red ? rgb565x(0xff0000u) : (mag ? rgb565x(0xff00ffu) : v[k]);
        }
      }
      if (GUIDES && gbits[u]) {  // the guide lines' pixels of this unit (draw_guides' colour)
#pragma unroll
        for (int k = 0; k < PX; ++k) v[k] = (gbits[u] >> k) & 1u ? rgb565x(0xff00ffu) : v[k];
      }
      if (ff[u] < nf) {
        uint8_t* dst = a.previews + (uint64_t)ff[u] * (uint32_t)a.preview_stride +
                       (__umul24(rr[u], (uint32_t)a.out_ll) + 2u * PX * qq[u]);
        // nontemporal stores: the preview is written once and not read back
        // here (630 MB per 4096 VGA frames; plain stores left back-to-back
        // batches waiting on the write-backs: 0.51 -> 0.45-0.47 ms,
        // scripts/ab/r05zc_preview_nt.py)
#pragma unroll
        for (int h = 0; h < PX / 4; ++h) {
          u32x2 o;
          o.x = v[4 * h] | (v[4 * h + 1] << 16);
          o.y = v[4 * h + 2] | (v[4 * h + 3] << 16);
          __builtin_nontemporal_store(o, reinterpret_cast<u32x2*>(dst + 8 * h));
        }
      }
    }
  }
}

// One wave per frame.  All guide-line pixels have one colour and all circle
// pixels another, so within each phase the write order is immaterial; only
// "lines before circle" (WSEQ:476-494) is kept, by the barrier.
template <bool LDSMAP>
__global__ __launch_bounds__(64) void overlay_kernel(PreviewArgs a, const TrikHsvTargetSums* sums,
                                                     int sums_pitch) {
  extern __shared__ uint32_t smaps[];
  const int f = blockIdx.x, lane = threadIdx.x;
  const Canvas cv = stage_canvas<LDSMAP>(smaps, a.previews + (int64_t)f * a.preview_stride, a.out_ll, a.width,
                                         a.height, a.wi2wo, a.hi2ho, lane);
  if (!a.guides_drawn) draw_guides(cv, lane, 64);  // WSEQ:471-485 (else the 2:1 kernel drew them)
  __syncthreads();
  const TrikHsvTargetSums s = sums[(int64_t)f * sums_pitch];
  const uint32_t n = (uint32_t)s.points;
  if (n == 0 || lane >= 8) return;
  // WSEQ:486-490 (as targets_kernel): unsigned division, IEEE fp32 radius
  const int32_t cx = (int32_t)((uint32_t)(int32_t)s.sum_x / n);
  const int32_t cy = (int32_t)((uint32_t)(int32_t)s.sum_y / n);
  const int32_t radius = (int32_t)(uint32_t)ceilf(__fsqrt_rn(__fdiv_rn((float)n, 3.1415927f)));
  // drawOutputCircle, WSEQ:91-134 (midpoint circle), colour 0xffff00; lane
  // o draws octant o of every step (and one of the four axis points)
  const uint32_t rgb = 0xffff00;
  const int sx = (lane & 1) ? -1 : 1, sy = (lane & 2) ? -1 : 1;
  const bool swap = (lane & 4) != 0;
  if (lane < 4) {
    const int32_t ax[4] = {0, 0, radius, -radius}, ay[4] = {radius, -radius, 0, 0};
    cv.px(cx + ax[lane], cy + ay[lane], rgb);
  }
  int32_t err = 1 - radius, err_y = 1, err_x = -2 * radius, x = radius, y = 0;
  while (y < x) {
    if (err >= 0) {
      x -= 1;
      err_x += 2;
      err += err_x;
    }
    y += 1;
    err_y += 2;
    err += err_y;
    cv.px(cx + sx * (swap ? y : x), cy + sy * (swap ? x : y), rgb);
  }
}

constexpr int kRangeBlock = 256;
constexpr int kRangeWideFrames = 32;  // batches up to this size: 1024 lanes per frame

// H, S, V bytes of one pixel (WSEQ:207-249), branch-free as the hot kernel's
// phase1 (clamp8_shift6 on v_dot4 presums, the hue case as selects), with
// LUT43 / LUT255 in LDS.
__device__ __forceinline__ void hsv_bytes(const uint8_t* fr, const AutoRangeArgs& a, int row, int col,
                                          const uint16_t* l43, const uint16_t* l255, uint32_t (&hsv)[3]) {
  using stripe_px::clamp8_shift6;
  uint32_t w;  // the pixel as a YUYV word with its Y in byte 0
  if (a.layout == TRIK_HSV_LAYOUT_YUYV && a.aligned4) {
    w = *reinterpret_cast<const uint32_t*>(fr + (int64_t)row * a.line_length + 4 * (col >> 1));
    if (col & 1) w = __builtin_amdgcn_perm(w, w, 0x03020102u);
  } else {
    int Y, U, V;
    fetch_yuv(fr, a.height, a.line_length, a.layout, row, col, Y, U, V);
    w = (uint32_t)Y | ((uint32_t)U << 8) | ((uint32_t)V << 24);
  }
  const uint32_t wc = w ^ 0xFF00FF00u;
  const int r = clamp8_shift6(__builtin_amdgcn_udot4(w, 74u | (102u << 24), (uint32_t)-14248, false));
  const int g = clamp8_shift6(__builtin_amdgcn_udot4(wc, 74u | (25u << 8) | (52u << 24), (uint32_t)-10939, false));
  const int b = clamp8_shift6(__builtin_amdgcn_udot4(w, 74u | (129u << 8), (uint32_t)-17672, false));
  const int mx = max(r, max(g, b)), mn = min(r, min(g, b));
  const bool eqG = mx == g, eqB = mx == b;  // priority G > B > R (WSEQ:226-246)
  const int diff = eqG ? b - r : (eqB ? r - g : g - b);
  const int base = eqG ? 21845 : (eqB ? 43690 : 0);
  const int h = base + (int)l43[mx - mn] * diff;
  hsv[0] = ((uint32_t)h >> 8) & 0xFFu;
  hsv[1] = ((uint32_t)l255[mx] * (uint32_t)(mx - mn)) >> 8;
  hsv[2] = (uint32_t)mx;
}

// One H (or S, V) value per lane into the histograms, for a wave whose active
// lanes are a prefix and hold consecutive zone pixels (the zone walk): equal
// values of neighbouring lanes -- runs, the common case on camera frames --
// take one atomic by the run's first lane (count = the run's length, last
// position = its last lane's, the latest in scan order).  A run head is a
// lane whose left neighbour (DPP wave_shr:1) holds another value.
template <bool kLast>
__device__ __forceinline__ void bin_add_runs(uint32_t* cnt, uint32_t* lst, uint32_t v, uint32_t pos) {
  const uint32_t lane = __lane_id();
  const uint32_t left = (uint32_t)__builtin_amdgcn_update_dpp((int)0xFFFFFFFFu, (int)v, 0x138, 0xF, 0xF, false);
  const bool head = lane == 0 || v != left;
  const unsigned long long heads = __ballot(head);
  const unsigned long long active = __ballot(true);  // a prefix of the wave
  const unsigned long long above = lane == 63 ? 0ull : heads & (~0ull << (lane + 1));
  const uint32_t end = above ? (uint32_t)__ffsll((long long)above) - 1u : (uint32_t)__popcll(active);
  uint32_t p_last = 0;
  if (kLast) p_last = (uint32_t)__shfl((int)pos, (int)(head ? end - 1u : lane), 64);
  if (head) {
    atomicAdd(&cnt[v], end - lane);
    if (kLast) atomicMax(&lst[v], p_last);
  }
}

// One pass over the zone: per-wave count histograms (same-bin LDS atomics
// contend only within a wave) and one last-position histogram per workgroup
// (atomicMax by run heads; the waves seldom meet on a bin); the winner is,
// among the values with the maximum count M, the one with the earliest last
// occurrence (see the file comment).  (Round 2 had a second pass over the
// zone recording last positions for the count-M values only, and per-wave
// last-position sets: with the run-aggregated atomics one pass is 37 % faster
// on scenes, 7 % on uniform bytes.)
template <int kBlock>
__global__ __launch_bounds__(kBlock) void auto_range_kernel(AutoRangeArgs a) {
  constexpr int kWaves = kBlock / 64;
  constexpr int kLastSets = 1;
  __shared__ uint32_t cnt[kWaves][3][256];
  __shared__ uint32_t lst[kLastSets][3][256];
  __shared__ uint32_t best_n[3];
  __shared__ uint64_t best[3];
  __shared__ uint16_t l43[256], l255[256];
  const int f = blockIdx.x, tid = threadIdx.x, wave = tid >> 6;
  for (int i = tid; i < kWaves * 3 * 256; i += blockDim.x) (&cnt[0][0][0])[i] = 0;
  for (int i = tid; i < kLastSets * 3 * 256; i += blockDim.x) (&lst[0][0][0])[i] = 0;
  for (int i = tid; i < 256; i += blockDim.x) {
    l43[i] = c_luts.l43[i];
    l255[i] = c_luts.l255[i];
  }
  if (tid < 3) {
    best_n[tid] = 0;
    best[tid] = ~0ull;
  }
  __syncthreads();
  // zone: c_lo < col < c_hi, r_lo < row < r_hi (uint16 bounds, hpp:88-108)
  const int c0 = max(a.c_lo + 1, 0), c1 = min(a.c_hi, a.width);  // [c0, c1)
  const int r0 = max(a.r_lo + 1, 0), r1 = min(a.r_hi, a.height);
  const int zw = c1 - c0, zh = r1 - r0;
  const int64_t zn = zw > 0 && zh > 0 ? (int64_t)zw * zh : 0;
  const uint8_t* fr = a.frames + (int64_t)f * a.frame_stride;
  // the zone in scan order, thread tid taking pixels tid, tid + block, ...:
  // (row, col) advanced incrementally (no division per pixel)
  auto zone = [&](auto fn) {
    if (zn <= 0) return;
    const uint32_t zwu = (uint32_t)zw, sq = (uint32_t)kBlock / zwu, sr = (uint32_t)kBlock % zwu;
    uint32_t zr = (uint32_t)tid / zwu, zc = (uint32_t)tid % zwu;
    for (uint32_t i = (uint32_t)tid; i < (uint32_t)zn; i += kBlock) {
      fn(r0 + (int)zr, c0 + (int)zc);
      zc += sr;
      zr += sq;
      if (zc >= zwu) { zc -= zwu; ++zr; }
    }
  };
  zone([&](int row, int col) {
    uint32_t hv[3];
    hsv_bytes(fr, a, row, col, l43, l255, hv);
    const uint32_t pos = (uint32_t)((int64_t)row * a.width + col);  // scan order of s_rgb888hsv
#pragma unroll
    for (int k = 0; k < 3; ++k) bin_add_runs<true>(cnt[wave][k], lst[0][k], hv[k], pos);
  });
  __syncthreads();
  // merge the waves: counts add, last positions take the maximum
  for (int i = tid; i < 3 * 256; i += blockDim.x) {
    uint32_t n = 0, l = 0;
#pragma unroll
    for (int w = 0; w < kWaves; ++w) n += (&cnt[w][0][0])[i];
#pragma unroll
    for (int w = 0; w < kLastSets; ++w) l = max(l, (&lst[w][0][0])[i]);
    (&cnt[0][0][0])[i] = n;
    (&lst[0][0][0])[i] = l;
    if (n) atomicMax(&best_n[i >> 8], n);
  }
  __syncthreads();
  for (int i = tid; i < 3 * 256; i += blockDim.x) {
    const int k = i >> 8, v = i & 255;
    const uint32_t n = cnt[0][k][v];
    if (n && n == best_n[k])
      atomicMin(reinterpret_cast<unsigned long long*>(&best[k]), ((unsigned long long)lst[0][k][v] << 8) | (unsigned)v);
  }
  __syncthreads();
  if (tid == 0) {
    uint32_t win[3];
    for (int k = 0; k < 3; ++k) win[k] = best[k] != ~0ull ? (uint32_t)(best[k] & 0xFFu) : 0u;  // none: m_max* = 0
    uint16_t* o = a.out + (int64_t)f * 6;  // hpp:190-195: float constants promoted to double
    o[0] = (uint16_t)((double)win[0] * (double)1.4f);
    o[1] = 15;
    o[2] = (uint16_t)((double)win[1] * (double)0.39f);
    o[3] = 30;
    o[4] = (uint16_t)((double)win[2] * (double)0.39f);
    o[5] = 30;
  }
}

// autoDetectHsv on 16-byte aligned batches (frames, frame stride and line
// length): the same result as auto_range_kernel, organised for throughput.
//  * The zone is cut into 16-byte chunks of its rows (YUYV: 4 words = 8
//    pixels; ov7670: 16 luma + 16 chroma bytes = 16 pixels); a lane takes
//    chunks tid, tid + 256, ... in batches of kVecBatch with every load of a
//    batch in flight (the one-pixel-per-lane walk waited one load latency per
//    pixel).
//  * Pass 1 counts only: a lane run-length encodes each of H, S, V of its
//    pixels in scan order and adds each run once to its wave's LDS
//    histogram of that channel (one atomic per run, not per pixel); the two
//    pixels of a word share one packed HSV computation (hsv_pair).
//  * The winner of a channel whose maximum count M is held by one value is
//    that value.  Only channels where several values reach M need their last
//    occurrences (see the file comment): pass 2 recomputes the zone's HSV and
//    takes atomicMax of the scan position for pixels of those values alone.
constexpr int kVecBatch = 4;
struct AutoVecGeom {
  int32_t r0, c0, c1;  // zone rows [r0, r0 + rows), pixel columns [c0, c1)
  int32_t k0;          // first chunk column
  FastDiv per_row;     // chunks per zone row
  uint32_t total;      // zone rows * chunks per row
  int32_t lo_f, hi_l;  // a row's first chunk: pixels p < lo_f lie left of the zone; its last: p >= hi_l right of it
};

// Two pixels in the 16-bit halves of one register (packed VOP3P arithmetic;
// plain vector types and builtins, so the compiler schedules the packed ops
// and inserts their wait states -- an inline-asm form computed wrong S values
// under another schedule, scripts/ab/r06u_hsv3.py)
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
typedef short i16x2 __attribute__((ext_vector_type(2)));

// One of R, G, B for both pixels of a word: Y holds Y0 and Y1 in its halves,
// c the channel's chroma term (its low 16 bits, used for both).  (74 Y + c)
// mod 2^16 is the reference's 16-bit _add2 sum (the B channel's wrap
// included), then >> 6 with the sign of bit 15 and the clamp to [0, 255]
// (WSEQ:181-205; clamp8_shift6 per pixel).
__device__ __forceinline__ i16x2 pk_chan(u16x2 Y, uint32_t c) {
  const u16x2 cc = {(unsigned short)c, (unsigned short)c};
  const u16x2 x = Y * (u16x2){74, 74} + cc;
  const i16x2 s = __builtin_bit_cast(i16x2, x) >> (i16x2){6, 6};
  return __builtin_elementwise_min(__builtin_elementwise_max(s, (i16x2){0, 0}), (i16x2){255, 255});
}

// H, S, V of both pixels of the YUYV-ordered word w (Y0 U Y1 V), one value
// per channel: WSEQ:207-249 for two pixels at once.  R, G, B, their max, min and the
// three hue differences in packed halves; the hue case selects, LUT43 /
// LUT255 reads and products per pixel.  ~54 VALU per word and no branches,
// against 66 and two divergent branches per pixel for hsv_bytes' form.
__device__ __forceinline__ void hsv_pair(uint32_t w, const uint16_t* l43, const uint16_t* l255, uint32_t (&p0)[3],
                                         uint32_t (&p1)[3]) {
  const uint32_t wc = w ^ 0xFF00FF00u;
  // the chroma terms (Y weight 0); their low 16 bits are the wrapped sums' offsets
  const uint32_t cr = __builtin_amdgcn_udot4(w, 102u << 24, (uint32_t)-14248, false);
  const uint32_t cg = __builtin_amdgcn_udot4(wc, (25u << 8) | (52u << 24), (uint32_t)-10939, false);
  const uint32_t cb = __builtin_amdgcn_udot4(w, 129u << 8, (uint32_t)-17672, false);
  const u16x2 Y = __builtin_bit_cast(u16x2, w & 0x00FF00FFu);
  const i16x2 R = pk_chan(Y, cr), G = pk_chan(Y, cg), B = pk_chan(Y, cb);
  const i16x2 MX = __builtin_elementwise_max(__builtin_elementwise_max(R, G), B);
  const i16x2 MN = __builtin_elementwise_min(__builtin_elementwise_min(R, G), B);
  const i16x2 D = MX - MN, dBR = B - R, dRG = R - G, dGB = G - B;
  // priority G > B > R (WSEQ:226-246)
  const bool eg0 = MX.x == G.x, eb0 = MX.x == B.x, eg1 = MX.y == G.y, eb1 = MX.y == B.y;
  const i16x2 df0 = eg0 ? dBR : (eb0 ? dRG : dGB), df1 = eg1 ? dBR : (eb1 ? dRG : dGB);
  const int b0 = eg0 ? 21845 : (eb0 ? 43690 : 0), b1 = eg1 ? 21845 : (eb1 ? 43690 : 0);
  const uint32_t d0 = (uint16_t)D.x, d1 = (uint16_t)D.y, m0 = (uint16_t)MX.x, m1 = (uint16_t)MX.y;
  const int h0 = b0 + (int)l43[d0] * (int)df0.x, h1 = b1 + (int)l43[d1] * (int)df1.y;
  p0[0] = ((uint32_t)h0 >> 8) & 0xFFu;
  p1[0] = ((uint32_t)h1 >> 8) & 0xFFu;
  p0[1] = ((uint32_t)l255[m0] * d0) >> 8;  // (< 256)
  p1[1] = ((uint32_t)l255[m1] * d1) >> 8;
  p0[2] = m0;
  p1[2] = m1;
}

template <int LAYOUT>
__global__ __launch_bounds__(kRangeBlock) void auto_range_vec_kernel(AutoRangeArgs a, AutoVecGeom g) {
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  constexpr int kWaves = kRangeBlock / 64;
  constexpr bool YUYV = LAYOUT == TRIK_HSV_LAYOUT_YUYV;
  constexpr int NW = YUYV ? 4 : 8;  // words (pixel pairs) per chunk
  __shared__ uint32_t cnt[kWaves][3][256];
  __shared__ uint32_t lst[3][256];
  __shared__ uint32_t top_n[3], n_top[3];
  __shared__ unsigned long long best[3];
  __shared__ uint16_t l43[256], l255[256];
  const int f = blockIdx.x, tid = threadIdx.x, wave = tid >> 6;
  for (int i = tid; i < kWaves * 3 * 256; i += kRangeBlock) (&cnt[0][0][0])[i] = 0;
  for (int i = tid; i < 3 * 256; i += kRangeBlock) (&lst[0][0])[i] = 0;
  for (int i = tid; i < 256; i += kRangeBlock) {
    l43[i] = c_luts.l43[i];
    l255[i] = c_luts.l255[i];
  }
  if (tid < 3) {
    top_n[tid] = 0;
    n_top[tid] = 0;
    best[tid] = ~0ull;
  }
  __syncthreads();
  const uint8_t* fr = a.frames + (int64_t)f * a.frame_stride;
  const int64_t plane = (int64_t)a.height * a.line_length;
  // one batch of chunks: their words (a chunk past the zone re-reads the
  // lane's first chunk and is masked), rows and first pixel columns
  auto load_batch = [&](uint32_t j0, uint32_t (&w)[kVecBatch][NW], int (&row)[kVecBatch], int (&x0)[kVecBatch],
                        bool (&ok)[kVecBatch]) {
#pragma unroll
    for (int b = 0; b < kVecBatch; ++b) {
      const uint32_t j = j0 + (uint32_t)(b * kRangeBlock);
      ok[b] = j < g.total;
      const uint32_t jj = ok[b] ? j : (uint32_t)tid;
      const uint32_t zr = fdiv(jj, g.per_row);
      const uint32_t kc = (uint32_t)g.k0 + (jj - zr * g.per_row.d);
      row[b] = g.r0 + (int)zr;
      x0[b] = (int)kc * 2 * NW;
      const uint8_t* p = fr + (int64_t)row[b] * a.line_length + 16 * (int64_t)kc;
      const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
      if (YUYV) {
        w[b][0] = v.x; w[b][1] = v.y; w[b][2] = v.z; w[b][3] = v.w;
      } else {  // 16 luma bytes, 16 chroma bytes: words (Y0, U = odd chroma, Y1, V = even chroma)
        const u32x4 c = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p + plane));
        const uint32_t yy[4] = {v.x, v.y, v.z, v.w}, cc[4] = {c.x, c.y, c.z, c.w};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          w[b][2 * k] = __builtin_amdgcn_perm(cc[k], yy[k], 0x04010500u);
          w[b][2 * k + 1] = __builtin_amdgcn_perm(cc[k], yy[k], 0x06030702u);
        }
      }
    }
  };
  // the zone's pixels of this lane, in scan order, through fn(key, pos)
  auto walk = [&](auto fn) {
    for (uint32_t j0 = (uint32_t)tid; j0 < g.total; j0 += kVecBatch * kRangeBlock) {
      uint32_t w[kVecBatch][NW];
      int row[kVecBatch], x0[kVecBatch];
      bool ok[kVecBatch];
      load_batch(j0, w, row, x0, ok);
#pragma unroll
      for (int b = 0; b < kVecBatch; ++b) {
        // a batch slot past the zone for the whole wave: no HSV to compute
        // (the last batch of a VGA frame's 3,180 chunks fills 108 of its
        // 1,024 slots)
        if (__builtin_amdgcn_ballot_w64(ok[b]) == 0ull) continue;
#pragma unroll
        for (int i = 0; i < NW; ++i) {
          const int c = x0[b] + 2 * i;
          const uint32_t pos = (uint32_t)row[b] * (uint32_t)a.width + (uint32_t)c;
          uint32_t h0[3], h1[3];
          hsv_pair(w[b][i], l43, l255, h0, h1);
          if (ok[b] && c >= g.c0 && c < g.c1) fn(h0, pos);
          if (ok[b] && c + 1 >= g.c0 && c + 1 < g.c1) fn(h1, pos + 1u);
        }
      }
    }
  };
  // pass 1: run-length encoded counts per channel
  // (each channel on its own: a triple's run breaks whenever any channel
  // changes -- on scene gradients nearly every pixel, on uniform bytes every
  // one; per channel, uniform frames -32 %, scripts/ab/r06q_hsv2.py).  Every
  // pixel of a chunk is counted; the few outside the zone's columns (a row's
  // first chunk p < lo_f, its last p >= hi_l: kernel-wide constants) are
  // subtracted again, so no pixel carries a column test (-7 %,
  // scripts/ab/r06ab_range_attr.py).  A run's length is added when the next
  // run starts (the first add of each channel adds 0 to bin 0).
  uint32_t rk3[3] = {0u, 0u, 0u}, rl3[3] = {0u, 0u, 0u};
  auto count = [&](const uint32_t (&hv)[3]) {
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const uint32_t v = hv[c];
      const bool brk = v != rk3[c];
      if (brk) atomicAdd(&cnt[wave][c][rk3[c]], rl3[c]);
      rl3[c] = brk ? 1u : rl3[c] + 1u;
      rk3[c] = v;
    }
  };
  auto uncount = [&](uint64_t m, const uint32_t (&hv)[3]) {  // lanes of m: this pixel lies outside the zone
    if (m == 0) return;
    if (__builtin_amdgcn_inverse_ballot_w64(m)) {
#pragma unroll
      for (int c = 0; c < 3; ++c) atomicSub(&cnt[wave][c][hv[c]], 1u);
    }
  };
  const uint32_t kc_last = (uint32_t)(g.k0 + (int)g.per_row.d - 1);
  for (uint32_t j0 = (uint32_t)tid; j0 < g.total; j0 += kVecBatch * kRangeBlock) {
    uint32_t w[kVecBatch][NW];
    int row[kVecBatch], x0[kVecBatch];
    bool ok[kVecBatch];
    load_batch(j0, w, row, x0, ok);
#pragma unroll
    for (int b = 0; b < kVecBatch; ++b) {
      const uint64_t okm = __builtin_amdgcn_ballot_w64(ok[b]);
      if (okm == 0ull) continue;
      const uint32_t kc = (uint32_t)x0[b] / (uint32_t)(2 * NW);
      const uint64_t firstm = __builtin_amdgcn_ballot_w64(ok[b] && kc == (uint32_t)g.k0);
      const uint64_t lastm = __builtin_amdgcn_ballot_w64(ok[b] && kc == kc_last);
      if (ok[b]) {
#pragma unroll
        for (int i = 0; i < NW; ++i) {
          uint32_t h0[3], h1[3];
          hsv_pair(w[b][i], l43, l255, h0, h1);
          count(h0);
          count(h1);
          uncount((2 * i < g.lo_f ? firstm : 0ull) | (2 * i >= g.hi_l ? lastm : 0ull), h0);
          uncount((2 * i + 1 < g.lo_f ? firstm : 0ull) | (2 * i + 1 >= g.hi_l ? lastm : 0ull), h1);
        }
      }
    }
  }
#pragma unroll
  for (int c = 0; c < 3; ++c) atomicAdd(&cnt[wave][c][rk3[c]], rl3[c]);
  __syncthreads();
  for (int i = tid; i < 3 * 256; i += kRangeBlock) {
    uint32_t n = 0;
#pragma unroll
    for (int w = 0; w < kWaves; ++w) n += (&cnt[w][0][0])[i];
    (&cnt[0][0][0])[i] = n;
    if (n) atomicMax(&top_n[i >> 8], n);
  }
  __syncthreads();
  for (int i = tid; i < 3 * 256; i += kRangeBlock) {
    const int k = i >> 8;
    const uint32_t n = (&cnt[0][0][0])[i];
    if (n && n == top_n[k]) {
      atomicAdd(&n_top[k], 1u);
      atomicMin(&best[k], (unsigned long long)(i & 255));
    }
  }
  __syncthreads();
  const uint32_t tie = (n_top[0] > 1u ? 1u : 0u) | (n_top[1] > 1u ? 2u : 0u) | (n_top[2] > 1u ? 4u : 0u);
  if (tie) {  // (workgroup-uniform) pass 2: the last occurrences of the tied values
    walk([&](const uint32_t (&hv)[3], uint32_t pos) {
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        const uint32_t v = hv[k];
        if (((tie >> k) & 1u) && cnt[0][k][v] == top_n[k]) atomicMax(&lst[k][v], pos);
      }
    });
    __syncthreads();
    if (tid < 3 && ((tie >> tid) & 1u)) best[tid] = ~0ull;
    __syncthreads();
    for (int i = tid; i < 3 * 256; i += kRangeBlock) {
      const int k = i >> 8, v = i & 255;
      if (((tie >> k) & 1u) && cnt[0][k][v] == top_n[k])
        atomicMin(&best[k], ((unsigned long long)lst[k][v] << 8) | (unsigned)v);
    }
    __syncthreads();
  }
  if (tid == 0) {
    uint32_t win[3];
    for (int k = 0; k < 3; ++k) win[k] = best[k] != ~0ull ? (uint32_t)(best[k] & 0xFFu) : 0u;  // none: m_max* = 0
    uint16_t* o = a.out + (int64_t)f * 6;  // hpp:190-195: float constants promoted to double
    o[0] = (uint16_t)((double)win[0] * (double)1.4f);
    o[1] = 15;
    o[2] = (uint16_t)((double)win[1] * (double)0.39f);
    o[3] = 30;
    o[4] = (uint16_t)((double)win[2] * (double)0.39f);
    o[5] = 30;
  }
}

}  // namespace

// The 2:1 row kernel when the maps, layout and alignment allow (see
// preview_rows2_kernel); hipErrorNotSupported otherwise.
static int launch_rows2(const PreviewArgs& a, hipStream_t s, bool guides = false) {
  const bool yuyv = a.layout == TRIK_HSV_LAYOUT_YUYV;
  const int px = 8;  // output pixels per unit
  if (a.rows2_first < 0 || (!yuyv && a.layout != TRIK_HSV_LAYOUT_OV7670) || a.out_w % px || a.out_ll != 2 * a.out_w ||
      (!a.meta && !a.tables))
    return hipErrorNotSupported;
  // every unit loads source pixels 2c .. 2c + 1 of each of its output columns
  // c < out_w, written or not (WIN masks the unwritten ones after the load):
  // they must lie in the row, or the last row of the last frame reads past
  // the buffer (e.g. a 480-wide frame under a 320-wide preview)
  if (2LL * a.out_w > a.width) return hipErrorNotSupported;
  const auto al = [](int64_t v, int64_t m) { return v % m == 0; };
  if (!al((int64_t)reinterpret_cast<uintptr_t>(a.frames), 16) || !al(a.line_length, 16) ||
      (a.n_frames > 1 && !al(a.frame_stride, 16)) || !al((int64_t)reinterpret_cast<uintptr_t>(a.previews), 8) ||
      (a.n_frames > 1 && !al(a.preview_stride, 8)))
    return hipErrorNotSupported;
  const int64_t gpr = a.out_w / px, total = (int64_t)a.n_frames * a.out_h * gpr;
  if (total >= (1ll << 31)) return hipErrorNotSupported;
  // the kernel's 32-bit strides and in-frame offsets, 24-bit row indices and line lengths
  const int64_t frame_bytes = (int64_t)a.height * a.line_length * (yuyv ? 1 : 2);
  if (a.frame_stride >= (1ll << 32) || a.preview_stride >= (1ll << 32) || frame_bytes >= (1ll << 32) ||
      (int64_t)a.out_h * a.out_ll >= (1ll << 32) || a.line_length >= (1 << 24) || a.out_ll >= (1 << 24) ||
      a.height >= (1 << 24))
    return hipErrorNotSupported;
  if (total == 0) return hipSuccess;
  const bool win = a.rows2_c0 > 0 || a.rows2_c1 < a.out_w, hue_free = a.hue_free && !a.meta;
  const bool ovl = a.ovl_sums != nullptr;
  if (ovl && (!a.ovl_ok || !hue_free)) return hipErrorNotSupported;  // the line sensors' previews only
  using Kern = void (*)(PreviewArgs, PreviewRowsGeom);
  static const Kern ovl_kerns[2][2] = {
      {preview_rows2_kernel<TRIK_HSV_LAYOUT_YUYV, false, true, true>,
       preview_rows2_kernel<TRIK_HSV_LAYOUT_YUYV, true, true, true>},
      {preview_rows2_kernel<TRIK_HSV_LAYOUT_OV7670, false, true, true>,
       preview_rows2_kernel<TRIK_HSV_LAYOUT_OV7670, true, true, true>}};
  static const Kern kerns[2][2][2] = {
      {{preview_rows2_kernel<TRIK_HSV_LAYOUT_YUYV, false, false>, preview_rows2_kernel<TRIK_HSV_LAYOUT_YUYV, false, true>},
       {preview_rows2_kernel<TRIK_HSV_LAYOUT_YUYV, true, false>, preview_rows2_kernel<TRIK_HSV_LAYOUT_YUYV, true, true>}},
      {{preview_rows2_kernel<TRIK_HSV_LAYOUT_OV7670, false, false>,
        preview_rows2_kernel<TRIK_HSV_LAYOUT_OV7670, false, true>},
       {preview_rows2_kernel<TRIK_HSV_LAYOUT_OV7670, true, false>,
        preview_rows2_kernel<TRIK_HSV_LAYOUT_OV7670, true, true>}}};
  // the object sensors' preview with its guide lines drawn in the same pass
  static const Kern guide_kerns[2][2][2] = {
      {{preview_rows2_kernel<TRIK_HSV_LAYOUT_YUYV, false, false, false, true>,
        preview_rows2_kernel<TRIK_HSV_LAYOUT_YUYV, false, true, false, true>},
       {preview_rows2_kernel<TRIK_HSV_LAYOUT_YUYV, true, false, false, true>,
        preview_rows2_kernel<TRIK_HSV_LAYOUT_YUYV, true, true, false, true>}},
      {{preview_rows2_kernel<TRIK_HSV_LAYOUT_OV7670, false, false, false, true>,
        preview_rows2_kernel<TRIK_HSV_LAYOUT_OV7670, false, true, false, true>},
       {preview_rows2_kernel<TRIK_HSV_LAYOUT_OV7670, true, false, false, true>,
        preview_rows2_kernel<TRIK_HSV_LAYOUT_OV7670, true, true, false, true>}}};
  if (guides && (ovl || a.meta || !a.guide_bits)) return hipErrorInvalidValue;
  // the multi-blob preview (metapixel flags)
  static const Kern meta_kerns[2][2] = {
      {preview_rows2_kernel<TRIK_HSV_LAYOUT_YUYV, false, false, false, false, true>,
       preview_rows2_kernel<TRIK_HSV_LAYOUT_YUYV, true, false, false, false, true>},
      {preview_rows2_kernel<TRIK_HSV_LAYOUT_OV7670, false, false, false, false, true>,
       preview_rows2_kernel<TRIK_HSV_LAYOUT_OV7670, true, false, false, false, true>}};
  const Kern kern = ovl      ? ovl_kerns[yuyv ? 0 : 1][win ? 1 : 0]
                    : a.meta ? meta_kerns[yuyv ? 0 : 1][win ? 1 : 0]
                    : guides ? guide_kerns[yuyv ? 0 : 1][win ? 1 : 0][hue_free ? 1 : 0]
                             : kerns[yuyv ? 0 : 1][win ? 1 : 0][hue_free ? 1 : 0];
  hipError_t e = set_dynamic_lds(reinterpret_cast<const void*>(kern), 80 * 1024);
  if (e != hipSuccess) return e;
  PreviewRowsGeom g;
  g.per_frame = make_div((uint32_t)(a.out_h * gpr));
  g.per_row = make_div((uint32_t)gpr);
  g.total = (uint32_t)total;
  const int64_t blocks = (total + 1024LL * kRowsQ - 1) / (1024LL * kRowsQ), slots = 2LL * device_cus();
  const int64_t grid = blocks < slots ? blocks : slots;
  {  // the grid's lane count as (frames, rows, groups): the kernel's per-unit step
    const int64_t T = grid * 1024, pf = (int64_t)a.out_h * gpr;
    g.step_f = (uint32_t)(T / pf);
    g.step_r = (uint32_t)((T % pf) / gpr);
    g.step_q = (uint32_t)(T % gpr);
  }
  const size_t lds = a.meta ? 0 : sizeof(StripeTables);
  hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(1024), lds, s, a, g);
  return hipGetLastError();
}

static int launch_gather(const PreviewArgs& a, hipStream_t s) {
  {  // the 2:1 row kernel where it applies
    const int e = launch_rows2(a, s);
    if (e != hipErrorNotSupported) return e;
  }
  const int64_t qpr = (a.out_ll + 3) / 4, total = (int64_t)a.n_frames * a.out_h * qpr;
  if (total >= (1ll << 31) || (!a.meta && !a.tables)) return hipErrorInvalidValue;
  if (total == 0) return hipSuccess;
  {
    hipError_t e = set_dynamic_lds(reinterpret_cast<const void*>(preview_gather_kernel), 80 * 1024);
    if (e != hipSuccess) return e;
  }
  const int cus = device_cus();
  PreviewGeom g;
  g.per_frame = make_div((uint32_t)(a.out_h * qpr));
  g.per_row = make_div((uint32_t)qpr);
  g.total = (uint32_t)total;
  // the maps in LDS behind the tables when they fit two workgroups per CU and
  // every source coordinate fits u16
  const uint32_t tables_bytes = a.meta ? 16u : (uint32_t)sizeof(StripeTables);
  const int64_t map_bytes = 2LL * (a.out_w + a.out_h);
  g.map_off = a.width < 65535 && a.height < 65535 &&
                      tables_bytes + map_bytes <= 80 * 1024
                  ? tables_bytes
                  : 0u;
  const size_t lds = g.map_off ? (size_t)(tables_bytes + map_bytes) : (a.meta ? 0 : sizeof(StripeTables));
  const int64_t blocks = (total + 1024LL * kPreviewQ - 1) / (1024LL * kPreviewQ), slots = 2LL * cus;
  hipLaunchKernelGGL(preview_gather_kernel, dim3((unsigned)(blocks < slots ? blocks : slots)), dim3(1024),
                     lds, s, a, g);
  return hipGetLastError();
}

int launch_preview_rows2(const PreviewArgs& a, hipStream_t s) {
  if (a.n_frames <= 0 || a.out_w <= 0 || a.out_h <= 0) return hipSuccess;
  return launch_rows2(a, s);
}

int launch_preview_body(const PreviewArgs& a, hipStream_t s) {
  if (a.n_frames <= 0 || a.out_w <= 0 || a.out_h <= 0) return hipSuccess;
  return launch_gather(a, s);
}

int launch_preview(const PreviewArgs& pa, const TrikHsvTargetSums* sums, int sums_pitch, hipStream_t s) {
  if (pa.n_frames <= 0 || pa.out_w <= 0 || pa.out_h <= 0) return hipSuccess;
  PreviewArgs a = pa;
  // the 2:1 row kernel draws the guide lines too where their bits exist
  hipError_t e = hipErrorNotSupported;
  if (a.guide_bits && !a.meta) {
    e = (hipError_t)launch_rows2(a, s, true);
    a.guides_drawn = e == hipSuccess ? 1 : 0;
  }
  if (e == hipErrorNotSupported) e = (hipError_t)launch_gather(a, s);
  if (e != hipSuccess || a.width <= 0 || a.height <= 0) return e;
  const size_t map_bytes = sizeof(uint32_t) * ((size_t)a.width + (size_t)a.height);
  if (map_bytes <= kMapLdsBytes)
    hipLaunchKernelGGL(overlay_kernel<true>, dim3((unsigned)a.n_frames), dim3(64), map_bytes, s, a, sums, sums_pitch);
  else
    hipLaunchKernelGGL(overlay_kernel<false>, dim3((unsigned)a.n_frames), dim3(64), 0, s, a, sums, sums_pitch);
  return hipGetLastError();
}

int launch_auto_range(const AutoRangeArgs& a, hipStream_t s) {
  if (a.n_frames <= 0) return hipSuccess;
  // 16-byte aligned batches: the chunked two-pass kernel
  const bool yuyv = a.layout == TRIK_HSV_LAYOUT_YUYV;
  if ((yuyv || a.layout == TRIK_HSV_LAYOUT_OV7670) && (reinterpret_cast<uintptr_t>(a.frames) % 16) == 0 &&
      (a.n_frames <= 1 || a.frame_stride % 16 == 0) && a.line_length % 16 == 0) {
    const int pxc = yuyv ? 8 : 16;
    AutoVecGeom g;
    g.c0 = a.c_lo + 1 > 0 ? a.c_lo + 1 : 0;
    g.c1 = a.c_hi < a.width ? a.c_hi : a.width;
    g.r0 = a.r_lo + 1 > 0 ? a.r_lo + 1 : 0;
    const int r1 = a.r_hi < a.height ? a.r_hi : a.height;
    const int zw = g.c1 - g.c0, zh = r1 - g.r0;
    int cpr = 0;
    if (zw > 0 && zh > 0) {
      g.k0 = g.c0 / pxc;
      cpr = (g.c1 - 1) / pxc + 1 - g.k0;
    } else {
      g.k0 = 0;
    }
    // (the zone's last chunk must lie in its row)
    if ((int64_t)16 * (g.k0 + cpr) <= a.line_length) {
      g.per_row = make_div((uint32_t)(cpr > 0 ? cpr : 1));
      g.total = (uint32_t)(cpr > 0 ? (int64_t)cpr * zh : 0);
      g.lo_f = g.c0 - g.k0 * pxc;                  // (0 .. pxc - 1)
      g.hi_l = g.c1 - (g.k0 + (cpr > 0 ? cpr : 1) - 1) * pxc;  // (1 .. pxc)
      if (yuyv)
        hipLaunchKernelGGL(auto_range_vec_kernel<TRIK_HSV_LAYOUT_YUYV>, dim3((unsigned)a.n_frames), dim3(kRangeBlock), 0,
                           s, a, g);
      else
        hipLaunchKernelGGL(auto_range_vec_kernel<TRIK_HSV_LAYOUT_OV7670>, dim3((unsigned)a.n_frames),
                           dim3(kRangeBlock), 0, s, a, g);
      return hipGetLastError();
    }
  }
  // one workgroup per frame; a few frames (process() takes one) get 1024
  // lanes each: the pass over the zone is a latency-bound chain per lane, 4x
  // shorter
  if (a.n_frames <= kRangeWideFrames)
    hipLaunchKernelGGL(auto_range_kernel<1024>, dim3((unsigned)a.n_frames), dim3(1024), 0, s, a);
  else
    hipLaunchKernelGGL(auto_range_kernel<kRangeBlock>, dim3((unsigned)a.n_frames), dim3(kRangeBlock), 0, s, a);
  return hipGetLastError();
}

}  // namespace trik_hsv
