// trik_hsv_line.hip -- the ov7670 line sensor, LSEQ =
// trik/ov7670/line_sensor/include/internal/cv_line_detector_seqpass.hpp:
//
//  line_vec_kernel      the fast form: lanes own fixed 8-pixel column units
//                       and walk rows; V = max(R, G, B) computed on packed
//                       16-bit pairs (two pixels per VALU op), per-column
//                       non-detection counters, sums formed once per
//                       workgroup (below).
//  line_sums_kernel     generic form (misaligned input): detection by V only (hue/sat bounds 0..255, LSEQ:
//                       391-396) in columns 5 <= col <= W-5 (LSEQ:288), per
//                       frame {N, sumX, crossPoints}; cross points are the
//                       detections of rows bandStart..bandStop (LSEQ:298-299).
//  line_targets_kernel  OutArgs of LSEQ:455-474 (all 0 unless N > 10).
//  line_overlay_kernel  guide lines (LSEQ:433-436), band lines (LSEQ:442-443)
//                       and the 3-pixel target line (LSEQ:467), one wave per
//                       frame; magenta before red as the reference.
// The preview body is trik_hsv_operator.hip's preview_kernel with the
// window-restricted inverse maps (only window columns are written, LSEQ:288-291).
#include <hip/hip_runtime.h>

#include "trik_hsv_internal.h"
#include "trik_hsv_pixel.h"

namespace trik_hsv {

namespace {

constexpr int kLineBlock = 256;
constexpr int kLineRows = 8;  // rows per workgroup

__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

// ---------------------------------------------------------------------------
// line_vec_kernel.  V = clamp8(max(R', G', B') >> 6) with R' = 74Y + 102V -
// 14248, G' = 74Y - 52V - 25U + 8696, B' = sext16(74Y + 129U - 17672): clamp8
// and >>6 are monotone, so they commute with the max (LSEQ:191-215 computes
// clamp8 of each channel first).  R' and G' lie in int16 range and B' is the
// reference's 16-bit wrap (_add2), so all three are exact in 16-bit lanes.
// The V test lo <= clamp8(m >> 6) <= hi is then mlo <= m <= mhi on int16 m
// (host: mlo = lo ? 64 lo : -32768, mhi = hi < 255 ? 64 hi + 63 : 32767),
// i.e. (u16)(m - mlo) <= (u16)(mhi - mlo) -- a saturating subtract is 0 iff
// detected.  A lane holds 8 pixels as four u16x2 groups whose halves are
// pixels 2 apart (so each half has its own chroma pair, no broadcast):
// group g = 2h + k holds pixels 4h + k and 4h + k + 2 of the unit.
// ---------------------------------------------------------------------------
typedef short s16x2 __attribute__((ext_vector_type(2)));
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));

struct LineGeom {
  int32_t units;      // 8-pixel column units per row (W / 8)
  int32_t cu;         // units one workgroup row covers
  int32_t rpi;        // rows per iteration (lanes = rpi x cu)
  int32_t chunks;     // column chunks per frame
  int32_t segs;       // row segments per frame
  int32_t seg_rows;   // rows per segment (multiple of rpi)
  int16_t mlo;
  uint16_t kspan;     // (u16)(mhi - mlo)
};

__device__ __forceinline__ void line_px8(uint32_t yw, uint32_t cw, int h, u16x2 mlo, u16x2 kspan,
                                         u16x2 (&acc)[4]) {
  // 16-bit lane arithmetic in unsigned vectors (defined wrap); only the max is signed.
  // chroma bytes V0 U0 V1 U1 (ov7670: V even, U odd; OSEQ:369-373)
  const u16x2 V = __builtin_bit_cast(u16x2, __builtin_amdgcn_perm(0u, cw, 0x0c020c00u));
  const u16x2 U = __builtin_bit_cast(u16x2, __builtin_amdgcn_perm(0u, cw, 0x0c030c01u));
  const u16x2 cR = V * (unsigned short)102 + (unsigned short)(65536 - 14248);
  const u16x2 cG = (unsigned short)8696 - V * (unsigned short)52 - U * (unsigned short)25;
  const u16x2 cB = U * (unsigned short)129 + (unsigned short)(65536 - 17672);
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const u16x2 Y =
        __builtin_bit_cast(u16x2, __builtin_amdgcn_perm(0u, yw, k ? 0x0c030c01u : 0x0c020c00u));
    const u16x2 y74 = Y * (unsigned short)74;
    const s16x2 r = __builtin_bit_cast(s16x2, (u16x2)(y74 + cR));
    const s16x2 gg = __builtin_bit_cast(s16x2, (u16x2)(y74 + cG));
    const s16x2 b = __builtin_bit_cast(s16x2, (u16x2)(y74 + cB));
    const u16x2 m = __builtin_bit_cast(u16x2, __builtin_elementwise_max(__builtin_elementwise_max(r, gg), b));
    // nd = min(sat(d - kspan), 1): 0 iff detected, else 1.  In asm: LLVM
    // rewrites this pair into per-half compares + selects (4+ ops instead of 2).
    uint32_t nd;
    asm volatile("v_pk_sub_u16 %0, %1, %2 clamp\n\tv_pk_min_u16 %0, %0, %3"
                 : "=&v"(nd)
                 : "v"(__builtin_bit_cast(uint32_t, (u16x2)(m - mlo))), "v"(__builtin_bit_cast(uint32_t, kspan)),
                   "v"(0x00010001u));
    acc[2 * h + k] += __builtin_bit_cast(u16x2, nd);
  }
}

// rows [r_lo, r_hi) of this lane (rows base + k*rpi): non-detections into acc
__device__ __forceinline__ int line_rows(const uint8_t* yp, int64_t cofs, int64_t step, int base, int rpi,
                                         int r_lo, int r_hi, u16x2 mlo, u16x2 kspan, u16x2 (&acc)[4]) {
  if (r_hi <= r_lo) return 0;
  const int k0 = r_lo > base ? (r_lo - base + rpi - 1) / rpi : 0;
  const int k1 = r_hi > base ? (r_hi - base + rpi - 1) / rpi : 0;
  const uint8_t* p = yp + (int64_t)k0 * step;
  int k = k0;
  for (; k + 4 <= k1; k += 4, p += 4 * step) {
    uint2 y[4], c[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      // streaming loads (nontemporal: 8 % faster than plain, scripts/ab/r05l_line.py)
      typedef unsigned int v2 __attribute__((ext_vector_type(2)));
      const v2 ty = __builtin_nontemporal_load(reinterpret_cast<const v2*>(p + i * step));
      const v2 tc = __builtin_nontemporal_load(reinterpret_cast<const v2*>(p + i * step + cofs));
      y[i] = make_uint2(ty.x, ty.y);
      c[i] = make_uint2(tc.x, tc.y);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      line_px8(y[i].x, c[i].x, 0, mlo, kspan, acc);
      line_px8(y[i].y, c[i].y, 1, mlo, kspan, acc);
    }
  }
  for (; k < k1; ++k, p += step) {
    const uint2 y = *reinterpret_cast<const uint2*>(p);
    const uint2 c = *reinterpret_cast<const uint2*>(p + cofs);
    line_px8(y.x, c.x, 0, mlo, kspan, acc);
    line_px8(y.y, c.y, 1, mlo, kspan, acc);
  }
  return k1 > k0 ? k1 - k0 : 0;
}

__device__ __forceinline__ uint64_t wave_sum_u64(uint64_t v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

__global__ __launch_bounds__(1024) void line_vec_kernel(LineArgs a, LineGeom g) {
  const int wg = blockIdx.x;
  const int s = wg % g.segs;
  const int fc = wg / g.segs;
  const int ch = fc % g.chunks;
  const int f = fc / g.chunks;
  const int tid = threadIdx.x;
  const int r_off = tid / g.cu;
  const int unit = ch * g.cu + (tid - r_off * g.cu);
  uint64_t n = 0, sx = 0, cross = 0;
  if (r_off < g.rpi && unit < g.units) {
    const int row0 = s * g.seg_rows;
    const int row_end = min(a.height, row0 + g.seg_rows);
    // band rows: (uint32)row in [band_start, band_stop] (LSEQ:298), clipped to the segment
    const int64_t bs64 = (int64_t)(uint32_t)a.band_start, be64 = (int64_t)(uint32_t)a.band_stop + 1;
    const int b_lo = (int)max((int64_t)row0, min(bs64, (int64_t)row_end));
    const int b_hi = (int)max((int64_t)b_lo, min(be64, (int64_t)row_end));
    const int base = row0 + r_off;
    const int64_t ll = a.line_length;
    const uint8_t* yp = a.frames + (int64_t)f * a.frame_stride + (int64_t)base * ll + 8 * unit;
    const int64_t cofs = (int64_t)a.height * ll, step = (int64_t)g.rpi * ll;
    const u16x2 mlo = (u16x2)(unsigned short)g.mlo;
    const u16x2 kspan = (u16x2)g.kspan;
    u16x2 acc[4] = {};
    int rows = line_rows(yp, cofs, step, base, g.rpi, row0, b_lo, mlo, kspan, acc);
    u16x2 before[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) before[i] = acc[i];
    const int brows = line_rows(yp, cofs, step, base, g.rpi, b_lo, b_hi, mlo, kspan, acc);
    u16x2 band_nd[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) band_nd[i] = acc[i] - before[i];
    rows += brows + line_rows(yp, cofs, step, base, g.rpi, b_hi, row_end, mlo, kspan, acc);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int col = 8 * unit + 4 * (i >> 1) + (i & 1) + 2 * j;
        if (col >= 5 && col <= a.width - 5) {  // LSEQ:288
          const uint32_t det = (uint32_t)rows - acc[i][j];
          n += det;
          sx += (uint64_t)det * (uint32_t)col;
          cross += (uint32_t)brows - band_nd[i][j];
        }
      }
  }
  n = wave_sum_u64(n);
  sx = wave_sum_u64(sx);
  cross = wave_sum_u64(cross);
  if ((tid & 63) == 0) {
    TrikHsvTargetSums* d = a.sums + f;
    if (n) atomicAdd(reinterpret_cast<unsigned long long*>(&d->points), (unsigned long long)n);
    if (sx) atomicAdd(reinterpret_cast<unsigned long long*>(&d->sum_x), (unsigned long long)sx);
    if (cross) atomicAdd(reinterpret_cast<unsigned long long*>(&d->sum_y), (unsigned long long)cross);
  }
}

__global__ __launch_bounds__(kLineBlock) void line_sums_kernel(LineArgs a) {
  const int groups = (a.height + kLineRows - 1) / kLineRows;
  const int f = blockIdx.x / groups;
  const int r0 = (blockIdx.x - f * groups) * kLineRows;
  const uint8_t* fr = a.frames + (int64_t)f * a.frame_stride;
  const int pairs = a.width / 2;
  uint32_t n = 0, sx = 0, cross = 0;
  for (int i = threadIdx.x; i < kLineRows * pairs; i += blockDim.x) {
    const int row = r0 + i / pairs, q = i % pairs;
    if (row >= a.height) break;
    // ov7670 planes (OSEQ:360-373 / LSEQ:211-234): U = odd chroma byte, V = even
    const uint8_t* yrow = fr + (int64_t)row * a.line_length;
    const uint8_t* crow = fr + (int64_t)a.line_length * a.height + (int64_t)row * a.line_length;
    const int U = crow[2 * q + 1], V = crow[2 * q];
    uint32_t row_n = 0, row_x = 0;
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int col = 2 * q + k;
      const PixelRgb p = pixel_rgb(yrow[col], U, V);
      const uint32_t mx = (uint32_t)max(p.r, max(p.g, p.b));
      const uint32_t det = (col >= 5 && col <= a.width - 5 && mx >= a.val_lo && mx <= a.val_hi) ? 1u : 0u;
      row_n += det;
      row_x += det ? (uint32_t)col : 0u;
    }
    n += row_n;
    sx += row_x;
    if ((uint32_t)row >= (uint32_t)a.band_start && (uint32_t)row <= (uint32_t)a.band_stop) cross += row_n;
  }
  n = wave_sum_u32(n);
  sx = wave_sum_u32(sx);
  cross = wave_sum_u32(cross);
  if ((threadIdx.x & 63) == 0) {
    TrikHsvTargetSums* d = a.sums + f;
    if (n) atomicAdd(reinterpret_cast<unsigned long long*>(&d->points), (unsigned long long)n);
    if (sx) atomicAdd(reinterpret_cast<unsigned long long*>(&d->sum_x), (unsigned long long)sx);
    if (cross) atomicAdd(reinterpret_cast<unsigned long long*>(&d->sum_y), (unsigned long long)cross);
  }
}

// cross = false: the webcam line sensor (LSEQW:401-417: targetY stays 0,
// the sum_y slot holds the plain row sums)
__global__ void line_targets_kernel(int n_frames, int width, int height, const TrikHsvTargetSums* sums,
                                    TrikHsvTarget* targets, int cross = 1) {
  const int f = blockIdx.x * blockDim.x + threadIdx.x;
  if (f >= n_frames) return;
  const TrikHsvTargetSums s = sums[f];
  TrikHsvTarget t = {0, 0, 0, 0};
  const uint32_t n = (uint32_t)s.points;
  if (n > 10) {  // LSEQ:462-474 (crossSize LSEQ:452, step 40)
    const int32_t cx = (int32_t)((uint32_t)(int32_t)s.sum_x / n);
    t.x = (int8_t)(((cx - width / 2) * 100 * 2) / width);
    t.y = cross ? (int8_t)(int)((uint32_t)((uint32_t)s.sum_y * 100u) / (uint32_t)(width * 2 * 40)) : (int8_t)0;
    t.size = (uint8_t)((uint32_t)(n * 100u) / (uint32_t)(height * width));
  }
  targets[f] = t;
}

// band = false: the webcam line sensor (LSEQW:396-399, 405-413): the four
// thin lines and the target line, no band lines
__global__ __launch_bounds__(64) void line_overlay_kernel(PreviewArgs a, const TrikHsvTargetSums* sums,
                                                          int band = 1) {
  const int f = blockIdx.x, lane = threadIdx.x;
  uint8_t* out = a.previews + (int64_t)f * a.preview_stride;
  const int W = a.width, H = a.height, step = 40;
  auto px = [&](int32_t col, int32_t row, uint32_t rgb) {  // drawOutputPixelBound, LSEQ:61-76
    const int32_t sc = col < 0 ? 0 : (col > W - 1 ? W - 1 : col);
    const int32_t sr = row < 0 ? 0 : (row > H - 1 ? H - 1 : row);
    write_px565(out + (int64_t)(int32_t)a.hi2ho[sr] * a.out_ll + (int64_t)(int32_t)a.wi2wo[sc] * 2, rgb);
  };
  const int hw = W / 2, hh = H / 2;
  const int32_t cols[4] = {hw - step, hw + step, hw - 2 * step, hw + 2 * step};
  for (int k = lane; k < 4 * H; k += 64) px(cols[k / H], k % H, 0xff00ff);  // drawRgbThinLine, rows 0..H-1
  __syncthreads();
  if (band)
    for (int k = lane; k < 2 * W; k += 64) px(k % W, k < W ? hh : hh + 2 * step, 0xff0000);  // band lines
  const TrikHsvTargetSums s = sums[f];
  const uint32_t n = (uint32_t)s.points;
  if (n > 10) {  // drawRgbTargetCenterLine(targetX, 0), LSEQ:88-102
    const int32_t cx = (int32_t)((uint32_t)(int32_t)s.sum_x / n);
    for (int k = lane; k < 3 * H; k += 64) px(cx - 1 + k % 3, k / 3, 0xff0000);
  }
}

}  // namespace

// Workgroup shape for line_vec_kernel: rpi rows x cu units, lanes a multiple
// of 64 where possible (640 px: 4 rows x 80 units = 320 lanes); row segments
// only when frames x chunks alone would leave the chip underfilled.
static bool line_geom(const LineArgs& a, LineGeom& g, int& block) {
  const uintptr_t base = reinterpret_cast<uintptr_t>(a.frames);
  if (a.width % 8 || a.line_length % 8 || base % 8 || (a.n_frames > 1 && a.frame_stride % 8)) return false;
  g.units = a.width / 8;
  g.cu = g.units < 1024 ? g.units : 1024;
  g.chunks = (g.units + g.cu - 1) / g.cu;
  g.rpi = 1;
  double best = 2.0;
  for (int r = 1; r * g.cu <= 1024; ++r) {  // least idle lane fraction, then fewest rows
    const int lanes = r * g.cu, padded = (lanes + 63) / 64 * 64;
    const double idle = (double)(padded - lanes) / padded;
    if (idle < best - 1e-9) { best = idle; g.rpi = r; }
    if (padded == lanes) break;
  }
  block = ((g.rpi * g.cu + 63) / 64) * 64;
  const int64_t base_wgs = (int64_t)a.n_frames * g.chunks;
  const int max_segs = (a.height + g.rpi * 8 - 1) / (g.rpi * 8);  // >= 8 iterations per lane
  int segs = base_wgs >= 1024 ? 1 : (int)((2048 + base_wgs - 1) / base_wgs);
  segs = segs < 1 ? 1 : (segs > max_segs ? (max_segs < 1 ? 1 : max_segs) : segs);
  int seg_rows = (a.height + segs - 1) / segs;
  seg_rows = (seg_rows + g.rpi - 1) / g.rpi * g.rpi;
  if (seg_rows / g.rpi > 32767) return false;  // 16-bit per-column counters
  g.seg_rows = seg_rows;
  g.segs = (a.height + seg_rows - 1) / seg_rows;
  // V window in the pre-shift domain (see line_vec_kernel)
  const int lo = (int)a.val_lo, hi = (int)a.val_hi;
  const int mlo = lo ? 64 * lo : -32768, mhi = hi < 255 ? 64 * hi + 63 : 32767;
  g.mlo = (int16_t)mlo;
  g.kspan = (uint16_t)(mhi - mlo);
  return base_wgs * g.segs <= 0x7FFFFFFF;
}

int launch_line(const LineArgs& a, hipStream_t s) {
  if (a.n_frames <= 0 || a.width <= 0 || a.height <= 0) return hipSuccess;
  LineGeom g;
  int block = 0;
  if (a.val_lo > a.val_hi) {
    // empty V range: nothing detected; the sums were zeroed by the caller
  } else if (line_geom(a, g, block)) {
    const int64_t wgs = (int64_t)a.n_frames * g.chunks * g.segs;
    hipLaunchKernelGGL(line_vec_kernel, dim3((unsigned)wgs), dim3(block), 0, s, a, g);
  } else {
    const int64_t blocks = (int64_t)a.n_frames * ((a.height + kLineRows - 1) / kLineRows);
    if (blocks > 0x7FFFFFFF) return hipErrorInvalidValue;
    hipLaunchKernelGGL(line_sums_kernel, dim3((unsigned)blocks), dim3(kLineBlock), 0, s, a);
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess || !a.targets) return e;
  hipLaunchKernelGGL(line_targets_kernel, dim3((unsigned)((a.n_frames + 255) / 256)), dim3(256), 0, s,
                     a.n_frames, a.width, a.height, a.sums, a.targets);
  return hipGetLastError();
}

int launch_wline_targets(int n_frames, int width, int height, const TrikHsvTargetSums* sums, TrikHsvTarget* targets,
                         hipStream_t s) {
  if (n_frames <= 0 || !targets) return hipSuccess;
  hipLaunchKernelGGL(line_targets_kernel, dim3((unsigned)((n_frames + 255) / 256)), dim3(256), 0, s, n_frames, width,
                     height, sums, targets, 0);
  return hipGetLastError();
}

int launch_wline_overlay(const PreviewArgs& a, const TrikHsvTargetSums* sums, hipStream_t s) {
  if (a.n_frames <= 0 || a.width <= 0 || a.height <= 0) return hipSuccess;
  hipLaunchKernelGGL(line_overlay_kernel, dim3((unsigned)a.n_frames), dim3(64), 0, s, a, sums, 0);
  return hipGetLastError();
}

int launch_line_overlay(const PreviewArgs& a, const TrikHsvTargetSums* sums, hipStream_t s) {
  if (a.n_frames <= 0 || a.width <= 0 || a.height <= 0) return hipSuccess;
  hipLaunchKernelGGL(line_overlay_kernel, dim3((unsigned)a.n_frames), dim3(64), 0, s, a, sums);
  return hipGetLastError();
}

// The whole line-sensor preview: with the 2:1 maps the overlay is drawn by
// preview_rows2_kernel in the same pass (the previews are written once);
// otherwise the preview body, then line_overlay_kernel.
int launch_line_preview(PreviewArgs a, const TrikHsvTargetSums* sums, int band, hipStream_t s) {
  if (a.ovl_ok && sums) {
    a.ovl_sums = sums;
    if (!band) a.ovl_band[0] = a.ovl_band[1] = -1;
    const int e = launch_preview_rows2(a, s);
    if (e != hipErrorNotSupported) return e;
    a.ovl_sums = nullptr;
  }
  const int e = launch_preview_body(a, s);
  if (e != hipSuccess) return e;
  return band ? launch_line_overlay(a, sums, s) : launch_wline_overlay(a, sums, s);
}

}  // namespace trik_hsv
