// trik_hsv_line.hip -- the ov7670 line sensor, LSEQ =
// trik/ov7670/line_sensor/include/internal/cv_line_detector_seqpass.hpp:
//
//  line_sums_kernel     detection by V only (hue/sat bounds 0..255, LSEQ:
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

__global__ void line_targets_kernel(int n_frames, int width, int height, const TrikHsvTargetSums* sums,
                                    TrikHsvTarget* targets) {
  const int f = blockIdx.x * blockDim.x + threadIdx.x;
  if (f >= n_frames) return;
  const TrikHsvTargetSums s = sums[f];
  TrikHsvTarget t = {0, 0, 0, 0};
  const uint32_t n = (uint32_t)s.points;
  if (n > 10) {  // LSEQ:462-474 (crossSize LSEQ:452, step 40)
    const int32_t cx = (int32_t)((uint32_t)(int32_t)s.sum_x / n);
    t.x = (int8_t)(((cx - width / 2) * 100 * 2) / width);
    t.y = (int8_t)(int)((uint32_t)((uint32_t)s.sum_y * 100u) / (uint32_t)(width * 2 * 40));
    t.size = (uint8_t)((uint32_t)(n * 100u) / (uint32_t)(height * width));
  }
  targets[f] = t;
}

__device__ __forceinline__ void write_px565(uint8_t* dst, uint32_t rgb888) {
  const uint32_t v = ((rgb888 >> 19) & 0x001fu) | ((rgb888 >> 5) & 0x07e0u) | ((rgb888 << 8) & 0xf800u);
  dst[0] = (uint8_t)v;
  dst[1] = (uint8_t)(v >> 8);
}

__global__ __launch_bounds__(64) void line_overlay_kernel(PreviewArgs a, const TrikHsvTargetSums* sums) {
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
  for (int k = lane; k < 2 * W; k += 64) px(k % W, k < W ? hh : hh + 2 * step, 0xff0000);  // band lines
  const TrikHsvTargetSums s = sums[f];
  const uint32_t n = (uint32_t)s.points;
  if (n > 10) {  // drawRgbTargetCenterLine(targetX, 0), LSEQ:88-102
    const int32_t cx = (int32_t)((uint32_t)(int32_t)s.sum_x / n);
    for (int k = lane; k < 3 * H; k += 64) px(cx - 1 + k % 3, k / 3, 0xff0000);
  }
}

}  // namespace

int launch_line(const LineArgs& a, hipStream_t s) {
  if (a.n_frames <= 0 || a.width <= 0 || a.height <= 0) return hipSuccess;
  const int64_t blocks = (int64_t)a.n_frames * ((a.height + kLineRows - 1) / kLineRows);
  if (blocks > 0x7FFFFFFF) return hipErrorInvalidValue;
  hipLaunchKernelGGL(line_sums_kernel, dim3((unsigned)blocks), dim3(kLineBlock), 0, s, a);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess || !a.targets) return e;
  hipLaunchKernelGGL(line_targets_kernel, dim3((unsigned)((a.n_frames + 255) / 256)), dim3(256), 0, s,
                     a.n_frames, a.width, a.height, a.sums, a.targets);
  return hipGetLastError();
}

int launch_line_overlay(const PreviewArgs& a, const TrikHsvTargetSums* sums, hipStream_t s) {
  if (a.n_frames <= 0 || a.width <= 0 || a.height <= 0) return hipSuccess;
  hipLaunchKernelGGL(line_overlay_kernel, dim3((unsigned)a.n_frames), dim3(64), 0, s, a, sums);
  return hipGetLastError();
}

}  // namespace trik_hsv
