// trik_hsv_kernels.hip -- CDNA4 (gfx950) kernels of the TRIK HSV path.
//
//  reduce_kernel   the generic form of the hot path, used when the optimised
//                  stripe_kernel (trik_hsv_stripe.hip) does not apply (input
//                  not 16-byte aligned, width > 8192): one read-once pass
//                  over N frames of packed YUYV (or ov7670 planes) fusing
//                  WSEQ:251-284 (YUV->RGB->HSV) with WSEQ:316-354 (threshold +
//                  per-row count / sumX / sumY) for up to 4 ranges, reduced
//                  per frame.
//  targets_kernel  WSEQ:486-505 epilogue in IEEE fp32, one thread per
//                  (frame, range).
//  synth_kernel    device-side synthetic frames (bit-identical to the CPU
//                  generator in oracle/trik_oracle.c).
//
// Paths are relative to the reference checkout; WSEQ/OSEQ as in trik_hsv.h.
#include <hip/hip_runtime.h>

#include "trik_hsv_internal.h"
#include "trik_hsv_pixel.h"

namespace trik_hsv {

constexpr int kBlock = 512;           // 8 waves; 2 workgroups per CU (66 KB LDS each)
constexpr int kBlocksPerCU = 2;
constexpr int kTileChunks = 4096;     // 16-byte chunks (8 pixels) per tile, about 64 KB of YUYV

template <int NR>
struct Acc {
  uint32_t n[NR], sx[NR], sy[NR];
  __device__ __forceinline__ void zero() {
#pragma unroll
    for (int k = 0; k < NR; ++k) n[k] = sx[k] = sy[k] = 0;
  }
  __device__ __forceinline__ void add(uint32_t det, uint32_t x, uint32_t y) {
#pragma unroll
    for (int k = 0; k < NR; ++k) {
      const uint32_t d = (det >> k) & 1u;
      n[k] += d;
      sx[k] += d ? x : 0u;
      sy[k] += d ? y : 0u;
    }
  }
};

__device__ __forceinline__ uint64_t wave_sum(uint64_t v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

// Block-wide reduction of the per-lane accumulators into sums[frame] (one
// 64-bit atomic per value per workgroup and frame).
template <int NR>
__device__ void flush(Acc<NR>& acc, int frame, const KernelArgs& a, uint64_t* scratch) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  constexpr int kVals = 3 * NR;
  uint64_t v[kVals];
#pragma unroll
  for (int k = 0; k < NR; ++k) {
    v[3 * k + 0] = wave_sum(acc.n[k]);
    v[3 * k + 1] = wave_sum(acc.sx[k]);
    v[3 * k + 2] = wave_sum(acc.sy[k]);
  }
  if (lane == 0) {
#pragma unroll
    for (int k = 0; k < kVals; ++k) scratch[wave * kVals + k] = v[k];
  }
  __syncthreads();
  if (threadIdx.x < kVals) {
    uint64_t s = 0;
    for (int w = 0; w < kBlock / 64; ++w) s += scratch[w * kVals + threadIdx.x];
    if (s) {
      const int k = threadIdx.x / 3, q = threadIdx.x % 3;
      TrikHsvTargetSums* dst = a.sums + (int64_t)frame * a.sums_ranges + a.range_offset + k;
      unsigned long long* p = reinterpret_cast<unsigned long long*>(&dst->points) + q;
      atomicAdd(p, (unsigned long long)s);
    }
  }
  __syncthreads();
  acc.zero();
}

// One chunk = 8 pixels of one row: 16 bytes of YUYV, or 8 luma + 8 chroma bytes.
template <int LAYOUT, bool ALIGNED>
__device__ __forceinline__ void load_chunk(const uint8_t* fr, int64_t row_off, int64_t plane,
                                           int col, uint32_t w[4]) {
  if (LAYOUT == TRIK_HSV_LAYOUT_YUYV) {
    const uint8_t* p = fr + row_off + (int64_t)col * 16;
    if (ALIGNED) {
      const uint4 v = *reinterpret_cast<const uint4*>(p);
      w[0] = v.x; w[1] = v.y; w[2] = v.z; w[3] = v.w;
    } else {
#pragma unroll
      for (int k = 0; k < 4; ++k)
        w[k] = (uint32_t)p[4 * k] | ((uint32_t)p[4 * k + 1] << 8) | ((uint32_t)p[4 * k + 2] << 16) |
               ((uint32_t)p[4 * k + 3] << 24);
    }
  } else {
    // OSEQ:369-373: pair k = luma bytes (2k, 2k+1), U = chroma byte 2k+1, V = chroma byte 2k.
    const uint8_t* py = fr + row_off + (int64_t)col * 8;
    const uint8_t* pc = py + plane;
    uint32_t y[2], c[2];
    if (ALIGNED) {
      const uint2 vy = *reinterpret_cast<const uint2*>(py);
      const uint2 vc = *reinterpret_cast<const uint2*>(pc);
      y[0] = vy.x; y[1] = vy.y; c[0] = vc.x; c[1] = vc.y;
    } else {
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        y[k] = (uint32_t)py[4 * k] | ((uint32_t)py[4 * k + 1] << 8) | ((uint32_t)py[4 * k + 2] << 16) |
               ((uint32_t)py[4 * k + 3] << 24);
        c[k] = (uint32_t)pc[4 * k] | ((uint32_t)pc[4 * k + 1] << 8) | ((uint32_t)pc[4 * k + 2] << 16) |
               ((uint32_t)pc[4 * k + 3] << 24);
      }
    }
    // rebuild the YUYV word the reference assembles: b0=Y0, b1=U, b2=Y1, b3=V
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      w[2 * k + 0] = __builtin_amdgcn_perm(c[k], y[k], 0x04010500u);  // Y0, C1(U), Y1, C0(V)
      w[2 * k + 1] = __builtin_amdgcn_perm(c[k], y[k], 0x06030702u);  // Y2, C3(U), Y3, C2(V)
    }
  }
}

template <int LAYOUT, int NR, bool MASKS, bool ALIGNED>
__global__ __launch_bounds__(kBlock) void reduce_kernel(KernelArgs a, int64_t n_tiles,
                                                        int band, int tiles_per_frame) {
  if (gated_out(a.gate, a.gate_max, a.gate_le)) return;
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  RangeTables& tab = *reinterpret_cast<RangeTables*>(lds);
  uint64_t* scratch = reinterpret_cast<uint64_t*>(lds + sizeof(RangeTables));

  {  // stage the 66 KB of tables in LDS once per persistent workgroup
    const uint4* src = reinterpret_cast<const uint4*>(a.tables);
    uint4* dst = reinterpret_cast<uint4*>(lds);
    for (int i = threadIdx.x; i < (int)(sizeof(RangeTables) / 16); i += kBlock) dst[i] = src[i];
  }
  __syncthreads();

  const int cpr = a.width >> 3;  // chunks per row
  const int64_t plane = (int64_t)a.height * a.line_length;
  const int64_t t_begin = n_tiles * blockIdx.x / gridDim.x;
  const int64_t t_end = n_tiles * (blockIdx.x + 1) / gridDim.x;

  Acc<NR> acc;
  acc.zero();
  int cur = t_begin < t_end ? (int)(t_begin / tiles_per_frame) : -1;
  for (int64_t t = t_begin; t < t_end; ++t) {
    const int f = (int)(t / tiles_per_frame);
    if (f != cur) {
      flush<NR>(acc, cur, a, scratch);
      cur = f;
    }
    const int r0 = (int)(t - (int64_t)f * tiles_per_frame) * band;
    const int rows = min(band, a.height - r0);
    const int n = rows * cpr;
    const uint8_t* fr = a.frames + (int64_t)f * a.frame_stride;
    for (int i = threadIdx.x; i < n; i += kBlock) {
      const int row = i / cpr, col = i - row * cpr;
      const int y = r0 + row;
      uint32_t w[4];
      load_chunk<LAYOUT, ALIGNED>(fr, (int64_t)y * a.line_length, plane, col, w);
      uint32_t dets[8];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int Y0 = w[k] & 0xFF, U = (w[k] >> 8) & 0xFF, Y1 = (w[k] >> 16) & 0xFF, V = w[k] >> 24;
        dets[2 * k] = detect_pixel(Y0, U, V, tab);
        dets[2 * k + 1] = detect_pixel(Y1, U, V, tab);
      }
      const uint32_t x0 = (uint32_t)col * 8;
#pragma unroll
      for (int j = 0; j < 8; ++j) acc.add(dets[j], x0 + j, (uint32_t)y);
      if (MASKS) {
        uint8_t* mp = a.masks + ((int64_t)f * a.height + y) * a.width + x0;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const uint8_t bits = (uint8_t)(dets[j] << a.mask_shift);
          mp[j] = a.mask_shift ? (uint8_t)(mp[j] | bits) : bits;
        }
      }
    }
  }
  if (cur >= 0) flush<NR>(acc, cur, a, scratch);
}

// ---------------------------------------------------------------------------
// Epilogue, WSEQ:486-505.
// ---------------------------------------------------------------------------
__global__ void targets_kernel(int n, int width, int height, const TrikHsvTargetSums* sums,
                               TrikHsvTarget* out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const TrikHsvTargetSums s = sums[i];
  out[i] = target_of((uint64_t)s.points, (uint64_t)s.sum_x, (uint64_t)s.sum_y, width, height);
}

// ---------------------------------------------------------------------------
// Synthetic frames (oracle/trik_oracle.c: trik_oracle_synth).
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

__constant__ uint8_t k_palette[6][3] = {
    {81, 90, 240}, {145, 54, 34}, {41, 240, 110}, {210, 16, 146}, {170, 166, 16}, {106, 202, 222}};

__device__ void scene_pixel(uint64_t smix, int f, int x, int y, int w, int h, uint32_t& Y,
                            uint32_t& U, uint32_t& V) {
  Y = (uint32_t)(x * 3 + y * 2 + f * 7) & 0xFFu;
  U = (uint32_t)(128 + ((x - w / 2) * 64) / (w > 0 ? w : 1));
  V = (uint32_t)(128 + ((y - h / 2) * 64) / (h > 0 ? h : 1));
  for (int k = 0; k < 6; ++k) {
    const uint64_t r = splitmix64(smix ^ ((uint64_t)(uint32_t)f << 8) ^ (uint64_t)k);
    const int cx = (int)(r % (uint64_t)(w > 0 ? w : 1));
    const int cy = (int)((r >> 20) % (uint64_t)(h > 0 ? h : 1));
    const int rad = 8 + (int)((r >> 40) % (uint64_t)(h / 6 + 1));
    const int dx = x - cx, dy = y - cy;
    if (dx * dx + dy * dy <= rad * rad) {
      Y = k_palette[k][0];
      U = k_palette[k][1];
      V = k_palette[k][2];
    }
  }
}

__global__ void synth_uniform_kernel(uint8_t* frames, int64_t stride, int first_frame,
                                     int n_frames, int64_t frame_bytes, uint64_t smix) {
  const int64_t words = (frame_bytes + 7) / 8;
  const int64_t total = words * n_frames;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int fi = (int)(i / words);
    const int64_t w = i - (int64_t)fi * words;
    const uint64_t v = splitmix64(smix ^ ((uint64_t)(uint32_t)(first_frame + fi) << 32) ^ (uint64_t)w);
    uint8_t* p = frames + (int64_t)fi * stride + w * 8;
    const int64_t left = frame_bytes - w * 8;
    if (left >= 8 && (reinterpret_cast<uintptr_t>(p) & 7) == 0) {
      *reinterpret_cast<uint64_t*>(p) = v;
    } else {
      for (int k = 0; k < 8 && k < left; ++k) p[k] = (uint8_t)(v >> (8 * k));
    }
  }
}

__global__ void synth_scene_kernel(uint8_t* frames, int64_t stride, int first_frame, int n_frames,
                                   int width, int height, int line_length, int layout,
                                   uint64_t smix) {
  const int pairs = width / 2;
  const int64_t total = (int64_t)pairs * height * n_frames;
  const int64_t plane = (int64_t)height * line_length;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int fi = (int)(i / ((int64_t)pairs * height));
    const int64_t rem = i - (int64_t)fi * pairs * height;
    const int y = (int)(rem / pairs), q = (int)(rem - (int64_t)y * pairs);
    const int f = first_frame + fi, x = 2 * q;
    uint32_t Y0, U, V, Y1, U1, V1;
    scene_pixel(smix, f, x, y, width, height, Y0, U, V);
    scene_pixel(smix, f, x + 1, y, width, height, Y1, U1, V1);
    uint8_t* fr = frames + (int64_t)fi * stride;
    if (layout == TRIK_HSV_LAYOUT_OV7670) {
      fr[(int64_t)y * line_length + x] = (uint8_t)Y0;
      fr[(int64_t)y * line_length + x + 1] = (uint8_t)Y1;
      fr[plane + (int64_t)y * line_length + x] = (uint8_t)V;
      fr[plane + (int64_t)y * line_length + x + 1] = (uint8_t)U;
    } else {
      uint8_t* p = fr + (int64_t)y * line_length + 2 * x;
      p[0] = (uint8_t)Y0; p[1] = (uint8_t)U; p[2] = (uint8_t)Y1; p[3] = (uint8_t)V;
    }
  }
}

// ---------------------------------------------------------------------------
// Launchers
// ---------------------------------------------------------------------------
static int cu_count() { return device_cus(); }

template <int LAYOUT, int NR, bool MASKS, bool ALIGNED>
static int launch_variant(const KernelArgs& a, hipStream_t s) {
  const int cpr = a.width >> 3;
  const int band = max(1, min(a.height, kTileChunks / max(cpr, 1)));
  const int tiles_per_frame = (a.height + band - 1) / band;
  const int64_t n_tiles = (int64_t)tiles_per_frame * a.n_frames;
  if (n_tiles == 0 || cpr == 0) return hipSuccess;
  const int64_t cap = (int64_t)cu_count() * kBlocksPerCU;
  const int64_t grid = n_tiles < cap ? n_tiles : cap;
  const size_t lds = sizeof(RangeTables) + (kBlock / 64) * 3 * NR * sizeof(uint64_t);
  auto kern = reduce_kernel<LAYOUT, NR, MASKS, ALIGNED>;
  {
    hipError_t e = set_dynamic_lds(reinterpret_cast<const void*>(kern), 80 * 1024);
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(kBlock), lds, s, a, n_tiles, band,
                     tiles_per_frame);
  return hipGetLastError();
}

template <int LAYOUT, bool MASKS, bool ALIGNED>
static int dispatch_nr(const KernelArgs& a, hipStream_t s) {
  switch (a.n_ranges) {
    case 1: return launch_variant<LAYOUT, 1, MASKS, ALIGNED>(a, s);
    case 2: return launch_variant<LAYOUT, 2, MASKS, ALIGNED>(a, s);
    case 3: return launch_variant<LAYOUT, 3, MASKS, ALIGNED>(a, s);
    case 4: return launch_variant<LAYOUT, 4, MASKS, ALIGNED>(a, s);
  }
  return hipErrorInvalidValue;
}

template <int LAYOUT, bool MASKS>
static int dispatch_aligned(const KernelArgs& a, hipStream_t s) {
  const int64_t need = LAYOUT == TRIK_HSV_LAYOUT_YUYV ? 16 : 8;
  const bool aligned = (reinterpret_cast<uintptr_t>(a.frames) % need) == 0 &&
                       (a.frame_stride % need) == 0 && (a.line_length % need) == 0;
  return aligned ? dispatch_nr<LAYOUT, MASKS, true>(a, s) : dispatch_nr<LAYOUT, MASKS, false>(a, s);
}

int launch_reduce(const KernelArgs& a, bool write_masks, hipStream_t s) {
  if (a.layout == TRIK_HSV_LAYOUT_YUYV)
    return write_masks ? dispatch_aligned<TRIK_HSV_LAYOUT_YUYV, true>(a, s)
                       : dispatch_aligned<TRIK_HSV_LAYOUT_YUYV, false>(a, s);
  return write_masks ? dispatch_aligned<TRIK_HSV_LAYOUT_OV7670, true>(a, s)
                     : dispatch_aligned<TRIK_HSV_LAYOUT_OV7670, false>(a, s);
}

// One workgroup of 256 per (group, mx) row: the range tables of
// compile_tables (trik_hsv_tables.cpp) and the stripe kernel's tables of
// compile_stripe_tables, from the packed ranges (WSEQ:425-445) -- the same
// per-range tests: hue by the wrap-aware "outside" pattern, S and V by their
// byte intervals, sv[mx][mn] when mn <= mx, V = mx in [fv, tv] and
// S = (LUT255[mx] (mx - mn)) >> 8 in [fs, ts] (WSEQ:389-407).  Row mx = 0 of
// each group also writes the per-value tables.
__global__ __launch_bounds__(256) void compile_tables_kernel(TableBuildArgs a, RangeTables* tabs, StripeTables* strs) {
  const int g = (int)blockIdx.y, mx = (int)blockIdx.x, mn = (int)threadIdx.x;
  const int n0 = 4 * g, cnt = a.n_ranges - n0 < 4 ? a.n_ranges - n0 : 4;
  RangeTables& t = tabs[g];
  StripeTables& st = strs[g];
  auto outside = [](uint32_t x, uint32_t lo, uint32_t hi) { return x < lo || x > hi; };
  const uint32_t l255 = mx ? (255u * 256u) / (uint32_t)mx : 0u;
  uint32_t sv = 0;
  for (int r = 0; r < cnt; ++r) {
    const uint32_t from = a.from[n0 + r], to = a.to[n0 + r];
    const uint32_t fs = (from >> 8) & 0xFFu, ts = (to >> 8) & 0xFFu;
    const uint32_t fv = (from >> 16) & 0xFFu, tv = (to >> 16) & 0xFFu;
    const uint32_t S = (l255 * (uint32_t)(mx - mn)) >> 8;
    if (mn <= mx && !outside((uint32_t)mx, fv, tv) && !outside(S, fs, ts)) sv |= 1u << r;
  }
  t.sv[mx * 256 + mn] = (uint8_t)sv;
  st.sv[mx * kSvStride + mn] = (uint8_t)sv;
  if (mn < kSvStride - 256) st.sv[mx * kSvStride + 256 + mn] = 0;
  if (mx == 0) {  // the per-value tables, index i = mn
    const uint32_t i = (uint32_t)mn;
    uint8_t hue = 0, sm = 0, vm = 0;
    for (int r = 0; r < cnt; ++r) {
      const uint32_t from = a.from[n0 + r], to = a.to[n0 + r];
      const uint8_t bit = (uint8_t)(1u << r);
      if ((outside(i, from & 0xFFu, to & 0xFFu) ? 1u : 0u) == (a.expect[n0 + r] & 1u)) hue |= bit;
      if (!outside(i, (from >> 8) & 0xFFu, (to >> 8) & 0xFFu)) sm |= bit;
      if (!outside(i, (from >> 16) & 0xFFu, (to >> 16) & 0xFFu)) vm |= bit;
    }
    const uint16_t l43 = i ? (uint16_t)((43u * 256u) / i) : (uint16_t)0;
    t.hue[i] = hue;
    t.smask[i] = sm;
    t.vmask[i] = vm;
    t.lut43[i] = l43;
    t.lut255[i] = i ? (uint16_t)((255u * 256u) / i) : (uint16_t)0;
    uint32_t spread = 0;
    for (int r = 0; r < cnt; ++r) spread |= ((uint32_t)(hue >> r) & 1u) << (8 * r);
    for (int c = 0; c < kHueCopies; ++c) st.hue[i * kHueCopies + c] = spread;
    for (int c = 0; c < kM43Copies; ++c) st.m43[i * kM43Copies + c] = l43;
  }
}

int launch_compile_tables(const TableBuildArgs& args, int groups, RangeTables* d_tables, StripeTables* d_stripe,
                          hipStream_t s) {
  if (groups <= 0 || groups > kTableGroups) return hipErrorInvalidValue;
  hipLaunchKernelGGL(compile_tables_kernel, dim3(256, groups), dim3(256), 0, s, args, d_tables, d_stripe);
  return hipGetLastError();
}

int launch_targets(const TrikHsvFrameBatch& b, int n_ranges, const TrikHsvTargetSums* sums,
                   TrikHsvTarget* targets, hipStream_t s) {
  const int n = b.n_frames * n_ranges;
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(targets_kernel, dim3((n + 255) / 256), dim3(256), 0, s, n, b.width, b.height,
                     sums, targets);
  return hipGetLastError();
}

// Per-target batch totals (the one value exchanged between
// ranks): totals[r] = sum over frames of sums[f][r], field by field, int64.
// One 256-lane workgroup per (range, field); the same order on every call.
__global__ __launch_bounds__(256) void totals_kernel(int n_frames, int n_ranges, const TrikHsvTargetSums* sums,
                                                     TrikHsvTargetSums* totals) {
  const int r = blockIdx.x / 3, c = blockIdx.x % 3;
  const long long* src = reinterpret_cast<const long long*>(sums) + (int64_t)r * 3 + c;
  long long acc = 0;
  for (int f = threadIdx.x; f < n_frames; f += blockDim.x) acc += src[(int64_t)f * n_ranges * 3];
  __shared__ long long part[256];
  part[threadIdx.x] = acc;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) part[threadIdx.x] += part[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) reinterpret_cast<long long*>(totals)[(int64_t)r * 3 + c] = part[0];
}

int launch_totals(int n_frames, int n_ranges, const TrikHsvTargetSums* sums, TrikHsvTargetSums* totals,
                  hipStream_t s) {
  if (n_ranges <= 0) return hipSuccess;
  hipLaunchKernelGGL(totals_kernel, dim3(3 * n_ranges), dim3(256), 0, s, n_frames, n_ranges, sums, totals);
  return hipGetLastError();
}

int launch_synth(const TrikHsvFrameBatch& b, uint8_t* frames, int first_frame, int kind,
                 uint64_t seed, hipStream_t s) {
  const uint64_t smix = [&] {
    uint64_t x = seed + 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
  }();
  const int64_t plane = (int64_t)b.height * b.line_length;
  const int64_t frame_bytes = plane * (b.layout == TRIK_HSV_LAYOUT_OV7670 ? 2 : 1);
  const int grid = cu_count() * 8;
  if (b.n_frames <= 0 || frame_bytes <= 0) return hipSuccess;
  if (kind == 0) {
    hipLaunchKernelGGL(synth_uniform_kernel, dim3(grid), dim3(256), 0, s, frames, b.frame_stride,
                       first_frame, b.n_frames, frame_bytes, smix);
  } else {
    for (int i = 0; i < b.n_frames; ++i) {
      hipError_t e = hipMemsetAsync(frames + (int64_t)i * b.frame_stride, 0, (size_t)frame_bytes, s);
      if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(synth_scene_kernel, dim3(grid), dim3(256), 0, s, frames, b.frame_stride,
                       first_frame, b.n_frames, b.width, b.height, b.line_length, b.layout, smix);
  }
  return hipGetLastError();
}

}  // namespace trik_hsv
