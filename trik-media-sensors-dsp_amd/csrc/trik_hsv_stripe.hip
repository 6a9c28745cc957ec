// trik_hsv_stripe.hip -- the optimised hot kernel for gfx950.
//
// One read-once pass over N frames fusing the reference's two loops
// (WSEQ:251-284 convert, WSEQ:316-354 threshold + centroid; WSEQ/OSEQ as in
// include/trik_hsv.h) for up to 4 HSV ranges.  Design:
//
//  * Column stripes.  A workgroup of B <= 1024 threads covers k = 1024/cpr
//    rows of cpr 16-byte chunks (8 pixels each); lane t owns chunk column
//    t % cpr for the whole tile and walks rows t / cpr, +k, +2k, ...  Loads are
//    coalesced dwordx4 (YUYV) or 2 x dwordx2 (ov7670 planes), the next row's
//    chunk prefetched while the current one computes.
//  * Per pixel, branch-free, ~30 VALU ops: YUV -> RGB presums with
//    v_dot4_u32_u8, clamp via v_bfe_i32 + v_med3_i32 (the 16-bit wrap of
//    _add2 falls out of bfe), max3/min3, the hue case select as v_cndmask,
//    h = m*diff + base as v_mad_i32_i24, and three LDS lookups: LUT43 and the
//    sat&val mask by (max, min), then the byte-spread hue mask by H.  A step's
//    8 pixels issue their first two lookups before any hue index is formed,
//    so LDS latency overlaps (4 waves/SIMD cannot hide it otherwise).  No
//    per-range work per pixel.
//  * Accumulation with fixed columns needs no per-pixel x weight: per lane,
//    pairs of pixels add into byte-packed counters with v_add3_u32 (range t in
//    byte t), odd pixels into one more counter, and a prefix-of-prefix counter
//    gives the sum over rows of y * count.  About one VALU op
//    per pixel; unpacked to 32-bit per range once per tile.
//  * Per tile: DPP wave reduction, one 64-bit atomic per value per wave.
#include <hip/hip_runtime.h>

#include <type_traits>

#include "trik_hsv_internal.h"
#include "trik_hsv_stripe_px.h"

namespace trik_hsv {

namespace {

using namespace stripe_px;

constexpr int kMaxBlock = 1024;
constexpr uint32_t kLdsReduce = sizeof(StripeTables);          // u64 [16 waves][3 * 4]: flush_frame
constexpr uint32_t kLdsStripe = kLdsReduce + 16 * 12 * 8;        // the dynamic LDS of one workgroup
static_assert(2 * kLdsStripe <= 160 * 1024, "two workgroups per CU");
constexpr int kMaxSteps = 63;  // byte counters: P_i <= 2*63, O <= 4*63 (a VGA frame is one 40-step tile)
constexpr int kQFlush = 7;     // steps per Q block: block-relative sums <= 8*(1+...+7) = 224

struct StripeGeom {
  int32_t cpr;              // 16-byte chunks per row (width / 8)
  int32_t k;                // rows per step
  int32_t steps;            // steps per tile (<= kMaxSteps)
  int32_t tiles_per_frame;
  int64_t n_tiles;
};

// Sum each of N values over the 64 lanes of the wave (result valid in lane
// 63).  DPP row_shr 1,2,4,8 builds row prefixes, row_bcast15/31 folds rows.
// The N reductions are interleaved so independent DPP ops hide each other's
// hazards.
template <int N>
__device__ __forceinline__ void wave_sums(uint32_t (&v)[N]) {
#pragma unroll
  for (int i = 0; i < N; ++i) v[i] += __builtin_amdgcn_update_dpp(0u, v[i], 0x111, 0xF, 0xF, true);
#pragma unroll
  for (int i = 0; i < N; ++i) v[i] += __builtin_amdgcn_update_dpp(0u, v[i], 0x112, 0xF, 0xF, true);
#pragma unroll
  for (int i = 0; i < N; ++i) v[i] += __builtin_amdgcn_update_dpp(0u, v[i], 0x114, 0xF, 0xF, true);
#pragma unroll
  for (int i = 0; i < N; ++i) v[i] += __builtin_amdgcn_update_dpp(0u, v[i], 0x118, 0xF, 0xF, true);
#pragma unroll
  for (int i = 0; i < N; ++i) v[i] += __builtin_amdgcn_update_dpp(0u, v[i], 0x142, 0xA, 0xF, false);
#pragma unroll
  for (int i = 0; i < N; ++i) v[i] += __builtin_amdgcn_update_dpp(0u, v[i], 0x143, 0xC, 0xF, false);
}

// Wave-reduce the per-lane accumulators of one tile and add them to sums[frame].
template <int NR>
__device__ __forceinline__ void flush_frame(uint32_t (&acc)[3 * NR], int frame, const KernelArgs& a) {
  // wave sums, then the workgroup's sum in LDS (64-bit: 16 waves' 32-bit
  // sums may not fit 32 bits), then one atomic per value per workgroup -- a
  // frame split into many short tiles (small batches) would otherwise pile
  // 12 atomics per wave onto the same 12 addresses
  wave_sums<3 * NR>(acc);
  typedef __attribute__((address_space(3))) unsigned long long* lds_u64_ptr;
  const lds_u64_ptr red = (lds_u64_ptr)(uintptr_t)kLdsReduce;
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 63) {
#pragma unroll
    for (int v = 0; v < 3 * NR; ++v) red[w * 3 * NR + v] = acc[v];
  }
  __syncthreads();
  if (threadIdx.x < 3 * NR) {
    unsigned long long sum = 0;
    for (int j = 0; j < (int)(blockDim.x >> 6); ++j) sum += red[j * 3 * NR + threadIdx.x];
    if (sum) {
      TrikHsvTargetSums* dst = a.sums + (int64_t)frame * a.sums_ranges + a.range_offset;
      atomicAdd(reinterpret_cast<unsigned long long*>(&dst[threadIdx.x / 3].points) + (threadIdx.x % 3), sum);
    }
  }
  __syncthreads();  // the slots are written again at the next tile's flush
#pragma unroll
  for (int v = 0; v < 3 * NR; ++v) acc[v] = 0;
}

template <int LAYOUT>
__device__ __forceinline__ void load_chunk(const uint8_t* p, int64_t plane, uint32_t w[4]) {
  if (LAYOUT == TRIK_HSV_LAYOUT_YUYV) {
    const uint4 v = *reinterpret_cast<const uint4*>(p);
    w[0] = v.x; w[1] = v.y; w[2] = v.z; w[3] = v.w;
  } else {
    const uint2 vy = *reinterpret_cast<const uint2*>(p);
    const uint2 vc = *reinterpret_cast<const uint2*>(p + plane);
    // OSEQ:369-373: U = odd chroma byte, V = even chroma byte
    w[0] = __builtin_amdgcn_perm(vc.x, vy.x, 0x04010500u);
    w[1] = __builtin_amdgcn_perm(vc.x, vy.x, 0x06030702u);
    w[2] = __builtin_amdgcn_perm(vc.y, vy.y, 0x04010500u);
    w[3] = __builtin_amdgcn_perm(vc.y, vy.y, 0x06030702u);
  }
}

// byte-spread mask -> bit mask (range t -> bit t)
__device__ __forceinline__ uint32_t pack_bits(uint32_t e) {
  return ((e * 0x01020408u) >> 24) & 0xFu;  // bit 8t lands on bit 24+t
}

// MODE (KernelArgs::detect_mode): the detection a launch group needs.
//  kDetectFull  the full pixel path above.
//  kDetectSV    every range accepts every hue (the S- and V-band sets): the
//               sat&val mask alone -- no hue case select, no LUT43 or hue
//               lookup (~15 instead of ~29 VALU per pixel); only sv is staged.
//  kDetectV     every range also accepts every saturation (V bands, the webcam
//               line sensor): the value test alone.  V = clamp8(max(R', G', B')
//               >> 6) over the unclamped presums (clamp8 and >>6 are monotone;
//               R', G' lie in int16, B' is the reference's 16-bit wrap), read
//               from a 1024-entry byte-spread table indexed by (m >> 6) + 512
//               whose ends hold the clamped values (~8 VALU per pixel); the
//               table is built in LDS from RangeTables::vmask.
template <int LAYOUT, int NR, bool MASKS, int MODE>
__global__ __launch_bounds__(kMaxBlock) __attribute__((amdgpu_waves_per_eu(8)))
void stripe_kernel(KernelArgs a, StripeGeom g) {
  if (gated_out(a.gate, a.gate_max, a.gate_le)) return;
  {  // stage the tables at LDS address 0 (dynamic LDS, sizeof(StripeTables))
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
    const u32x4* src = reinterpret_cast<const u32x4*>(a.stripe_tables);
    typedef __attribute__((address_space(3))) u32x4* lds_u128_wptr;
    lds_u128_wptr dst = (lds_u128_wptr)(uintptr_t)0;
    if constexpr (MODE == kDetectV) {
      typedef __attribute__((address_space(3))) uint32_t* lds_u32_wptr;
      const uint32_t keep = (1u << NR) - 1u;
      for (int i = threadIdx.x; i < 1024; i += blockDim.x) {
        const int v = i < 512 ? 0 : (i > 767 ? 255 : i - 512);
        ((lds_u32_wptr)(uintptr_t)0)[i] = combine(0x01010101u, a.tables->vmask[v] & keep);
      }
    } else {
      constexpr int kStage = MODE == kDetectFull ? (int)(sizeof(StripeTables) / 16) : (int)(sizeof(StripeTables::sv) / 16);
      for (int i = threadIdx.x; i < kStage; i += blockDim.x) dst[i] = src[i];
    }
  }
  __syncthreads();

  const int t = threadIdx.x;
  const uint32_t hue_lane = (uint32_t)offsetof(StripeTables, hue) + ((t % kHueCopies) << 2);
  const uint32_t m43_lane = (uint32_t)offsetof(StripeTables, m43) + ((t % kM43Copies) << 2);
  const bool active = t < g.k * g.cpr;
  const int col = active ? t % g.cpr : 0;
  const int ro = active ? t / g.cpr : 0;
  const int64_t plane = (int64_t)a.height * a.line_length;
  const int64_t rowstep = (int64_t)g.k * a.line_length;
  const int col_bytes = LAYOUT == TRIK_HSV_LAYOUT_YUYV ? col * 16 : col * 8;
  const uint32_t x0 = (uint32_t)col * 8;
  const uint32_t voff = (uint32_t)ro * (uint32_t)a.line_length + (uint32_t)col_bytes;  // < 2^32 (geometry)

  const int64_t t_begin = g.n_tiles * blockIdx.x / gridDim.x;
  const int64_t t_end = g.n_tiles * (blockIdx.x + 1) / gridDim.x;
  for (int64_t tile = t_begin; tile < t_end; ++tile) {
    const int f = (int)(tile / g.tiles_per_frame);
    const int r0 = (int)(tile - (int64_t)f * g.tiles_per_frame) * g.k * g.steps;
    const int y0 = r0 + ro;
    // steps that hold at least one valid row of this tile (uniform per block)
    const int steps = min(g.steps, (a.height - r0 + g.k - 1) / g.k);
    const uint8_t* p = a.frames + (int64_t)f * a.frame_stride + (int64_t)y0 * a.line_length + col_bytes;

    // Byte-packed per-lane counters (range t in byte t):
    //   P_i : pixels 2i and 2i+1 of the chunk    O : odd pixels
    //   Q   : sum over the current block of steps of (cumulative count - CumS),
    //         CumS = cumulative count at the block start.  Q's byte fields may
    //         carry into each other while adding; the block-end value
    //         Q - nb*CumS has true fields in [0, 224], and packed arithmetic
    //         is exact mod 2^32, so the fields come out right.
    //   Qa/Qb, Ba/Bb : 16-bit fields (ranges 0,2 / 1,3) collecting, per block,
    //         the sums above and nb*CumS.  CumS's byte fields may exceed 255
    //         past 31 steps (it only enters mod-2^32 linear terms); CumA/CumB
    //         hold the same counts in 16-bit fields for Ba/Bb and the totals.
    uint32_t P0 = 0, P1 = 0, P2 = 0, P3 = 0, O = 0, Q = 0, CumS = 0, CumA = 0, CumB = 0;
    uint32_t Qa = 0, Qb = 0, Ba = 0, Bb = 0;
    int nb = 0;
    // Software pipeline, one row ahead (8 waves per SIMD hide the rest).
    // Loads are unconditional (a row past the frame end re-reads the tile's
    // first row) so the compiler can wait with a counted vmcnt.
    const uint8_t* pf = active ? p : a.frames + (int64_t)f * a.frame_stride;
    const int vsteps = active ? min(steps, (a.height - y0 + g.k - 1) / g.k) : 0;  // valid steps, this lane
    // The step loop, in two forms: FULL when every lane of the block is active
    // and every row of the tile lies in the frame (the common case: no
    // per-lane validity, a uniform loop counter, loads from a uniform row base
    // plus a per-lane 32-bit offset); otherwise per-lane row validity.
    const bool full = (r0 + steps * g.k <= a.height) && (g.k * g.cpr) % 64 == 0;
    const uint8_t* tbase = a.frames + (int64_t)f * a.frame_stride + (int64_t)r0 * a.line_length;
    auto run = [&](auto full_c) {
      constexpr bool FULL = decltype(full_c)::value;
      // 4 pixels (words w0, w1) of row y0 + s*k at chunk pixel offset 4*half
      auto half_step = [&](uint32_t w0, uint32_t w1, int s, int half, uint32_t& Pa, uint32_t& Pb) {
        const bool valid = FULL || s < vsteps;
        uint32_t e[4];
        if constexpr (MODE == kDetectFull) {
          Phase1 p[4];
          uint32_t m[4], sv[4];
          p[0] = phase1<0>(w0, w0 ^ 0xFF00FF00u, m43_lane);
          p[1] = phase1<1>(w0, w0 ^ 0xFF00FF00u, m43_lane);
          p[2] = phase1<0>(w1, w1 ^ 0xFF00FF00u, m43_lane);
          p[3] = phase1<1>(w1, w1 ^ 0xFF00FF00u, m43_lane);
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            m[j] = lds_u32(p[j].m43_addr);
            sv[j] = lds_u8(p[j].sv_addr);
          }
#pragma unroll
          for (int j = 0; j < 4; ++j) e[j] = combine(lds_u32(phase2_addr(m[j], p[j], hue_lane)), sv[j]);
        } else if constexpr (MODE == kDetectV) {
          e[0] = lds_u32(v_addr<0>(w0, w0 ^ 0xFF00FF00u));
          e[1] = lds_u32(v_addr<1>(w0, w0 ^ 0xFF00FF00u));
          e[2] = lds_u32(v_addr<0>(w1, w1 ^ 0xFF00FF00u));
          e[3] = lds_u32(v_addr<1>(w1, w1 ^ 0xFF00FF00u));
        } else {
          const uint32_t a0 = sv_addr_only<0>(w0, w0 ^ 0xFF00FF00u), a1 = sv_addr_only<1>(w0, w0 ^ 0xFF00FF00u);
          const uint32_t a2 = sv_addr_only<0>(w1, w1 ^ 0xFF00FF00u), a3 = sv_addr_only<1>(w1, w1 ^ 0xFF00FF00u);
          e[0] = combine(0x01010101u, lds_u8(a0));
          e[1] = combine(0x01010101u, lds_u8(a1));
          e[2] = combine(0x01010101u, lds_u8(a2));
          e[3] = combine(0x01010101u, lds_u8(a3));
        }
        if (MASKS && valid) {
          const int y = y0 + s * g.k;
          uint8_t* mp = a.masks + ((int64_t)f * a.height + y) * a.width + x0 + 4 * half;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const uint8_t bits = (uint8_t)(pack_bits(e[j]) << a.mask_shift);
            mp[j] = a.mask_shift ? (uint8_t)(mp[j] | bits) : bits;
          }
        }
        if (valid) {  // false only for rows past the frame end and idle lanes
          Pa = Pa + e[0] + e[1];
          Pb = Pb + e[2] + e[3];
          O = O + e[1] + e[3];
        }
      };
      auto step = [&](const uint32_t (&cw)[4], int s) {
        half_step(cw[0], cw[1], s, 0, P0, P1);
        half_step(cw[2], cw[3], s, 1, P2, P3);
        Q = Q + P0 + P1;
        Q = Q + P2 + P3;
        ++nb;
        if (nb == kQFlush || s + 1 == steps) {  // uniform across the block
          const uint32_t T = Q - (uint32_t)nb * CumS;
          Qa += T & 0x00FF00FFu;
          Qb += (T >> 8) & 0x00FF00FFu;
          Ba += (uint32_t)nb * CumA;
          Bb += (uint32_t)nb * CumB;
          CumS = P0 + P1 + P2 + P3;
          CumA = (P0 & 0x00FF00FFu) + (P1 & 0x00FF00FFu) + (P2 & 0x00FF00FFu) + (P3 & 0x00FF00FFu);
          CumB = ((P0 >> 8) & 0x00FF00FFu) + ((P1 >> 8) & 0x00FF00FFu) + ((P2 >> 8) & 0x00FF00FFu) +
                 ((P3 >> 8) & 0x00FF00FFu);
          Q = 0;
          nb = 0;
        }
      };
      // FULL: a uniform row base advanced by rowstep per step (scalar adds),
      // plus the lane's 32-bit offset
      const uint8_t* rb = tbase;
      auto row_ptr = [&](int s) -> const uint8_t* {
        if (FULL) return rb + voff;
        return s < vsteps ? pf + (int64_t)s * rowstep : pf;
      };
      uint32_t wa[4], wb[4];  // two buffers rotate statically (unroll by 2)
      load_chunk<LAYOUT>(row_ptr(0), plane, wa);
      for (int s = 0; s < steps; s += 2) {
        if (FULL && s + 1 < steps) rb += rowstep;
        load_chunk<LAYOUT>(row_ptr(s + 1), plane, wb);
        step(wa, s);
        if (s + 1 >= steps) break;
        if (FULL && s + 2 < steps) rb += rowstep;
        load_chunk<LAYOUT>(row_ptr(s + 2), plane, wa);
        step(wb, s + 1);
      }
    };
    if (full) run(std::true_type{});
    else run(std::false_type{});
    Qa += Ba;  // sum over steps of the cumulative count, 16-bit fields
    Qb += Bb;

    // unpack per range, wave-reduce, one atomic per value per wave and tile
    uint32_t acc[3 * NR];
    // the last step always flushed, so CumA/CumB hold the tile's counts
#pragma unroll
    for (int rr = 0; rr < NR; ++rr) {
      const int sh = 8 * rr;
      const uint32_t c = ((rr & 1) ? (CumB >> ((rr >> 1) * 16)) : (CumA >> ((rr >> 1) * 16))) & 0xFFFFu;
      const uint32_t wx = 2u * ((P1 >> sh) & 0xFFu) + 4u * ((P2 >> sh) & 0xFFu) +
                          6u * ((P3 >> sh) & 0xFFu) + ((O >> sh) & 0xFFu);
      const uint32_t qq = ((rr & 1) ? (Qb >> ((rr >> 1) * 16)) : (Qa >> ((rr >> 1) * 16))) & 0xFFFFu;
      acc[3 * rr + 0] = c;
      acc[3 * rr + 1] = x0 * c + wx;
      // sum over steps of (y0 + k*s) * c_s = y0*C + k*(steps*C - sum of prefix counts)
      acc[3 * rr + 2] = (uint32_t)y0 * c + (uint32_t)g.k * ((uint32_t)steps * c - qq);
    }
    flush_frame<NR>(acc, f, a);
  }
}

// two workgroups per CU (LDS and VGPR budgets)
int64_t stripe_slots() { return 2LL * device_cus(); }

// Tiles of <= kMaxSteps steps; small batches split each frame into more
// (shorter) tiles until the grid fills the chip's workgroup slots -- one VGA
// frame is 40 one-step tiles instead of one 40-step tile on a single CU.
bool geometry(const KernelArgs& a, StripeGeom& g, int64_t slots) {
  const int cpr = a.width >> 3;
  if (cpr <= 0 || cpr > kMaxBlock || a.height <= 0) return false;
  const int k = kMaxBlock / cpr;
  const int steps_total = (a.height + k - 1) / k;
  int64_t tiles = (steps_total + kMaxSteps - 1) / kMaxSteps;
  if (a.n_frames > 0 && tiles * a.n_frames < slots) {
    const int64_t want = (slots + a.n_frames - 1) / a.n_frames;
    tiles = want < steps_total ? want : steps_total;
  }
  g.cpr = cpr;
  g.k = k;
  g.steps = (int)((steps_total + tiles - 1) / tiles);
  g.tiles_per_frame = (steps_total + g.steps - 1) / g.steps;
  g.n_tiles = (int64_t)g.tiles_per_frame * a.n_frames;
  return true;
}

template <int LAYOUT, int NR, bool MASKS, int MODE>
int launch_t(const KernelArgs& a, const StripeGeom& g, hipStream_t s) {
  auto kern = stripe_kernel<LAYOUT, NR, MASKS, MODE>;
  {
    hipError_t e = set_dynamic_lds(reinterpret_cast<const void*>(kern), (int)kLdsStripe);
    if (e != hipSuccess) return e;
  }
  const int block = ((g.k * g.cpr + 63) / 64) * 64;
  const int64_t slots = stripe_slots();
  const int64_t grid = g.n_tiles < slots ? g.n_tiles : slots;
  hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(block), kLdsStripe, s, a, g);
  return hipGetLastError();
}

template <int LAYOUT, bool MASKS, int MODE>
int launch_nr(const KernelArgs& a, const StripeGeom& g, hipStream_t s) {
  switch (a.n_ranges) {
    case 1: return launch_t<LAYOUT, 1, MASKS, MODE>(a, g, s);
    case 2: return launch_t<LAYOUT, 2, MASKS, MODE>(a, g, s);
    case 3: return launch_t<LAYOUT, 3, MASKS, MODE>(a, g, s);
    case 4: return launch_t<LAYOUT, 4, MASKS, MODE>(a, g, s);
  }
  return hipErrorInvalidValue;
}

template <int LAYOUT, bool MASKS>
int launch_hue(const KernelArgs& a, const StripeGeom& g, hipStream_t s) {
  switch (a.detect_mode) {
    case kDetectSV: return launch_nr<LAYOUT, MASKS, kDetectSV>(a, g, s);
    case kDetectV: return launch_nr<LAYOUT, MASKS, kDetectV>(a, g, s);
  }
  return launch_nr<LAYOUT, MASKS, kDetectFull>(a, g, s);
}

}  // namespace

int launch_stripe(const KernelArgs& a, bool write_masks, hipStream_t s) {
  StripeGeom g;
  if (!geometry(a, g, stripe_slots())) return hipErrorNotSupported;
  const int64_t need = a.layout == TRIK_HSV_LAYOUT_YUYV ? 16 : 8;
  if ((reinterpret_cast<uintptr_t>(a.frames) % need) || (a.frame_stride % need) ||
      (a.line_length % need))
    return hipErrorNotSupported;
  if (g.n_tiles == 0) return hipSuccess;
  if (a.layout == TRIK_HSV_LAYOUT_YUYV)
    return write_masks ? launch_hue<TRIK_HSV_LAYOUT_YUYV, true>(a, g, s)
                       : launch_hue<TRIK_HSV_LAYOUT_YUYV, false>(a, g, s);
  return write_masks ? launch_hue<TRIK_HSV_LAYOUT_OV7670, true>(a, g, s)
                     : launch_hue<TRIK_HSV_LAYOUT_OV7670, false>(a, g, s);
}

}  // namespace trik_hsv
