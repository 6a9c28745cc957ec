// trik_hsv_blob.hip -- the ov7670 multi-blob object sensor (SURVEY 8(f) row
// 3).  OSEQ = trik/ov7670/object_sensor/include/internal/
// cv_ball_detector_seqpass.hpp, BMB = .../cv_bitmap_builder_reference.hpp,
// CLU = .../cv_clusterizer_reference.hpp.
//
//  blob_meta_kernel  per-pixel HSV + the sticky range, counted per 4x4
//                    metapixel (BMB:171-190); set when more than 2 of 16
//                    (CLU:185-186).  A lane per (metapixel, row of it): four
//                    lanes sum with two xor-shuffles.
//  blob_ccl_kernel   Clusterizer::run + postProcessing + the target epilogue,
//                    one wave per frame, reproducing the reference's
//                    sequential scan exactly:
//    * labels: a set metapixel takes the smallest non-zero label among left,
//      up-left, up and up-right (CLU:44-52, 70-84), else a new one.  Which
//      metapixels open labels depends only on the bitmap (no set causal
//      neighbour), so new labels are numbered by a prefix sum; along a row,
//      labels are a prefix minimum over runs of set metapixels of the
//      up-row minima -- one segmented min-scan per row across the wave;
//    * statistics: every non-opening set metapixel adds (c, r, 1) to its
//      label (CLU:91-95; the opening one is not counted, CLU:98-112), with
//      one atomic per run of equal labels in a lane -- one 64-bit atomic of
//      the packed (size, sum x, sum y) when the frame's maxima fit 63 bits
//      (VGA: 15 + 21 + 21), else three 32-bit ones;
//    * the bitmap row r + 1 is loaded while row r is labelled;
//    * equivalences: eq[a] = eq[L] for each non-zero neighbour a (equal to
//      the reference's conditional form, CLU:92-96), in raster order; only
//      metapixels with a neighbour label other than L can change anything,
//      and they are replayed serially by the owning lane, lane by lane;
//    * postProcessing (CLU:115-127), in place on the own statistics in
//      ascending chunks of 64 labels: label k ends with its own x, y (size
//      only if eq[k] == k) plus the own sums of every j with eq[j] == k,
//      j != k (eq[j] <= j, so j's sums are its own when it is folded);
//    * the 8 largest by size, ties by label (std::sort's order among equals
//      is unspecified in the reference) -- eight wave-maximum passes over
//      the folded sizes, in LDS when they fit 16 bits -- and OSEQ:563-590's
//      arithmetic.
//  blob_overlay_kernel  guide lines, then a 3x3 red mark per kept target.
#include <hip/hip_runtime.h>

#include <type_traits>

#include "trik_hsv_internal.h"
#include "trik_hsv_pixel.h"
#include "trik_hsv_stripe_px.h"

namespace trik_hsv {

namespace {

using namespace stripe_px;

struct MetaGeom {
  FastDiv per_frame;  // bw * bh
  FastDiv per_row;    // bw
  uint32_t total;     // n_frames * bw * bh
};

// The metapixel flags with the hot kernel's per-pixel arithmetic and its
// StripeTables image (range 0 = the sticky range) staged at LDS address 0:
// four lanes per metapixel (one per pixel row of it, 4 pixels each), 256
// metapixels per 1024-lane workgroup per iteration, grid-stride over all
// metapixels of the batch; two workgroups per CU as stripe_kernel.
__global__ __launch_bounds__(1024) __attribute__((amdgpu_waves_per_eu(8)))
void blob_meta_kernel(BlobArgs a, MetaGeom g) {
  if (gated_out(a.gate, a.gate_max, a.gate_le)) return;
  {
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
    const u32x4* src = reinterpret_cast<const u32x4*>(a.tables);
    typedef __attribute__((address_space(3))) u32x4* lds_u128_wptr;
    lds_u128_wptr dst = (lds_u128_wptr)(uintptr_t)0;
    for (int i = threadIdx.x; i < (int)(sizeof(StripeTables) / 16); i += blockDim.x) dst[i] = src[i];
  }
  __syncthreads();
  const int t = threadIdx.x;
  const uint32_t hue_lane = (uint32_t)offsetof(StripeTables, hue) + ((t % kHueCopies) << 2);
  const uint32_t m43_lane = (uint32_t)offsetof(StripeTables, m43) + ((t % kM43Copies) << 2);
  const int rr = t & 3;
  const uint32_t bw = g.per_row.d;
  const int64_t ll = a.line_length;
  for (uint32_t base = blockIdx.x * 256u; base < g.total; base += gridDim.x * 256u) {
    const uint32_t m = base + (uint32_t)(t >> 2);
    const bool valid = m < g.total;
    uint32_t cnt = 0;
    if (valid) {
      const uint32_t f = fdiv(m, g.per_frame), rem = m - f * g.per_frame.d;
      const uint32_t mr = fdiv(rem, g.per_row), mc = rem - mr * bw;
      const uint8_t* yp = a.frames + (int64_t)f * a.frame_stride + (int64_t)(4 * mr + rr) * ll + 4 * mc;
      const uint8_t* cp = yp + (int64_t)a.height * ll;
      uint32_t yy, cc;
      if (a.aligned4) {
        yy = *reinterpret_cast<const uint32_t*>(yp);
        cc = *reinterpret_cast<const uint32_t*>(cp);
      } else {
        yy = (uint32_t)yp[0] | ((uint32_t)yp[1] << 8) | ((uint32_t)yp[2] << 16) | ((uint32_t)yp[3] << 24);
        cc = (uint32_t)cp[0] | ((uint32_t)cp[1] << 8) | ((uint32_t)cp[2] << 16) | ((uint32_t)cp[3] << 24);
      }
      uint32_t w0, w1;
      ov7670_words(yy, cc, w0, w1);
      Phase1 p[4];
      p[0] = phase1<0>(w0, w0 ^ 0xFF00FF00u, m43_lane);
      p[1] = phase1<1>(w0, w0 ^ 0xFF00FF00u, m43_lane);
      p[2] = phase1<0>(w1, w1 ^ 0xFF00FF00u, m43_lane);
      p[3] = phase1<1>(w1, w1 ^ 0xFF00FF00u, m43_lane);
      uint32_t mm[4], sv[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        mm[j] = lds_u32(p[j].m43_addr);
        sv[j] = lds_u8(p[j].sv_addr);
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) cnt += combine(lds_u32(phase2_addr(mm[j], p[j], hue_lane)), sv[j]) & 1u;
    }
    cnt += __shfl_xor(cnt, 1, 64);
    cnt += __shfl_xor(cnt, 2, 64);
    if (rr == 0 && valid) a.meta[m] = cnt > 2 ? 1 : 0;  // (f, mr, mc) is m itself
  }
}

constexpr uint32_t kInf = 0xFFFFu;

// Inclusive wave scans with DPP (row_shr 1/2/4/8 inside 16-lane rows, then
// row_bcast 15/31 across rows): VALU-latency steps instead of LDS permutes.
// A lane whose source is outside its row (or whose row is masked) reads the
// operator's identity.
template <int CTRL, int ROWS>
__device__ __forceinline__ uint32_t dpp_from(uint32_t identity, uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp((int)identity, (int)v, CTRL, ROWS, 0xF, false);
}
__device__ __forceinline__ uint32_t wave_incl_sum(uint32_t v) {
  v += dpp_from<0x111, 0xF>(0u, v);
  v += dpp_from<0x112, 0xF>(0u, v);
  v += dpp_from<0x114, 0xF>(0u, v);
  v += dpp_from<0x118, 0xF>(0u, v);
  v += dpp_from<0x142, 0xA>(0u, v);
  v += dpp_from<0x143, 0xC>(0u, v);
  return v;
}
// segmented minimum over (break, min) pairs: (b1, m1) then (b2, m2) combine to
// (b1 | b2, b2 ? m2 : min(m1, m2))
template <int CTRL, int ROWS>
__device__ __forceinline__ void seg_step(uint32_t& b, uint32_t& m) {
  const uint32_t tb = dpp_from<CTRL, ROWS>(0u, b), tm = dpp_from<CTRL, ROWS>(kInf, m);
  m = b ? m : min(tm, m);
  b |= tb;
}
__device__ __forceinline__ void wave_incl_segmin(uint32_t& b, uint32_t& m) {
  seg_step<0x111, 0xF>(b, m);
  seg_step<0x112, 0xF>(b, m);
  seg_step<0x114, 0xF>(b, m);
  seg_step<0x118, 0xF>(b, m);
  seg_step<0x142, 0xA>(b, m);
  seg_step<0x143, 0xC>(b, m);
}

// lane l gets lane l - 1's v (lane 0: first); lane l gets lane l + 1's v
// (lane 63: 0) -- DPP wave shifts (wave_shr:1 / wave_shl:1), no LDS permute
__device__ __forceinline__ uint32_t from_prev_lane(uint32_t v, uint32_t first) {
  return (uint32_t)__builtin_amdgcn_update_dpp((int)first, (int)v, 0x138, 0xF, 0xF, false);
}
__device__ __forceinline__ uint32_t from_next_lane(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x130, 0xF, 0xF, false);
}

__device__ __forceinline__ uint64_t wave_max_u64(uint64_t v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const uint64_t o = __shfl_xor(v, off, 64);
    v = o > v ? o : v;
  }
  return v;
}

// OSEQ:563-590 for one cluster: kept when the size percentage exceeds 4;
// (x, y) = the mark's source point (getX/getY, CLU:139-147).
__device__ __forceinline__ bool blob_target(int32_t size, int32_t sx, int32_t sy, int bw, int bh, int& pct,
                                            int32_t& x, int32_t& y) {
  const int root = (int)__fsqrt_rn((float)(uint16_t)size);  // getSize() is uint16_t
  const uint32_t radius = (uint32_t)ceilf(__fdiv_rn((float)root, 3.1415927f));
  pct = (int)((radius * 100u * 4u) / (uint32_t)(bw + bh));
  if (pct <= 4) return false;
  x = (sx / (size + 1)) * 4;
  y = (sy / (size + 1)) * 4;
  return true;
}

// Register form: lane l owns columns c0 = l*K .. c0+K-1 (K <= KMAX) and keeps
// their set flags, up-row minima and the labels of rows r-1 / r in registers
// (fully unrolled loops over KMAX with a j < K guard; EXACT: K == KMAX, the
// guards fold away -- VGA's 160 metapixel columns are K = 3); the boundary
// values of the neighbouring lanes come by one-lane shifts.  LDS holds eq
// (and the staged bitmap).
template <int KMAX, bool EXACT, bool STAGED>
__global__ __launch_bounds__(64) void blob_ccl_kernel(BlobArgs a) {
  extern __shared__ uint16_t smem[];
  const int f = blockIdx.x, lane = threadIdx.x;
  const int bw = a.width >> 2, bh = a.height >> 2;
  const int ml = a.max_labels;
  uint16_t* eq = smem;  // [ml]
  // the frame's bitmap: staged in LDS when it fits (bw*bh is a multiple of 8)
  if (STAGED) {
    uint32_t* dst = reinterpret_cast<uint32_t*>(eq + ((ml + 1) & ~1));
    const uint32_t* src = reinterpret_cast<const uint32_t*>(a.meta + (int64_t)f * bw * bh);
    for (int i = lane; i < bw * bh / 4; i += 64) dst[i] = src[i];
    __syncthreads();
  }
  // own statistics (zeroed by the launcher; folded in place at the end):
  // packed, own64[k] = size | x << pack_sx | y << pack_sy; else
  // own[3k + {0,1,2}] = x, y, size
  int32_t* own = a.stats + (int64_t)f * 3 * ml;
  unsigned long long* own64 = reinterpret_cast<unsigned long long*>(a.stats) + (int64_t)f * ml;
  const bool packed = a.pack_sx != 0;
  auto add_own = [&](uint32_t L, int32_t x, int32_t y, int32_t n) {
    if (packed) {
      atomicAdd(own64 + L, (unsigned long long)(uint32_t)n | ((unsigned long long)(uint32_t)x << a.pack_sx) |
                               ((unsigned long long)(uint32_t)y << a.pack_sy));
    } else {
      atomicAdd(&own[3 * L], x);
      atomicAdd(&own[3 * L + 1], y);
      atomicAdd(&own[3 * L + 2], n);
    }
  };
  // subtract size sz from label k's own size (the field holds at least sz:
  // no borrow into the packed x field)
  auto sub_own_size = [&](uint32_t k, int32_t sz) {
    if (packed) atomicAdd(own64 + k, (unsigned long long)(-(long long)sz));
    else atomicAdd(&own[3 * k + 2], -sz);
  };
  auto get_own = [&](int k, int32_t& x, int32_t& y, int32_t& n) {
    if (packed) {
      const unsigned long long v = own64[k];
      n = (int32_t)(v & ((1ull << a.pack_sx) - 1ull));
      x = (int32_t)((v >> a.pack_sx) & ((1ull << (a.pack_sy - a.pack_sx)) - 1ull));
      y = (int32_t)(v >> a.pack_sy);
    } else {
      x = own[3 * k];
      y = own[3 * k + 1];
      n = own[3 * k + 2];
    }
  };
  uint16_t* labels = a.labels ? a.labels + (int64_t)f * bw * bh : nullptr;

  const int K = EXACT ? KMAX : (bw + 63) / 64;
  const int c0 = lane * K;
  uint32_t prv[KMAX], cur[KMAX], dd[KMAX], up[KMAX];
#pragma unroll
  for (int j = 0; j < KMAX; ++j) prv[j] = 0;
  if (lane == 0) eq[0] = 0;
  // The bitmap rows come in batches of RB: batch b + 1's loads are in flight
  // while batch b is labelled, and the wait for them comes once per batch.
  // (Each wait is a full drain: the label stores and statistics atomics issued
  // since are memory operations of another kind.  Waiting per row exposed a
  // memory latency on every row, all of it on the empty rows of camera-like
  // frames.)  bt: the current batch, row r's columns first (shifted up a row
  // per row); pf: the next batch.  Loads take clamped columns and rows (no
  // branches); columns past the row are masked when a batch is taken.
  constexpr int RB = KMAX <= 5 ? 8 : 1;
  uint32_t pf[RB][KMAX], bt[KMAX];  // bt: the current batch as bits (bit i = its row i), shifted a row per row
  // (LDS-staged or global: separate paths, so that neither is a flat load --
  // a flat load in flight would hold every LDS wait of the row too)
  // (the staged copy at its LDS offset: the dynamic LDS starts at 0)
  typedef const __attribute__((address_space(3))) uint8_t* lds_u8_ptr;
  typedef const __attribute__((address_space(1))) uint8_t* glb_u8_ptr;
  const lds_u8_ptr meta_l = (lds_u8_ptr)(uintptr_t)(2u * (uint32_t)((ml + 1) & ~1));
  const glb_u8_ptr meta_g = (glb_u8_ptr)(a.meta + (int64_t)f * bw * bh);
  uint32_t colc[KMAX];  // the lane's columns, clamped into the row
#pragma unroll
  for (int j = 0; j < KMAX; ++j) colc[j] = (uint32_t)min(c0 + j, bw - 1);
  auto load_batch = [&](int r0) {
#pragma unroll
    for (int i = 0; i < RB; ++i) {
      const int rr = min(r0 + i, bh - 1);  // (wave-uniform: a scalar row base, the column as the offset)
#pragma unroll
      for (int j = 0; j < KMAX; ++j)
        pf[i][j] = STAGED ? meta_l[(uint32_t)(rr * bw) + colc[j]] : (meta_g + (int64_t)rr * bw)[colc[j]];
    }
  };
  if (bh > 0) load_batch(0);
  int next = 1;  // next new label (wave-uniform)
  // the lane's statistics run: label acc_l's (x, y, size) so far, added to
  // the label's sums when the lane meets another label (in its columns, row
  // after row) and at the end -- a blob's columns keep their label for many
  // rows, so a lane adds once per blob, not once per row (the adds in flight
  // sit in every row batch's memory wait)
  uint32_t acc_l = 0;
  int32_t ax = 0, ay = 0, an = 0;
  for (int r = 0; r < bh; ++r) {
    if (r % RB == 0) {  // take the batch in flight, start the next one
#pragma unroll
      for (int j = 0; j < KMAX; ++j) {
        uint32_t v = 0;
#pragma unroll
        for (int i = 0; i < RB; ++i) v |= (pf[i][j] & 1u) << i;
        bt[j] = (j < K && c0 + j < bw) ? v : 0u;
      }
      load_batch(r + RB);  // (unconditional: past the last row it re-reads it; a branch here
                           // made the compiler copy, and so wait for, the new loads)
    }
    uint32_t prev_last = 0, d_last = 0;
#pragma unroll
    for (int j = 0; j < KMAX; ++j) {
      dd[j] = bt[j] & 1u;
      bt[j] >>= 1;
      if (j == K - 1) {
        prev_last = prv[j];
        d_last = dd[j];
      }
    }
    // a row without a set metapixel opens, joins and counts nothing (CLU:98-112
    // only acts on set ones): its labels are 0 -- skip the scans (camera-like
    // frames are mostly such rows)
    {
      uint32_t any = 0;
#pragma unroll
      for (int j = 0; j < KMAX; ++j) any |= dd[j];
      if (__builtin_amdgcn_ballot_w64(any != 0u) == 0ull) {
#pragma unroll
        for (int j = 0; j < KMAX; ++j) {
          if (labels && j < K && c0 + j < bw) labels[(int64_t)r * bw + c0 + j] = 0;
          prv[j] = 0;
        }
        continue;
      }
    }
    // the neighbours' boundary columns (CLU:70-84 reads c-1 and c+1)
    const uint32_t l_prev = from_prev_lane(prev_last, 0u), l_d = from_prev_lane(d_last, 0u);
    const uint32_t r_prev = from_next_lane(prv[0]);
    // up-row minima of the set metapixels; opening ones (no set causal neighbour)
    uint32_t nseed = 0;
    {
      uint32_t left = l_d;
#pragma unroll
      for (int j = 0; j < KMAX; ++j) {
        const uint32_t pl = j == 0 ? l_prev : prv[j > 0 ? j - 1 : 0];
        const uint32_t pr = j + 1 < K ? prv[j + 1 < KMAX ? j + 1 : j] : r_prev;
        uint32_t u = kInf;
        if (dd[j] && r > 0) {
          if (pl) u = pl;
          if (prv[j] && prv[j] < u) u = prv[j];
          if (pr && pr < u) u = pr;
        }
        up[j] = u;
        if (j < K && dd[j] && !left && u == kInf) ++nseed;
        left = dd[j];
      }
    }
    // new labels in raster order: exclusive prefix sum of the lanes' counts
    const uint32_t incl = wave_incl_sum(nseed);
    const uint32_t total = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
    const uint32_t label_next = (uint32_t)next + incl - nseed;
    // segmented min-scan over runs of set metapixels: this lane's summary is
    // (the chunk holds an unset one, the minimum after the last unset one)
    uint32_t cb = 0, cm = kInf;
    {
      uint32_t lbl = label_next, left = l_d;
#pragma unroll
      for (int j = 0; j < KMAX; ++j) {
        if (j < K) {
          if (!dd[j]) {
            cb = 1;
            cm = kInf;
          } else {
            const bool open = !left && up[j] == kInf;
            cm = min(cm, open ? lbl++ : up[j]);
          }
        }
        left = dd[j];
      }
    }
    wave_incl_segmin(cb, cm);
    const uint32_t carry = from_prev_lane(cm, kInf);  // exclusive: lanes before this one
    // labels; open the new labels (eq[L] = L)
    uint32_t seeds = 0, cur_last = 0;
    {
      uint32_t lbl = label_next, run = carry, left = l_d;
#pragma unroll
      for (int j = 0; j < KMAX; ++j) {
        if (!dd[j]) {
          run = kInf;
          cur[j] = 0;
        } else if (!left && up[j] == kInf) {  // CLU:98-112
          eq[lbl] = (uint16_t)lbl;
          seeds |= 1u << j;
          run = lbl++;
          cur[j] = run;
        } else {
          run = min(run, up[j]);
          cur[j] = run;
        }
        left = dd[j];
        if (j == K - 1) cur_last = cur[j];
      }
    }
    next += (int)total;
    const uint32_t l_cur = from_prev_lane(cur_last, 0u);
    // statistics of the non-opening metapixels, one atomic per run of equal
    // labels; equivalence events flagged
    uint32_t events = 0;  // bit j: column c0 + j has a neighbour label != L
    {
#pragma unroll
      for (int j = 0; j < KMAX; ++j) {
        const uint32_t L = cur[j];
        if (L && !((seeds >> j) & 1u)) {
          if (L != acc_l) {
            if (an) add_own(acc_l, ax, ay, an);
            acc_l = L;
            ax = ay = an = 0;
          }
          ax += c0 + j;
          ay += r;
          ++an;
          const uint32_t n0 = j == 0 ? l_cur : cur[j > 0 ? j - 1 : 0];
          const uint32_t n1 = j == 0 ? l_prev : prv[j > 0 ? j - 1 : 0];
          const uint32_t n2 = prv[j];
          const uint32_t n3 = j + 1 < K ? prv[j + 1 < KMAX ? j + 1 : j] : r_prev;
          if ((n0 && n0 != L) || (n1 && n1 != L) || (n2 && n2 != L) || (n3 && n3 != L)) events |= 1u << j;
        }
        if (labels && j < K && c0 + j < bw) labels[(int64_t)r * bw + c0 + j] = (uint16_t)L;
      }
    }
    // equivalence events in raster order: lane by lane, each lane in column
    // order (CLU:92-96 as eq[a] = eq[L] for every non-zero neighbour a)
    uint64_t pending = __ballot(events != 0);
    while (pending) {
      const int l = __ffsll((unsigned long long)pending) - 1;
      pending &= pending - 1;
      if (lane == l) {
#pragma unroll
        for (int j = 0; j < KMAX; ++j) {
          if (!((events >> j) & 1u)) continue;
          const uint16_t e = eq[cur[j]];
          const uint32_t nb[4] = {j == 0 ? l_cur : cur[j > 0 ? j - 1 : 0],
                                  j == 0 ? l_prev : prv[j > 0 ? j - 1 : 0], prv[j],
                                  j + 1 < K ? prv[j + 1 < KMAX ? j + 1 : j] : r_prev};
          // (unconditional: an absent neighbour (0) writes eq[0], which no
          // scan step reads -- the writes go back to back, no branch and no
          // wait between them)
#pragma unroll
          for (int i = 0; i < 4; ++i) eq[nb[i]] = e;
        }
      }
      __builtin_amdgcn_wave_barrier();
    }
#pragma unroll
    for (int j = 0; j < KMAX; ++j) prv[j] = cur[j];
  }
  if (an) add_own(acc_l, ax, ay, an);
  __threadfence();
  __syncthreads();
  const int n = next;
  // postProcessing (CLU:115-127) in place, in ascending chunks of 64 labels:
  // a label k with eq[k] != k adds its own (x, y, size) to eq[k] and keeps x
  // and y with size 0.  CLU forwards what k holds when its turn comes, which
  // is its own sums: every label that adds into k (eq[j] == k) is higher
  // (eq[j] <= j), so it lies in k's chunk -- whose reads all precede its
  // adds -- or in a later one.
  for (int k0 = 0; k0 < n; k0 += 64) {
    const int k = k0 + lane;
    int32_t x = 0, y = 0, sz = 0;
    int e = 0;
    const bool live = k < n && k != 0;
    if (live) {
      e = eq[k];
      get_own(k, x, y, sz);
    }
    if (live && e != k) {
      add_own((uint32_t)e, x, y, sz);
      sub_own_size((uint32_t)k, sz);
    }
  }
  // the adds performed (at L2) before the reads below; the L1 invalidated
  __threadfence();
  __syncthreads();
  // the 8 largest (size desc, label asc): key = size << 32 | ~label (unique,
  // never 0), eight passes over the labels, each a wave maximum below the
  // last one.  When every size fits 16 bits the folded sizes are first copied
  // into LDS over eq (dead after the fold), so the passes read LDS, not
  // memory.
  const bool lds_sizes = bw * bh < 65536;
  if (lds_sizes) {
#pragma unroll 4
    for (int k = lane; k < n; k += 64) {
      int32_t x, y, sz;
      get_own(k, x, y, sz);
      eq[k] = (uint16_t)sz;
    }
    __syncthreads();
  }
  auto size_of = [&](int k) -> uint32_t {
    if (lds_sizes) return eq[k];
    int32_t x, y, sz;
    get_own(k, x, y, sz);
    return (uint32_t)sz;
  };
  uint64_t last = ~0ull;
  int32_t* top = a.top + (int64_t)f * 24;
  TrikHsvTarget* tg = a.targets + (int64_t)f * 8;
  for (int i = 0; i < 8; ++i) {
    uint64_t best = 0;
#pragma unroll 4
    for (int k = lane; k < n; k += 64) {
      const uint64_t key = ((uint64_t)size_of(k) << 32) | (uint32_t)(0xFFFFFFFFu - (uint32_t)k);
      best = key < last && key > best ? key : best;
    }
    best = wave_max_u64(best);
    last = best;
    if (lane == 0) {
      int32_t size = 0, sx = 0, sy = 0;
      if (best) {
        get_own((int)(0xFFFFFFFFu - (uint32_t)best), sx, sy, size);
      }
      top[3 * i] = size;
      top[3 * i + 1] = sx;
      top[3 * i + 2] = sy;
      TrikHsvTarget t = {0, 0, 0, 0};
      int pct;
      int32_t x, y;
      if (best && blob_target(size, sx, sy, bw, bh, pct, x, y)) {  // OSEQ:574-583
        t.size = (uint8_t)pct;
        t.x = (int8_t)(((x - a.width / 2) * 100 * 2) / a.width);
        t.y = (int8_t)(((y - a.height / 2) * 100 * 2) / a.height);
      }
      tg[i] = t;
    }
  }
  if (lane == 0 && a.n_labels) a.n_labels[f] = n;
  // leave the own statistics zero for the next launch: this frame used labels
  // 1 .. n - 1 only (every read of them above has returned: lane 0's last
  // reads fed the stores before this loop), so zeroing those restores the
  // all-zero buffer launch_blob relies on -- no memset of all max_labels
  // slots per frame (157 MB for 4096 VGA frames) before every batch
  for (int k = lane; k < n; k += 64) {
    if (packed) own64[k] = 0ull;
    else own[3 * k] = own[3 * k + 1] = own[3 * k + 2] = 0;
  }
}

template <bool LDSMAP>
__global__ __launch_bounds__(64) void blob_overlay_kernel(PreviewArgs a, const int32_t* top) {
  extern __shared__ uint32_t smaps[];
  const int f = blockIdx.x, lane = threadIdx.x;
  const Canvas cv = stage_canvas<LDSMAP>(smaps, a.previews + (int64_t)f * a.preview_stride, a.out_ll, a.width,
                                         a.height, a.wi2wo, a.hi2ho, lane);
  draw_guides(cv, lane, 64);  // OSEQ:548-561
  __syncthreads();
  // drawFatPixel (OSEQ:92-108) per kept target, in target order: lane 9*i + j
  // draws point j of target i; marks may overlap, so targets go in order
  const int32_t* t = top + (int64_t)f * 24;
  const int bw = a.width >> 2, bh = a.height >> 2;
  for (int i = 0; i < 8; ++i) {
    int pct;
    int32_t x, y;
    if (blob_target(t[3 * i], t[3 * i + 1], t[3 * i + 2], bw, bh, pct, x, y) && lane < 9)
      cv.px(x + lane / 3 - 1, y + lane % 3 - 1, 0xff0000);
    __syncthreads();
  }
}

}  // namespace

int launch_blob(const BlobArgs& a, hipStream_t s) {
  if (a.n_frames <= 0 || a.width <= 0 || a.height <= 0) return hipSuccess;
  const int bw = a.width >> 2, bh = a.height >> 2;
  if (bw > 64 * 32) return hipErrorInvalidValue;  // events mask: 32 columns per lane
  // own statistics: one packed u64 per label when the frame's maxima (size
  // <= bw*bh, sum x <= bh*bw(bw-1)/2, sum y <= bw*bh(bh-1)/2) fit 63 bits
  BlobArgs b = a;
  {
    auto bits = [](uint64_t v) {
      int n = 0;
      while (n < 64 && (v >> n)) ++n;
      return n;
    };
    const uint64_t w = (uint64_t)bw, h = (uint64_t)bh;
    const int bn = bits(w * h), bx = bits(h * w * (w ? w - 1 : 0) / 2), by = bits(w * h * (h ? h - 1 : 0) / 2);
    b.pack_sx = b.pack_sy = 0;
    if (bn > 0 && bn + bx + by <= 63) {
      b.pack_sx = bn;
      b.pack_sy = bn + bx;
    }
  }
  // own statistics start at zero (at the front of stats): the buffer is
  // zeroed when it is allocated (ensure_blob_scratch) and every clusterer
  // launch zeroes the labels it used before it ends
  const int64_t total = (int64_t)a.n_frames * bw * bh;
  if (total >= (1ll << 31) || !a.tables) return hipErrorInvalidValue;
  {
    hipError_t e = set_dynamic_lds(reinterpret_cast<const void*>(blob_meta_kernel), (int)sizeof(StripeTables));
    if (e != hipSuccess) return e;
  }
  const int cus = device_cus();
  if (total > 0 && !a.meta_ready) {
    MetaGeom g;
    g.per_frame = make_div((uint32_t)(bw * bh));
    g.per_row = make_div((uint32_t)bw);
    g.total = (uint32_t)total;
    const int64_t chunks = (total + 255) / 256, slots = 2LL * cus;
    hipLaunchKernelGGL(blob_meta_kernel, dim3((unsigned)(chunks < slots ? chunks : slots)), dim3(1024),
                       sizeof(StripeTables), s, a, g);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  size_t lds = sizeof(uint16_t) * (size_t)((a.max_labels + 1) & ~1);
  if (lds > 64 * 1024) return hipErrorInvalidValue;
  // the frame's bitmap staged in LDS when it fits and the batch is small
  // (latency); large batches read it from L2 instead, so that the eq table
  // alone bounds the residency (VGA: 16 frames per CU instead of 5; 4096
  // frames 1.59 -> 1.30 ms with the chroma-run bitmap kernel)
  b.meta_lds = a.n_frames < 2 * cus && lds + (size_t)bw * bh <= 40 * 1024 ? 1 : 0;
  if (b.meta_lds) lds += (size_t)bw * bh;
  const int K = (bw + 63) / 64;
  auto pick = [&](auto staged) {
    constexpr bool S = decltype(staged)::value;
    return K == 1 ? blob_ccl_kernel<1, true, S> : K == 2 ? blob_ccl_kernel<2, true, S>
         : K == 3 ? blob_ccl_kernel<3, true, S> : K == 4 ? blob_ccl_kernel<4, true, S>
         : K == 5 ? blob_ccl_kernel<5, true, S> : K <= 8 ? blob_ccl_kernel<8, false, S>
         : K <= 16 ? blob_ccl_kernel<16, false, S> : blob_ccl_kernel<32, false, S>;
  };
  auto kern = b.meta_lds ? pick(std::true_type{}) : pick(std::false_type{});
  hipLaunchKernelGGL(kern, dim3((unsigned)a.n_frames), dim3(64), lds, s, b);
  return hipGetLastError();
}

int launch_blob_overlay(const PreviewArgs& a, const int32_t* top, hipStream_t s) {
  if (a.n_frames <= 0 || a.width <= 0 || a.height <= 0) return hipSuccess;
  const size_t map_bytes = sizeof(uint32_t) * ((size_t)a.width + (size_t)a.height);
  if (map_bytes <= kMapLdsBytes)
    hipLaunchKernelGGL(blob_overlay_kernel<true>, dim3((unsigned)a.n_frames), dim3(64), map_bytes, s, a, top);
  else
    hipLaunchKernelGGL(blob_overlay_kernel<false>, dim3((unsigned)a.n_frames), dim3(64), 0, s, a, top);
  return hipGetLastError();
}

}  // namespace trik_hsv
