// Microbenchmark (development): the 2:1 preview's memory pattern alone --
// 4096 VGA YUYV frames, every other source row read (1280 B), 320x240x2 B
// written per frame -- in two lane mappings, no pixel arithmetic:
//   pairs:     lane = one 8-pixel output unit: its 32 source bytes as two
//              16-B loads (lanes 32 B apart, as preview_rows2_kernel), one
//              16-B store;
//   coalesced: the 64 lanes of a wave take 128 consecutive 16-B source pieces
//              (4 output pixels each), lane l pieces l and l + 64 (lanes 16 B
//              apart: 1 KiB contiguous per load instruction), two 8-B stores.
// build: hipcc -O3 --offload-arch=gfx950 -o preview_pattern preview_pattern.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

typedef unsigned int v4 __attribute__((ext_vector_type(4)));
typedef unsigned int v2 __attribute__((ext_vector_type(2)));
constexpr int W = 640, H = 480, LL = 1280, OW = 320, OH = 240, PPR = LL / 16;  // 80 pieces per row
constexpr int UNITS_ROW = OW / 8;                                               // 40 units per output row

__device__ __forceinline__ uint32_t fold(v4 a) { return a.x ^ (a.y << 1) ^ (a.z << 2) ^ (a.w << 3); }

__global__ __launch_bounds__(1024) void pv_pairs(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst,
                                                 int frames) {
  const uint32_t total = (uint32_t)frames * OH * UNITS_ROW;
  for (uint32_t u = blockIdx.x * blockDim.x + threadIdx.x; u < total; u += gridDim.x * blockDim.x) {
    const uint32_t f = u / (OH * UNITS_ROW), rem = u % (OH * UNITS_ROW), r = rem / UNITS_ROW, q = rem % UNITS_ROW;
    const uint8_t* p = src + (size_t)f * H * LL + (size_t)(2 * r + 1) * LL + 32 * q;
    const v4 a = __builtin_nontemporal_load(reinterpret_cast<const v4*>(p));
    const v4 b = __builtin_nontemporal_load(reinterpret_cast<const v4*>(p + 16));
    v4 o = {fold(a), fold(b), a.x ^ b.y, a.z ^ b.w};
    *reinterpret_cast<v4*>(dst + (size_t)f * OH * OW * 2 + (size_t)r * OW * 2 + 16 * q) = o;
  }
}

__global__ __launch_bounds__(1024) void pv_coalesced(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst,
                                                     int frames) {
  constexpr uint32_t PF = OH * PPR;  // pieces per frame (19200 = 150 x 128)
  const uint32_t total = (uint32_t)frames * PF;
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6, waves = gridDim.x * blockDim.x / 64;
  for (uint32_t blk = wave * 128; blk < total; blk += waves * 128) {
    uint32_t j[2] = {blk + lane, blk + 64 + lane};
    v4 a[2];
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const uint32_t f = j[k] / PF, rem = j[k] % PF, r = rem / PPR, c = rem % PPR;
      a[k] = __builtin_nontemporal_load(
          reinterpret_cast<const v4*>(src + (size_t)f * H * LL + (size_t)(2 * r + 1) * LL + 16 * c));
    }
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const uint32_t f = j[k] / PF, rem = j[k] % PF;
      v2 o = {fold(a[k]), a[k].x ^ a[k].w};
      *reinterpret_cast<v2*>(dst + (size_t)f * OH * OW * 2 + 8 * (size_t)rem) = o;
    }
  }
}

template <typename K>
void run(const char* name, K k, const uint8_t* s, uint8_t* d, int frames, int cus) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int per_cu : {1, 2, 4}) {
    const int grid = cus * per_cu;
    for (int w = 0; w < 2; ++w) hipLaunchKernelGGL(k, dim3(grid), dim3(1024), 0, 0, s, d, frames);
    float best = 1e9;
    for (int r = 0; r < 5; ++r) {
      hipEventRecord(a);
      hipLaunchKernelGGL(k, dim3(grid), dim3(1024), 0, 0, s, d, frames);
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms;
      hipEventElapsedTime(&ms, a, b);
      if (ms < best) best = ms;
    }
    const double bytes = (double)frames * (H / 2 * LL + OH * OW * 2);
    printf("%-10s wg/CU=%d: %.4f ms  %.0f GB/s (%.1f %% of 8 TB/s)\n", name, per_cu, best, bytes / best / 1e6,
           bytes / best / 1e6 / 80.0);
  }
}

int main() {
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  const int frames = 4096;
  uint8_t *s, *d;
  if (hipMalloc(&s, (size_t)frames * H * LL) || hipMalloc(&d, (size_t)frames * OH * OW * 2)) return 1;
  hipMemset(s, 7, (size_t)frames * H * LL);
  run("pairs", pv_pairs, s, d, frames, cus);
  run("coalesced", pv_coalesced, s, d, frames, cus);
  run("pairs", pv_pairs, s, d, frames, cus);
  run("coalesced", pv_coalesced, s, d, frames, cus);
  return hipDeviceSynchronize() != hipSuccess;
}
