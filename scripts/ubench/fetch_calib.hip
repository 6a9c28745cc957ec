// Calibration of FETCH_SIZE for the chroma kernel's access pattern (round 5,
// attribute the 82.8 MB of HBM reads above the algorithmic bytes).
// Kernels over the C3 batch size (2,516,582,400 B), 256 workgroups of 1024
// lanes (one per CU, as the chroma kernel), each run 3 times:
//   calib_stream        -- lane-interleaved pairs: each lane reads a 32-B
//                          chunk as two nontemporal 16-B loads (lanes 32 B
//                          apart, so one load instruction covers half of each
//                          of 16 cache lines), two chunks in flight;
//   calib_stage         -- only the LDS-image staging: every workgroup reads
//                          the same 139,264-B table with plain 16-B loads
//                          (8 run chunks + 1 block chunk per lane, as
//                          stage_chroma_image) into LDS;
//   calib_stage_stream  -- both, in that order;
//   calib_rows          -- the chroma kernel's own pattern (VGA geometry): a
//                          workgroup walks 640-lane tiles of 80 16-B columns
//                          x 8 rows, each lane loading its column in row y
//                          and row y + 8 (two nontemporal 16-B loads, lanes
//                          16 B apart: 1 KiB contiguous per instruction), 16
//                          rows per step, the next step's loads in flight.
// rocprofv3 --pmc FETCH_SIZE on this binary gives the per-dispatch counter for
// a known byte count in the same pattern.
// build: hipcc -O3 --offload-arch=gfx950 -o fetch_calib fetch_calib.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

typedef unsigned int u32x4v __attribute__((ext_vector_type(4)));
constexpr int kThreads = 1024;
constexpr int kTableChunks = 139264 / 16;  // 8704 = 8.5 per lane

__device__ __forceinline__ uint32_t stage(const u32x4v* __restrict__ tab) {
  __shared__ u32x4v img[kTableChunks];
  const int t = threadIdx.x;
  u32x4v r[9];
#pragma unroll
  for (int k = 0; k < 9; ++k) {
    const int i = t + kThreads * k;
    r[k] = i < kTableChunks ? tab[i] : u32x4v{0u, 0u, 0u, 0u};
  }
#pragma unroll
  for (int k = 0; k < 9; ++k) {
    const int i = t + kThreads * k;
    if (i < kTableChunks) img[i] = r[k];
  }
  __syncthreads();
  const u32x4v v = img[(t * 37) % kTableChunks];
  return v.x ^ v.w;
}

__device__ __forceinline__ uint32_t stream(const u32x4v* __restrict__ p, size_t n32) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t acc = 0;
  for (; i + stride < n32; i += 2 * stride) {
    const u32x4v* q0 = p + 2 * i;
    const u32x4v* q1 = p + 2 * (i + stride);
    const u32x4v a0 = __builtin_nontemporal_load(q0), b0 = __builtin_nontemporal_load(q0 + 1);
    const u32x4v a1 = __builtin_nontemporal_load(q1), b1 = __builtin_nontemporal_load(q1 + 1);
    acc ^= a0.x + a0.y + a0.z + a0.w + b0.x + b0.y + b0.z + b0.w;
    acc ^= a1.x + a1.y + a1.z + a1.w + b1.x + b1.y + b1.z + b1.w;
  }
  for (; i < n32; i += stride) {
    const u32x4v a = __builtin_nontemporal_load(p + 2 * i), b = __builtin_nontemporal_load(p + 2 * i + 1);
    acc ^= a.x + a.y + a.z + a.w + b.x + b.y + b.z + b.w;
  }
  return acc;
}

__global__ __launch_bounds__(kThreads) void calib_stream(const u32x4v* p, size_t n32, uint32_t* out) {
  const uint32_t acc = stream(p, n32);
  if (acc == 0x12345678u) out[0] = acc;
}

__global__ __launch_bounds__(kThreads) void calib_stage(const u32x4v* tab, uint32_t* out) {
  const uint32_t acc = stage(tab);
  if (acc == 0x12345678u) out[0] = acc;
}

__global__ __launch_bounds__(kThreads) void calib_stage_stream(const u32x4v* tab, const u32x4v* p, size_t n32,
                                                               uint32_t* out) {
  uint32_t acc = stage(tab);
  acc ^= stream(p, n32);
  if (acc == 0x12345678u) out[0] = acc;
}

// the chroma kernel's tile walk at VGA: 1280-B rows, 80 columns of 16 B, 8
// rows per half step, 30 steps per 480-row frame, one tile per frame; the
// 1024-lane workgroup runs 640-lane tiles with lanes 640..1023 idle (the
// kernel's 16 waves pull 10-wave units instead; the bytes and their order
// per instruction are the same)
__global__ __launch_bounds__(kThreads) void calib_rows(const u32x4v* __restrict__ p, int frames, uint32_t* out) {
  const int t = threadIdx.x;
  if (t >= 640) return;
  const int col = t % 80, ro = t / 80;
  uint32_t acc = 0;
  for (int f = blockIdx.x; f < frames; f += gridDim.x) {
    const u32x4v* fr = p + (size_t)f * (480 * 80) + ro * 80 + col;
    u32x4v a = __builtin_nontemporal_load(fr), b = __builtin_nontemporal_load(fr + 8 * 80);
    for (int s = 0; s < 30; ++s) {
      const int sn = s + 1 < 30 ? s + 1 : s;
      const u32x4v na = __builtin_nontemporal_load(fr + sn * 16 * 80);
      const u32x4v nb = __builtin_nontemporal_load(fr + sn * 16 * 80 + 8 * 80);
      acc ^= a.x + a.y + a.z + a.w + b.x + b.y + b.z + b.w;
      a = na;
      b = nb;
    }
  }
  if (acc == 0x12345678u) out[0] = acc;
}

int main() {
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  const size_t bytes = 4096ull * 640 * 480 * 2;
  u32x4v *p, *tab;
  uint32_t* out;
  if (hipMalloc(&p, bytes) || hipMalloc(&tab, 16 * kTableChunks) || hipMalloc(&out, 64)) return 1;
  hipMemset(p, 1, bytes);
  hipMemset(tab, 3, 16 * kTableChunks);
  const size_t n32 = bytes / 32;
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int which = 0; which < 4; ++which)
    for (int r = 0; r < 3; ++r) {
      hipEventRecord(a);
      if (which == 0) hipLaunchKernelGGL(calib_stream, dim3(cus), dim3(kThreads), 0, 0, p, n32, out);
      if (which == 1) hipLaunchKernelGGL(calib_stage, dim3(cus), dim3(kThreads), 0, 0, tab, out);
      if (which == 2) hipLaunchKernelGGL(calib_stage_stream, dim3(cus), dim3(kThreads), 0, 0, tab, p, n32, out);
      if (which == 3) hipLaunchKernelGGL(calib_rows, dim3(cus), dim3(kThreads), 0, 0, p, 4096, out);
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms = 0;
      hipEventElapsedTime(&ms, a, b);
      printf("kernel %d rep %d: %.4f ms\n", which, r, ms);
    }
  printf("stream bytes %zu, staging bytes per workgroup %d, workgroups %d\n", bytes, 16 * kTableChunks, cus);
  return hipDeviceSynchronize() != hipSuccess;
}
