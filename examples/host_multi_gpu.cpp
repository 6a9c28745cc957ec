// host_multi_gpu.cpp -- a C++ host driving several GPUs through the C ABI's
// multi-GPU layer (include/trik_hsv.h, Layer 3): a batch of frames is split
// by frame index over the devices, each device's shard stays in its own HBM,
// and the per-target totals are summed with one RCCL all-reduce
// (trik_hsv_group_process).  One host worker thread and one stream per
// device live inside the group; this program only allocates, fills and
// checks.
//
// usage: host_multi_gpu [TOTAL_FRAMES [WIDTH [HEIGHT [ITERS [N_DEVICES]]]]]
//   defaults 4096 640 480 20 (all visible devices); 4 ranges (bench.py's).
// Prints one JSON line: devices, frames, ms per batch (host clock around
// ITERS back-to-back group calls + sync), Mpix/s, the totals, and "ok": the
// totals equal on every device and equal to the sum of all per-frame sums.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <chrono>
#include <vector>

#include "trik_hsv.h"

#define CK(x)                                                                         \
  do {                                                                                \
    hipError_t e_ = (x);                                                              \
    if (e_ != hipSuccess) {                                                           \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      return 2;                                                                       \
    }                                                                                 \
  } while (0)
#define TK(x)                                                                         \
  do {                                                                                \
    int32_t r_ = (x);                                                                 \
    if (r_ != 0) {                                                                    \
      fprintf(stderr, "%s failed (%d): %s\n", #x, (int)r_, trik_hsv_last_error());    \
      return 3;                                                                       \
    }                                                                                 \
  } while (0)

int main(int argc, char** argv) {
  const int total = argc > 1 ? atoi(argv[1]) : 4096;
  const int w = argc > 2 ? atoi(argv[2]) : 640;
  const int h = argc > 3 ? atoi(argv[3]) : 480;
  const int iters = argc > 4 ? atoi(argv[4]) : 20;
  int n_dev = 0;
  CK(hipGetDeviceCount(&n_dev));
  if (argc > 5 && atoi(argv[5]) < n_dev) n_dev = atoi(argv[5]);
  if (n_dev < 1 || total < 0 || iters < 1) {
    fprintf(stderr, "need a GPU, TOTAL_FRAMES >= 0, ITERS >= 1\n");
    return 2;
  }
  const int T = 4, ll = 2 * w;
  const int64_t fb = (int64_t)h * ll;
  TRIK_VIDTRANSCODE_CV_InArgsAlg ranges[T] = {{0, 30, 50, 100, 30, 100, 0},
                                              {90, 150, 40, 100, 20, 100, 0},
                                              {200, 260, 40, 100, 20, 100, 0},
                                              {330, 20, 30, 100, 30, 100, 0}};
  std::vector<int32_t> devs(n_dev);
  std::vector<TrikHsvFrameBatch> batches(n_dev);
  std::vector<uint8_t*> frames(n_dev);
  std::vector<TrikHsvTargetSums*> sums(n_dev), totals(n_dev);
  std::vector<TrikHsvTarget*> targets(n_dev);
  for (int d = 0; d < n_dev; ++d) {
    devs[d] = d;
    // frame shard: contiguous, sizes differ by at most one (trik_hsv.shard.frame_shard)
    const int lo = (int)((int64_t)total * d / n_dev), hi = (int)((int64_t)total * (d + 1) / n_dev);
    const int n = hi - lo;
    CK(hipSetDevice(d));
    CK(hipMalloc(&frames[d], (size_t)(n > 0 ? n : 1) * fb));
    CK(hipMalloc(&sums[d], sizeof(TrikHsvTargetSums) * (size_t)(n > 0 ? n : 1) * T));
    CK(hipMalloc(&targets[d], sizeof(TrikHsvTarget) * (size_t)(n > 0 ? n : 1) * T));
    CK(hipMalloc(&totals[d], sizeof(TrikHsvTargetSums) * T));
    batches[d] = TrikHsvFrameBatch{frames[d], fb, n, w, h, ll, TRIK_HSV_LAYOUT_YUYV};
    TK(trik_hsv_synth(&batches[d], lo, 0, 0x7A1C, nullptr));  // global frame index lo + i
    CK(hipDeviceSynchronize());
  }
  TRIK_HSV_GroupHandle g = nullptr;
  TK(trik_hsv_group_create(n_dev, devs.data(), &g));
  // one warm-up batch (tables compiled and built), then ITERS timed batches
  TK(trik_hsv_group_process(g, batches.data(), ranges, T, sums.data(), targets.data(), totals.data()));
  TK(trik_hsv_group_sync(g));
  const auto t0 = std::chrono::steady_clock::now();
  for (int i = 0; i < iters; ++i)
    TK(trik_hsv_group_process(g, batches.data(), ranges, T, sums.data(), targets.data(), totals.data()));
  TK(trik_hsv_group_sync(g));
  const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count() / iters;

  // check: every device holds the same totals, equal to the sum of all frames' sums
  std::vector<long long> want(3 * T, 0), got0(3 * T, 0);
  bool ok = true;
  for (int d = 0; d < n_dev; ++d) {
    CK(hipSetDevice(d));
    const int n = batches[d].n_frames;
    std::vector<TrikHsvTargetSums> s((size_t)(n > 0 ? n : 0) * T), t(T);
    if (n > 0) CK(hipMemcpy(s.data(), sums[d], sizeof(TrikHsvTargetSums) * s.size(), hipMemcpyDeviceToHost));
    CK(hipMemcpy(t.data(), totals[d], sizeof(TrikHsvTargetSums) * T, hipMemcpyDeviceToHost));
    for (size_t k = 0; k < s.size(); ++k) {
      want[3 * (k % T) + 0] += s[k].points;
      want[3 * (k % T) + 1] += s[k].sum_x;
      want[3 * (k % T) + 2] += s[k].sum_y;
    }
    for (int r = 0; r < T; ++r) {
      const long long v[3] = {(long long)t[r].points, (long long)t[r].sum_x, (long long)t[r].sum_y};
      for (int c = 0; c < 3; ++c) {
        if (d == 0) got0[3 * r + c] = v[c];
        else ok = ok && got0[3 * r + c] == v[c];
      }
    }
  }
  ok = ok && want == got0;
  printf("{\"devices\": %d, \"frames\": %d, \"width\": %d, \"height\": %d, \"ms_per_batch\": %.4f, "
         "\"mpix_per_s\": %.1f, \"ok\": %s, \"totals\": [",
         n_dev, total, w, h, ms, (double)total * w * h / (ms * 1e-3) / 1e6, ok ? "true" : "false");
  for (int k = 0; k < 3 * T; ++k) printf("%s%lld", k ? ", " : "", got0[k]);
  printf("]}\n");
  TK(trik_hsv_group_delete(g));
  for (int d = 0; d < n_dev; ++d) {
    CK(hipSetDevice(d));
    CK(hipFree(frames[d]));
    CK(hipFree(sums[d]));
    CK(hipFree(targets[d]));
    CK(hipFree(totals[d]));
  }
  return ok ? 0 : 1;
}
