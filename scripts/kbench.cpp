// kbench -- development A/B timer for libtrik_hsv.so variants (no torch).
//
// Loads each library given on the command line (dlopen, RTLD_LOCAL), fills one
// device batch with the library's own synthetic-frame generator (first library),
// and times trik_hsv_batch_sums with HIP events on one stream, interleaving the
// variants round by round.  Every variant's sums are compared with the first
// variant's (bit for bit).  Development only: not part of the product or tests.
//
// build: hipcc -O2 -std=c++17 --offload-arch=gfx950 -o scripts/kbench scripts/kbench.cpp -ldl
// usage: kbench [-f frames] [-w W] [-h H] [-t targets] [-k kind] [-n iters] [-r rounds]
//               [-m hot] [-l layout] lib.so [lib.so ...]
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include <algorithm>
#include <string>
#include <vector>

#include "../include/trik_hsv.h"

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(2);                                                                  \
    }                                                                           \
  } while (0)

struct Lib {
  std::string path;
  void* so = nullptr;
  decltype(&TRIK_VIDTRANSCODE_CV_create) create;
  decltype(&trik_hsv_batch_sums) sums;
  decltype(&trik_hsv_process_batch_totals) step = nullptr;
  decltype(&trik_hsv_synth) synth;
  decltype(&trik_hsv_set_hot_kernel) set_hot;
  decltype(&trik_hsv_last_error) last_error;
  decltype(&trik_hsv_chroma_share) share;
  TRIK_VIDTRANSCODE_CV_Handle h = nullptr;
  std::vector<float> ms;
  void* (*trace_ptr)() = nullptr;  // timing variants only: the per-wave timestamp trace
};

template <typename F>
static void sym(void* so, const char* name, F& f) {
  f = reinterpret_cast<F>(dlsym(so, name));
  if (!f) {
    fprintf(stderr, "missing %s: %s\n", name, dlerror());
    exit(2);
  }
}

int main(int argc, char** argv) {
  int frames = 4096, W = 640, H = 480, T = 4, kind = 0, iters = 20, rounds = 3, hot = 2, layout = 0, full = 0;
  int opt;
  int b2b = 0;
  while ((opt = getopt(argc, argv, "f:w:h:t:k:n:r:m:l:sb")) != -1) {
    switch (opt) {
      case 'f': frames = atoi(optarg); break;
      case 'w': W = atoi(optarg); break;
      case 'h': H = atoi(optarg); break;
      case 't': T = atoi(optarg); break;
      case 'k': kind = atoi(optarg); break;
      case 'n': iters = atoi(optarg); break;
      case 'r': rounds = atoi(optarg); break;
      case 'm': hot = atoi(optarg); break;
      case 'l': layout = atoi(optarg); break;
      case 's': full = 1; break;  // time the full step (trik_hsv_process_batch_totals)
      case 'b': b2b = 1; break;   // also back to back: per step without and with per-launch events
      default: return 2;
    }
  }
  std::vector<Lib> libs;
  for (int i = optind; i < argc; ++i) {
    Lib L;
    L.path = argv[i];
    L.so = dlopen(argv[i], RTLD_NOW | RTLD_LOCAL);
    if (!L.so) {
      fprintf(stderr, "dlopen %s: %s\n", argv[i], dlerror());
      return 2;
    }
    sym(L.so, "TRIK_VIDTRANSCODE_CV_create", L.create);
    sym(L.so, "trik_hsv_batch_sums", L.sums);
    if (full) sym(L.so, "trik_hsv_process_batch_totals", L.step);
    sym(L.so, "trik_hsv_synth", L.synth);
    sym(L.so, "trik_hsv_set_hot_kernel", L.set_hot);
    sym(L.so, "trik_hsv_last_error", L.last_error);
    sym(L.so, "trik_hsv_chroma_share", L.share);
    L.trace_ptr = reinterpret_cast<void* (*)()>(dlsym(L.so, "trik_trace_ptr"));
    libs.push_back(L);
  }
  if (libs.empty()) return 2;
  const TRIK_VIDTRANSCODE_CV_InArgsAlg all[4] = {
      {0, 30, 50, 100, 30, 100, 0}, {90, 150, 40, 100, 20, 100, 0},
      {200, 260, 40, 100, 20, 100, 0}, {330, 20, 30, 100, 30, 100, 0}};
  const int ll = layout == 0 ? 2 * W : W;
  const int64_t fb = (int64_t)H * ll * (layout == 0 ? 1 : 2);
  uint8_t* d_frames = nullptr;
  CK(hipMalloc(&d_frames, fb * frames));
  TrikHsvTargetSums* d_sums = nullptr;
  const size_t sb = sizeof(TrikHsvTargetSums) * (size_t)frames * T;
  CK(hipMalloc(&d_sums, sb));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  TrikHsvTarget* d_targets = nullptr;
  TrikHsvTargetSums* d_totals = nullptr;
  CK(hipMalloc(&d_targets, sizeof(TrikHsvTarget) * (size_t)frames * T));
  CK(hipMalloc(&d_totals, sizeof(TrikHsvTargetSums) * T));
  TrikHsvFrameBatch b = {d_frames, fb, frames, W, H, ll, layout};
  if (libs[0].synth(&b, 0, kind, 0x7A1Cull, s)) {
    fprintf(stderr, "synth: %s\n", libs[0].last_error());
    return 2;
  }
  std::vector<TrikHsvTargetSums> ref(sb / sizeof(TrikHsvTargetSums)), got(ref.size());
  for (size_t i = 0; i < libs.size(); ++i) {
    Lib& L = libs[i];
    if (L.create(nullptr, &L.h)) return 2;
    L.set_hot(L.h, hot);
    CK(hipMemsetAsync(d_sums, 0, sb, s));
    if ((full ? L.step(L.h, &b, all, T, d_sums, d_targets, d_totals, s) : L.sums(L.h, &b, all, T, d_sums, s))) {
      fprintf(stderr, "%s: %s\n", L.path.c_str(), L.last_error());
      return 2;
    }
    CK(hipStreamSynchronize(s));
    CK(hipMemcpy(i ? got.data() : ref.data(), d_sums, sb, hipMemcpyDeviceToHost));
    if (i && memcmp(got.data(), ref.data(), sb)) {
      size_t k = 0;
      while (k < ref.size() && !memcmp(&got[k], &ref[k], sizeof got[k])) ++k;
      printf("MISMATCH %s vs %s at frame %zu range %zu\n", L.path.c_str(), libs[0].path.c_str(), k / T, k % T);
    }
  }
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int r = 0; r < rounds; ++r)
    for (Lib& L : libs) {
      L.set_hot(L.h, hot);
      for (int w = 0; w < 3; ++w) (full ? L.step(L.h, &b, all, T, d_sums, d_targets, d_totals, s) : L.sums(L.h, &b, all, T, d_sums, s));
      for (int k = 0; k < iters; ++k) {
        CK(hipEventRecord(e0, s));
        (full ? L.step(L.h, &b, all, T, d_sums, d_targets, d_totals, s) : L.sums(L.h, &b, all, T, d_sums, s));
        CK(hipEventRecord(e1, s));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        L.ms.push_back(ms);
      }
    }
  if (b2b) {  // steps enqueued back to back (as bench.py's timed loop), K = 200
    const int K = 200;
    std::vector<hipEvent_t> ev(2 * K);
    for (auto& e : ev) CK(hipEventCreate(&e));
    for (Lib& L : libs) {
      auto launch = [&]() { (full ? L.step(L.h, &b, all, T, d_sums, d_targets, d_totals, s) : L.sums(L.h, &b, all, T, d_sums, s)); };
      for (int w = 0; w < 10; ++w) launch();
      CK(hipStreamSynchronize(s));
      CK(hipEventRecord(e0, s));
      for (int k = 0; k < K; ++k) launch();
      CK(hipEventRecord(e1, s));
      CK(hipEventSynchronize(e1));
      float bare = 0;
      CK(hipEventElapsedTime(&bare, e0, e1));
      CK(hipEventRecord(e0, s));
      for (int k = 0; k < K; ++k) {
        CK(hipEventRecord(ev[2 * k], s));
        launch();
        CK(hipEventRecord(ev[2 * k + 1], s));
      }
      CK(hipEventRecord(e1, s));
      CK(hipEventSynchronize(e1));
      float with = 0, kern = 0;
      CK(hipEventElapsedTime(&with, e0, e1));
      for (int k = 0; k < K; ++k) {
        float ms = 0;
        CK(hipEventElapsedTime(&ms, ev[2 * k], ev[2 * k + 1]));
        kern += ms;
      }
      printf("%-40s back to back: %.4f ms/step bare, %.4f ms/step with per-launch events, launch %.4f ms, gap %.2f us\n",
             L.path.c_str(), bare / K, with / K, kern / K, 1e3 * (with - kern) / K);
    }
  }
  for (Lib& L : libs) {  // per-wave timestamps of one launch in a back-to-back run (trace variants)
    if (!L.trace_ptr) continue;
    constexpr int kRec = 6, kMaxWaves = 8192;
    uint64_t* d_tr = static_cast<uint64_t*>(L.trace_ptr());
    auto launch = [&]() { (full ? L.step(L.h, &b, all, T, d_sums, d_targets, d_totals, s) : L.sums(L.h, &b, all, T, d_sums, s)); };
    for (int w = 0; w < 10; ++w) launch();
    CK(hipMemsetAsync(d_tr, 0, sizeof(uint64_t) * kRec * kMaxWaves, s));
    launch();
    launch();  // (the traced launch: the one before it overwrote nothing it reads)
    CK(hipStreamSynchronize(s));
    std::vector<uint64_t> tr((size_t)kRec * kMaxWaves);
    CK(hipMemcpy(tr.data(), d_tr, sizeof(uint64_t) * tr.size(), hipMemcpyDeviceToHost));
    // records: t0 kernel start, t1 image staged, t2 unit loop left, t3 wave end, units, workgroup
    std::vector<int> ws;
    uint64_t t0min = ~0ull, tend = 0;
    for (int i = 0; i < kMaxWaves; ++i)
      if (tr[kRec * i]) {
        ws.push_back(i);
        t0min = std::min(t0min, tr[kRec * i]);
        tend = std::max(tend, tr[kRec * i + 3]);
      }
    if (ws.empty()) continue;
    auto us = [&](uint64_t t) { return (t - t0min) / 100.0; };  // s_memrealtime: 100 MHz
    std::vector<double> st, stg, le, en, un;
    for (int i : ws) {
      st.push_back(us(tr[kRec * i]));
      stg.push_back((tr[kRec * i + 1] - tr[kRec * i]) / 100.0);
      le.push_back(us(tr[kRec * i + 2]));
      en.push_back(us(tr[kRec * i + 3]));
      un.push_back((double)tr[kRec * i + 4]);
    }
    auto pct = [](std::vector<double> v, double q) { std::sort(v.begin(), v.end()); return v[(size_t)(q * (v.size() - 1))]; };
    const double span = us(tend);
    double idle = 0;
    for (double x : le) idle += span - x;
    idle /= (double)ws.size() * span;
    printf("%-40s trace: %zu waves, span %.1f us; start p50/max %.1f/%.1f; staging p50/max %.1f/%.1f; "
           "loop end min/p10/p50/p90/max %.1f/%.1f/%.1f/%.1f/%.1f; idle after loop %.1f %%; units/wave min/max %.0f/%.0f\n",
           L.path.c_str(), ws.size(), span, pct(st, 0.5), pct(st, 1.0), pct(stg, 0.5), pct(stg, 1.0), pct(le, 0.0),
           pct(le, 0.1), pct(le, 0.5), pct(le, 0.9), pct(le, 1.0), 100 * idle, pct(un, 0.0), pct(un, 1.0));
    // per workgroup: its first and last wave out of the loop
    std::vector<double> wfirst(kMaxWaves, 1e30), wlast(kMaxWaves, 0);
    int nwg = 0;
    for (int i : ws) {
      const int g = (int)tr[kRec * i + 5];
      nwg = std::max(nwg, g + 1);
      wfirst[g] = std::min(wfirst[g], us(tr[kRec * i + 2]));
      wlast[g] = std::max(wlast[g], us(tr[kRec * i + 2]));
    }
    std::vector<double> spread, lastv;
    for (int g = 0; g < nwg; ++g)
      if (wlast[g] > 0) {
        spread.push_back(wlast[g] - wfirst[g]);
        lastv.push_back(wlast[g]);
      }
    printf("%-40s trace: %d workgroups; in-workgroup loop-end spread p50/p90/max %.1f/%.1f/%.1f us; "
           "workgroup end min/p50/max %.1f/%.1f/%.1f us\n",
           L.path.c_str(), nwg, pct(spread, 0.5), pct(spread, 0.9), pct(spread, 1.0), pct(lastv, 0.0), pct(lastv, 0.5),
           pct(lastv, 1.0));
    // workgroup end by XCD (blockIdx % 8 under round-robin placement) and the
    // units each workgroup's waves took
    printf("%-40s trace: workgroup end by blockIdx %% 8 (p50/max):", L.path.c_str());
    for (int x = 0; x < 8; ++x) {
      std::vector<double> v;
      for (int g = x; g < nwg; g += 8)
        if (wlast[g] > 0) v.push_back(wlast[g]);
      if (!v.empty()) printf(" %d:%.1f/%.1f", x, pct(v, 0.5), pct(v, 1.0));
    }
    printf("\n");
  }
  const double bytes = (double)fb * frames;
  for (Lib& L : libs) {
    std::vector<float> v = L.ms;
    std::sort(v.begin(), v.end());
    double mean = 0;
    for (float x : v) mean += x;
    mean /= v.size();
    const double med = v[v.size() / 2];
    double sh = -1;
    L.share(L.h, &sh);
    printf("%-40s T=%d kind=%d share %.4f  median %.4f ms  mean %.4f  min %.4f  frac %.4f\n", L.path.c_str(), T, kind, sh, med,
           mean, v[0], bytes / (med * 1e-3) / 8e12);
  }
  return 0;
}
