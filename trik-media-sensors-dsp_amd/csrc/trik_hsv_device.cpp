// trik_hsv_device.cpp -- per-device facts the launchers need, cached
// thread-safely per device (a process may drive several GPUs from several
// threads, one handle each).
#include <hip/hip_runtime.h>

#include <map>
#include <mutex>
#include <utility>

#include "trik_hsv_internal.h"

namespace trik_hsv {

namespace {
std::mutex g_mu;
std::map<int, int> g_cus;                                     // device -> CUs
std::map<std::pair<int, const void*>, int> g_lds;             // (device, kernel) -> dynamic LDS bytes set
}  // namespace

int device_cus() {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 256;
  std::lock_guard<std::mutex> lock(g_mu);
  auto it = g_cus.find(dev);
  if (it != g_cus.end()) return it->second;
  int n = 0;
  if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
  g_cus[dev] = n;
  return n;
}

int stream_cus(hipStream_t s) {
  const int all = device_cus();
  if (!s) return all;
  // a stream created with a CU mask (hipExtStreamCreateWithCUMask) runs its
  // kernels on the masked CUs only: one workgroup per CU means one per
  // masked CU (the rest would wait for a second round)
  uint32_t m[32] = {};
  if (hipExtStreamGetCUMask(s, 32, m) != hipSuccess) return all;
  int n = 0;
  for (uint32_t w : m) n += __builtin_popcount(w);
  return n > 0 && n < all ? n : all;
}

hipError_t set_dynamic_lds(const void* kern, int bytes) {
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  std::lock_guard<std::mutex> lock(g_mu);
  auto key = std::make_pair(dev, kern);
  auto it = g_lds.find(key);
  if (it != g_lds.end() && it->second >= bytes) return hipSuccess;
  e = hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
  if (e == hipSuccess) g_lds[key] = bytes;
  return e;
}

}  // namespace trik_hsv
