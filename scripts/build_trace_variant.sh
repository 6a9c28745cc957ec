#!/bin/bash
# Timing variant of the chroma-run kernel with per-wave timestamps (development
# only): s_memrealtime at the kernel start, after the image is staged, when the
# wave leaves its unit loop and at its end, plus its unit count and workgroup,
# into a device array that scripts/kbench reads through trik_trace_ptr().
#   bash scripts/build_trace_variant.sh NAME
set -eu
cd "$(dirname "$0")/.."
bash scripts/build_variant.sh "$1" trik_hsv_chroma.hip \
 'template <int LAYOUT, int NR, bool MASKS>\n__global__ __launch_bounds__\(kMaxBlock\) void chroma_kernel=>__device__ unsigned long long g_trace[6 * 8192];\nextern "C" void* trik_trace_ptr() { void* p = nullptr; (void)hipGetSymbolAddress(&p, HIP_SYMBOL(g_trace)); return p; }\ntemplate <int LAYOUT, int NR, bool MASKS>\n__global__ __launch_bounds__(kMaxBlock) void chroma_kernel' \
 'stage_chroma_image\(ct, a.tables, t\);=>const uint64_t tr0 = __builtin_amdgcn_s_memrealtime(); stage_chroma_image(ct, a.tables, t);' \
 '  if \(t < 3\) \*\(lds32_t\)\(uintptr_t\)\(kLdsWords \+ 4 \* t\) = 0u;\n  __syncthreads\(\);=>  if (t < 3) *(lds32_t)(uintptr_t)(kLdsWords + 4 * t) = 0u;\n  __syncthreads();\n  const uint64_t tr1 = __builtin_amdgcn_s_memrealtime(); uint32_t trn = 0;' \
 'pend_f = f;=>pend_f = f; ++trn;' \
 "  if \(a.fused\) \{  // this wave's last counts=>  const uint64_t tr2 = __builtin_amdgcn_s_memrealtime();\n  if (a.fused) {  // this wave's last counts" \
 '  if \(!a.fused\) return;=>  { const uint64_t tr3 = __builtin_amdgcn_s_memrealtime(); const uint32_t wi = blockIdx.x * 16u + wave; if (lane == 0 && wi < 8192u) { unsigned long long* T = g_trace + 6u * wi; T[0] = tr0; T[1] = tr1; T[2] = tr2; T[3] = tr3; T[4] = trn; T[5] = blockIdx.x; } }\n  if (!a.fused) return;'
