# timing variant of chroma_kernel with per-wave timestamps (kbench reads them
# through trik_trace_ptr): kernel start, image staged, unit loop left, wave end,
# units, workgroup -- development only
FILE = "trik_hsv_chroma.hip"
VARIANTS = {
    "trace": [
        ("template <int LAYOUT, int NR, bool MASKS>\n__global__ __launch_bounds__(kMaxBlock) void chroma_kernel",
         "__device__ unsigned long long g_trace[6 * 8192];\n"
         "extern \"C\" void* trik_trace_ptr() { void* p = nullptr; (void)hipGetSymbolAddress(&p, HIP_SYMBOL(g_trace)); return p; }\n"
         "template <int LAYOUT, int NR, bool MASKS>\n__global__ __launch_bounds__(kMaxBlock) void chroma_kernel"),
        ("  if (gated_out(a.gate, a.gate_max, a.gate_le)) return;\n  constexpr int CW = kChunkWords;",
         "  if (gated_out(a.gate, a.gate_max, a.gate_le)) return;\n  const uint64_t tr0 = __builtin_amdgcn_s_memrealtime();\n  constexpr int CW = kChunkWords;"),
        ("  const int lane = t & 63;\n  const uint32_t wave = (uint32_t)(t >> 6);\n  const uint32_t rw_s",
         "  const uint64_t tr1 = __builtin_amdgcn_s_memrealtime(); uint32_t trn = 0;\n  const int lane = t & 63;\n  const uint32_t wave = (uint32_t)(t >> 6);\n  const uint32_t rw_s"),
        ("    if (a.fused) pend_f = f;", "    if (a.fused) pend_f = f;\n    ++trn;"),
        ("  if (a.fused) {  // this wave's last counts", "  const uint64_t tr2 = __builtin_amdgcn_s_memrealtime();\n  if (a.fused) {  // this wave's last counts"),
        ("  if (!a.fused) return;\n  // fused step: the per-target totals",
         "  { const uint64_t tr3 = __builtin_amdgcn_s_memrealtime(); const uint32_t wi = blockIdx.x * 16u + wave; "
         "if (lane == 0 && wi < 8192u) { unsigned long long* T = g_trace + 6u * wi; T[0] = tr0; T[1] = tr1; T[2] = tr2; "
         "T[3] = tr3; T[4] = trn; T[5] = blockIdx.x; } }\n  if (!a.fused) return;\n  // fused step: the per-target totals"),
    ],
}
