# attribution of auto_range_vec_kernel (timing-only variants: results differ)
FILE = "trik_hsv_operator.hip"
PASS1 = """  walk([&](uint32_t key, uint32_t) {
    if (rl && key == rk) {
      ++rl;
    } else {
      flush();
      rk = key;
      rl = 1u;
    }
  });"""
VARIANTS = {
    "ar2_base": [("constexpr int kVecBatch = 4;", "constexpr int kVecBatch = 4;")],
    "ar2_hsv": [(PASS1, """  walk([&](uint32_t key, uint32_t) { rk ^= key; });
  if (rk == 0x12345678u) cnt[0][0][0] = 1;""")],
    "ar2_nop2": [("  const uint32_t tie = (n_top[0] > 1u ? 1u : 0u) | (n_top[1] > 1u ? 2u : 0u) | (n_top[2] > 1u ? 4u : 0u);",
                  "  const uint32_t tie = 0u;")],
    "ar2_b8": [("constexpr int kVecBatch = 4;", "constexpr int kVecBatch = 8;")],
}
