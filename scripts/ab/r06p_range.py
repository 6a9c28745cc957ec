# round-6 A/B, autoDetectHsv (auto_range_vec_kernel), cost only: where the
# 0.156 ms per 4096 VGA scene frames goes.
#  nohsv   the pixel's key is its raw (Y, U, V) bytes (no HSV arithmetic):
#          loads + zone walk + run-length counting + atomics
#  nocount the HSV keys folded into one XOR per lane (no run-length counting,
#          no histogram atomics): loads + zone walk + HSV
FILE = "trik_hsv_operator.hip"
_KEYS = ("          const uint32_t k0 = hsv_key<0>(w[b][i], l43, l255), k1 = hsv_key<1>(w[b][i], l43, l255);\n",)
_P1 = ("  walk([&](uint32_t key, uint32_t) {\n    if (rl && key == rk) {\n",)
VARIANTS = {
    "r6p_base": [("kVecBatch = 4;", "kVecBatch = 4;")],
    "nohsv": [(_KEYS[0], "          const uint32_t k0 = w[b][i] & 0xFFFFFFu, k1 = (w[b][i] >> 8) & 0xFFFFFFu;\n")],
    "nocount": [("  walk([&](uint32_t key, uint32_t) {\n    if (rl && key == rk) {\n      ++rl;\n    } else {\n      flush();\n      rk = key;\n      rl = 1u;\n    }\n  });\n  flush();\n",
                 "  uint32_t xk = 0;\n  walk([&](uint32_t key, uint32_t) { xk ^= key; });\n"
                 "  if (xk == 0x12345678u) atomicAdd(&cnt[wave][0][0], 1u + rk + rl);\n")],
}
