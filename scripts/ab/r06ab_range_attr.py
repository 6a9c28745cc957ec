# round-6 A/B, autoDetectHsv (current form), cost only: where ~58 VALU per
# pixel-lane go on scenes.
#  nozone   no per-pixel zone-column test (edge chunks' outside pixels counted)
#  nocount  pass 1 folds the H, S, V values into one XOR per lane (no runs, no atomics)
#  nohsv    H, S, V from the raw bytes (no HSV arithmetic)
FILE = "trik_hsv_operator.hip"
_WALK = ("          if (ok[b] && c >= g.c0 && c < g.c1) fn(h0, pos);\n          if (ok[b] && c + 1 >= g.c0 && c + 1 < g.c1) fn(h1, pos + 1u);\n",)
_P1 = ('''  walk([&](const uint32_t (&hv)[3], uint32_t) {
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const uint32_t v = hv[c];
      if (v != rk3[c]) {
        if (rl3[c]) atomicAdd(&cnt[wave][c][rk3[c]], rl3[c]);
        rk3[c] = v;
        rl3[c] = 1u;
      } else {
        ++rl3[c];
      }
    }
  });
''',)
VARIANTS = {
    "r6ab_base": [("kVecBatch = 4;", "kVecBatch = 4;")],
    "nozone": [(_WALK[0], "          if (ok[b]) fn(h0, pos);\n          if (ok[b]) fn(h1, pos + 1u);\n")],
    "nocount": [(_P1[0], "  uint32_t xk = 0;\n  walk([&](const uint32_t (&hv)[3], uint32_t) { xk ^= hv[0] ^ (hv[1] << 8) ^ (hv[2] << 16); });\n"
                         "  if (xk == 0x12345678u) rl3[0] = 7u;\n")],
    "nohsv": [("          hsv_pair(w[b][i], l43, l255, h0, h1);\n",
               "          h0[0] = w[b][i] & 0xFFu; h0[1] = (w[b][i] >> 8) & 0xFFu; h0[2] = w[b][i] >> 24;\n"
               "          h1[0] = (w[b][i] >> 16) & 0xFFu; h1[1] = h0[1]; h1[2] = h0[2];\n")],
}
