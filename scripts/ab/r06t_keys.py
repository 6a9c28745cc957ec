# round-6 A/B, autoDetectHsv: the batch slot's keys (4 words, 8 pixels) all
# computed before the run-length updates, so the four words' HSV chains can
# be interleaved (each word's chain ended at the updates' branches: its LDS
# reads' latency and the packed-math wait states were exposed per word)
#  keysfirst
FILE = "trik_hsv_operator.hip"
VARIANTS = {
    "r6t_base": [("kVecBatch = 4;", "kVecBatch = 4;")],
    "keysfirst": [("#pragma unroll\n        for (int i = 0; i < NW; ++i) {\n          const int c = x0[b] + 2 * i;\n"
                   "          const uint32_t pos = (uint32_t)row[b] * (uint32_t)a.width + (uint32_t)c;\n"
                   "          uint32_t k0, k1;\n          hsv_key2(w[b][i], l43, l255, k0, k1);\n",
                   "        uint32_t kk[2 * NW];\n#pragma unroll\n        for (int i = 0; i < NW; ++i) hsv_key2(w[b][i], l43, l255, kk[2 * i], kk[2 * i + 1]);\n"
                   "#pragma unroll\n        for (int i = 0; i < NW; ++i) {\n          const int c = x0[b] + 2 * i;\n"
                   "          const uint32_t pos = (uint32_t)row[b] * (uint32_t)a.width + (uint32_t)c;\n"
                   "          const uint32_t k0 = kk[2 * i], k1 = kk[2 * i + 1];\n")],
}
