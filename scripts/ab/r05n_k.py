# round-5 A/B: fewer, longer units per frame (the per-unit epilogue -- the
# wave reduction of 12 sums, their atomics, the unit setup -- is ~6 % of the
# C3 kernel): at VGA k = 8 rows per half step (10 units of 30 steps per frame)
# instead of k = 12 (15 units of 20 steps)
FILE = "trik_hsv_chroma.hip"
VARIANTS = {
    "k_base": [("kMaxBlock = 1024;", "kMaxBlock = 1024;")],
    "k640": [("  int k = kHotLanes / cpr;\n", "  int k = 640 / cpr;\n")],
    "k320": [("  int k = kHotLanes / cpr;\n", "  int k = 320 / cpr;\n")],
}
