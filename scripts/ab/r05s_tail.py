# round-5 A/B: the load past a tile's last step (unconditional, so the step's
# wait stays "this step's data") reads a fixed L2-resident region (the
# ChromaTables block) instead of re-reading the tile's last rows from HBM:
# FETCH_SIZE showed 1.022 x the algorithmic bytes where the kernel's own
# pattern calibrates to 1.000 x (1 extra step of 30 per unit = 3.3 %)
FILE = "trik_hsv_chroma.hip"
TAIL = [
    ("        if (FULL && s + 1 < steps) rb += rowstep;\n",
     "        if (FULL) rb = s + 1 < steps ? rb + rowstep : (g.tail_ok ? tail : rb);\n"),
    ("        if (FULL && s + 2 < steps) rb += rowstep;\n",
     "        if (FULL) rb = s + 2 < steps ? rb + rowstep : (g.tail_ok ? tail : rb);\n"),
    ("      const uint8_t* rb = tbase;\n",
     "      const uint8_t* rb = tbase;\n      const uint8_t* const tail = reinterpret_cast<const uint8_t*>(ct);\n"),
    ("  int32_t units;  // wave-sized units per tile",
     "  int32_t tail_ok;  // the past-the-end loads fit inside the ChromaTables block\n  int32_t units;  // wave-sized units per tile"),
    ("  g.units = (g.k * g.cpr + 63) / 64;",
     "  g.units = (g.k * g.cpr + 63) / 64;\n  g.tail_ok = (int64_t)(g.k + g.dy) * a.line_length + 2LL * g.dx + 16 <= (int64_t)sizeof(ChromaTables);"),
]
VARIANTS = {
    "t_base": [("kMaxBlock = 1024;", "kMaxBlock = 1024;")],
    "t_tail": TAIL,
}
