# round-5 A/B: loads two steps ahead (a third chunk buffer) and the chroma
# index formed as c << 8 (the run-descriptor address by one cheap right shift
# instead of a 4-cycle left shift)
FILE = "trik_hsv_chroma.hip"
PRE3 = [("""      uint32_t wa[CW], wb[CW];
      ld(0, wa);
      for (int s = 0; s < steps; s += 2) {
        if (FULL && s + 1 < steps) rb += rowstep;
        ld(s + 1, wb);
        step(wa, s);
        if (s + 1 >= steps) break;
        if (FULL && s + 2 < steps) rb += rowstep;
        ld(s + 2, wa);
        step(wb, s + 1);
      }""", """      uint32_t wa[CW], wb[CW], wc[CW];
      ld(0, wa);
      if (FULL && 1 < steps) rb += rowstep;
      ld(1, wb);
      for (int s = 0; s < steps; s += 3) {
        if (FULL && s + 2 < steps) rb += rowstep;
        ld(s + 2, wc);
        step(wa, s);
        if (s + 1 >= steps) break;
        if (FULL && s + 3 < steps) rb += rowstep;
        ld(s + 3, wa);
        step(wb, s + 1);
        if (s + 2 >= steps) break;
        if (FULL && s + 4 < steps) rb += rowstep;
        ld(s + 4, wb);
        step(wc, s + 2);
      }""")]
PERM8 = [("""        for (int i = 0; i < CW; ++i) c[i] = chroma_of(cw[i]);
#pragma unroll
        for (int i = 0; i < CW; ++i) {
          d[i] = ld16(kLdsRuns + 2u * c[i]);
          // the block word: the pair's palette offset | the cut << 8
          cut[i] = ld16(kLdsBlocks + ((c[i] >> 3) & 0x1FFEu));""",
          """        for (int i = 0; i < CW; ++i) c[i] = __builtin_amdgcn_perm(cw[i], cw[i], 0x0C03010Cu);  // U << 8 | V << 16
#pragma unroll
        for (int i = 0; i < CW; ++i) {
          d[i] = ld16(kLdsRuns + (c[i] >> 7));
          // the block word: the pair's palette offset | the cut << 8
          cut[i] = ld16(kLdsBlocks + ((c[i] >> 11) & 0x1FFEu));""")]
VARIANTS = {
    "base": [("kMaxBlock = 1024;", "kMaxBlock = 1024;")],
    "pre3": PRE3,
    "perm8": PERM8,
    "pre3perm8": PRE3 + PERM8,
}
