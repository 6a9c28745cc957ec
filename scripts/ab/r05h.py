# round-5 timing variants of chroma_kernel (sums differ: cost measurements only)
FILE = "trik_hsv_chroma.hip"
VARIANTS = {
    "base": [("kMaxBlock = 1024;", "kMaxBlock = 1024;")],
    # VERDICT r4 lever (b): a u8 block index (one shift from the chroma) and a
    # 256-entry palette of (M1, M2, cut) read as ds_read_b128 -- emulated on the
    # real index distribution (the block table's bytes) and a 4 KB region
    "pal128": [("""          cut[i] = ld16(kLdsBlocks + ((c[i] >> 3) & 0x1FFEu));
          pr[i] = cut[i] & 0xFFu;
        }
#pragma unroll
        for (int i = 0; i < CW; ++i) mm[i] = ld64(kLdsPairs + pr[i]);""",
                """          pr[i] = ld8(kLdsBlocks + (c[i] >> 4));
        }
#pragma unroll
        for (int i = 0; i < CW; ++i) {
          const u32x4 pe = *(lds128_t)(uintptr_t)(kLdsRuns + 16u * pr[i]);
          mm[i].x = pe.x;
          mm[i].y = pe.y;
          cut[i] = pe.z;
        }""")],
    # what the exception-code compare costs (no exception flags)
    "noexc": [("""  "v_cmp_eq_u32_e64 %[x], %[k], %[d]\\n\\t"                                                       \\""",
               """  "s_mov_b64 %[x], 0\\n\\t"                                                                          \\""")],
}
