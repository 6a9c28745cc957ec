# round-6 A/B, hot kernel, cost only (sums wrong): which of the fast path's
# three LDS lookups per word carries the bank-conflict cost that r06c's
# cf_blocks priced at C3 -5.7 % (the block word and, through its palette
# offset, the palette read)?
#  cf_pal    the palette reads at lane-fixed slots (block words real)
#  cf_blk    the block reads at conflict-free addresses, the palette offset
#            taken from the run descriptor (random slots, no dependency on
#            the block read)
#  nopal     no palette read: the mask pair made from the block word by two
#            VALU ops (prices the read and its dependent latency)
FILE = "trik_hsv_chroma.hip"
_PAL = ("        for (int i = 0; i < CW; ++i) mm[i] = ld64(kLdsPairs + pr[i]);\n",)
_CUT = "          cut[i] = ld16(kLdsBlocks + ((c[i] >> 11) & 0x1FFEu));\n          pr[i] = cut[i] & 0xFFu;\n"
VARIANTS = {
    "r6j_base": [("kMaxBlock = 1024;", "kMaxBlock = 1024;")],
    "cf_pal": [(_PAL[0], "        for (int i = 0; i < CW; ++i) mm[i] = ld64(kLdsPairs + 8u * ((uint32_t)lane & 31u) + 0u * pr[i]);\n")],
    "cf_blk": [(_CUT, "          cut[i] = ld16(kLdsBlocks + 4u * (uint32_t)lane + 256u * (uint32_t)i + (c[i] >> 31));\n"
                      "          pr[i] = d[i] & 0xF8u;\n")],
    "nopal": [(_PAL[0], "        for (int i = 0; i < CW; ++i) { mm[i].x = pr[i] * 0x01010101u; mm[i].y = pr[i] >> 3; }\n")],
}
# r06c's cf_blocks on the current tree
VARIANTS["cf_blocks"] = [(_CUT, "          cut[i] = ld16(kLdsBlocks + 4u * (uint32_t)lane + 256u * (uint32_t)i + (c[i] >> 31));\n"
                                "          pr[i] = cut[i] & 0xFFu;\n")]
# r06c's cf_runs on the current tree
VARIANTS["cf_runs"] = [("          d[i] = ld16(kLdsRuns + (c[i] >> 7));\n",
                        "          d[i] = ld16(kLdsRuns + 4u * (uint32_t)lane + 256u * (uint32_t)i);\n")]
