# round-6 A/B, hot kernel: the block word -> palette read is a dependent LDS
# chain (r06j: the palette reads at addresses that do not depend on the block
# word, cost only, C3 -3.6 %).  The compiler interleaves the 8 run and 8 block
# reads and waits for nearly all 16 before the first palette read.
#  blkfirst  the 8 block reads issued first (a memory clobber keeps them
#            ahead of the run reads): the palette reads wait only for them
#  blkfirst4 the same in two halves of 4 words (blocks A, runs A, blocks B,
#            palette A, runs B, palette B)
FILE = "trik_hsv_chroma.hip"
_OLD = ("#pragma unroll\n        for (int i = 0; i < CW; ++i) {\n"
        "          d[i] = ld16(kLdsRuns + (c[i] >> 7));\n"
        "          // the block word: the pair's palette offset | the cut << 8\n"
        "          cut[i] = ld16(kLdsBlocks + ((c[i] >> 11) & 0x1FFEu));\n"
        "          pr[i] = cut[i] & 0xFFu;\n        }\n"
        "#pragma unroll\n        for (int i = 0; i < CW; ++i) mm[i] = ld64(kLdsPairs + pr[i]);\n")
_BF = ("#pragma unroll\n        for (int i = 0; i < CW; ++i) cut[i] = ld16(kLdsBlocks + ((c[i] >> 11) & 0x1FFEu));\n"
       "        asm volatile(\"\" ::: \"memory\");\n"
       "#pragma unroll\n        for (int i = 0; i < CW; ++i) d[i] = ld16(kLdsRuns + (c[i] >> 7));\n"
       "        asm volatile(\"\" ::: \"memory\");\n"
       "#pragma unroll\n        for (int i = 0; i < CW; ++i) { pr[i] = cut[i] & 0xFFu; mm[i] = ld64(kLdsPairs + pr[i]); }\n")
_BF4 = ("#pragma unroll\n        for (int i = 0; i < 4; ++i) cut[i] = ld16(kLdsBlocks + ((c[i] >> 11) & 0x1FFEu));\n"
        "        asm volatile(\"\" ::: \"memory\");\n"
        "#pragma unroll\n        for (int i = 0; i < 4; ++i) d[i] = ld16(kLdsRuns + (c[i] >> 7));\n"
        "        asm volatile(\"\" ::: \"memory\");\n"
        "#pragma unroll\n        for (int i = 4; i < CW; ++i) cut[i] = ld16(kLdsBlocks + ((c[i] >> 11) & 0x1FFEu));\n"
        "        asm volatile(\"\" ::: \"memory\");\n"
        "#pragma unroll\n        for (int i = 0; i < 4; ++i) { pr[i] = cut[i] & 0xFFu; mm[i] = ld64(kLdsPairs + pr[i]); }\n"
        "        asm volatile(\"\" ::: \"memory\");\n"
        "#pragma unroll\n        for (int i = 4; i < CW; ++i) d[i] = ld16(kLdsRuns + (c[i] >> 7));\n"
        "        asm volatile(\"\" ::: \"memory\");\n"
        "#pragma unroll\n        for (int i = 4; i < CW; ++i) { pr[i] = cut[i] & 0xFFu; mm[i] = ld64(kLdsPairs + pr[i]); }\n")
VARIANTS = {
    "r6k_base": [("kMaxBlock = 1024;", "kMaxBlock = 1024;")],
    "blkfirst": [(_OLD, _BF)],
    "blkfirst4": [(_OLD, _BF4)],
}
