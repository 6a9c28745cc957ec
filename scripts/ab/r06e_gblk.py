# round-6 A/B, hot kernel: the LDS array is a co-bottleneck (r06c: the block
# word reads at conflict-free addresses, cost only, C3 -5.7 %).  These move
# the block-word lookups off the LDS onto the vector memory path (an 8 KiB
# table, L1-resident): one global_load_ushort per word.
#  reorder   control: the next step's frame loads issued inside the step,
#            after its chroma indices (blocks still from LDS)
#  gblk      block words by global loads, issued before the next step's frame
#            loads (vmcnt completes in order: the wait for them must not
#            include the HBM prefetch)
FILE = "trik_hsv_chroma.hip"
_STEP = [
    ("      auto step = [&](const uint32_t (&cw)[CW], int s) {\n",
     "      auto step = [&](const uint32_t (&cw)[CW], int s, auto&& pre) {\n"),
    ("        for (int i = 0; i < CW; ++i) c[i] = chroma_of8(cw[i]);\n#pragma unroll\n        for (int i = 0; i < CW; ++i) {\n",
     "        for (int i = 0; i < CW; ++i) c[i] = chroma_of8(cw[i]);\n        BLK_LOADS\n        pre();\n#pragma unroll\n        for (int i = 0; i < CW; ++i) {\n"),
    ("        if (FULL) rb = s + 1 < steps ? rb + rowstep : (g.tail_ok ? tail : rb);\n        ld(s + 1, wb);\n        step(wa, s);\n",
     "        step(wa, s, [&]() {\n          if (FULL) rb = s + 1 < steps ? rb + rowstep : (g.tail_ok ? tail : rb);\n          ld(s + 1, wb);\n        });\n"),
    ("        if (FULL) rb = s + 2 < steps ? rb + rowstep : (g.tail_ok ? tail : rb);\n        ld(s + 2, wa);\n        step(wb, s + 1);\n",
     "        step(wb, s + 1, [&]() {\n          if (FULL) rb = s + 2 < steps ? rb + rowstep : (g.tail_ok ? tail : rb);\n          ld(s + 2, wa);\n        });\n"),
]
def _with(blk_loads, lds_read):
    out = []
    for old, new in _STEP:
        out.append((old, new.replace("BLK_LOADS", blk_loads)))
    out.append(("          cut[i] = ld16(kLdsBlocks + ((c[i] >> 11) & 0x1FFEu));\n", lds_read))
    return out
VARIANTS = {
    "r6e_base": [("kMaxBlock = 1024;", "kMaxBlock = 1024;")],
    "reorder": _with("", "          cut[i] = ld16(kLdsBlocks + ((c[i] >> 11) & 0x1FFEu));\n"),
    "gblk": _with("uint32_t gcut[CW];\n#pragma unroll\n        for (int i = 0; i < CW; ++i) gcut[i] = "
                  "ct->blocks[c[i] >> 12];",
                  "          cut[i] = gcut[i];\n"),
}
