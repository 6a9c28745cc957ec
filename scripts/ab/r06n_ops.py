# round-6 A/B, hot kernel: fewer VALU per word/step (r06m: one more VOP2 per
# word costs C3 +2 %, one more VOP3/VOPC +3 %).
#  u8pal    the palette offset read as its own byte (ds_read_u8 at the block
#           word's address) instead of masked out of the block word: one LDS
#           read more, one v_and less per word
#  appsb    appends: the lane's rank from mbcnt alone and the queue's base
#           (+ 16 or 4 x count) formed in SALU: no v_mov of the count per append
FILE = "trik_hsv_chroma.hip"
VARIANTS = {
    "r6n_base": [("kMaxBlock = 1024;", "kMaxBlock = 1024;")],
    "u8pal": [("          pr[i] = cut[i] & 0xFFu;\n",
               "          pr[i] = ld8(kLdsBlocks + ((c[i] >> 11) & 0x1FFEu));\n")],
    "appsb": [("      const uint32_t idx =\n          __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, (uint32_t)qn));\n"
               "      store_record(m, rw_s + 16u * idx, w4, rm_s + 4u * idx, meta);\n",
               "      const uint32_t rk = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));\n"
               "      const uint32_t bw_ = __builtin_amdgcn_readfirstlane(rw_s + 16u * (uint32_t)qn);\n"
               "      const uint32_t bm_ = __builtin_amdgcn_readfirstlane(rm_s + 4u * (uint32_t)qn);\n"
               "      store_record(m, bw_ + 16u * rk, w4, bm_ + 4u * rk, meta);\n")],
}
