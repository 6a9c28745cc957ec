# round-6 A/B, hot kernel:
#  addc      the records' flag bits shifted in by one v_addc_co_u32 per word
#            (carry-in = the word's flag mask) instead of a v_cndmask per word
#            and a v_or3 per two words; the drain reads word 3 - bit
#  cf_runs   cost only (sums wrong): the run-descriptor reads at conflict-free
#            addresses (lane l reads dword l) -- prices the LDS bank conflicts
#            of the random descriptor lookups (VERDICT r5 lever d)
#  cf_blocks cost only: the block-word reads at conflict-free addresses
#  cf_both   cost only: both
FILE = "trik_hsv_chroma.hip"
_SHIFT = (
    "// 4-bit mask (range t -> bit t) -> byte-spread (range t -> bit 8t)\n",
    "__device__ __forceinline__ uint32_t shift_in(uint32_t v, uint64_t m) {\n"
    "  uint32_t r;\n  uint64_t co;\n"
    "  asm volatile(\"v_addc_co_u32_e64 %0, %1, %2, %2, %3\" : \"=v\"(r), \"=&s\"(co) : \"v\"(v), \"s\"(m));\n"
    "  return r;\n}\n"
    "// 4-bit mask (range t -> bit t) -> byte-spread (range t -> bit 8t)\n")
_ADDC = [
    _SHIFT,
    ("        uint32_t fa = meta_a, fb = meta_a + meta_b;\n",
     "        uint32_t fa = meta_a >> 4, fb = (meta_a + meta_b) >> 4;\n"),
    ("            fa |= lane_bit(bal, 1u << i);\n            if (i & 1) asm volatile(\"\" : \"+v\"(fa));  // (two words per v_or3)\n",
     "            fa = shift_in(fa, bal);\n"),
    ("            fb |= lane_bit(bal, 1u << (i - 4));\n            if (i & 1) asm volatile(\"\" : \"+v\"(fb));\n",
     "            fb = shift_in(fb, bal);\n"),
    ("        const uint32_t i = (uint32_t)__builtin_ctz(fl);\n",
     "        const uint32_t i = 3u - (uint32_t)__builtin_ctz(fl);\n"),
]
_CFR = ("          d[i] = ld16(kLdsRuns + (c[i] >> 7));\n",
        "          d[i] = ld16(kLdsRuns + 4u * (uint32_t)lane + 256u * (uint32_t)i);\n")
_CFB = ("          cut[i] = ld16(kLdsBlocks + ((c[i] >> 11) & 0x1FFEu));\n",
        "          cut[i] = ld16(kLdsBlocks + 4u * (uint32_t)lane + 256u * (uint32_t)i + (c[i] >> 31));\n")
VARIANTS = {
    "r6base": [("kMaxBlock = 1024;", "kMaxBlock = 1024;")],
    "addc": _ADDC,
    "cf_runs": [_CFR],
    "cf_blocks": [_CFB],
    "cf_both": [_CFR, _CFB],
}
