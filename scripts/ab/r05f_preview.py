# round-5 attribution of preview_rows2_kernel (timing-only variants)
FILE = "trik_hsv_operator.hip"
VARIANTS = {
    "pv_base": [("constexpr int kRangeBlock = 256;", "constexpr int kRangeBlock = 256;")],
    # no detection lookups (every pixel its colour)
    "pv_nodet": [("          det = lds_u32(phase2_addr(m, p, hue_lane)) & sv & 1u;  // range 0 (combine keeps bit 0 in place)",
                  "          det = 0u; (void)m; (void)sv;")],
    # loads and stores only: the output is the source word's low half
    "pv_nocomp": [("        v[k] = det ? 0xFFE0u : c565;", "        v[k] = ws[k] & 0xFFFFu; (void)det; (void)c565;")],
}
