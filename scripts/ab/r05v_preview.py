# round-5 preview_rows2_kernel: one 16-byte store per unit instead of two
# 8-byte ones (consecutive lanes' units are 16 B apart, so each 8-byte store
# instruction covered every other 8 bytes of a 1 KiB span)
FILE = "trik_hsv_operator.hip"
ST16 = [("""#pragma unroll
        for (int h = 0; h < PX / 4; ++h) {
          uint2 o;
          o.x = v[4 * h] | (v[4 * h + 1] << 16);
          o.y = v[4 * h + 2] | (v[4 * h + 3] << 16);
          *reinterpret_cast<uint2*>(dst + 8 * h) = o;
        }""", """        uint4 o;
        o.x = v[0] | (v[1] << 16);
        o.y = v[2] | (v[3] << 16);
        o.z = v[4] | (v[5] << 16);
        o.w = v[6] | (v[7] << 16);
        *reinterpret_cast<uint4*>(dst) = o;""")]
NOCOMP = [("        v[k] = det ? 0xFFE0u : c565;", "        v[k] = ws[k] & 0xFFFFu; (void)det; (void)c565;")]
NOGUIDE = [("      if (GUIDES) gbits[u] = a.guide_bits[r * gpr + q];  // (the same bytes for every frame: cached)",
            "      if (GUIDES) gbits[u] = 0u;")]
VARIANTS = {
    "pv_base": [("constexpr int kRangeBlock = 256;", "constexpr int kRangeBlock = 256;")],
    "pv_st16": ST16,
    "pv_nocomp": NOCOMP,
    "pv_st16_nocomp": ST16 + NOCOMP,
    "pv_noguide": NOGUIDE,
}
