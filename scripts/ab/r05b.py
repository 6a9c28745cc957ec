# round-5 A/B: the cross-unit prefetch and the SGPR append tail, separately
FILE = "trik_hsv_chroma.hip"
NOPRE = [("    const bool nx_pre = u_nx < u_end && first_chunk(u_nx, nx_base, nx_off);",
          "    const bool nx_pre = false && first_chunk(u_nx, nx_base, nx_off);")]
NOAPP = [("""      const uint32_t idx = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
      const uint32_t tw = __builtin_amdgcn_readfirstlane(rw_s + 16u * (uint32_t)qn);
      const uint32_t tm = __builtin_amdgcn_readfirstlane(rm_s + 4u * (uint32_t)qn);
      store_record(m, tw + 16u * idx, w4, tm + 4u * idx, meta);""",
          """      const uint32_t idx =
          __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, (uint32_t)qn));
      store_record(m, rw_s + 16u * idx, w4, rm_s + 4u * idx, meta);""")]
ADD2C = [("          d[i] = ld16(kLdsRuns + 2u * c[i]);",
          """          uint32_t c2;
          asm("v_add_u32 %0, %1, %1" : "=v"(c2) : "v"(c[i]));
          d[i] = ld16(kLdsRuns + c2);""")]
VARIANTS = {
    "base": ["REV=HEAD", ("kMaxBlock = 1024;", "kMaxBlock = 1024;")],
    "nopre": NOPRE,
    "noapp": NOAPP,
    "none": NOPRE + NOAPP,
    "add2c": ADD2C,
}
PLAIN = [("""    const u32x4 va = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
    const u32x4 vb = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(pb));""",
          """    const u32x4 va = *reinterpret_cast<const u32x4*>(p);
    const u32x4 vb = *reinterpret_cast<const u32x4*>(pb);""")]
VARIANTS["plain"] = PLAIN
