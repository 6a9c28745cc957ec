# round-5 A/B: nontemporal loads in the ov7670 line sensor's kernel
FILE = "trik_hsv_line.hip"
NT = [("""      y[i] = *reinterpret_cast<const uint2*>(p + i * step);
      c[i] = *reinterpret_cast<const uint2*>(p + i * step + cofs);""",
       """      typedef unsigned int v2 __attribute__((ext_vector_type(2)));
      const v2 ty = __builtin_nontemporal_load(reinterpret_cast<const v2*>(p + i * step));
      const v2 tc = __builtin_nontemporal_load(reinterpret_cast<const v2*>(p + i * step + cofs));
      y[i] = make_uint2(ty.x, ty.y);
      c[i] = make_uint2(tc.x, tc.y);""")]
VARIANTS = {
    "ln_base": [("if (r_hi <= r_lo) return 0;", "if (r_hi <= r_lo) return 0;")],
    "ln_nt": NT,
}
