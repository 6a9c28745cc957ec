# round-5 A/B: nontemporal frame loads in the stripe kernel (band sets) -- the
# chroma kernel's streaming loads are nontemporal (2.7 % faster), the
# multi-blob bitmap kernel's became so (9 %)
FILE = "trik_hsv_stripe.hip"
VARIANTS = {
    "st_base": [("const uint4 v = *reinterpret_cast<const uint4*>(p);", "const uint4 v = *reinterpret_cast<const uint4*>(p);")],
    "st_nt": [("""    const uint4 v = *reinterpret_cast<const uint4*>(p);
    w[0] = v.x; w[1] = v.y; w[2] = v.z; w[3] = v.w;
  } else {
    const uint2 vy = *reinterpret_cast<const uint2*>(p);
    const uint2 vc = *reinterpret_cast<const uint2*>(p + plane);""",
               """    typedef unsigned int v4 __attribute__((ext_vector_type(4)));
    const v4 v = __builtin_nontemporal_load(reinterpret_cast<const v4*>(p));
    w[0] = v.x; w[1] = v.y; w[2] = v.z; w[3] = v.w;
  } else {
    typedef unsigned int v2 __attribute__((ext_vector_type(2)));
    const v2 vy = __builtin_nontemporal_load(reinterpret_cast<const v2*>(p));
    const v2 vc = __builtin_nontemporal_load(reinterpret_cast<const v2*>(p + plane));""")],
}
