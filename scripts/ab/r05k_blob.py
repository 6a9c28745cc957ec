# round-5 A/B of the multi-blob bitmap kernel (blob_chroma_meta_kernel): its
# two row loads nontemporal (the chroma kernel's streaming loads)
FILE = "trik_hsv_chroma.hip"
VARIANTS = {
    "blob_base": [("kMaxBlock = 1024;", "kMaxBlock = 1024;")],
    "blob_nt": [("""      by[(r + 1) & 1] = *reinterpret_cast<const uint4*>(np);
      bc[(r + 1) & 1] = *reinterpret_cast<const uint4*>(np + plane);""",
                 """      {
        typedef unsigned int v4 __attribute__((ext_vector_type(4)));
        const v4 ty = __builtin_nontemporal_load(reinterpret_cast<const v4*>(np));
        const v4 tc = __builtin_nontemporal_load(reinterpret_cast<const v4*>(np + plane));
        by[(r + 1) & 1] = make_uint4(ty.x, ty.y, ty.z, ty.w);
        bc[(r + 1) & 1] = make_uint4(tc.x, tc.y, tc.z, tc.w);
      }""")],
}
