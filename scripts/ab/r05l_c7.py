# round-5 A/B: nontemporal loads in the chroma kernel's ov7670 layout
FILE = "trik_hsv_chroma.hip"
VARIANTS = {
    "c7_base": [("kMaxBlock = 1024;", "kMaxBlock = 1024;")],
    "c7_nt": [("""    const uint4 vy = *reinterpret_cast<const uint4*>(p);
    const uint4 vc = *reinterpret_cast<const uint4*>(p + plane);""",
               """    const uint4 vy = ld_nt16(p);
    const uint4 vc = ld_nt16(p + plane);""")],
}
