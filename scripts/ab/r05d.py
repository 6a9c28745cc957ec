# round-5 attribution of the hot kernel (timing-only variants: sums differ)
FILE = "trik_hsv_chroma.hip"
VARIANTS = {
    "base": [("kMaxBlock = 1024;", "kMaxBlock = 1024;")],
    "noappend": [("""        append(ma, wa, fa);
        append(mb, wb, fb);""", "")],
    "nodrain": [("    auto drain = [&](int take) {\n", "    auto drain = [&](int take) {\n      qn -= take; if (take < 1000) return;\n")],
    "noflags": [("            fa |= lane_bit(bal, 1u << i);", ""), ("            fb |= lane_bit(bal, 1u << (i - 4));", "")],
    "nofinal": [("    while (qn > 0) drain(qn < 64 ? qn : 64);\n    Qa += Ba;", "    qn = 0;\n    Qa += Ba;")],
    "noepi": [("    emit(acc);\n    if (a.fused) pend_f = f;", "    if (a.fused) pend_f = f;")],
}
