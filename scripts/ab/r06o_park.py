# round-6 A/B, hot kernel, VERDICT r5 lever (c): amortise the appends.  Each
# lane parks one flagged piece (its 4 words + meta) in VGPRs; the wave's
# compaction (append) runs only when a lane with a parked piece flags another
# one (then all parked pieces go to the queue at once) and at the unit end.
#  park    one VGPR slot per lane (5 VGPRs), parking by EXEC-masked v_mov
FILE = "trik_hsv_chroma.hip"
_DECL = ("    int qn = 0;\n    ExcSums ex;\n",
         "    int qn = 0;\n    ExcSums ex;\n"
         "    uint64_t occ = 0;  // lanes with a parked piece\n"
         "    uint32_t sw0 = 0, sw1 = 0, sw2 = 0, sw3 = 0, smeta = 0;  // the parked piece's words and meta\n")
_APP = ("        append(ma, wa, fa);\n        append(mb, wb, fb);\n",
        "        park(ma, wa, fa);\n        park(mb, wb, fb);\n")
_PARK = ("    // a row inside the frame for lanes whose rows run past it (re-read, masked)\n",
         "    auto flush_parked = [&]() {\n"
         "      if (occ == 0) return;\n"
         "      u32x4 s4;\n      s4.x = sw0; s4.y = sw1; s4.z = sw2; s4.w = sw3;\n"
         "      append(occ, s4, smeta);\n      occ = 0;\n    };\n"
         "    auto park = [&](uint64_t m, u32x4 w4, uint32_t meta) {\n"
         "      if (m == 0) return;\n"
         "      if (m & occ) flush_parked();\n"
         "      uint64_t sv;\n"
         "      asm volatile(\n"
         "          \"s_and_saveexec_b64 %[sv], %[m]\\n\\t\"\n"
         "          \"v_mov_b32 %[a], %[x]\\n\\t\"\n"
         "          \"v_mov_b32 %[b], %[y]\\n\\t\"\n"
         "          \"v_mov_b32 %[c], %[z]\\n\\t\"\n"
         "          \"v_mov_b32 %[d], %[w]\\n\\t\"\n"
         "          \"v_mov_b32 %[e], %[mt]\\n\\t\"\n"
         "          \"s_mov_b64 exec, %[sv]\"\n"
         "          : [sv] \"=&s\"(sv), [a] \"+v\"(sw0), [b] \"+v\"(sw1), [c] \"+v\"(sw2), [d] \"+v\"(sw3), [e] \"+v\"(smeta)\n"
         "          : [m] \"s\"(m), [x] \"v\"(w4.x), [y] \"v\"(w4.y), [z] \"v\"(w4.z), [w] \"v\"(w4.w), [mt] \"v\"(meta)\n"
         "          : \"scc\");\n"
         "      occ |= m;\n"
         "    };\n"
         "    // a row inside the frame for lanes whose rows run past it (re-read, masked)\n")
_END = ("    while (qn > 0) drain(qn < 64 ? qn : 64);\n    Qa += Ba;\n",
        "    flush_parked();\n    while (qn > 0) drain(qn < 64 ? qn : 64);\n    Qa += Ba;\n")
VARIANTS = {
    "r6o_base": [("kMaxBlock = 1024;", "kMaxBlock = 1024;")],
    "park": [_DECL, _PARK, _APP, _END],
}
