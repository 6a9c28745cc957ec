# round-6 A/B, autoDetectHsv pass 1: every pixel of a chunk counted, the few
# outside the zone's columns (a row's first / last chunk, kernel-wide pixel
# bounds lo_f / hi_l) subtracted again -- no per-pixel column test; the run
# update branch-free except the add itself.
#  count2   the work tree;  r6ac_head: the committed form (REV=HEAD)
FILE = "trik_hsv_operator.hip"
VARIANTS = {
    "r6ac_head": ["REV=HEAD"],
    "count2": [("kVecBatch = 4;", "kVecBatch = 4;")],
}
# count2 with the old branchy run update (rk3 initialised to ~0, an add only when
# the run was non-empty): the column-test removal alone
_NEW_RUN = ("      const bool brk = v != rk3[c];\n      if (brk) atomicAdd(&cnt[wave][c][rk3[c]], rl3[c]);\n"
            "      rl3[c] = brk ? 1u : rl3[c] + 1u;\n      rk3[c] = v;\n")
_OLD_RUN = ("      if (v != rk3[c]) {\n        if (rl3[c]) atomicAdd(&cnt[wave][c][rk3[c]], rl3[c]);\n        rk3[c] = v;\n"
            "        rl3[c] = 1u;\n      } else {\n        ++rl3[c];\n      }\n")
VARIANTS["count2_oldrun"] = [(_NEW_RUN, _OLD_RUN)]
# count2 with V (channel 2) added per pixel without a run (V breaks its run on
# nearly every pixel of a gradient)
_LOOP = ("#pragma unroll\n    for (int c = 0; c < 3; ++c) {\n      const uint32_t v = hv[c];\n      const bool brk = v != rk3[c];\n",)
VARIANTS["vdirect"] = [(_LOOP[0], "    atomicAdd(&cnt[wave][2][hv[2]], 1u);\n#pragma unroll\n    for (int c = 0; c < 2; ++c) {\n      const uint32_t v = hv[c];\n      const bool brk = v != rk3[c];\n")]
