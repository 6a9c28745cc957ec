# round-5 attribution of auto_range_kernel (timing-only variants: results differ)
FILE = "trik_hsv_operator.hip"
VARIANTS = {
    "ar_base": [("constexpr int kRangeBlock = 256;", "constexpr int kRangeBlock = 256;")],
    # no last-position tracking (no shfl, no atomicMax)
    "ar_nolast": [("for (int k = 0; k < 3; ++k) bin_add_runs<true>(cnt[wave][k], lst[0][k], hv[k], pos);",
                   "for (int k = 0; k < 3; ++k) bin_add_runs<false>(cnt[wave][k], lst[0][k], hv[k], pos);")],
    # plain per-pixel atomics, no run aggregation
    "ar_noruns": [("for (int k = 0; k < 3; ++k) bin_add_runs<true>(cnt[wave][k], lst[0][k], hv[k], pos);",
                   "for (int k = 0; k < 3; ++k) { atomicAdd(&cnt[wave][k][hv[k]], 1u); atomicMax(&lst[0][k][hv[k]], pos); }")],
    # plain count atomics only
    "ar_cntonly": [("for (int k = 0; k < 3; ++k) bin_add_runs<true>(cnt[wave][k], lst[0][k], hv[k], pos);",
                    "for (int k = 0; k < 3; ++k) atomicAdd(&cnt[wave][k][hv[k]], 1u);")],
    # the HSV arithmetic and loads only
    "ar_hsvonly": [("for (int k = 0; k < 3; ++k) bin_add_runs<true>(cnt[wave][k], lst[0][k], hv[k], pos);",
                    "for (int k = 0; k < 1; ++k) if ((hv[0] ^ hv[1] ^ hv[2] ^ pos) == 0x7fffffffu) cnt[wave][0][0] = 1;")],
}
