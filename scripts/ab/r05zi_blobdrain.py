# round-5 cost-only variant of blob_chroma_meta_kernel: no partial drain at
# each item's end (the item's counts then miss its queued words -- results
# wrong, timing only): what the per-item final drain costs
FILE = "trik_hsv_chroma.hip"
VARIANTS = {
    "bd_base": [("kMaxBlock = 1024;", "kMaxBlock = 1024;")],
    "bd_nofinal": [("""    while (qn > 0) drain(qn < 64 ? qn : 64);
    __builtin_amdgcn_wave_barrier();
    const uint32_t extra = *(lds32_t)(uintptr_t)my_counts;""",
                    """    if (qn > 64) drain(64);
    __builtin_amdgcn_wave_barrier();
    const uint32_t extra = *(lds32_t)(uintptr_t)my_counts;""")],
}
